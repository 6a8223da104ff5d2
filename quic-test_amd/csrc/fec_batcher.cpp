// fec_batcher.cpp — process-wide, deadline-bounded batching of FEC groups (SURVEY.md §8(f)
// item 1; include/fec_hip.h "batcher").
//
// The reference encodes one group per cgo call: every QUIC stream owns a HybridFECEncoder
// and calls EncodeBatch with a single group on its 10th packet (encoder_hybrid.go:71-73,
// :115), at --rate packets/s per stream (main.go:32, client.go:1140-1143).  A GPU launch per
// group costs ~15 us against ~0.6 us for the reference's AVX2 loop, so the GPU only pays with
// many groups per launch.  A batcher is shared by every stream of the process: a stream
// submits a finished group and gets a ticket; the batch is encoded when `max_groups` groups
// are pending OR `deadline_us` has passed since the oldest pending group arrived, whichever
// comes first, so no repair waits longer than the deadline plus one encode.
//
// Memory: a ring of `slabs` page-locked slabs (fec_alloc_slab), each max_groups groups of k
// slots of `slot_bytes`, plus its parity; the kernels read and write them in place over PCIe
// (the zero-copy path of fec_encode_batch_rs), so a batch costs one launch and one
// synchronize.  While one slab is being encoded the next one fills.  When every slab is busy,
// submitters wait (backpressure).
//
// Threads: submitters copy their group into the open slab under the batcher lock; one
// flusher thread per batcher closes slabs (full or deadline), encodes them on the batcher's
// own context and publishes every group's r repair payloads (maxLen bytes each, the group's
// longest packet, as the reference's repair length, encoder_hybrid.go:91-98) under its ticket.
// fec_batcher_wait hands a ticket's payloads to the caller and forgets them.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "fec_hip.h"

#define QFEC_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

using Clock = std::chrono::steady_clock;

struct GroupMeta {
  int64_t ticket;
  uint32_t count;    // packets in the group (slots count..k-1 are zero)
  uint32_t max_len;  // longest packet: the repair payload length
  Clock::time_point t_submit;
};

struct Slab {
  uint8_t* data = nullptr;    // max_groups * k * slot, page-locked
  uint8_t* parity = nullptr;  // max_groups * r * slot, page-locked
  std::vector<GroupMeta> groups;
};

struct Result {
  int rc = FEC_OK;
  uint32_t len = 0;
  std::vector<uint8_t> bytes;  // r rows of len bytes
  std::string err;             // the failed batch's message
};

}  // namespace

struct FECBatcher {
  uint32_t k = 0, r = 0, slot = 0, max_groups = 0;
  std::chrono::microseconds deadline{0};
  FECEncoderCtx* ctx = nullptr;
  std::vector<Slab> slabs;
  int open = -1;                 // slab accepting groups, -1 while every slab is busy
  std::deque<int> free_slabs;    // empty slabs
  std::deque<int> closed;        // full or due slabs waiting for the flusher
  int64_t next_ticket = 0;
  std::unordered_map<int64_t, Result> results;
  FECBatcherStats stats{};
  bool stop = false;
  std::mutex mu;
  std::condition_variable cv_flusher, cv_done, cv_free;
  std::thread flusher;

  ~FECBatcher() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv_flusher.notify_all();
    if (flusher.joinable()) flusher.join();
    for (auto& s : slabs) {
      if (s.data) fec_free_slab(s.data);
      if (s.parity) fec_free_repair_buffer(s.parity);
    }
    if (ctx) fec_encoder_free(ctx);
  }

  // Moves the open slab to the flusher's queue and opens the next free one (or none).
  // Caller holds mu.
  void close_open(bool full) {
    if (open < 0 || slabs[open].groups.empty()) return;
    closed.push_back(open);
    ++(full ? stats.full_flushes : stats.deadline_flushes);
    if (!free_slabs.empty()) {
      open = free_slabs.front();
      free_slabs.pop_front();
    } else {
      open = -1;
    }
  }

  void encode_slab(int si) {
    Slab& s = slabs[si];
    const uint32_t n = static_cast<uint32_t>(s.groups.size());
    const int rc = fec_encode_batch_rs(ctx, s.data, nullptr, n, k, r, slot, s.parity);
    std::string err;
    if (rc != FEC_OK) {
      char buf[512];
      fec_ctx_last_error(ctx, buf, sizeof(buf));
      err = buf;
    }
    // Repair payloads out of the slab (so it can be refilled at once), outside the lock.
    std::vector<std::pair<int64_t, Result>> out(n);
    for (uint32_t g = 0; g < n; ++g) {
      const GroupMeta& m = s.groups[g];
      Result& res = out[g].second;
      out[g].first = m.ticket;
      res.rc = rc;
      if (rc != FEC_OK) {
        res.err = err;
        continue;
      }
      res.len = m.max_len;
      res.bytes.resize(size_t(r) * m.max_len);
      for (uint32_t i = 0; i < r; ++i)
        std::memcpy(res.bytes.data() + size_t(i) * m.max_len, s.parity + (size_t(g) * r + i) * slot, m.max_len);
    }
    std::lock_guard<std::mutex> lk(mu);
    for (auto& kv : out) results.emplace(kv.first, std::move(kv.second));
    ++stats.batches;
    stats.groups += n;
    if (n > stats.max_batch) stats.max_batch = n;
    s.groups.clear();
    if (open < 0) {
      open = si;
    } else {
      free_slabs.push_back(si);
    }
    cv_free.notify_all();
    cv_done.notify_all();
  }

  void run() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      if (!closed.empty()) {
        const int si = closed.front();
        closed.pop_front();
        lk.unlock();
        encode_slab(si);
        lk.lock();
        continue;
      }
      const bool pending = open >= 0 && !slabs[open].groups.empty();
      if (stop) {
        if (!pending) return;
        close_open(false);  // shutdown: encode what is pending, then leave
        continue;
      }
      if (pending) {
        const Clock::time_point due = slabs[open].groups.front().t_submit + deadline;
        if (Clock::now() >= due) {
          close_open(false);
          continue;
        }
        cv_flusher.wait_until(lk, due);
      } else {
        cv_flusher.wait(lk);
      }
    }
  }
};

namespace {

thread_local std::string g_batcher_error;

void berr(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_batcher_error = buf;
}

}  // namespace

QFEC_EXPORT FECBatcher* fec_batcher_new(int device, uint32_t k, uint32_t r, uint32_t slot_bytes, uint32_t max_groups,
                                        uint32_t deadline_us, uint32_t slabs) {
  if (k == 0 || r == 0 || k + r > 256 || slot_bytes == 0 || max_groups == 0) {
    berr("fec_batcher_new: unsupported k=%u r=%u slot=%u max_groups=%u", k, r, slot_bytes, max_groups);
    return nullptr;
  }
  auto* b = new FECBatcher();
  b->k = k;
  b->r = r;
  b->slot = slot_bytes;
  b->max_groups = max_groups;
  b->deadline = std::chrono::microseconds(deadline_us);
  b->ctx = device < 0 ? fec_encoder_new(0.10, max_groups) : fec_encoder_new_device(0.10, max_groups, device);
  if (!b->ctx) {
    berr("fec_batcher_new: %s", fec_hip_last_error());
    delete b;
    return nullptr;
  }
  const uint32_t nslabs = slabs < 2 ? 2 : slabs;
  b->slabs.resize(nslabs);
  for (uint32_t i = 0; i < nslabs; ++i) {
    Slab& s = b->slabs[i];
    s.data = static_cast<uint8_t*>(fec_alloc_slab(size_t(max_groups) * k * slot_bytes));
    s.parity = static_cast<uint8_t*>(fec_alloc_repair_buffer(size_t(max_groups) * r * slot_bytes));
    if (!s.data || !s.parity) {
      berr("fec_batcher_new: page-locked slab allocation failed (%s)", fec_hip_last_error());
      delete b;
      return nullptr;
    }
    s.groups.reserve(max_groups);
    if (i > 0) b->free_slabs.push_back(static_cast<int>(i));
  }
  b->open = 0;
  b->flusher = std::thread([b] { b->run(); });
  return b;
}

QFEC_EXPORT void fec_batcher_free(FECBatcher* b) { delete b; }

QFEC_EXPORT int64_t fec_batcher_submit(FECBatcher* b, const uint8_t* packed, const uint32_t* lens, uint32_t count) {
  if (!b || !lens || (!packed && count > 0)) return FEC_ERR_NULL;
  if (count == 0 || count > b->k) {
    berr("fec_batcher_submit: %u packets (group size k=%u)", count, b->k);
    return FEC_ERR_RANGE;
  }
  uint32_t max_len = 0;
  for (uint32_t j = 0; j < count; ++j) {
    if (lens[j] > b->slot) {
      berr("fec_batcher_submit: packet of %u bytes exceeds the %u-byte slot", lens[j], b->slot);
      return FEC_ERR_RANGE;
    }
    max_len = std::max(max_len, lens[j]);
  }
  if (max_len == 0) {  // encoder_hybrid.go:95-97
    berr("fec_batcher_submit: empty packets");
    return FEC_ERR_RANGE;
  }
  std::unique_lock<std::mutex> lk(b->mu);
  b->cv_free.wait(lk, [b] { return b->open >= 0 || b->stop; });
  if (b->stop) return FEC_ERR_RANGE;
  Slab& s = b->slabs[b->open];
  const size_t g = s.groups.size();
  uint8_t* dst = s.data + g * b->k * size_t(b->slot);
  const uint8_t* src = packed;
  for (uint32_t j = 0; j < b->k; ++j) {  // packets zero-padded to the slot, absent slots zero
    uint8_t* d = dst + size_t(j) * b->slot;
    const uint32_t n = j < count ? lens[j] : 0;
    if (n) std::memcpy(d, src, n);
    std::memset(d + n, 0, b->slot - n);
    src += n;
  }
  const int64_t ticket = b->next_ticket++;
  s.groups.push_back(GroupMeta{ticket, count, max_len, Clock::now()});
  if (s.groups.size() == b->max_groups) {
    b->close_open(true);
    b->cv_flusher.notify_one();
  } else if (g == 0) {
    b->cv_flusher.notify_one();  // a deadline starts
  }
  return ticket;
}

QFEC_EXPORT int fec_batcher_wait(FECBatcher* b, int64_t ticket, uint8_t* out, uint32_t out_stride, int64_t timeout_us) {
  if (!b) return FEC_ERR_NULL;
  std::unique_lock<std::mutex> lk(b->mu);
  if (ticket < 0 || ticket >= b->next_ticket) {
    berr("fec_batcher_wait: unknown ticket %lld", static_cast<long long>(ticket));
    return FEC_ERR_RANGE;
  }
  auto ready = [&] { return b->results.count(ticket) != 0; };
  if (timeout_us < 0) {
    b->cv_done.wait(lk, ready);
  } else if (!b->cv_done.wait_for(lk, std::chrono::microseconds(timeout_us), ready)) {
    return FEC_ERR_AGAIN;
  }
  auto it = b->results.find(ticket);
  Result res = std::move(it->second);
  b->results.erase(it);
  lk.unlock();
  if (res.rc != FEC_OK) {
    berr("fec_batcher_wait: the batch of ticket %lld failed with code %d: %s", static_cast<long long>(ticket), res.rc,
         res.err.c_str());
    return res.rc;
  }
  if (out) {
    if (out_stride < res.len) {
      berr("fec_batcher_wait: out_stride %u < repair length %u", out_stride, res.len);
      return FEC_ERR_RANGE;
    }
    for (uint32_t i = 0; i < b->r; ++i)
      std::memcpy(out + size_t(i) * out_stride, res.bytes.data() + size_t(i) * res.len, res.len);
  }
  return static_cast<int>(res.len);
}

QFEC_EXPORT int fec_batcher_flush(FECBatcher* b) {
  if (!b) return FEC_ERR_NULL;
  {
    std::lock_guard<std::mutex> lk(b->mu);
    b->close_open(false);
  }
  b->cv_flusher.notify_one();
  return FEC_OK;
}

QFEC_EXPORT int fec_batcher_stats(FECBatcher* b, FECBatcherStats* out) {
  if (!b || !out) return FEC_ERR_NULL;
  std::lock_guard<std::mutex> lk(b->mu);
  *out = b->stats;
  return FEC_OK;
}

QFEC_EXPORT const char* fec_batcher_last_error(void) { return g_batcher_error.c_str(); }
