// fec_batcher.cpp — process-wide, deadline-bounded batching of FEC groups (SURVEY.md §8(f)
// item 1; include/fec_hip.h "batcher").
//
// The reference encodes one group per cgo call: every QUIC stream owns a HybridFECEncoder
// and calls EncodeBatch with a single group on its 10th packet (encoder_hybrid.go:71-73,
// :115), at --rate packets/s per stream (main.go:32, client.go:1140-1143).  A GPU launch per
// group costs ~15 us against well under a microsecond for the reference's AVX2 loop, so the
// GPU only pays with many groups per launch.  A batcher is shared by every stream of the
// process: a stream submits a finished group and gets a ticket; the batch is encoded when
// `max_groups` groups are pending OR `deadline_us` has passed since the oldest pending group
// arrived, whichever comes first, so no repair waits longer than the deadline plus one encode.
//
// Memory: a ring of `slabs` page-locked slabs (fec_alloc_slab), each max_groups groups of k
// slots of `slot_bytes`, plus its parity; the kernels read and write them in place over PCIe
// (the zero-copy path of fec_encode_batch_rs), so a batch costs one launch and one
// synchronize.  While one slab is being encoded the next ones fill.  When every slab is busy,
// submitters wait (backpressure).
//
// Threads.  A submitter reserves its group's slot under the batcher lock and copies the
// packets in after releasing it, so streams copy in parallel; the slab is encoded once every
// reserved copy has landed.  One flusher thread per batcher closes slabs (full or due),
// encodes them on the batcher's own context and publishes each group's r repair payloads
// (maxLen bytes each, the group's longest packet: the reference's repair length,
// encoder_hybrid.go:91-98) into a ring of result entries indexed by ticket, which waiters read
// without the lock.  A result not collected before 2 * slabs * max_groups newer groups are
// published is dropped (the late wait gets FEC_ERR_RANGE; stats.expired counts them).
#include <hip/hip_runtime.h>
#include <sys/prctl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
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
  uint8_t* d_data = nullptr;  // the same memory as the kernels address it (zero-copy)
  uint8_t* d_parity = nullptr;
  hipEvent_t done = nullptr;  // the slab's encode has finished
  int rc = FEC_OK;            // its launch status
  std::vector<GroupMeta> groups;         // reserved groups (under the batcher lock)
  std::atomic<uint32_t> committed{0};    // groups whose packets have been copied in
};

// One published result.  `ticket` is -1 while the entry is being (re)written, else the
// ticket whose payloads it holds; a reader copies, then re-checks `ticket` (a rewrite in
// between makes the copy invalid) and claims it by swapping in -1.
struct Entry {
  std::atomic<int64_t> ticket{-1};
  int rc = FEC_OK;
  uint32_t len = 0;
  std::vector<uint8_t> bytes;  // r rows of len bytes
};

}  // namespace

struct FECBatcher {
  uint32_t k = 0, r = 0, slot = 0, max_groups = 0;
  std::chrono::microseconds deadline{0};
  FECEncoderCtx* ctx = nullptr;
  std::vector<std::unique_ptr<Slab>> slabs;
  int open = -1;                 // slab accepting groups, -1 while every slab is busy
  std::deque<int> free_slabs;    // empty slabs
  std::deque<int> closed;        // full or due slabs waiting for the flusher
  std::deque<int> in_flight;     // encodes launched, results not yet published (launch order)
  int device = 0;
  hipStream_t stream = nullptr;  // the flusher's launches
  std::atomic<int64_t> next_ticket{0};
  std::atomic<int64_t> published_upto{0};  // every ticket below this has been published (in order)
  std::vector<Entry> ring;       // results, entry ticket % ring.size()
  FECBatcherStats stats{};
  std::string last_batch_error;  // message of the last failed batch (under mu)
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
      if (s->data) fec_free_slab(s->data);
      if (s->parity) fec_free_repair_buffer(s->parity);
      if (s->done) (void)hipEventDestroy(s->done);
    }
    if (stream) (void)hipStreamDestroy(stream);
    if (ctx) fec_encoder_free(ctx);
  }

  // Moves the open slab to the flusher's queue and opens the next free one (or none).
  // Caller holds mu.
  void close_open(bool full) {
    if (open < 0 || slabs[open]->groups.empty()) return;
    closed.push_back(open);
    ++(full ? stats.full_flushes : stats.deadline_flushes);
    if (!free_slabs.empty()) {
      open = free_slabs.front();
      free_slabs.pop_front();
    } else {
      open = -1;
    }
  }

  // Stage 1 (flusher, no lock): once every reserved copy has landed, launch the slab's
  // encode asynchronously on the batcher's stream (the kernels read the page-locked slab
  // and write its parity in place over PCIe) and record its completion event.
  void launch_slab(int si) {
    Slab& s = *slabs[si];
    const uint32_t n = static_cast<uint32_t>(s.groups.size());  // closed: no more reservations
    while (s.committed.load(std::memory_order_acquire) < n) std::this_thread::yield();  // copies in flight
    s.rc = fec_encode_batch_rs_dev(ctx, s.d_data, n, k, r, slot, s.d_parity, stream);
    if (s.rc == FEC_OK && hipEventRecord(s.done, stream) != hipSuccess) s.rc = FEC_ERR_HIP;
  }

  // Stage 2 (flusher, no lock until the end): wait for the slab's encode, copy every group's
  // payloads into the result ring, then hand the slab back for refilling.  While the flusher
  // waits here, the next slab's encode is already queued behind this one (stage 1 runs first
  // whenever a slab is closed), so the GPU never waits for the copies.
  void publish_slab(int si) {
    Slab& s = *slabs[si];
    const uint32_t n = static_cast<uint32_t>(s.groups.size());
    int rc = s.rc;
    if (rc == FEC_OK && hipEventSynchronize(s.done) != hipSuccess) rc = FEC_ERR_HIP;
    std::string err;
    if (rc != FEC_OK) {
      char buf[512];
      fec_ctx_last_error(ctx, buf, sizeof(buf));
      err = buf[0] ? buf : "the batch's encode failed on the device";
    }
    for (uint32_t g = 0; g < n; ++g) {
      const GroupMeta& m = s.groups[g];
      Entry& e = ring[static_cast<size_t>(m.ticket) % ring.size()];
      const int64_t prev = e.ticket.exchange(-1, std::memory_order_acq_rel);
      if (prev >= 0) ++dropped;  // never collected: dropped
      e.rc = rc;
      e.len = rc == FEC_OK ? m.max_len : 0;
      e.bytes.resize(size_t(r) * e.len);
      for (uint32_t i = 0; i < r && rc == FEC_OK; ++i)
        std::memcpy(e.bytes.data() + size_t(i) * e.len, s.parity + (size_t(g) * r + i) * slot, e.len);
      e.ticket.store(m.ticket, std::memory_order_release);
    }
    std::lock_guard<std::mutex> lk(mu);
    ++stats.batches;
    stats.groups += n;
    if (n > stats.max_batch) stats.max_batch = n;
    stats.expired += dropped;
    dropped = 0;
    if (n > 0) published_upto.store(s.groups.back().ticket + 1, std::memory_order_release);
    if (rc != FEC_OK) last_batch_error = err;
    s.groups.clear();
    s.committed.store(0, std::memory_order_relaxed);
    if (open < 0) {
      open = si;
    } else {
      free_slabs.push_back(si);
    }
    cv_free.notify_all();
    cv_done.notify_all();
  }

  void run() {
    // Wake at the deadline itself, not up to the default 50 us timer slack later.
    prctl(PR_SET_TIMERSLACK, 1UL, 0, 0, 0);
    (void)hipSetDevice(device);  // the events and stream live on the batcher's device
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      if (!closed.empty()) {  // launch first: keep the GPU busy while results are copied
        const int si = closed.front();
        closed.pop_front();
        in_flight.push_back(si);
        lk.unlock();
        launch_slab(si);
        lk.lock();
        continue;
      }
      if (!in_flight.empty()) {
        const int si = in_flight.front();
        in_flight.pop_front();
        lk.unlock();
        publish_slab(si);
        lk.lock();
        continue;
      }
      const bool pending = open >= 0 && !slabs[open]->groups.empty();
      if (stop) {
        if (!pending) return;
        close_open(false);  // shutdown: encode what is pending, then leave
        continue;
      }
      if (pending) {
        const Clock::time_point due = slabs[open]->groups.front().t_submit + deadline;
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

  uint64_t dropped = 0;  // flusher only
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
  b->device = fec_encoder_device(b->ctx);
  int prev_dev = -1;
  (void)hipGetDevice(&prev_dev);
  auto restore = [&] {
    if (prev_dev >= 0) (void)hipSetDevice(prev_dev);
  };
  if (hipSetDevice(b->device) != hipSuccess ||
      hipStreamCreateWithFlags(&b->stream, hipStreamNonBlocking) != hipSuccess) {
    berr("fec_batcher_new: cannot create a stream on device %d", b->device);
    restore();
    delete b;
    return nullptr;
  }
  const uint32_t nslabs = slabs < 2 ? 2 : slabs;
  for (uint32_t i = 0; i < nslabs; ++i) {
    b->slabs.push_back(std::make_unique<Slab>());
    Slab& s = *b->slabs.back();
    s.data = static_cast<uint8_t*>(fec_alloc_slab(size_t(max_groups) * k * slot_bytes));
    s.parity = static_cast<uint8_t*>(fec_alloc_repair_buffer(size_t(max_groups) * r * slot_bytes));
    void *dd = nullptr, *dp = nullptr;
    if (!s.data || !s.parity || hipHostGetDevicePointer(&dd, s.data, 0) != hipSuccess ||
        hipHostGetDevicePointer(&dp, s.parity, 0) != hipSuccess ||
        hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess) {
      berr("fec_batcher_new: page-locked slab setup failed (%s)", fec_hip_last_error());
      restore();
      delete b;
      return nullptr;
    }
    s.d_data = static_cast<uint8_t*>(dd);
    s.d_parity = static_cast<uint8_t*>(dp);
    s.groups.reserve(max_groups);
    if (i > 0) b->free_slabs.push_back(static_cast<int>(i));
  }
  // Results of two full rounds of slabs stay collectable.
  b->ring = std::vector<Entry>(size_t(2) * nslabs * max_groups);
  // Warm-up: the first launch loads the code object and the (k, r) tables; do it here, not
  // in the first stream's repair delay.
  std::memset(b->slabs[0]->data, 0, size_t(k) * slot_bytes);
  if (fec_encode_batch_rs(b->ctx, b->slabs[0]->data, nullptr, 1, k, r, slot_bytes, b->slabs[0]->parity) != FEC_OK) {
    char buf[512];
    fec_ctx_last_error(b->ctx, buf, sizeof(buf));
    berr("fec_batcher_new: warm-up encode failed: %s", buf);
    restore();
    delete b;
    return nullptr;
  }
  restore();
  b->open = 0;
  b->flusher = std::thread([b] { b->run(); });
  return b;
}

QFEC_EXPORT void fec_batcher_free(FECBatcher* b) { delete b; }

namespace {

// Shared by both submit forms: packet j is at src(j).
template <class Src>
int64_t submit_group(FECBatcher* b, Src&& src, const uint32_t* lens, uint32_t count) {
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
    if (lens[j] > 0 && src(j) == nullptr) return FEC_ERR_NULL;
    max_len = std::max(max_len, lens[j]);
  }
  if (max_len == 0) {  // encoder_hybrid.go:95-97
    berr("fec_batcher_submit: empty packets");
    return FEC_ERR_RANGE;
  }
  // Reserve the slot under the lock ...
  Slab* s = nullptr;
  size_t g = 0;
  int64_t ticket = 0;
  {
    std::unique_lock<std::mutex> lk(b->mu);
    b->cv_free.wait(lk, [b] { return b->open >= 0 || b->stop; });
    if (b->stop) return FEC_ERR_RANGE;
    s = b->slabs[b->open].get();
    g = s->groups.size();
    ticket = b->next_ticket.fetch_add(1, std::memory_order_relaxed);
    s->groups.push_back(GroupMeta{ticket, count, max_len, Clock::now()});
    if (s->groups.size() == b->max_groups) {
      b->close_open(true);
      b->cv_flusher.notify_one();
    } else if (g == 0) {
      b->cv_flusher.notify_one();  // a deadline starts
    }
  }
  // ... and copy without it (the flusher encodes a slab once every reserved copy landed).
  uint8_t* dst = s->data + g * b->k * size_t(b->slot);
  for (uint32_t j = 0; j < b->k; ++j) {  // packets zero-padded to the slot, absent slots zero
    uint8_t* d = dst + size_t(j) * b->slot;
    const uint32_t n = j < count ? lens[j] : 0;
    if (n) std::memcpy(d, src(j), n);
    std::memset(d + n, 0, b->slot - n);
  }
  s->committed.fetch_add(1, std::memory_order_release);
  return ticket;
}

}  // namespace

QFEC_EXPORT int64_t fec_batcher_submit(FECBatcher* b, const uint8_t* packed, const uint32_t* lens, uint32_t count) {
  if (!b || !lens || (!packed && count > 0)) return FEC_ERR_NULL;
  // packed back to back: prefix sums of the lengths
  uint64_t offs[256];
  uint64_t o = 0;
  for (uint32_t j = 0; j < count && j < 256; ++j) {
    offs[j] = o;
    o += lens[j];
  }
  return submit_group(b, [&](uint32_t j) { return packed + offs[j]; }, lens, count);
}

QFEC_EXPORT int64_t fec_batcher_submit_packets(FECBatcher* b, const uint8_t* const* packets, const uint32_t* lens,
                                               uint32_t count) {
  if (!b || !lens || (!packets && count > 0)) return FEC_ERR_NULL;
  return submit_group(b, [&](uint32_t j) { return packets[j]; }, lens, count);
}

namespace {

// Copies a published result out of the ring and claims it: 1 done, 0 not published yet,
// negative code on failure.  *len = payload length.
int take(FECBatcher* b, int64_t ticket, uint8_t* out, uint32_t out_stride, int* len) {
  Entry& e = b->ring[static_cast<size_t>(ticket) % b->ring.size()];
  if (e.ticket.load(std::memory_order_acquire) != ticket) return 0;
  const int rc = e.rc;
  const uint32_t n = e.len;
  if (rc == FEC_OK && out) {
    if (out_stride < n) {
      berr("fec_batcher_wait: out_stride %u < repair length %u", out_stride, n);
      return FEC_ERR_RANGE;
    }
    for (uint32_t i = 0; i < b->r; ++i) std::memcpy(out + size_t(i) * out_stride, e.bytes.data() + size_t(i) * n, n);
  }
  int64_t expect = ticket;
  if (!e.ticket.compare_exchange_strong(expect, -1, std::memory_order_acq_rel)) {
    berr("fec_batcher_wait: result of ticket %lld was overwritten while read", static_cast<long long>(ticket));
    return FEC_ERR_RANGE;
  }
  if (rc != FEC_OK) {
    std::lock_guard<std::mutex> lk(b->mu);
    berr("fec_batcher_wait: the batch of ticket %lld failed with code %d: %s", static_cast<long long>(ticket), rc,
         b->last_batch_error.c_str());
    return rc;
  }
  *len = static_cast<int>(n);
  return 1;
}

}  // namespace

QFEC_EXPORT int fec_batcher_wait(FECBatcher* b, int64_t ticket, uint8_t* out, uint32_t out_stride, int64_t timeout_us) {
  if (!b) return FEC_ERR_NULL;
  int len = 0;
  int st = ticket >= 0 ? take(b, ticket, out, out_stride, &len) : 0;
  if (st == 1) return len;
  if (st < 0) return st;
  // A poll of a ticket not published yet needs no lock.
  if (timeout_us == 0 && ticket >= b->published_upto.load(std::memory_order_acquire) &&
      ticket < b->next_ticket.load(std::memory_order_relaxed))
    return FEC_ERR_AGAIN;
  std::unique_lock<std::mutex> lk(b->mu);
  if (ticket < 0 || ticket >= b->next_ticket.load(std::memory_order_relaxed)) {
    berr("fec_batcher_wait: unknown ticket %lld", static_cast<long long>(ticket));
    return FEC_ERR_RANGE;
  }
  // Results are published between a batch's ring writes and its cv_done signal (under mu),
  // in ticket order, so checking under mu and waiting on cv_done misses none.
  const auto until = Clock::now() + std::chrono::microseconds(timeout_us > 0 ? timeout_us : 0);
  Entry& e = b->ring[static_cast<size_t>(ticket) % b->ring.size()];
  for (;;) {
    if (e.ticket.load(std::memory_order_acquire) == ticket) break;
    if (ticket < b->published_upto.load(std::memory_order_acquire)) {
      berr("fec_batcher_wait: ticket %lld was already collected or its result expired (more than %zu newer "
           "groups encoded)", static_cast<long long>(ticket), b->ring.size());
      return FEC_ERR_RANGE;
    }
    if (timeout_us < 0) {
      b->cv_done.wait(lk);
    } else if (timeout_us == 0 || b->cv_done.wait_until(lk, until) == std::cv_status::timeout) {
      if (e.ticket.load(std::memory_order_acquire) == ticket) break;
      return FEC_ERR_AGAIN;
    }
  }
  lk.unlock();
  st = take(b, ticket, out, out_stride, &len);
  if (st == 1) return len;
  if (st == 0) {
    berr("fec_batcher_wait: ticket %lld was already collected", static_cast<long long>(ticket));
    return FEC_ERR_RANGE;
  }
  return st;
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
