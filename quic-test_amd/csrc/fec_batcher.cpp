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
// slots of `slot_bytes`, and one page-locked parity ring of C = 3 * slabs * max_groups group
// slots (r * slot_bytes each; ticket t's parity sits in slot t % C); the kernels read a slab
// and write its groups' parity slots in place over PCIe (the zero-copy path of
// fec_encode_batch_rs), so a batch costs one launch (two where it wraps the ring) and one
// synchronize.  While one slab is being encoded the next ones fill.  When every slab is
// busy, submitters wait (backpressure).
//
// Threads.  A submitter reserves its group's slot with one atomic add on the open slab's
// reservation word (no lock: the global lock serialised 16 saturating streams), copies the
// packets in, and counts itself committed; the slab is encoded once every reserved copy has
// landed.  The lock is taken only by a slab's first group (its deadline starts), by the group
// that fills it, and while every slab is busy.  One flusher thread per batcher closes slabs (full or due),
// encodes them on the batcher's own context and publishes each group's result (where its r
// repair payloads of maxLen bytes sit -- the group's longest packet: the reference's repair
// length, encoder_hybrid.go:91-98) into a ring of C entries indexed by ticket.  Waiters copy
// the payloads straight out of the parity ring without the lock and then check that no encode
// covering ticket + C has been launched meanwhile (a seqlock on `launched_upto`), so the
// flusher copies nothing per group.  A result not collected before C newer groups are
// launched (at least 2 * slabs * max_groups newer groups encoded) is dropped: the late wait
// gets FEC_ERR_RANGE and stats.expired counts it.
//
// Decoder batchers (fec_batcher_new_decoder) do the same for the receiving side, whose
// FECDecoder rebuilds one group per call (decoder.go:216-287): a connection submits a group's
// received shards (NULL for the lost ones), the slab also holds the received parity rows and
// the erasure masks, the batch runs fec_recover_batch_rs_dev, and the rebuilt data packets
// land in the output ring (ticket t: r slots at t % C) next to a status byte per ticket.
//
// Several GPUs (fec_batcher_new_multi / fec_batcher_new_decoder_multi): one such batcher per
// device, each with its own context, slabs, output ring and flusher, behind one handle.  A
// host-resident batch is bound by its GPU's PCIe link (the kernels read the page-locked slab
// over it), so N devices give N links.  Groups are dealt round robin (skipping a device whose
// slabs are all busy while another has room); ticket t of device i of n is handed out as
// t * n + i, so a wait goes straight to its device.
#include <hip/hip_runtime.h>
#include <sys/prctl.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
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
  uint32_t count;    // packets in the group (slots count..k-1 are zero); decoder: unused
  uint32_t max_len;  // longest packet: the repair payload length; decoder: the symbol length
  uint64_t mask;     // decoder: lost shards (bit s = shard s)
};

// Reservation word of a slab: bit 63 set once the slab is closed, the low bits count the
// reservations attempted (they may run past max_groups; those attempts back off).
constexpr uint64_t kClosed = 1ull << 63;

struct Slab {
  uint8_t* data = nullptr;    // max_groups * k * slot, page-locked
  uint8_t* d_data = nullptr;  // the same memory as the kernels address it (zero-copy)
  uint8_t* rparity = nullptr;   // decoder: the received parity rows, max_groups * r * slot
  uint8_t* d_rparity = nullptr;
  uint64_t* masks = nullptr;    // decoder: erasure masks, max_groups
  uint64_t* d_masks = nullptr;
  hipEvent_t done = nullptr;  // the slab's encode has finished
  int rc = FEC_OK;            // its launch status
  std::vector<GroupMeta> groups;       // max_groups entries; entry g written by its submitter
  std::atomic<uint64_t> state{kClosed};
  int64_t base = 0;                    // ticket of entry 0 (set when the slab opens)
  uint32_t n = 0;                      // groups in the batch (set when it closes)
  bool started = false;                // its first group arrived (under mu)
  Clock::time_point t_first;           // when (under mu): the deadline runs from here
  std::atomic<uint32_t> committed{0};  // groups whose packets have been copied in
};

// One published result.  `ticket` is -1 while the entry is being (re)written, else the
// ticket whose result it describes (r rows of `len` bytes in the ticket's parity slot).  A
// reader copies, checks the slot was not rewritten meanwhile, and claims the result by
// swapping in -1.
// The fields are atomics (relaxed; `ticket` orders them) because a late reader may still load
// them while the flusher rewrites the entry for ticket + C; its ticket re-check discards
// what it read then.
struct Entry {
  std::atomic<int64_t> ticket{-1};
  std::atomic<int> rc{FEC_OK};
  std::atomic<uint32_t> len{0};
  std::atomic<uint64_t> mask{0};  // decoder: the group's lost shards
};

}  // namespace

struct FECBatcher {
  uint32_t k = 0, r = 0, slot = 0, max_groups = 0;
  bool decoder = false;
  std::chrono::microseconds deadline{0};
  FECEncoderCtx* ctx = nullptr;
  std::vector<std::unique_ptr<Slab>> slabs;
  uint8_t* parity = nullptr;     // the output ring: C group slots of r * slot bytes, page-locked
  uint8_t* d_parity = nullptr;   // as the kernels address it (encoder: parity; decoder: rebuilt)
  uint8_t* status = nullptr;     // decoder: a status byte per ring slot (1 = unrecoverable)
  uint8_t* d_status = nullptr;
  uint64_t cap = 0;              // C
  std::atomic<int64_t> launched_upto{0};  // encodes of every ticket below this have been launched
  std::atomic<int> open{-1};     // slab accepting groups, -1 while every slab is busy (written under mu)
  int64_t next_base = 0;         // ticket of the next slab's first group while none is open (under mu)
  std::deque<int> free_slabs;    // empty slabs
  std::deque<int> closed;        // full or due slabs waiting for the flusher
  std::deque<int> in_flight;     // encodes launched, results not yet published (launch order)
  int device = 0;
  hipStream_t stream = nullptr;  // the flusher's launches
  std::atomic<int64_t> published_upto{0};  // every ticket below this has been published (in order)
  std::vector<Entry> ring;       // results, entry ticket % ring.size()
  FECBatcherStats stats{};
  std::string last_batch_error;  // message of the last failed batch (under mu)
  bool stop = false;
  std::mutex mu;
  std::condition_variable cv_flusher, cv_done, cv_free;
  std::thread flusher;
  // Multi-device handle: the per-device batchers (everything above is unused then).
  std::vector<FECBatcher*> parts;
  std::atomic<uint64_t> rr{0};

  ~FECBatcher() {
    for (FECBatcher* p : parts) delete p;
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv_flusher.notify_all();
    if (flusher.joinable()) flusher.join();
    for (auto& s : slabs) {
      if (s->data) fec_free_slab(s->data);
      if (s->rparity) fec_free_slab(s->rparity);
      if (s->masks) fec_free_slab(s->masks);
      if (s->done) (void)hipEventDestroy(s->done);
    }
    if (parity) fec_free_repair_buffer(parity);
    if (status) fec_free_slab(status);
    if (stream) (void)hipStreamDestroy(stream);
    if (ctx) fec_encoder_free(ctx);
  }

  // Opens slab si for reservations; its tickets continue the previous batch's.  Caller holds mu.
  void open_slab(int si) {
    Slab& s = *slabs[si];
    s.base = next_base;
    s.n = 0;
    s.started = false;
    s.committed.store(0, std::memory_order_relaxed);
    s.state.store(0, std::memory_order_release);
    open.store(si, std::memory_order_release);
    cv_free.notify_all();
  }

  // Closes the open slab (if it has groups), queues it for the flusher and opens the next
  // free one (or none).  Caller holds mu.
  void close_open(bool full) {
    const int si = open.load(std::memory_order_relaxed);
    if (si < 0) return;
    Slab& s = *slabs[si];
    // A slab closes once its first group has started the deadline or, when full, as soon as
    // every slot is reserved: the first reserver records its start under mu only after its
    // lock-free reservation, and a full slab must not wait out the deadline meanwhile.
    if (!s.started && !(full && (s.state.load(std::memory_order_acquire) & ~kClosed) >= max_groups)) return;
    const uint64_t old = s.state.fetch_or(kClosed, std::memory_order_acq_rel);
    s.n = static_cast<uint32_t>(std::min<uint64_t>(old & ~kClosed, max_groups));
    next_base = s.base + s.n;
    closed.push_back(si);
    ++(full ? stats.full_flushes : stats.deadline_flushes);
    if (!free_slabs.empty()) {
      const int nx = free_slabs.front();
      free_slabs.pop_front();
      open_slab(nx);
    } else {
      open.store(-1, std::memory_order_release);
    }
  }

  // Every ticket below this has been handed out (or is being).  Caller holds mu.
  int64_t issued_bound() const {
    const int si = open.load(std::memory_order_relaxed);
    if (si < 0) return next_base;
    const Slab& s = *slabs[si];
    return s.base + static_cast<int64_t>(std::min<uint64_t>(s.state.load(std::memory_order_acquire) & ~kClosed, max_groups));
  }

  // Stage 1 (flusher, no lock): once every reserved copy has landed, launch the slab's
  // encode asynchronously on the batcher's stream (the kernels read the page-locked slab and
  // write its groups' parity slots in place over PCIe; a slab's tickets are consecutive, so
  // that is one range of the ring, split in two where it wraps) and record its completion
  // event.  `launched_upto` moves first: the results of tickets C below expire.
  void launch_slab(int si) {
    Slab& s = *slabs[si];
    const uint32_t n = s.n;  // closed: no more reservations
    while (s.committed.load(std::memory_order_acquire) < n) std::this_thread::yield();  // copies in flight
    const int64_t t0 = s.base;
    launched_upto.store(t0 + n, std::memory_order_relaxed);
    std::atomic_thread_fence(std::memory_order_seq_cst);
    const uint64_t first_slot = static_cast<uint64_t>(t0) % cap;
    const uint32_t n1 = static_cast<uint32_t>(std::min<uint64_t>(n, cap - first_slot));
    const size_t group_parity = size_t(r) * slot;
    auto part = [&](uint32_t g0, uint32_t cnt, uint64_t slot0) {
      if (!decoder)
        return fec_encode_batch_rs_dev(ctx, s.d_data + size_t(g0) * k * slot, cnt, k, r, slot,
                                       d_parity + slot0 * group_parity, stream);
      return fec_recover_batch_rs_dev(ctx, s.d_data + size_t(g0) * k * slot, s.d_rparity + size_t(g0) * r * slot,
                                      s.d_masks + g0, cnt, k, r, slot, d_parity + slot0 * group_parity,
                                      d_status + slot0, stream);
    };
    s.rc = part(0, n1, first_slot);
    if (s.rc == FEC_OK && n1 < n) s.rc = part(n1, n - n1, 0);
    if (s.rc == FEC_OK && hipEventRecord(s.done, stream) != hipSuccess) s.rc = FEC_ERR_HIP;
  }

  // Stage 2 (flusher, no lock until the end): wait for the slab's encode, publish where every
  // group's payloads sit, then hand the slab back for refilling.  While the flusher waits
  // here, the next slab's encode is already queued behind this one (stage 1 runs first
  // whenever a slab is closed).
  void publish_slab(int si) {
    Slab& s = *slabs[si];
    const uint32_t n = s.n;
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
      const int64_t ticket = s.base + g;
      Entry& e = ring[static_cast<size_t>(ticket) % ring.size()];
      const int64_t prev = e.ticket.exchange(-1, std::memory_order_acq_rel);
      if (prev >= 0) ++dropped;  // never collected: dropped
      const bool unrecoverable = decoder && rc == FEC_OK && status[static_cast<uint64_t>(ticket) % cap] != 0;
      e.rc.store(unrecoverable ? FEC_ERR_UNRECOVERABLE : rc, std::memory_order_relaxed);
      e.len.store(rc == FEC_OK ? m.max_len : 0, std::memory_order_relaxed);
      e.mask.store(m.mask, std::memory_order_relaxed);
      e.ticket.store(ticket, std::memory_order_release);
    }
    std::lock_guard<std::mutex> lk(mu);
    ++stats.batches;
    stats.groups += n;
    if (n > stats.max_batch) stats.max_batch = n;
    stats.expired += dropped;
    dropped = 0;
    published_upto.store(s.base + n, std::memory_order_release);
    if (rc != FEC_OK) last_batch_error = err;
    if (open.load(std::memory_order_relaxed) < 0) {
      open_slab(si);
    } else {
      free_slabs.push_back(si);
    }
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
      const int si = open.load(std::memory_order_relaxed);
      const bool pending = si >= 0 && slabs[si]->started;
      if (stop) {
        if (!pending) return;
        close_open(false);  // shutdown: encode what is pending, then leave
        continue;
      }
      if (pending) {
        const Clock::time_point due = slabs[si]->t_first + deadline;
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

namespace {

// Page-locked allocation and its device address (zero-copy); false on failure.
template <class T>
bool alloc_mapped(size_t bytes, T** host, T** dev) {
  *host = static_cast<T*>(fec_alloc_slab(bytes));
  void* d = nullptr;
  if (!*host || hipHostGetDevicePointer(&d, *host, 0) != hipSuccess) return false;
  *dev = static_cast<T*>(d);
  return true;
}

FECBatcher* create(bool decoder, int device, uint32_t k, uint32_t r, uint32_t slot_bytes, uint32_t max_groups,
                   uint32_t deadline_us, uint32_t slabs) {
  const char* fn = decoder ? "fec_batcher_new_decoder" : "fec_batcher_new";
  if (k == 0 || r == 0 || k + r > (decoder ? 64u : 256u) || slot_bytes == 0 || max_groups == 0) {
    berr("%s: unsupported k=%u r=%u slot=%u max_groups=%u", fn, k, r, slot_bytes, max_groups);
    return nullptr;
  }
  auto* b = new FECBatcher();
  b->decoder = decoder;
  b->k = k;
  b->r = r;
  b->slot = slot_bytes;
  b->max_groups = max_groups;
  b->deadline = std::chrono::microseconds(deadline_us);
  b->ctx = device < 0 ? fec_encoder_new(0.10, max_groups) : fec_encoder_new_device(0.10, max_groups, device);
  if (!b->ctx) {
    berr("%s: %s", fn, fec_hip_last_error());
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
    berr("%s: cannot create a stream on device %d", fn, b->device);
    restore();
    delete b;
    return nullptr;
  }
  const uint32_t nslabs = slabs < 2 ? 2 : slabs;
  // QUICFEC_BATCHER_BLOCKING_SYNC=1: the flusher sleeps in its completion waits instead of
  // polling (frees a core, adds wake-up latency; no throughput gain measured,
  // profiles/r02_ab_batcher_blocking_sync.txt, so polling stays the default)
  const char* bs = std::getenv("QUICFEC_BATCHER_BLOCKING_SYNC");
  const bool blocking = bs && bs[0] == '1';
  for (uint32_t i = 0; i < nslabs; ++i) {
    b->slabs.push_back(std::make_unique<Slab>());
    Slab& s = *b->slabs.back();
    bool ok = alloc_mapped(size_t(max_groups) * k * slot_bytes, &s.data, &s.d_data);
    if (decoder)
      ok = ok && alloc_mapped(size_t(max_groups) * r * slot_bytes, &s.rparity, &s.d_rparity) &&
           alloc_mapped(size_t(max_groups) * sizeof(uint64_t), &s.masks, &s.d_masks);
    if (!ok ||
        hipEventCreateWithFlags(&s.done, hipEventDisableTiming | (blocking ? hipEventBlockingSync : 0u)) != hipSuccess) {
      berr("%s: page-locked slab setup failed (%s)", fn, fec_hip_last_error());
      restore();
      delete b;
      return nullptr;
    }
    s.groups.resize(max_groups);
    if (i > 0) b->free_slabs.push_back(static_cast<int>(i));
  }
  // Results of two full rounds of slabs stay collectable: a slot is rewritten when the batch
  // C tickets later is launched, and up to a round of slabs is launched ahead of publishing.
  b->cap = uint64_t(3) * nslabs * max_groups;
  b->parity = static_cast<uint8_t*>(fec_alloc_repair_buffer(b->cap * r * slot_bytes));
  void* dp = nullptr;
  if (!b->parity || hipHostGetDevicePointer(&dp, b->parity, 0) != hipSuccess ||
      (decoder && !alloc_mapped(b->cap, &b->status, &b->d_status))) {
    berr("%s: page-locked output ring setup failed (%s)", fn, fec_hip_last_error());
    restore();
    delete b;
    return nullptr;
  }
  b->d_parity = static_cast<uint8_t*>(dp);
  b->ring = std::vector<Entry>(b->cap);
  // Warm-up: the first launch loads the code object and the (k, r) tables (decoder: the
  // recovery codebook too); do it here, not in the first stream's repair delay.
  Slab& s0 = *b->slabs[0];
  std::memset(s0.data, 0, size_t(k) * slot_bytes);
  int wrc;
  if (!decoder) {
    wrc = fec_encode_batch_rs(b->ctx, s0.data, nullptr, 1, k, r, slot_bytes, b->parity);
  } else {
    std::memset(s0.rparity, 0, size_t(r) * slot_bytes);
    s0.masks[0] = 1;  // shard 0 lost
    wrc = fec_decode_prepare(b->ctx, k, r, nullptr);
    if (wrc == FEC_OK)
      wrc = fec_recover_batch_rs_dev(b->ctx, s0.d_data, s0.d_rparity, s0.d_masks, 1, k, r, slot_bytes, b->d_parity,
                                     b->d_status, b->stream);
    if (wrc == FEC_OK && hipStreamSynchronize(b->stream) != hipSuccess) wrc = FEC_ERR_HIP;
  }
  if (wrc != FEC_OK) {
    char buf[512];
    fec_ctx_last_error(b->ctx, buf, sizeof(buf));
    berr("%s: warm-up launch failed: %s", fn, buf);
    restore();
    delete b;
    return nullptr;
  }
  restore();
  {
    std::lock_guard<std::mutex> lk(b->mu);
    b->open_slab(0);
  }
  b->flusher = std::thread([b] { b->run(); });
  return b;
}

}  // namespace

QFEC_EXPORT FECBatcher* fec_batcher_new(int device, uint32_t k, uint32_t r, uint32_t slot_bytes, uint32_t max_groups,
                                        uint32_t deadline_us, uint32_t slabs) {
  return create(false, device, k, r, slot_bytes, max_groups, deadline_us, slabs);
}

QFEC_EXPORT FECBatcher* fec_batcher_new_decoder(int device, uint32_t k, uint32_t r, uint32_t slot_bytes,
                                                uint32_t max_groups, uint32_t deadline_us, uint32_t slabs) {
  return create(true, device, k, r, slot_bytes, max_groups, deadline_us, slabs);
}

namespace {

FECBatcher* create_multi(bool decoder, const int* devices, int ndevices, uint32_t k, uint32_t r, uint32_t slot_bytes,
                         uint32_t max_groups, uint32_t deadline_us, uint32_t slabs) {
  const char* fn = decoder ? "fec_batcher_new_decoder_multi" : "fec_batcher_new_multi";
  std::vector<int> devs;
  if (devices && ndevices > 0) {
    devs.assign(devices, devices + ndevices);
  } else {
    const int n = fec_hip_device_count();
    for (int i = 0; i < n; ++i) devs.push_back(i);
  }
  if (devs.empty()) {
    berr("%s: no GPU visible", fn);
    return nullptr;
  }
  if (devs.size() == 1) return create(decoder, devs[0], k, r, slot_bytes, max_groups, deadline_us, slabs);
  auto* b = new FECBatcher();
  b->decoder = decoder;
  b->k = k;
  b->r = r;
  b->slot = slot_bytes;
  b->max_groups = max_groups;
  for (const int d : devs) {
    FECBatcher* p = d < 0 ? nullptr : create(decoder, d, k, r, slot_bytes, max_groups, deadline_us, slabs);
    if (!p) {
      const std::string why = d < 0 ? "negative device ordinal" : g_batcher_error;
      delete b;
      berr("%s: device %d: %s", fn, d, why.c_str());
      return nullptr;
    }
    b->parts.push_back(p);
  }
  return b;
}

// Multi-device routing: the part that owns `ticket` and the part's own ticket.
FECBatcher* part_of(FECBatcher* b, int64_t ticket, int64_t* local) {
  if (b->parts.empty()) {
    *local = ticket;
    return b;
  }
  const int64_t n = static_cast<int64_t>(b->parts.size());
  *local = ticket < 0 ? ticket : ticket / n;
  return b->parts[static_cast<size_t>(ticket < 0 ? 0 : ticket % n)];
}

// The part the next group goes to: round robin, passing over parts whose slabs are all
// busy (their submitters would wait) while another part has an open slab.
size_t pick_part(FECBatcher* b) {
  const size_t n = b->parts.size();
  const size_t first = static_cast<size_t>(b->rr.fetch_add(1, std::memory_order_relaxed) % n);
  for (size_t i = 0; i < n; ++i) {
    const size_t c = (first + i) % n;
    if (b->parts[c]->open.load(std::memory_order_acquire) >= 0) return c;
  }
  return first;
}

// A part's ticket as the multi-device handle hands it out.
int64_t global_ticket(const FECBatcher* b, size_t part, int64_t t) {
  return t < 0 ? t : t * static_cast<int64_t>(b->parts.size()) + static_cast<int64_t>(part);
}

}  // namespace

QFEC_EXPORT FECBatcher* fec_batcher_new_multi(const int* devices, int ndevices, uint32_t k, uint32_t r,
                                              uint32_t slot_bytes, uint32_t max_groups, uint32_t deadline_us,
                                              uint32_t slabs) {
  return create_multi(false, devices, ndevices, k, r, slot_bytes, max_groups, deadline_us, slabs);
}

QFEC_EXPORT FECBatcher* fec_batcher_new_decoder_multi(const int* devices, int ndevices, uint32_t k, uint32_t r,
                                                      uint32_t slot_bytes, uint32_t max_groups, uint32_t deadline_us,
                                                      uint32_t slabs) {
  return create_multi(true, devices, ndevices, k, r, slot_bytes, max_groups, deadline_us, slabs);
}

QFEC_EXPORT int fec_batcher_devices(const FECBatcher* b) {
  if (!b) return FEC_ERR_NULL;
  return b->parts.empty() ? 1 : static_cast<int>(b->parts.size());
}

QFEC_EXPORT void fec_batcher_free(FECBatcher* b) { delete b; }

namespace {

// Shared by both submit forms: packet j is at src(j).
// A reserved slot of the open slab: group g of slab si.
struct Slot {
  Slab* s = nullptr;
  uint32_t g = 0;
  int si = -1;
  int64_t ticket = -1;  // read before the commit: once committed, the slab may be recycled
};

// Reserves a slot of the open slab with one atomic add, or waits, under the lock, until a
// slab with room is open.  The slab's first group starts its deadline.  FEC_ERR_RANGE once
// the batcher is stopping.
int reserve(FECBatcher* b, Slot* out) {
  for (;;) {
    const int si = b->open.load(std::memory_order_acquire);
    if (si >= 0) {
      Slab& cand = *b->slabs[si];
      const uint64_t old = cand.state.fetch_add(1, std::memory_order_acq_rel);
      if (!(old & kClosed) && old < b->max_groups) {
        *out = Slot{&cand, static_cast<uint32_t>(old), si, cand.base + static_cast<int64_t>(old)};
        break;
      }
    }
    std::unique_lock<std::mutex> lk(b->mu);
    if (b->stop) return FEC_ERR_RANGE;
    const int cur = b->open.load(std::memory_order_relaxed);
    if (cur >= 0 && cur != si) continue;  // another slab opened meanwhile
    if (cur >= 0) {
      const uint64_t st = b->slabs[cur]->state.load(std::memory_order_acquire);
      if (!(st & kClosed) && st < b->max_groups) continue;
    }
    b->cv_free.wait(lk);  // open_slab notifies; spurious wake-ups retry
  }
  if (out->g == 0) {  // a deadline starts (unless the slab filled and closed meanwhile)
    std::lock_guard<std::mutex> lk(b->mu);
    if (!(out->s->state.load(std::memory_order_acquire) & kClosed)) {
      out->s->t_first = Clock::now();
      out->s->started = true;
      b->cv_flusher.notify_one();
    }
  }
  return FEC_OK;
}

// The slot's bytes have landed: count it, and close the slab now if this group filled it
// (rather than at its deadline).  Nothing of the slab may be read after the count: the
// flusher may encode, publish and reopen it at once.
int64_t commit(FECBatcher* b, const Slot& sl) {
  sl.s->committed.fetch_add(1, std::memory_order_release);
  if (sl.g + 1 == b->max_groups) {
    std::lock_guard<std::mutex> lk(b->mu);
    // still this incarnation of the slab (it may have closed at its deadline and reopened)
    if (b->open.load(std::memory_order_relaxed) == sl.si && sl.s->base == sl.ticket - sl.g &&
        !(sl.s->state.load(std::memory_order_acquire) & kClosed)) {
      b->close_open(true);
      b->cv_flusher.notify_one();
    }
  }
  return sl.ticket;
}

// Shared by both encoder submit forms: packet j is at src(j).
template <class Src>
int64_t submit_group(FECBatcher* b, Src&& src, const uint32_t* lens, uint32_t count) {
  if (b->decoder) {
    berr("fec_batcher_submit: a decoder batcher takes fec_batcher_submit_shards");
    return FEC_ERR_RANGE;
  }
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
  Slot sl;
  if (reserve(b, &sl) != FEC_OK) return FEC_ERR_RANGE;
  sl.s->groups[sl.g] = GroupMeta{count, max_len, 0};
  // copied without the lock (the flusher encodes a slab once every reserved copy landed)
  uint8_t* dst = sl.s->data + size_t(sl.g) * b->k * b->slot;
  for (uint32_t j = 0; j < b->k; ++j) {  // packets zero-padded to the slot, absent slots zero
    uint8_t* d = dst + size_t(j) * b->slot;
    const uint32_t n = j < count ? lens[j] : 0;
    if (n) std::memcpy(d, src(j), n);
    std::memset(d + n, 0, b->slot - n);
  }
  return commit(b, sl);
}

}  // namespace

QFEC_EXPORT int64_t fec_batcher_submit(FECBatcher* b, const uint8_t* packed, const uint32_t* lens, uint32_t count) {
  if (!b || !lens || (!packed && count > 0)) return FEC_ERR_NULL;
  if (!b->parts.empty()) {
    const size_t i = pick_part(b);
    return global_ticket(b, i, fec_batcher_submit(b->parts[i], packed, lens, count));
  }
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
  if (!b->parts.empty()) {
    const size_t i = pick_part(b);
    return global_ticket(b, i, fec_batcher_submit_packets(b->parts[i], packets, lens, count));
  }
  return submit_group(b, [&](uint32_t j) { return packets[j]; }, lens, count);
}

QFEC_EXPORT int64_t fec_batcher_submit_shards(FECBatcher* b, const uint8_t* const* shards, uint32_t len) {
  if (!b || !shards) return FEC_ERR_NULL;
  if (!b->parts.empty() && b->decoder) {
    const size_t i = pick_part(b);
    return global_ticket(b, i, fec_batcher_submit_shards(b->parts[i], shards, len));
  }
  if (!b->decoder) {
    berr("fec_batcher_submit_shards: an encoder batcher takes fec_batcher_submit");
    return FEC_ERR_RANGE;
  }
  if (len == 0 || len > b->slot) {
    berr("fec_batcher_submit_shards: symbol length %u (slot %u bytes)", len, b->slot);
    return FEC_ERR_RANGE;
  }
  uint64_t mask = 0;
  for (uint32_t j = 0; j < b->k + b->r; ++j)
    if (!shards[j]) mask |= 1ull << j;
  Slot sl;
  if (reserve(b, &sl) != FEC_OK) return FEC_ERR_RANGE;
  sl.s->groups[sl.g] = GroupMeta{0, len, mask};
  sl.s->masks[sl.g] = mask;
  // received shards zero-padded to the slot (decoder.go:62-69); lost ones are never read
  uint8_t* dd = sl.s->data + size_t(sl.g) * b->k * b->slot;
  uint8_t* pd = sl.s->rparity + size_t(sl.g) * b->r * b->slot;
  for (uint32_t j = 0; j < b->k + b->r; ++j) {
    if (!shards[j]) continue;
    uint8_t* d = j < b->k ? dd + size_t(j) * b->slot : pd + size_t(j - b->k) * b->slot;
    std::memcpy(d, shards[j], len);
    std::memset(d + len, 0, b->slot - len);
  }
  return commit(b, sl);
}

namespace {

// Copies a published result out of the ring and claims it: 1 done, 0 not published yet,
// negative code on failure.  *len = payload length; *rows = rows copied (encoder: r;
// decoder: the group's lost data shards); *mask = the group's erasure mask (decoder).
int take(FECBatcher* b, int64_t ticket, uint8_t* out, uint32_t out_stride, int* len, uint32_t* rows,
         uint64_t* mask) {
  Entry& e = b->ring[static_cast<size_t>(ticket) % b->ring.size()];
  if (e.ticket.load(std::memory_order_acquire) != ticket) return 0;
  const int rc = e.rc.load(std::memory_order_relaxed);
  const uint32_t n = e.len.load(std::memory_order_relaxed);
  const uint64_t m = e.mask.load(std::memory_order_relaxed);
  const uint32_t nrows = b->decoder ? static_cast<uint32_t>(__builtin_popcountll(m & ((1ull << b->k) - 1))) : b->r;
  bool stale = false;
  if (rc == FEC_OK && out) {
    if (out_stride < n) {
      berr("fec_batcher_wait: out_stride %u < payload length %u", out_stride, n);
      return FEC_ERR_RANGE;
    }
    const uint8_t* src = b->parity + (static_cast<uint64_t>(ticket) % b->cap) * b->r * b->slot;
    for (uint32_t i = 0; i < nrows; ++i) std::memcpy(out + size_t(i) * out_stride, src + size_t(i) * b->slot, n);
    std::atomic_thread_fence(std::memory_order_acquire);
    // the slot is rewritten by the batch of ticket + C: launched already?
    stale = b->launched_upto.load(std::memory_order_relaxed) > ticket + static_cast<int64_t>(b->cap);
  }
  int64_t expect = ticket;
  if (stale || !e.ticket.compare_exchange_strong(expect, -1, std::memory_order_acq_rel)) {
    berr("fec_batcher_wait: result of ticket %lld expired while it was read", static_cast<long long>(ticket));
    return FEC_ERR_RANGE;
  }
  if (mask) *mask = m;
  if (rc == FEC_ERR_UNRECOVERABLE) {
    berr("fec_batcher_wait: ticket %lld lost more shards than parity rows survive (mask 0x%llx)",
         static_cast<long long>(ticket), static_cast<unsigned long long>(m));
    return rc;
  }
  if (rc != FEC_OK) {
    std::lock_guard<std::mutex> lk(b->mu);
    berr("fec_batcher_wait: the batch of ticket %lld failed with code %d: %s", static_cast<long long>(ticket), rc,
         b->last_batch_error.c_str());
    return rc;
  }
  *len = static_cast<int>(n);
  *rows = nrows;
  return 1;
}

// fec_batcher_wait's body: 1 and the result, or FEC_ERR_AGAIN / another negative code.
int wait_result(FECBatcher* b, int64_t ticket, uint8_t* out, uint32_t out_stride, int64_t timeout_us, int* len,
                uint32_t* rows, uint64_t* mask) {
  int st = ticket >= 0 ? take(b, ticket, out, out_stride, len, rows, mask) : 0;
  if (st != 0) return st;
  // A poll of a ticket not published yet needs no lock.
  if (timeout_us == 0 && ticket >= 0 && ticket >= b->published_upto.load(std::memory_order_acquire))
    return FEC_ERR_AGAIN;
  std::unique_lock<std::mutex> lk(b->mu);
  if (ticket < 0 || ticket >= b->issued_bound()) {
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
  st = take(b, ticket, out, out_stride, len, rows, mask);
  if (st == 0) {
    berr("fec_batcher_wait: ticket %lld was already collected", static_cast<long long>(ticket));
    return FEC_ERR_RANGE;
  }
  return st;
}

}  // namespace

QFEC_EXPORT int fec_batcher_wait(FECBatcher* b, int64_t ticket, uint8_t* out, uint32_t out_stride, int64_t timeout_us) {
  if (!b) return FEC_ERR_NULL;
  if (b->decoder) {
    berr("fec_batcher_wait: a decoder batcher's results are read with fec_batcher_wait_rebuilt");
    return FEC_ERR_RANGE;
  }
  int64_t local = 0;
  b = part_of(b, ticket, &local);
  int len = 0;
  uint32_t rows = 0;
  const int st = wait_result(b, local, out, out_stride, timeout_us, &len, &rows, nullptr);
  return st == 1 ? len : st;
}

QFEC_EXPORT int fec_batcher_wait_rebuilt(FECBatcher* b, int64_t ticket, uint8_t* out, uint32_t out_stride,
                                         uint64_t* lost_mask, int64_t timeout_us) {
  if (!b) return FEC_ERR_NULL;
  if (!b->decoder) {
    berr("fec_batcher_wait_rebuilt: an encoder batcher's results are read with fec_batcher_wait");
    return FEC_ERR_RANGE;
  }
  int64_t local = 0;
  b = part_of(b, ticket, &local);
  int len = 0;
  uint32_t rows = 0;
  const int st = wait_result(b, local, out, out_stride, timeout_us, &len, &rows, lost_mask);
  return st == 1 ? static_cast<int>(rows) : st;
}

QFEC_EXPORT int fec_batcher_flush(FECBatcher* b) {
  if (!b) return FEC_ERR_NULL;
  for (FECBatcher* p : b->parts) fec_batcher_flush(p);
  if (!b->parts.empty()) return FEC_OK;
  {
    std::lock_guard<std::mutex> lk(b->mu);
    b->close_open(false);
  }
  b->cv_flusher.notify_one();
  return FEC_OK;
}

QFEC_EXPORT int fec_batcher_stats(FECBatcher* b, FECBatcherStats* out) {
  if (!b || !out) return FEC_ERR_NULL;
  if (!b->parts.empty()) {  // sums over the devices (max_batch: the largest)
    FECBatcherStats sum{};
    for (FECBatcher* p : b->parts) {
      FECBatcherStats st{};
      fec_batcher_stats(p, &st);
      sum.groups += st.groups;
      sum.batches += st.batches;
      sum.full_flushes += st.full_flushes;
      sum.deadline_flushes += st.deadline_flushes;
      sum.max_batch = std::max(sum.max_batch, st.max_batch);
      sum.expired += st.expired;
    }
    *out = sum;
    return FEC_OK;
  }
  std::lock_guard<std::mutex> lk(b->mu);
  *out = b->stats;
  return FEC_OK;
}

QFEC_EXPORT const char* fec_batcher_last_error(void) { return g_batcher_error.c_str(); }
