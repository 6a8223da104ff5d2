// fec_coalesce.cpp — legacy fec_encode_batch calls of many contexts joined into shared launches
// (batching for the reference's *unchanged* call site).
//
// The reference encodes one group per cgo call: every QUIC stream owns a HybridFECEncoder,
// hence its own FECEncoderCXX and context, and calls EncodeBatch with a single group on its
// 10th packet (encoder_hybrid.go:71-73, :115 -> fec_cgo.go:138 -> fec_encode_batch).  On its
// own context each such call is one kernel launch plus one synchronize (~15 us, against
// ~0.6 us for the reference's AVX2 loop), and concurrent streams' calls never share a launch.
// Here every small host-resident legacy call of the process goes through one coalescer per
// (device, packet size):
//
//  * A caller reserves room for its groups in the open batch (under the lock), writes the
//    absolute device addresses of its 10 x G packets into the batch's page-locked address list
//    (without the lock; page-locked slabs -- fec_alloc_slab, which FECEncoderCXX uses -- are
//    read in place by the kernel, pageable ones are first copied into the batch's page-locked
//    staging), and then waits for the batch.
//  * Group commit, no flusher thread: the first waiting caller that finds fewer than
//    `max_inflight` batches in flight becomes the batch's leader.  It closes the batch (the
//    next one opens for new callers), waits for the batch's outstanding address writes,
//    launches the gather encode (encode_v16<10, 1, kAddr>: row 0 = XOR, as the reference) on
//    the coalescer's stream, waits for it and wakes the batch's callers.  While batches are in
//    flight the next one fills, so under load a launch carries every group that arrived during
//    the previous one; a lone caller leads its own one-group batch and pays no thread hand-off.
//  * Every caller copies its own repair rows out of the batch's page-locked output and returns
//    the legacy code (0, or the FEC_ERR_* of a failed launch).  The batch is reused once its
//    last caller has copied out.
//
// QUICFEC_COALESCE=0 turns it off; QUICFEC_COALESCE_MAX_GROUPS (default 64) bounds the calls
// it takes; QUICFEC_COALESCE_INFLIGHT (default 2) the batches in flight per coalescer.
//
// Resident server (the default for the Go wrapper's calls: page-locked slab, 1..8 groups, P >=
// 16).  A launch per batch costs the leader ~6-9 us of HIP API time and ~12 us until it sees
// the completion (profiles/r03_legacy_v3_tuning.jsonl), so batching alone only matches the
// per-context path.  Instead workgroups stay resident on each device and serve a ring of
// submission slots in page-locked coherent host memory (fec_kernels.hpp ServerSlot,
// legacy_server): a caller takes a sequence number, writes its packets' device addresses and
// its repair rows' address into slot seq % kServerSlots, every word tagged with the slot's lap,
// and polls the slot's done word; a workgroup takes every complete slot of its class in order
// each time it polls (one round trip reads the next 16 slots' headers and first groups), so
// concurrent callers share one pass without any host-side batch.  An instance is 8 workgroups
// (QUICFEC_RESIDENT_SERVERS), workgroup c serving the seqs with seq % 8 == c: eight
// independent poll -> serve -> done cycles; the host gives a call the class by the calls in
// flight (Resident::encode).
// VRAM ring (large-BAR devices, the default where setup_vram succeeds; QUICFEC_RESIDENT_VRAM=0
// keeps the page-locked ring): the slots live in uncached device memory the host writes
// through the BAR, and a call of <= 4 groups with P % 4 == 0 and P <= 1536 -- the Go wrapper's
// (1 group, 1200 B) -- has its packets copied into its slot as lap-tagged 16-B chunks
// (pack_inline).  The server's poll and packet loads are then device-local: the call's one
// PCIe crossing each way is the host's stores and the device's repair-row stores.  Any slab
// memory works for those calls, pageable included.
// No kernel launch per call: the resident instance leaves after QUICFEC_RESIDENT_IDLE_US
// (default 2000) without work or QUICFEC_RESIDENT_LIFE_US (default 50000) of life, and the next
// caller that finds it gone (its `exited` word equals the instance's generation) launches the
// next one from the served-up-to mark (`progress`).  QUICFEC_RESIDENT=0 turns it off.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <utility>
#include <chrono>
#include <vector>

#include "fec_hip.h"
#include "fec_internal.hpp"
#include "fec_kernels.hpp"
#include "fec_knobs.hpp"

#define QFEC_EXPORT extern "C" __attribute__((visibility("default")))

namespace qfec {
namespace {

constexpr uint32_t kPackets = 10;  // packets per group of the legacy call (fec_xor_simd.cpp:580)
constexpr uint32_t kMaxBatchGroups = 1024;
constexpr uint64_t kStageBudget = 16ull << 20;  // page-locked staging bytes per batch
constexpr size_t kMaxCoalescers = 16;           // (device, packet size) pairs
constexpr uint32_t kCoalesceMaxP = 16u << 10;   // larger packets: no shared launches (staging bound)
// FECCoalesceStats as published in round 4: calls .. resident_vram (15 words)
constexpr size_t kCoalesceStatsV4Bytes = 15 * sizeof(uint64_t);

long env_long(const char* name, long def) {
  const char* v = std::getenv(name);
  return v && *v ? std::atol(v) : def;
}

// Binds a device for the scope (HIP's current device is per thread).
struct BindDevice {
  int prev = -1;
  bool ok = false;
  explicit BindDevice(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    ok = hipSetDevice(dev) == hipSuccess;
    if (!ok) (void)hipGetLastError();
  }
  ~BindDevice() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// Page-locked host memory and the address kernels use for it.
struct Pinned {
  uint8_t* host = nullptr;
  uint8_t* dev = nullptr;
  Pinned() = default;
  Pinned(const Pinned&) = delete;
  Pinned& operator=(const Pinned&) = delete;
  ~Pinned() {
    if (host) (void)hipHostFree(host);
  }
  bool alloc(size_t bytes) {
    void* h = nullptr;
    if (hipHostMalloc(&h, bytes, hipHostMallocDefault) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    void* d = nullptr;
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || d == nullptr) {
      (void)hipGetLastError();
      d = h;  // unified addressing
    }
    host = static_cast<uint8_t*>(h);
    dev = static_cast<uint8_t*>(d);
    return true;
  }
};

struct Batch {
  enum State { kFree, kOpen, kClosed, kLaunched, kDone };
  std::atomic<int> state{kFree};  // transitions under the coalescer's lock, except kDone (leader)
  Pinned addr;    // cap * kPackets packet addresses (u64), read by the kernel in place
  Pinned stage;   // cap * kPackets * P bytes: packets of pageable callers (allocated on first need)
  Pinned out;     // cap * P: repair row of every group, written by the kernel in place
  hipEvent_t done = nullptr;
  uint32_t used = 0;     // groups reserved
  uint32_t calls = 0;    // callers in the batch
  std::atomic<uint32_t> copying{0};  // callers whose addresses / packets are not written yet
  uint32_t readers = 0;  // callers that have not copied their rows out
  int rc = FEC_OK;
  std::string err;
  std::condition_variable cv;  // callers that stopped spinning: done, or a launch slot came free
};

// A batch large enough for any packet size the coalescer takes: cap * P <= kStageBudget / 10
// (cap = max(8, min(kMaxBatchGroups, kStageBudget / (10 P))), P <= kCoalesceMaxP).
constexpr size_t kBatchOutMax = std::max<size_t>(kStageBudget / kPackets, size_t(8) * kCoalesceMaxP);

// The first batch of the device's first coalescer, made with the device's first context
// (coalesce_prepare) so that the first shared-launch call of a process pays no page-locked
// allocation (~0.35 ms; profiles/r05g): sized for any packet size.
std::mutex g_spare_mu;
std::map<int, std::unique_ptr<Batch>> g_spare;

bool alloc_batch(Batch& b, size_t groups, size_t out_bytes) {
  if (!b.addr.alloc(groups * kPackets * sizeof(uint64_t)) || !b.out.alloc(out_bytes) ||
      hipEventCreateWithFlags(&b.done, hipEventDisableTiming) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return true;
}

// The device's shared-launch stream, non-blocking: a batch holding other contexts' calls never
// waits on legacy null-stream work or on a leader context's own queued work.  Made
// with the first context too (a stream that needs a new hardware queue costs ~9 ms); nullptr
// when that failed (the leader then launches on its caller's context stream).  Never destroyed.
std::map<int, hipStream_t> g_launch_stream;

void prepare_spare_batch(int device) {
  std::lock_guard<std::mutex> lk(g_spare_mu);
  if (g_spare.count(device)) return;
  auto b = std::make_unique<Batch>();
  g_spare.emplace(device, alloc_batch(*b, kMaxBatchGroups, kBatchOutMax) ? std::move(b) : nullptr);
  hipStream_t s = nullptr;
  BindDevice bd(device);
  if (!bd.ok || hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
    (void)hipGetLastError();
    s = nullptr;
  }
  g_launch_stream[device] = s;
}

hipStream_t launch_stream_for(int device) {
  std::lock_guard<std::mutex> lk(g_spare_mu);
  auto it = g_launch_stream.find(device);
  return it == g_launch_stream.end() ? nullptr : it->second;
}

std::unique_ptr<Batch> take_spare_batch(int device) {
  std::lock_guard<std::mutex> lk(g_spare_mu);
  auto it = g_spare.find(device);
  if (it == g_spare.end()) return nullptr;
  return std::move(it->second);
}

std::atomic<uint64_t> g_calls{0}, g_groups{0}, g_batches{0}, g_max_batch{0}, g_max_calls{0};
std::atomic<uint64_t> g_close_ns{0}, g_launch_ns{0}, g_done_ns{0};

uint64_t now_ns() {
  return static_cast<uint64_t>(std::chrono::duration_cast<std::chrono::nanoseconds>(
                                   std::chrono::steady_clock::now().time_since_epoch())
                                   .count());
}

void atomic_max(std::atomic<uint64_t>& a, uint64_t v) {
  uint64_t cur = a.load(std::memory_order_relaxed);
  while (v > cur && !a.compare_exchange_weak(cur, v, std::memory_order_relaxed)) {
  }
}

class Coalescer {
 public:
  // NULL when the device or page-locked memory cannot be set up (the call then runs alone).
  // Nothing but the first batch's page-locked buffers and event is made here: no context and no
  // stream (the leader launches on the device's shared-launch stream, made with the first context,
  // launch_stream_for), further batches when concurrent
  // callers need them.  A context and a stream of its own each cost ~9 ms here (a stream that
  // needs a new hardware queue), and the first shared-launch call of a process paid both: 18-22 ms
  // against a p99 of 21-35 us (coalescer stamps, profiles/r05e/legacy_coalescer_*.err).
  static Coalescer* create(int device, uint32_t P) {
    // the test library's TestKnob::kCoalesceStamps: the creation's time to stderr (diagnostic)
    const uint64_t t0 = now_ns();
    std::unique_ptr<Coalescer> c(new Coalescer());
    c->device = device;
    c->P = P;
    const uint64_t fit = kStageBudget / (uint64_t(kPackets) * P);
    c->cap = static_cast<uint32_t>(std::max<uint64_t>(8, std::min<uint64_t>(kMaxBatchGroups, fit)));
    c->max_inflight = static_cast<int>(std::max(1L, std::min(8L, env_long("QUICFEC_COALESCE_INFLIGHT", 2))));
    c->launch_stream = launch_stream_for(device);
    BindDevice bd(device);
    if (!bd.ok || !c->add_batch()) return nullptr;
    std::lock_guard<std::mutex> lk(c->mu);
    c->open_free();
    if (test_knob(TestKnob::kCoalesceStamps, 0) != 0)
      std::fprintf(stderr, "{\"coalescer_create_us\": %.1f}\n", (now_ns() - t0) / 1e3);
    return c.release();
  }

  uint32_t capacity() const { return cap; }

  ~Coalescer() {  // only a Coalescer whose create() failed; never at exit (shutdown_all)
    BindDevice bd(device);
    for (auto& b : batches)
      if (b->done) (void)hipEventDestroy(b->done);
    batches.clear();
  }

  // The legacy call's body; slab_dev is the slab's device address when it is page-locked; stream:
  // the caller's context stream (a leader launches its batch there only when the device has no
  // shared-launch stream).
  int encode(const uint8_t* slab, const uint8_t* slab_dev, const uint32_t* offsets, uint32_t G, uint8_t* repair_out,
             hipStream_t stream) {
    std::unique_lock<std::mutex> lk(mu);
    if (!slab_dev && !staging_ready) {
      for (auto& b : batches)
        if (!b->stage.host && !b->stage.alloc(size_t(cap) * kPackets * P)) {
          set_last_error("fec_encode_batch: page-locked staging of the coalescer failed");
          return FEC_ERR_HIP;
        }
      staging_ready = true;
    }
    for (;;) {
      if (open < 0) open_free(true);
      if (open >= 0 && batches[open]->used + G <= cap) break;
      cv_room.wait(lk);
    }
    const int bi = open;
    Batch& b = *batches[bi];
    const uint32_t g0 = b.used;
    b.used += G;
    ++b.calls;
    b.copying.fetch_add(1, std::memory_order_relaxed);
    ++b.readers;
    lk.unlock();
    // the packets' addresses (and, from pageable memory, the packets); packet_size bytes from
    // every offset, as the reference reads them (fec_xor_simd.cpp:582-590)
    const uint64_t n = uint64_t(G) * kPackets;
    uint64_t* a = reinterpret_cast<uint64_t*>(b.addr.host) + uint64_t(g0) * kPackets;
    if (slab_dev) {
      const uint64_t base = reinterpret_cast<uint64_t>(slab_dev);
      for (uint64_t i = 0; i < n; ++i) a[i] = base + offsets[i];
    } else {
      const uint64_t first = uint64_t(g0) * kPackets;
      for (uint64_t i = 0; i < n; ++i) {
        std::memcpy(b.stage.host + (first + i) * P, slab + offsets[i], P);
        a[i] = reinterpret_cast<uint64_t>(b.stage.dev + (first + i) * P);
      }
    }
    b.copying.fetch_sub(1, std::memory_order_release);
    // Wait for the batch, or lead it once a launch slot is free.  Callers spin first (a
    // condition-variable wake costs several microseconds per hand-off, as much as the launch
    // itself), then yield, then sleep in short timed waits.
    for (uint32_t spins = 0;; ++spins) {
      const int st = b.state.load(std::memory_order_acquire);
      if (st == Batch::kDone) break;
      if (st == Batch::kOpen && inflight.load(std::memory_order_acquire) < max_inflight) {
        lk.lock();
        if (b.state.load(std::memory_order_relaxed) == Batch::kOpen &&
            inflight.load(std::memory_order_relaxed) < max_inflight)
          lead(b, lk, stream);  // returns with the lock released
        else
          lk.unlock();
        spins = 0;
        continue;
      }
      if (spins < spin_pause) {
        for (int i = 0; i < 16; ++i) __builtin_ia32_pause();
      } else if (spins < spin_pause + spin_yield) {
        std::this_thread::yield();
      } else {
        lk.lock();
        b.cv.wait_for(lk, std::chrono::microseconds(200));
        lk.unlock();
      }
    }
    const int rc = b.rc;  // written before kDone was stored (release)
    if (rc != FEC_OK) set_last_error(b.err.c_str());
    if (rc == FEC_OK) std::memcpy(repair_out, b.out.host + uint64_t(g0) * P, uint64_t(G) * P);
    lk.lock();
    if (--b.readers == 0) {
      b.state.store(Batch::kFree, std::memory_order_relaxed);
      if (open < 0) open_free();
    }
    return rc;
  }

 private:
  int device = 0;
  uint32_t P = 0, cap = 0;
  int max_inflight = 2;
  hipStream_t launch_stream = nullptr;  // the device's non-blocking shared-launch stream, if made
  std::atomic<int> stamps_left{test_knob(TestKnob::kCoalesceStamps, 0) != 0 ? 3 : 0};  // diagnostic: the first batches
  std::mutex mu;
  std::condition_variable cv_room;  // callers waiting for an open batch with room
  std::vector<std::unique_ptr<Batch>> batches;
  int open = -1;                    // the batch taking callers, -1 while none is free
  std::atomic<int> inflight{0};     // batches closed by a leader and not done yet
  bool staging_ready = false;
  // waiting callers' spin budget before they sleep (pause rounds, then yields)
  uint32_t spin_pause = static_cast<uint32_t>(test_knob(TestKnob::kCoalesceSpinPause, 256));
  uint32_t spin_yield = static_cast<uint32_t>(test_knob(TestKnob::kCoalesceSpinYield, 3840));

  // One more batch (its page-locked address list and output, its event, and staging when pageable
  // callers have needed it).  Caller holds mu, or owns the coalescer alone (create).
  bool add_batch() {
    std::unique_ptr<Batch> b = batches.empty() ? take_spare_batch(device) : nullptr;  // made at the first context
    if (!b) {
      b = std::make_unique<Batch>();
      if (!alloc_batch(*b, cap, size_t(cap) * P)) return false;
    }
    if (staging_ready && !b->stage.alloc(size_t(cap) * kPackets * P)) {
      (void)hipGetLastError();
      if (b->done) (void)hipEventDestroy(b->done);
      return false;
    }
    batches.push_back(std::move(b));
    return true;
  }

  // Opens a free batch for new callers, if there is one -- with grow, a new one while fewer than
  // the in-flight batches + the open one + one still being copied out exist (only callers that
  // need room grow the set: a leader closing its batch does not pay an allocation).  Caller holds
  // mu.
  void open_free(bool grow = false) {
    for (size_t i = 0;; ++i) {
      if (i == batches.size()) {
        if (!grow || batches.size() >= size_t(max_inflight) + 2) return;
        BindDevice bd(device);
        if (!bd.ok || !add_batch()) return;
      }
      Batch& b = *batches[i];
      if (b.state.load(std::memory_order_relaxed) != Batch::kFree) continue;
      b.used = b.calls = b.readers = 0;
      b.copying.store(0, std::memory_order_relaxed);
      b.rc = FEC_OK;
      b.err.clear();
      b.state.store(Batch::kOpen, std::memory_order_release);
      open = static_cast<int>(i);
      cv_room.notify_all();
      return;
    }
  }

  // Closes, launches and completes batch b.  Called with mu held through `lk`; returns with it
  // released.
  void lead(Batch& b, std::unique_lock<std::mutex>& lk, hipStream_t caller_stream) {
    const hipStream_t stream = launch_stream ? launch_stream : caller_stream;
    b.state.store(Batch::kClosed, std::memory_order_relaxed);
    open = -1;
    open_free();
    inflight.fetch_add(1, std::memory_order_acq_rel);
    const uint32_t n = b.used, calls = b.calls;  // closed: no more reservations
    lk.unlock();
    const uint64_t t0 = now_ns();
    while (b.copying.load(std::memory_order_acquire) > 0) __builtin_ia32_pause();
    b.state.store(Batch::kLaunched, std::memory_order_relaxed);
    const uint64_t t1 = now_ns();
    // the gather encode of the batch's groups, row 0 = XOR as the reference (no coefficient table)
    BindDevice bd(device);
    const EncodeLaunch a{nullptr, b.addr.dev, OffsetKind::kAddr, b.out.dev, n, kPackets, 1, P, nullptr};
    hipError_t le = bd.ok ? launch_encode(a, stream) : hipErrorInvalidDevice;
    int rc = le == hipSuccess ? FEC_OK : FEC_ERR_HIP;
    std::string err;
    uint64_t t2 = t1;
    if (rc != FEC_OK) {
      (void)hipGetLastError();
      err = std::string("fec_encode_batch (coalesced): ") + hipGetErrorString(le);
    } else {
      hipError_t e = hipEventRecord(b.done, stream);
      t2 = now_ns();
      // poll (a blocking wait adds its wake-up to every batch); yield once it takes a while
      for (uint32_t i = 0; e == hipSuccess; ++i) {
        e = hipEventQuery(b.done);
        if (e != hipErrorNotReady) break;
        e = hipSuccess;
        if (i < 4096) {
          for (int j = 0; j < 16; ++j) __builtin_ia32_pause();
        } else {
          std::this_thread::yield();
        }
      }
      if (e != hipSuccess) {
        (void)hipGetLastError();
        rc = FEC_ERR_HIP;
        err = std::string("fec_encode_batch (coalesced): ") + hipGetErrorString(e);
      }
    }
    const uint64_t t3 = now_ns();
    if (stamps_left.load(std::memory_order_relaxed) > 0 && stamps_left.fetch_sub(1) > 0) {  // TestKnob::kCoalesceStamps
      std::fprintf(stderr, "{\"coalescer_batch_us\": {\"close\": %.1f, \"launch\": %.1f, \"done\": %.1f}}\n", (t1 - t0) / 1e3,
                   (t2 - t1) / 1e3, (t3 - t2) / 1e3);
    }
    g_close_ns.fetch_add(t1 - t0, std::memory_order_relaxed);
    g_launch_ns.fetch_add(t2 - t1, std::memory_order_relaxed);
    g_done_ns.fetch_add(t3 - t2, std::memory_order_relaxed);
    g_batches.fetch_add(1, std::memory_order_relaxed);
    g_calls.fetch_add(calls, std::memory_order_relaxed);
    g_groups.fetch_add(n, std::memory_order_relaxed);
    atomic_max(g_max_batch, n);
    atomic_max(g_max_calls, calls);
    b.rc = rc;
    b.err = err;
    b.state.store(Batch::kDone, std::memory_order_release);
    inflight.fetch_sub(1, std::memory_order_acq_rel);
    lk.lock();
    b.cv.notify_all();
    if (open >= 0) batches[open]->cv.notify_all();  // a launch slot is free: the open batch may go
    lk.unlock();
  }
};

// Page-locked host memory the device reads and writes coherently (polling and flags).
bool alloc_coherent(Pinned& m, size_t bytes) {
  void* h = nullptr;
  if (hipHostMalloc(&h, bytes, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  std::memset(h, 0, bytes);
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || d == nullptr) {
    (void)hipGetLastError();
    d = h;
  }
  m.host = static_cast<uint8_t*>(h);
  m.dev = static_cast<uint8_t*>(d);
  return true;
}

constexpr uint32_t kResidentOutBytes = 16u << 10;  // per slot: repair rows of callers whose buffer is pageable
// per slot of the VRAM ring: an inline call's tagged repair chunks (kInlineMaxGroups x 128 x 16 B)
constexpr uint32_t kInlineOutBytes = kInlineMaxGroups * (kInlineMaxP / kInlinePayload) * 16;

std::atomic<uint64_t> g_res_calls{0}, g_res_launches{0}, g_res_pre_ns{0}, g_res_wait_ns{0}, g_res_post_ns{0};
std::atomic<uint64_t> g_res_inline{0}, g_res_vram{0};

// The stream the resident instance runs on.  A persistent kernel occupies its hardware queue:
// every later kernel on a stream that shares that queue waits until the instance leaves (up to
// the life bound).  On a plain non-blocking stream, the runtime's queue pool put other streams
// of the process behind it: their kernels' p99 launch-to-completion went from ~50 us to 33 ms
// while legacy calls were being served, the context's own stream's p50 to 48 ms
// (scripts/probe_resident_interference.py, profiles/r03_probe_resident_interference.txt).
// Streams of another priority come from another queue pool, so the instance runs on a
// non-blocking stream of the highest priority (other streams' p99 52 us, and the instance's
// relaunch is dispatched ahead of bulk work); a normal-priority stream of the caller never
// shares its queue.  (Also measured and not kept: the lowest priority, and a CU-masked stream,
// which always gets a queue of its own but is blocking: it orders against the legacy null
// stream.)
bool create_server_stream(hipStream_t* s) {
  int lo = 0, hi = 0;
  if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess) return false;
  return hipStreamCreateWithPriority(s, hipStreamNonBlocking, hi) == hipSuccess;
}

class Resident {
 public:
  static Resident* create(int device) {
    std::unique_ptr<Resident> r(new Resident());
    r->device = device;
    BindDevice bd(device);
    int khz = 0;
    if (!bd.ok || hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device) != hipSuccess || khz <= 0 ||
        !create_server_stream(&r->stream)) {
      (void)hipGetLastError();
      return nullptr;
    }
    const uint64_t per_us = static_cast<uint64_t>(khz) / 1000u;
    r->idle_ticks = per_us * static_cast<uint64_t>(std::max(10L, env_long("QUICFEC_RESIDENT_IDLE_US", 2000)));
    r->slow_ticks = per_us * static_cast<uint64_t>(std::max(1L, test_knob(TestKnob::kResidentSlowUs, 50)));
    r->life_ticks = per_us * static_cast<uint64_t>(std::max(100L, env_long("QUICFEC_RESIDENT_LIFE_US", 50000)));
    // The per-slot staging of pageable repair buffers (16 MB) comes with the first call that
    // needs it (ensure_outs): the first context of every process sets a Resident up
    // (coalesce_prepare), most never make such a call.
    if (!alloc_coherent(r->ring, sizeof(ServerSlot) * kServerSlots) ||
        !alloc_coherent(r->done, sizeof(uint64_t) * kServerSlots) || !alloc_coherent(r->ctl, sizeof(ServerControl)))
      return nullptr;
    r->ring_w = reinterpret_cast<ServerSlot*>(r->ring.host);
    r->ring_d = reinterpret_cast<ServerSlot*>(r->ring.dev);
    r->deadline = std::chrono::milliseconds(std::max(1L, env_long("QUICFEC_RESIDENT_DEADLINE_MS", 10000)));
    // Test switches (libfec_hip_test.so only; fec_knobs.hpp):
    // an instance that never serves (relaunch records a launch without launching);
    r->no_launch = test_knob(TestKnob::kResidentNoLaunch, 0) != 0;
    // a short tag epoch (fec_kernels.hpp server_tag), so the scrubs at its boundaries run within
    // a few thousand calls;
    const long ep = std::min<long>(kServerEpoch, std::max(1L, test_knob(TestKnob::kResidentEpoch, kServerEpoch)));
    r->epoch = 1u;
    while (r->epoch * 2 <= static_cast<uint32_t>(ep)) r->epoch *= 2;  // a power of two (server_tag)
    // every inline call lands one chunk in two 8-B pieces, the half with the tag first and the
    // other ~100 us after the slot's header (a write-combined store evicted in pieces);
    r->tear = test_knob(TestKnob::kResidentTear, 0) != 0;
    // the call of this number (0 = the Resident's first) fails as if its deadline had passed
    // (poisoning under load);
    r->fail_at = static_cast<uint64_t>(test_knob(TestKnob::kResidentFailAt, -1));
    // every call to the next class round robin, however few are in flight (one thread's n-th
    // call then takes seq n);
    r->spread = test_knob(TestKnob::kResidentSpread, 0) != 0;
    // the served batches' phase stamps, printed at exit.
    if (test_knob(TestKnob::kResidentStamps, 0) != 0 && !alloc_coherent(r->stamps, 256 * 8 * sizeof(uint64_t))) return nullptr;
    r->tick_khz = static_cast<uint64_t>(khz);
    // no word of a slot that was never written carries a tag (tags are 1 .. epoch; alloc_coherent zeroed it)
    std::memset(r->ring.host, 0, sizeof(ServerSlot) * kServerSlots);
    if (env_long("QUICFEC_RESIDENT_VRAM", 1) != 0) r->setup_vram();
    // Serving classes (fec_kernels.hpp kServerMaxClasses): QUICFEC_RESIDENT_SERVERS workgroups
    // (default 8 with the VRAM ring; 1 with the page-locked ring, whose every poll is a PCIe round
    // trip), a power of two up to 8 (rounded down); more than one share a few words of uncached
    // device memory, and without them the instance is one workgroup.  Same box,
    // alternating (profiles/r05{q,s}/ab_servers.jsonl): 16 streams 0.69-0.74 M groups/s with one
    // class, 1.15-1.16 M with 8; 64 streams 0.26-0.29 vs 0.39-0.42 M; one stream 7.9-8.1 vs
    // 8.5-8.7 us a call (a workgroup's poll takes 1.5-1.7 us instead of 1.3 while others poll).
    const long want = std::min<long>(kServerMaxClasses, std::max(1L, env_long("QUICFEC_RESIDENT_SERVERS", r->vinl ? 8 : 1)));
    while (r->classes * 2 <= static_cast<uint32_t>(want)) r->classes *= 2;
    if (r->classes > 1) {
      void* c = nullptr;
      if (hipExtMallocWithFlags(&c, sizeof(ServerCoord), hipDeviceMallocUncached) != hipSuccess ||
          hipMemsetAsync(c, 0, sizeof(ServerCoord), r->stream) != hipSuccess || hipStreamSynchronize(r->stream) != hipSuccess) {
        (void)hipGetLastError();
        if (c) (void)hipFree(c);
        c = nullptr;
        r->classes = 1;
      }
      r->coord = static_cast<ServerCoord*>(c);
    }
    for (uint32_t c = 0; c < kServerMaxClasses; ++c) r->class_next[c].store(c, std::memory_order_relaxed);
    r->collected.reset(new std::atomic<uint64_t>[kServerSlots]);
    for (uint32_t i = 0; i < kServerSlots; ++i) r->collected[i].store(0, std::memory_order_relaxed);
    return r.release();
  }

  // Whether a call of G groups of P bytes fits a slot (repair rows staged in the slot unless
  // the caller's buffer is page-locked).
  static bool fits(uint32_t G, uint32_t P, bool repair_pinned) {
    return G >= 1 && G <= kServerMaxGroups && P >= 16 && P <= 0xFFFFu &&
           (repair_pinned || uint64_t(G) * P <= kResidentOutBytes);
  }

  // False once a call timed out or a relaunch failed (poison): later legacy calls take the
  // coalescer / per-context paths, and no instance is launched again.
  bool usable() const { return !broken.load(std::memory_order_acquire); }

  // The server's diagnostic counters (ServerControl): retried slots and epoch scrubs.
  uint64_t bad_slots() const { return sum_classes(&ServerControl::bad_slots); }
  uint64_t scrubs() const { return sum_classes(&ServerControl::scrubs); }
  uint32_t serving_classes() const { return classes; }

  // The call's result, or kNotTaken when the Resident is (or just became) unusable before the
  // call published its slot: nothing of the caller's was handed to the device, and the caller
  // runs the call on another path.
  static constexpr int kNotTaken = 1;

  // Whether a call of G groups of P bytes can have its packets copied into its slot (the VRAM
  // ring): then the slab may be any host memory.
  bool inlines(uint32_t G, uint32_t P) const {
    return vinl != nullptr && G <= kInlineMaxGroups && P <= kInlineMaxP && P % 4 == 0;
  }

  // slab: the caller's slab; slab_dev: the device's address for it when it is page-locked, else
  // nullptr (the call is then taken only with its packets inline).
  int encode(const uint8_t* slab, const uint8_t* slab_dev, const uint32_t* offsets, uint32_t G, uint32_t P,
             uint8_t* repair_out, uint8_t* repair_dev, uint64_t t_enter) {
    const bool inline_pk = inlines(G, P);
    if (!inline_pk && slab_dev == nullptr) return kNotTaken;
    if (!inline_pk && !repair_dev && !ensure_outs()) return kNotTaken;
    const uint64_t base = reinterpret_cast<uint64_t>(slab_dev);
    // The call's serving class: while few calls are in flight only the lowest classes take them
    // (a lone caller's calls all go to class 0, whose workgroup stays busy, while the others poll
    // slowly: a poll is slower while other workgroups poll fast), under load all of
    // them, round robin.  Each class's seqs are c, c + classes, c + 2 * classes, ... in the order
    // taken, which is the order its workgroup serves them.
    struct InFlight {
      std::atomic<uint32_t>& n;
      uint32_t now;
      explicit InFlight(std::atomic<uint32_t>& c) : n(c), now(c.fetch_add(1, std::memory_order_relaxed) + 1) {}
      ~InFlight() { n.fetch_sub(1, std::memory_order_relaxed); }
    } inflight(in_flight);
    const uint32_t span = spread ? classes : std::min(classes, inflight.now);
    const uint32_t cls = span > 1 ? rr.fetch_add(1, std::memory_order_relaxed) % span : 0u;
    const uint64_t seq = class_next[cls].fetch_add(classes, std::memory_order_relaxed);
    const uint32_t si = static_cast<uint32_t>(seq % kServerSlots);
    const uint32_t tag16 = server_tag(seq, epoch);
    const uint64_t tag = uint64_t(tag16) << kServerTagShift;
    // the slot's previous occupant (seq - kServerSlots) has been served and collected; if that
    // does not happen within the deadline, or no instance can be launched to serve it, the
    // Resident is poisoned and this call is not taken (its slot stays untouched: overwriting it
    // would change the lap tag of a call the device has not served yet)
    const uint64_t* dw = reinterpret_cast<const uint64_t*>(done.host) + si;
    const auto t_reuse = std::chrono::steady_clock::now() + deadline;
    for (uint32_t spins = 0; seq >= kServerSlots && (collected[si].load(std::memory_order_acquire) != seq - kServerSlots + 1 ||
                                                     __atomic_load_n(dw, __ATOMIC_ACQUIRE) != seq - kServerSlots + 1);
         ++spins) {
      if (!usable()) return kNotTaken;
      if ((spins & 1023u) == 1023u) {
        if ((!instance_alive() && relaunch() != FEC_OK) || std::chrono::steady_clock::now() > t_reuse) {
          poison();
          return kNotTaken;
        }
      }
      backoff(spins);
    }
    if (!usable()) return kNotTaken;
    ServerSlot* sl = ring_w + si;
    const uint32_t nch = (P + kInlinePayload - 1) / kInlinePayload;
    uint8_t* const out_dev = inline_pk   ? iouts.dev + size_t(si) * kInlineOutBytes
                             : repair_dev ? repair_dev
                                          : outs.dev + size_t(si) * kResidentOutBytes;
    // The first lap of a tag epoch: no chunk the server wrote into this slot's output staging in
    // the previous epoch may carry a tag of this one (the server zeroed the slot's own words and
    // data area after serving its last lap; fec_kernels.hpp server_tag).  The previous occupant's
    // rows were all collected, so the device writes nothing here until this slot is published.
    if (vinl && seq >= kServerSlots && server_tag(seq, epoch) == 1u) {
      std::memset(iouts.host + size_t(si) * kInlineOutBytes, 0, kInlineOutBytes);
      std::atomic_thread_fence(std::memory_order_seq_cst);
    }
    uint64_t torn = ~0ull;  // test switch kResidentTear: the chunk whose low half is stored late
    if (inline_pk) {
      // the packets into the slot's data area (both halves of each chunk carry the tag), then the header
      uint8_t* const area = vinl + size_t(si) * kInlineSlotBytes;
      if (tear) torn = (seq * 7919u) % (uint64_t(G) * kServerPackets * nch);
      pack_inline(area, slab, offsets, G, P, tag16, torn);
      __atomic_store_n(&sl->out, reinterpret_cast<uint64_t>(out_dev) | tag, __ATOMIC_RELAXED);
      __atomic_store_n(&sl->shape, uint64_t(P) | (uint64_t(G) << 16) | kServerInline | tag, __ATOMIC_RELAXED);
      if (torn != ~0ull) {
        // the header out, the chunk's tagged high half landed, its low half ~100 us later
        std::atomic_thread_fence(std::memory_order_seq_cst);
        const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(100);
        while (std::chrono::steady_clock::now() < until) __builtin_ia32_pause();
        store_half(area + torn * 16, chunk_half(slab + offsets[torn / nch], P, uint32_t(torn % nch) * kInlinePayload, tag16));
      }
    } else {
      // groups after the first, then the first group and the header (every word tagged: the
      // device checks each one it reads, whatever order they land in)
      const bool late = tear && G > 1;  // tests: the later groups' words ~100 us after the header
      if (!late)
        for (uint32_t i = kServerPackets; i < G * kServerPackets; ++i) sl->addr[i] = (base + offsets[i]) | tag;
      std::atomic_thread_fence(std::memory_order_release);
      for (uint32_t i = 0; i < kServerPackets; ++i) __atomic_store_n(&sl->addr[i], (base + offsets[i]) | tag, __ATOMIC_RELAXED);
      __atomic_store_n(&sl->out, reinterpret_cast<uint64_t>(out_dev) | tag, __ATOMIC_RELAXED);
      __atomic_store_n(&sl->shape, uint64_t(P) | (uint64_t(G) << 16) | tag, __ATOMIC_RELEASE);
      if (late) {
        std::atomic_thread_fence(std::memory_order_seq_cst);
        const auto until = std::chrono::steady_clock::now() + std::chrono::microseconds(100);
        while (std::chrono::steady_clock::now() < until) __builtin_ia32_pause();
        for (uint32_t i = kServerPackets; i < G * kServerPackets; ++i)
          __atomic_store_n(&sl->addr[i], (base + offsets[i]) | tag, __ATOMIC_RELAXED);
      }
    }
    // through the BAR the stores sit in write-combining buffers until a serialising fence (mfence)
    if (vinl) std::atomic_thread_fence(std::memory_order_seq_cst);
    g_res_calls.fetch_add(1, std::memory_order_relaxed);
    if (inline_pk) g_res_inline.fetch_add(1, std::memory_order_relaxed);
    const uint64_t t_pub = now_ns();
    int rc = FEC_OK;
    const auto t_fail = std::chrono::steady_clock::now() + deadline;
    // An inline call's rows are complete when both 8-B halves of every chunk of its staging
    // carry the tag (the last chunk is watched first; chunks, and the halves of one chunk, land
    // in any order: the device's 16-B store is not assumed to arrive in one piece).
    const uint8_t* const stg = inline_pk ? iouts.host + size_t(si) * kInlineOutBytes : nullptr;
    uint32_t landed = 0;
    auto half_ok = [&](uint32_t h) {  // 8-B half h of the staging carries this lap's tag
      return (__atomic_load_n(reinterpret_cast<const uint64_t*>(stg) + h, __ATOMIC_ACQUIRE) >> 48) == tag16;
    };
    auto rows_landed = [&]() {
      if (!half_ok(2 * (G * nch - 1) + 1)) return false;
      while (landed < 2 * G * nch && half_ok(landed)) ++landed;
      return landed == 2 * G * nch;
    };
    // test switch kResidentFailAt: this call's deadline passes at once (no shared counter
    // otherwise: every call would pay one more contended atomic)
    if (fail_at != ~0ull && call_no.fetch_add(1, std::memory_order_relaxed) == fail_at) {
      set_last_error("fec_encode_batch: injected failure (test library)");
      rc = FEC_ERR_HIP;
    }
    for (uint32_t spins = 0; rc == FEC_OK; ++spins) {
      if (inline_pk ? rows_landed() : __atomic_load_n(dw, __ATOMIC_ACQUIRE) == seq + 1) break;
      // no instance serving (never launched, or it left): launch one from its progress mark
      if ((spins & 15u) == 0 && !instance_alive()) {
        rc = relaunch();
        if (rc != FEC_OK) break;
      }
      if ((spins & 1023u) == 1023u && std::chrono::steady_clock::now() > t_fail) {
        set_last_error("fec_encode_batch: the resident encoder did not serve the call within the deadline "
                       "(QUICFEC_RESIDENT_DEADLINE_MS); legacy calls now take the coalescer path");
        rc = FEC_ERR_HIP;
        break;
      }
      backoff(spins);
    }
    const uint64_t t_done = now_ns();
    if (rc != FEC_OK) {
      // Not served in time, or no instance can be launched (this call's deadline passed, or
      // another call poisoned the Resident).  Poison it (never relaunched; the stop word asks a
      // running instance to leave) and wait, bounded, until the instance has left: its done word
      // for this seq is then final.  The slot is not rewritten, so whether the device served it
      // never depends on a race with the host.  Served: the rows are in place (an instance's
      // stores are performed before its exited word), and the call succeeds.  Not served: the
      // device read nothing of this call's after the instance left, so the call is not taken and
      // runs on the coalescer path like every later legacy call.  An instance that does not leave
      // within the bound is hung: the call fails, and the caller's buffers handed to it must not
      // be reused (include/fec_xor_simd.h, fec_encode_batch).
      poison();
      const auto t_drain = std::chrono::steady_clock::now() + deadline;
      for (uint32_t spins = 0; instance_alive() && std::chrono::steady_clock::now() < t_drain; ++spins) backoff(spins);
      if (!instance_alive()) {
        const bool served = __atomic_load_n(dw, __ATOMIC_ACQUIRE) == seq + 1 && (!inline_pk || rows_landed());
        rc = served ? FEC_OK : kNotTaken;
      }
    }
    if (rc == FEC_OK && inline_pk) {
      // chunk c's 12 payload bytes to repair bytes [12c, 12c + 12): two 8-B copies per chunk,
      // in increasing order, each overwriting the previous one's two tag bytes, while the copy
      // stays inside the row (12c + 14 <= P); the last chunks byte-exact
      const uint32_t nfast = P >= 14 ? (P - 14) / kInlinePayload + 1 : 0;
      for (uint32_t g = 0; g < G; ++g) {
        const uint8_t* ch = stg + size_t(g) * nch * 16;
        uint8_t* dst = repair_out + size_t(g) * P;
        uint32_t c = 0;
        for (; c < nfast; ++c) {
          std::memcpy(dst + c * kInlinePayload, ch + c * 16, 8);
          std::memcpy(dst + c * kInlinePayload + 6, ch + c * 16 + 8, 8);
        }
        for (; c < nch; ++c) {
          const uint32_t n = std::min(kInlinePayload, P - c * kInlinePayload);
          std::memcpy(dst + c * kInlinePayload, ch + c * 16, std::min(6u, n));
          if (n > 6) std::memcpy(dst + c * kInlinePayload + 6, ch + c * 16 + 8, n - 6);
        }
      }
    } else if (rc == FEC_OK && !repair_dev) {
      std::memcpy(repair_out, outs.host + size_t(si) * kResidentOutBytes, size_t(G) * P);
    }
    collected[si].store(seq + 1, std::memory_order_release);
    if (rc == kNotTaken) {  // counted on the path that runs it
      g_res_calls.fetch_sub(1, std::memory_order_relaxed);
      if (inline_pk) g_res_inline.fetch_sub(1, std::memory_order_relaxed);
      return rc;
    }
    g_res_pre_ns.fetch_add(t_pub - t_enter, std::memory_order_relaxed);
    g_res_wait_ns.fetch_add(t_done - t_pub, std::memory_order_relaxed);
    g_res_post_ns.fetch_add(now_ns() - t_done, std::memory_order_relaxed);
    return rc;
  }

  // Process exit: ask the running instance to leave and wait, bounded, until its host-visible
  // `exited` word says it has.  No HIP call: under rocprofv3 the tool has finalised by the time
  // atexit handlers run, and a runtime call there aborted the process (f13ed47); the stream,
  // the page-locked ring and the device memory go with the process.  Never deleted.
  void shutdown() {
    __atomic_store_n(&reinterpret_cast<ServerControl*>(ctl.host)->stop, 1, __ATOMIC_RELEASE);
    if (gen.load(std::memory_order_acquire) == 0) return;
    const auto until = std::chrono::steady_clock::now() + std::chrono::milliseconds(200);
    while (instance_alive() && std::chrono::steady_clock::now() < until) std::this_thread::yield();
    if (stamps.host) print_stamps();
  }

  ~Resident() {  // only a Resident whose create() failed; never at exit (shutdown)
    if (stream) (void)hipStreamDestroy(stream);
  }

  // Test switch kResidentStamps: mean phase times of the last (up to) 256 served batches, to stderr.
  void print_stamps() const {
    const uint64_t* st = reinterpret_cast<const uint64_t*>(stamps.host);
    double sum[7] = {};
    uint32_t n = 0;
    for (uint32_t i = 0; i < 256; ++i) {
      if (st[i * 8 + 7] == 0) continue;
      for (int k = 0; k < 7; ++k) sum[k] += double(st[i * 8 + k]);
      ++n;
    }
    if (n == 0) return;
    const double us = 1000.0 / double(tick_khz);
    std::fprintf(stderr,
                 "{\"resident_stamps\": {\"batches\": %u, \"us\": {\"poll\": %.2f, \"acquire\": %.2f, \"loads\": %.2f, "
                 "\"store_issue\": %.2f, \"acked_barrier_done\": %.2f}, \"mean_slots\": %.2f, \"mean_polls\": %.2f}}\n",
                 n, sum[0] / n * us, sum[1] / n * us, sum[2] / n * us, sum[3] / n * us, sum[4] / n * us, sum[5] / n,
                 sum[6] / n);
  }

 private:
  int device = 0;
  hipStream_t stream = nullptr;
  uint64_t idle_ticks = 0, slow_ticks = 0, life_ticks = 0;
  Pinned ring, done, ctl, outs, stamps;
  uint64_t tick_khz = 100000;
  std::unique_ptr<std::atomic<uint64_t>[]> collected;  // per slot: seq + 1 of its last collected call
  std::atomic<uint64_t> class_next[kServerMaxClasses];  // the next seq of each class (c, then + classes)
  // every call updates both: each on a cache line of its own
  alignas(64) std::atomic<uint32_t> in_flight{0};       // calls inside encode()
  alignas(64) std::atomic<uint32_t> rr{0};              // round robin over the classes in use
  std::atomic<uint64_t> call_no{0};                     // calls so far (test switch kResidentFailAt)
  std::mutex mu;
  std::atomic<uint64_t> gen{0};  // generation of the last launched instance (0 = none yet)
  std::atomic<bool> broken{false};
  std::chrono::milliseconds deadline{10000};  // QUICFEC_RESIDENT_DEADLINE_MS
  bool no_launch = false;                     // test switch kResidentNoLaunch
  bool tear = false;                          // test switch kResidentTear
  uint64_t fail_at = ~0ull;                   // test switch kResidentFailAt
  bool spread = false;                        // test switch kResidentSpread
  uint32_t epoch = kServerEpoch;              // test switch kResidentEpoch
  uint32_t classes = 1;                       // QUICFEC_RESIDENT_SERVERS
  ServerCoord* coord = nullptr;               // device memory shared by the classes' workgroups
  std::atomic<bool> outs_ready{false};
  // The slots as the host writes them and as the device reads them: the page-locked ring, or
  // (setup_vram) one address for both, uncached device memory the host writes through the BAR.
  ServerSlot* ring_w = nullptr;
  ServerSlot* ring_d = nullptr;
  uint8_t* vinl = nullptr;  // VRAM ring: the slots' inline data areas (kInlineSlotBytes each)
  Pinned iouts;             // VRAM ring: the inline slots' tagged output staging (kInlineOutBytes each)

  // Moves the ring into VRAM when the host can store to device memory directly (a large-BAR
  // device; profiles/r04_probe_vram_host.jsonl: a host -> VRAM -> device -> host round trip in
  // 4.4 us, 8.1 us through page-locked memory).  Checked before it is used: the allocation must
  // be mapped in this process (/proc/self/maps) and a host store must reach the device's copy.
  // Any failure leaves the page-locked ring in place.  The device memory is never freed (like
  // the rest of a Resident, it goes with the process).
  void setup_vram() {
    int large_bar = 0;
    if (hipDeviceGetAttribute(&large_bar, hipDeviceAttributeIsLargeBar, device) != hipSuccess || !large_bar) {
      (void)hipGetLastError();
      return;
    }
    const size_t ring_bytes = sizeof(ServerSlot) * kServerSlots, inl_bytes = size_t(kInlineSlotBytes) * kServerSlots;
    void *vr = nullptr, *vi = nullptr;
    bool ok = hipExtMallocWithFlags(&vr, ring_bytes, hipDeviceMallocUncached) == hipSuccess &&
              hipExtMallocWithFlags(&vi, inl_bytes, hipDeviceMallocUncached) == hipSuccess && host_mapped(vr, ring_bytes) &&
              host_mapped(vi, inl_bytes);
    if (ok) {
      uint64_t probe[2] = {0x5EED0001CAFEF00Dull, 0x0123456789ABCDEFull}, back[2] = {0, 0};
      std::memcpy(vr, probe, sizeof(probe));
      std::atomic_thread_fence(std::memory_order_seq_cst);
      ok = hipMemcpy(back, vr, sizeof(back), hipMemcpyDeviceToHost) == hipSuccess && std::memcmp(back, probe, sizeof(back)) == 0;
    }
    // no word and no chunk half with a tag (tags are 1 .. epoch)
    ok = ok && hipMemsetAsync(vr, 0, ring_bytes, stream) == hipSuccess && hipMemsetAsync(vi, 0, inl_bytes, stream) == hipSuccess &&
         hipStreamSynchronize(stream) == hipSuccess;
    // the inline slots' output staging, only once the VRAM ring is usable (zeroed: no tagged half
    // before the device writes one)
    ok = ok && alloc_coherent(iouts, size_t(kInlineOutBytes) * kServerSlots);
    if (!ok) {
      (void)hipGetLastError();
      if (vr) (void)hipFree(vr);
      if (vi) (void)hipFree(vi);
      return;
    }
    ring_w = static_cast<ServerSlot*>(vr);
    ring_d = static_cast<ServerSlot*>(vr);
    vinl = static_cast<uint8_t*>(vi);
    g_res_vram.fetch_add(1, std::memory_order_relaxed);
  }

  // Whether [p, p + n) lies in one readable and writable mapping of this process.
  static bool host_mapped(const void* p, size_t n) {
    FILE* f = std::fopen("/proc/self/maps", "r");
    if (!f) return false;
    const uintptr_t a = reinterpret_cast<uintptr_t>(p);
    bool found = false;
    char line[512];
    while (!found && std::fgets(line, sizeof(line), f)) {
      unsigned long lo = 0, hi = 0;
      char perms[8] = {};
      if (std::sscanf(line, "%lx-%lx %7s", &lo, &hi, perms) == 3 && a >= lo && a + n <= hi)
        found = perms[0] == 'r' && perms[1] == 'w';
    }
    std::fclose(f);
    return found;
  }

  // One 8-B half of an inline chunk: payload bytes [off, off + 6) of a packet of P bytes (zero
  // past P) and the tag in the top two bytes (fec_kernels.hpp kServerInline).
  static uint64_t chunk_half(const uint8_t* src, uint32_t P, uint32_t off, uint32_t tag16) {
    uint64_t w = 0;
    if (off + 8 <= P) {
      std::memcpy(&w, src + off, 8);
      w &= 0x0000FFFFFFFFFFFFull;
    } else if (off < P) {
      std::memcpy(&w, src + off, std::min(6u, P - off));
    }
    return w | (uint64_t(tag16) << 48);
  }

  static void store_half(uint8_t* p, uint64_t w) { *reinterpret_cast<volatile uint64_t*>(p) = w; }

  // An inline slot's packets into its data area through the BAR (fec_kernels.hpp kServerInline):
  // packet p = g * 10 + j as nch 16-B chunks, each two 8-B halves of 6 payload bytes and the tag;
  // each chunk one 16-B store (write-combined).  torn (test switch kResidentTear): that
  // chunk gets only its high half here; the caller stores the low half after the header.
  static void pack_inline(uint8_t* area, const uint8_t* slab, const uint32_t* offsets, uint32_t G, uint32_t P,
                          uint32_t tag16, uint64_t torn) {
    typedef uint64_t v2u __attribute__((vector_size(16)));
    const uint32_t nch = (P + kInlinePayload - 1) / kInlinePayload;
    const uint32_t nfast = P >= 14 ? (P - 14) / kInlinePayload + 1 : 0;  // chunks whose two 8-B reads stay in the packet
    const uint64_t tg = uint64_t(tag16) << 48, lo48 = 0x0000FFFFFFFFFFFFull;
    for (uint32_t p = 0; p < G * kServerPackets; ++p) {
      const uint8_t* src = slab + offsets[p];
      volatile v2u* dst = reinterpret_cast<volatile v2u*>(area + size_t(p) * nch * 16);
      if (torn / nch == p) {
        // the test's torn packet: every chunk but the torn one whole; of that one only the tagged
        // high half, its low half left as the previous lap wrote it
        const uint32_t ct = static_cast<uint32_t>(torn % nch);
        for (uint32_t c = 0; c < nch; ++c)
          if (c != ct)
            dst[c] = v2u{chunk_half(src, P, c * kInlinePayload, tag16), chunk_half(src, P, c * kInlinePayload + 6, tag16)};
        store_half(area + (size_t(p) * nch + ct) * 16 + 8, chunk_half(src, P, ct * kInlinePayload + 6, tag16));
        continue;
      }
      uint32_t c = 0;
      for (; c < nfast; ++c) {
        uint64_t a, b;
        std::memcpy(&a, src + size_t(c) * kInlinePayload, 8);
        std::memcpy(&b, src + size_t(c) * kInlinePayload + 6, 8);
        dst[c] = v2u{(a & lo48) | tg, (b & lo48) | tg};
      }
      for (; c < nch; ++c)
        dst[c] = v2u{chunk_half(src, P, c * kInlinePayload, tag16), chunk_half(src, P, c * kInlinePayload + 6, tag16)};
    }
  }

  void poison() {
    broken.store(true, std::memory_order_release);
    __atomic_store_n(&reinterpret_cast<ServerControl*>(ctl.host)->stop, 1, __ATOMIC_RELEASE);
  }

  bool ensure_outs() {
    if (outs_ready.load(std::memory_order_acquire)) return true;
    std::lock_guard<std::mutex> lk(mu);
    if (!outs.host && !alloc_coherent(outs, size_t(kResidentOutBytes) * kServerSlots)) return false;
    outs_ready.store(true, std::memory_order_release);
    return true;
  }

  static void backoff(uint32_t spins) {
    if (spins < 2048) {
      for (int i = 0; i < 8; ++i) __builtin_ia32_pause();
    } else if (spins < 16384) {
      std::this_thread::yield();
    } else {
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }

  uint64_t sum_classes(uint64_t (ServerControl::*field)[kServerMaxClasses]) const {
    const ServerControl* c = reinterpret_cast<const ServerControl*>(ctl.host);
    uint64_t s = 0;
    for (uint32_t i = 0; i < kServerMaxClasses; ++i) s += __atomic_load_n(&(c->*field)[i], __ATOMIC_ACQUIRE);
    return s;
  }

  bool instance_alive() const {
    const uint64_t g = gen.load(std::memory_order_acquire);
    return g != 0 && __atomic_load_n(&reinterpret_cast<const ServerControl*>(ctl.host)->exited, __ATOMIC_ACQUIRE) != g;
  }

  // Launches the next instance unless another caller just did.
  int relaunch() {
    std::lock_guard<std::mutex> lk(mu);
    if (instance_alive()) return FEC_OK;
    const ServerControl* c = reinterpret_cast<const ServerControl*>(ctl.host);
    if (__atomic_load_n(&c->stop, __ATOMIC_ACQUIRE) || !usable()) {
      set_last_error("fec_encode_batch: the resident encoder is shutting down or out of service");
      return FEC_ERR_HIP;
    }
    const uint64_t g = gen.load(std::memory_order_relaxed) + 1;
    if (no_launch) {  // tests: an instance that is "alive" and never serves
      gen.store(g, std::memory_order_release);
      return FEC_OK;
    }
    // every class resumes from its own progress mark (ServerControl::progress, read by the instance)
    BindDevice bd(device);
    const hipError_t e = bd.ok ? launch_legacy_server(ring_d, vinl, reinterpret_cast<uint64_t*>(done.dev),
                                                      reinterpret_cast<ServerControl*>(ctl.dev), coord, classes, g,
                                                      idle_ticks, slow_ticks, life_ticks,
                                                      stamps.host ? reinterpret_cast<uint64_t*>(stamps.dev) : nullptr,
                                                      epoch, stream)
                               : hipErrorInvalidDevice;
    if (e != hipSuccess) {
      (void)hipGetLastError();
      set_last_error((std::string("fec_encode_batch: resident encoder launch failed: ") + hipGetErrorString(e)).c_str());
      return FEC_ERR_HIP;
    }
    gen.store(g, std::memory_order_release);
    g_res_launches.fetch_add(1, std::memory_order_relaxed);
    return FEC_OK;
  }
};

std::mutex g_reg_mu;
std::map<std::pair<int, uint32_t>, Coalescer*> g_reg;  // until process exit (shutdown_all)
constexpr int kResidentDevices = 64;
std::atomic<Resident*> g_resident_fast[kResidentDevices];  // set once per device
std::map<int, Resident*> g_resident;                   // per device; NULL when it cannot be set up

std::atomic<bool> g_shut{false};  // process exit: legacy calls run alone from here on
std::once_flag g_atexit_once;

// Process exit (std::atexit): stop every resident instance (a store to host memory and a
// bounded wait on its host-visible `exited` word).  No HIP call from here on: under a tool that
// tears the runtime down before atexit handlers run (rocprofv3), one aborted the process
// (f13ed47).  Residents, coalescers, their streams, events and page-locked buffers are left to
// process teardown (tests/csrc/exit_path_test.cpp counts the HIP calls made after exit begins).
void shutdown_all() {
  g_shut.store(true, std::memory_order_release);
  std::lock_guard<std::mutex> lk(g_reg_mu);
  for (int d = 0; d < kResidentDevices; ++d) g_resident_fast[d].store(nullptr, std::memory_order_release);
  for (auto& kv : g_resident)
    if (kv.second) kv.second->shutdown();
}

Resident* resident_for(int device) {
  if (device >= 0 && device < kResidentDevices) {
    if (Resident* r = g_resident_fast[device].load(std::memory_order_acquire)) return r;
  }
  std::call_once(g_atexit_once, [] { std::atexit(shutdown_all); });
  std::lock_guard<std::mutex> lk(g_reg_mu);
  if (g_shut.load(std::memory_order_acquire)) return nullptr;
  auto it = g_resident.find(device);
  if (it != g_resident.end()) return it->second;
  Resident* r = Resident::create(device);
  g_resident.emplace(device, r);
  if (r && device >= 0 && device < kResidentDevices) g_resident_fast[device].store(r, std::memory_order_release);
  return r;
}

// Set while this thread holds g_reg_mu in coalescer_for: Coalescer::create makes a context,
// whose first-context warm-up must not take g_reg_mu again (coalesce_prepare skips then).
thread_local bool t_holds_reg = false;

Coalescer* coalescer_for(int device, uint32_t P) {
  std::call_once(g_atexit_once, [] { std::atexit(shutdown_all); });
  std::lock_guard<std::mutex> lk(g_reg_mu);
  struct Flag {
    Flag() { t_holds_reg = true; }
    ~Flag() { t_holds_reg = false; }
  } flag;
  if (g_shut.load(std::memory_order_acquire)) return nullptr;
  const auto key = std::make_pair(device, P);
  auto it = g_reg.find(key);
  if (it != g_reg.end()) return it->second;
  if (g_reg.size() >= kMaxCoalescers) return nullptr;
  Coalescer* c = Coalescer::create(device, P);
  g_reg.emplace(key, c);  // NULL too: the pair is not retried on every call
  return c;
}

}  // namespace

void coalesce_prepare(int device) {
  if (t_holds_reg || env_long("QUICFEC_COALESCE", 1) == 0) return;
  prepare_spare_batch(device);
  if (env_long("QUICFEC_RESIDENT", 1) == 0) return;
  (void)resident_for(device);
}

bool coalesce_legacy_encode(int device, const uint8_t* slab, const uint32_t* offsets, uint32_t num_groups,
                            uint32_t packet_size, uint8_t* repair_out, int* rc, hipStream_t stream) {
  const uint64_t t_enter = now_ns();
  if (env_long("QUICFEC_COALESCE", 1) == 0 || g_shut.load(std::memory_order_acquire)) return false;
  if (num_groups > static_cast<uint64_t>(std::max(0L, env_long("QUICFEC_COALESCE_MAX_GROUPS", 64)))) return false;
  void *sdev = nullptr, *rdev = nullptr;
  const HostMem sm = classify_host_pointer(slab, &sdev);
  const HostMem rm = classify_host_pointer(repair_out, &rdev);
  if (sm == HostMem::kDevice || rm == HostMem::kDevice || classify_host_pointer(offsets, nullptr) == HostMem::kDevice)
    return false;  // device-resident callers batch by themselves
  const bool repair_pinned = rm == HostMem::kPinned;
  // The resident encoder: packets addressed in the caller's page-locked slab, or (VRAM ring)
  // copied into the slot from any host memory.
  const bool slab_addressable =
      sm == HostMem::kPinned && reinterpret_cast<uint64_t>(sdev) + 0xFFFFFFFFull + packet_size <= kServerAddrMask;
  if (env_long("QUICFEC_RESIDENT", 1) != 0 && Resident::fits(num_groups, packet_size, repair_pinned) &&
      reinterpret_cast<uint64_t>(rdev) <= kServerAddrMask) {
    Resident* r = resident_for(device);
    if (r && r->usable() && (slab_addressable || r->inlines(num_groups, packet_size))) {
      const int res = r->encode(slab, slab_addressable ? static_cast<const uint8_t*>(sdev) : nullptr, offsets, num_groups,
                                packet_size, repair_out, repair_pinned ? static_cast<uint8_t*>(rdev) : nullptr, t_enter);
      if (res != Resident::kNotTaken) {
        *rc = res;
        return true;
      }
    }
  }
  // Pageable packets are staged per batch at cap * 10 * P bytes (cap >= 8): past this size the
  // legacy call runs alone on its context (QUIC datagrams are <= 1500 B).
  if (packet_size > kCoalesceMaxP) return false;
  const uint64_t t_cls = now_ns();
  Coalescer* c = coalescer_for(device, packet_size);
  if (!c || num_groups > c->capacity() / 2) return false;
  const uint64_t t_for = now_ns();
  *rc = c->encode(slab, sm == HostMem::kPinned ? static_cast<const uint8_t*>(sdev) : nullptr, offsets, num_groups,
                  repair_out, stream);
  static std::atomic<int> stamps_left{test_knob(TestKnob::kCoalesceStamps, 0) != 0 ? 3 : 0};
  if (stamps_left.load(std::memory_order_relaxed) > 0 && stamps_left.fetch_sub(1) > 0)  // diagnostic
    std::fprintf(stderr, "{\"coalesced_call_us\": {\"classify\": %.1f, \"coalescer_for\": %.1f, \"encode\": %.1f}}\n",
                 (t_cls - t_enter) / 1e3, (t_for - t_cls) / 1e3, (now_ns() - t_for) / 1e3);
  return true;
}

}  // namespace qfec

// The totals are gathered into a full struct of this build and copied out at the caller's size:
// a binary built against an older fec_hip.h (a smaller struct) never has fields written past it.
QFEC_EXPORT int fec_coalesce_stats_sized(FECCoalesceStats* caller, size_t caller_bytes, int reset) {
  if (!caller) return FEC_ERR_NULL;
  using namespace qfec;
  if (caller_bytes < kCoalesceStatsV4Bytes) return FEC_ERR_RANGE;
  FECCoalesceStats full{};
  FECCoalesceStats* const out = &full;
  out->calls = g_calls.load();
  out->groups = g_groups.load();
  out->batches = g_batches.load();
  out->max_batch = g_max_batch.load();
  out->max_calls = g_max_calls.load();
  out->close_ns = g_close_ns.load();
  out->launch_ns = g_launch_ns.load();
  out->done_ns = g_done_ns.load();
  out->resident_calls = g_res_calls.load();
  out->resident_launches = g_res_launches.load();
  out->resident_pre_ns = g_res_pre_ns.load();
  out->resident_wait_ns = g_res_wait_ns.load();
  out->resident_post_ns = g_res_post_ns.load();
  out->resident_inline = g_res_inline.load();
  out->resident_vram = g_res_vram.load();
  out->resident_bad_slots = 0;
  out->resident_scrubs = 0;
  out->resident_servers = 0;
  {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    for (auto& kv : g_resident)
      if (kv.second) {
        out->resident_bad_slots += kv.second->bad_slots();
        out->resident_scrubs += kv.second->scrubs();
        out->resident_servers = std::max<uint64_t>(out->resident_servers, kv.second->serving_classes());
      }
  }
  if (reset) {
    g_res_calls = 0;
    g_res_launches = 0;
    g_res_pre_ns = 0;
    g_res_wait_ns = 0;
    g_res_post_ns = 0;
    g_res_inline = 0;
    g_close_ns = 0;
    g_launch_ns = 0;
    g_done_ns = 0;
    g_calls = 0;
    g_groups = 0;
    g_batches = 0;
    g_max_batch = 0;
    g_max_calls = 0;
  }
  std::memcpy(caller, &full, std::min(caller_bytes, sizeof(full)));
  return FEC_OK;
}

// The round-4 entry point: the 15 fields it was published with, never more (its callers' struct
// may end there).  New callers use fec_coalesce_stats_sized.
QFEC_EXPORT int fec_coalesce_stats(FECCoalesceStats* out, int reset) {
  return fec_coalesce_stats_sized(out, qfec::kCoalesceStatsV4Bytes, reset);
}
