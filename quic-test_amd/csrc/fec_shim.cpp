// fec_shim.cpp — C-ABI of libfec_hip.so (include/fec_xor_simd.h, include/fec_hip.h).
//
// Replaces the reference's native library internal/fec/fec_xor_simd.cpp behind the
// same eleven symbols, and adds the batch GF(2^8) encode/decode API.  All arithmetic
// runs in the gfx950 kernels of fec_kernels.hip; this file owns contexts, device
// buffers, host<->device staging, per-(k,r) plans and error reporting.
//
// Threading (SURVEY.md §8(b) "Threading"): one context per caller stream of work; every
// entry point locks its context and binds the context's device for the duration of the
// call (Go goroutines migrate between OS threads and the HIP current device is
// thread-local), restoring the caller's device afterwards.
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <shared_mutex>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "fec_hip.h"
#include "fec_internal.hpp"
#include "fec_kernels.hpp"
#include "fec_knobs.hpp"
#include "gf256.hpp"

#define QFEC_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

int hip_fail(hipError_t e, const char* what) {
  set_error("%s: %s", what, hipGetErrorString(e));
  return FEC_ERR_HIP;
}

#define QFEC_HIP(call)                                 \
  do {                                                 \
    const hipError_t qfec_e_ = (call);                 \
    if (qfec_e_ != hipSuccess) return hip_fail(qfec_e_, #call); \
  } while (0)

// Binds a device for the scope, restores the caller's device on exit.
struct DeviceGuard {
  int prev = -1;
  bool ok = false;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    ok = hipSetDevice(dev) == hipSuccess;
    if (!ok) (void)hipGetLastError();
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// Grow-only device buffer (freed with its owner).
struct DevBuf {
  void* ptr = nullptr;
  size_t cap = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() { release(); }
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (ptr) {
      (void)hipFree(ptr);
      ptr = nullptr;
      cap = 0;
    }
    size_t want = bytes < 256 ? 256 : bytes;
    hipError_t e = hipMalloc(&ptr, want);
    if (e != hipSuccess) {
      ptr = nullptr;
      return e;
    }
    cap = want;
    return hipSuccess;
  }
  void release() {
    if (ptr) (void)hipFree(ptr);
    ptr = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const { return static_cast<T*>(ptr); }
};

struct EncodePlan {
  DevBuf tables;  // (r-1) * k CoefEntry
};

struct DecodePlan {
  bool dense = false;          // dense codebook of every pattern (else: sparse per call)
  qfec::CodebookLayout layout;
  DevBuf codebook;
  qfec::CodebookLayout clayout;  // compact (coefficient-byte) book, built on first use
  DevBuf cbook;
  std::vector<uint8_t> M;      // parity matrix, for sparse per-call records
  DevBuf sparse_book;          // the last sparse call's records
};

constexpr uint64_t kCodebookCap = 2ull << 30;  // 2 GiB of recovery tables per (k, r)

// Grow-only page-locked host buffer (staging for the compacted host decode).
struct HostBuf {
  void* ptr = nullptr;
  void* dev = nullptr;   // the same memory as the kernels address it
  size_t cap = 0;
  HostBuf() = default;
  HostBuf(const HostBuf&) = delete;
  HostBuf& operator=(const HostBuf&) = delete;
  ~HostBuf() { release(); }
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    release();
    const size_t want = bytes < 4096 ? 4096 : bytes;
    const hipError_t e = hipHostMalloc(&ptr, want, hipHostMallocDefault);
    if (e != hipSuccess) {
      ptr = nullptr;
      return e;
    }
    cap = want;
    if (hipHostGetDevicePointer(&dev, ptr, 0) != hipSuccess || dev == nullptr) {
      (void)hipGetLastError();
      dev = ptr;  // unified addressing: the host pointer is the device address
    }
    return hipSuccess;
  }
  void release() {
    if (ptr) (void)hipHostFree(ptr);
    ptr = nullptr;
    dev = nullptr;
    cap = 0;
  }
  template <class T>
  T* as() const { return static_cast<T*>(ptr); }
  template <class T>
  T* dev_as() const { return static_cast<T*>(dev); }
};

// Host threads for the CPU side of the host-resident paths (gathering / scattering
// packets): QUICFEC_HOST_THREADS, default 8, at most the machine's.
unsigned host_threads() {
  static const unsigned n = [] {
    unsigned hw = std::thread::hardware_concurrency();
    if (hw == 0) hw = 1;
    unsigned want = 8;
    if (const char* v = std::getenv("QUICFEC_HOST_THREADS")) {
      const int x = std::atoi(v);
      if (x > 0) want = static_cast<unsigned>(x);
    }
    return want < hw ? want : hw;
  }();
  return n;
}

// f(begin, end) over [0, n) split across host_threads() threads (inline when small).
template <class F>
void parallel_for(uint64_t n, uint64_t min_per_thread, F&& f) {
  uint64_t nt = host_threads();
  if (min_per_thread > 0 && n / min_per_thread < nt) nt = n / min_per_thread;
  if (nt <= 1) {
    f(uint64_t(0), n);
    return;
  }
  std::vector<std::thread> th;
  th.reserve(nt - 1);
  for (uint64_t t = 1; t < nt; ++t) th.emplace_back([&f, n, nt, t] { f(n * t / nt, n * (t + 1) / nt); });
  f(uint64_t(0), n / nt);
  for (auto& x : th) x.join();
}

enum class Mem { kHost, kPinned, kDevice };

// Page-locked buffers this library handed out (fec_alloc_slab / _numa / fec_alloc_repair_buffer).
// The Go wrapper passes the same two of them to every legacy call (fec_cgo.go:64, :76, :138);
// finding them here keeps hipPointerGetAttributes -- a runtime lock and a lookup per pointer --
// off the per-call path.
struct PinnedRange {
  uintptr_t hi;   // one past the last byte
  uintptr_t dev;  // device address of the first byte
};
std::shared_mutex g_pin_mu;
std::map<uintptr_t, PinnedRange> g_pinned;  // by first byte

void pinned_register(void* p, size_t len) {
  if (!p || len == 0) return;
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, p, 0) != hipSuccess || d == nullptr) {
    (void)hipGetLastError();
    d = p;
  }
  std::unique_lock<std::shared_mutex> lk(g_pin_mu);
  g_pinned[reinterpret_cast<uintptr_t>(p)] = PinnedRange{reinterpret_cast<uintptr_t>(p) + len, reinterpret_cast<uintptr_t>(d)};
}

void pinned_unregister(void* p) {
  std::unique_lock<std::shared_mutex> lk(g_pin_mu);
  g_pinned.erase(reinterpret_cast<uintptr_t>(p));
}

bool pinned_lookup(const void* p, void** dev) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  std::shared_lock<std::shared_mutex> lk(g_pin_mu);
  auto it = g_pinned.upper_bound(a);
  if (it == g_pinned.begin()) return false;
  --it;
  if (a >= it->second.hi) return false;
  if (dev) *dev = reinterpret_cast<void*>(it->second.dev + (a - it->first));
  return true;
}

// `dev` (optional): for page-locked host memory, the address kernels use for `p`.
Mem classify_ptr(const void* p, void** dev = nullptr) {
  if (dev) *dev = nullptr;
  if (!p) return Mem::kHost;
  if (pinned_lookup(p, dev)) return Mem::kPinned;
  hipPointerAttribute_t attr;
  std::memset(&attr, 0, sizeof(attr));
  const hipError_t e = hipPointerGetAttributes(&attr, p);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return Mem::kHost;
  }
  if (attr.type == hipMemoryTypeDevice || attr.type == hipMemoryTypeManaged) return Mem::kDevice;
  if (attr.type == hipMemoryTypeHost) {
    if (dev) *dev = attr.devicePointer ? attr.devicePointer : const_cast<void*>(p);
    return Mem::kPinned;
  }
  return Mem::kHost;
}

// Host-resident calls up to small_call_bytes() (data + parity bytes) run zero-copy: the
// kernels address page-locked host memory directly over PCIe -- the caller's buffers when
// they are page-locked (fec_alloc_slab), else the context's page-locked staging, filled
// and drained by CPU memcpy.  No DMA copies: one kernel launch and one stream synchronize
// per call, where the DMA path pays a copy-engine round trip per buffer.  Measured
// (tools/latency.cpp, k=10 r=3 1200 B, profiles/r01_latency_sweep.txt): one group 33 -> 15 us
// (legacy fec_encode_batch).  With page-locked buffers zero-copy beats the DMA pipeline at
// every size (4096 groups: 942 vs 1013 us encode, 947 vs 1281 us decode; 1M groups, 12 GB:
// encode 52.0 vs 48.7 GiB/s, 2-erasure decode 52.4 vs 34.8, C5 sparse-loss decode 454 vs
// 243; profiles/r01_e2e_zero_copy.txt), so it has no limit; staged pageable buffers pay a
// CPU memcpy and break even near 3 MB.  QUICFEC_SMALL_CALL_BYTES overrides both limits
// (0 = always DMA).
constexpr uint64_t kZeroCopyPinnedBytes = ~0ull;

// Completion wait of the zero-copy calls.  The runtime's blocking wait: polling
// hipStreamQuery from the calling thread measured slower (one group: 20 vs 15.5 us;
// profiles/r01_latency_sweep.txt).
hipError_t wait_stream(hipStream_t s) { return hipStreamSynchronize(s); }

constexpr uint64_t kZeroCopyStagedBytes = 2ull << 20;
uint64_t small_call_bytes(bool all_pinned) {  // read per call: tests switch paths in one process
  const char* v = std::getenv("QUICFEC_SMALL_CALL_BYTES");
  const long long x = v && *v ? std::atoll(v) : -1;
  if (x >= 0) return static_cast<uint64_t>(x);
  return all_pinned ? kZeroCopyPinnedBytes : kZeroCopyStagedBytes;
}

}  // namespace

// One stage of the host<->device pipeline: its own stream and device buffers.
struct PipeSlot {
  hipStream_t s = nullptr;
  DevBuf in, par, mask, status, rec;
  HostBuf h_in, h_par, h_mask;          // compacted host decode staging
  std::vector<uint64_t> h_groups;        // the groups gathered into this slot's staging
};
constexpr int kPipeSlots = 3;
constexpr uint64_t kPipeChunkBytes = 64ull << 20;  // data bytes per pipelined chunk

// QUICFEC_PIPE_CHUNK_BYTES overrides the chunk size (tests use small chunks to run many).
uint64_t pipe_chunk_bytes() {
  const char* v = std::getenv("QUICFEC_PIPE_CHUNK_BYTES");
  const long long x = v ? std::atoll(v) : 0;
  return x > 0 ? static_cast<uint64_t>(x) : kPipeChunkBytes;
}
// Host-resident decode moves only the groups to rebuild when they are at most 1 in
// kCompactMaxShare of the batch; above that the whole batch streams through the pipeline.
constexpr uint64_t kCompactMaxShare = 2;

// A caller stream's decode workspace (stream_workspace).
struct StreamWorkspace {
  hipStream_t s = nullptr;
  DevBuf buf;
  uint64_t last_use = 0;
  // one-launch packed recover (recover_runs): ticket, chunk totals and look-back words, zeroed
  // when allocated; `epoch` = the last look-back epoch a launch on this stream used
  DevBuf runs;
  uint32_t epoch = 0;
};

struct FECEncoderCtx {
  double redundancy = 0.10;
  uint32_t max_groups = 1024;
  int device = 0;
  hipStream_t stream = nullptr;
  std::mutex mu;
  // staging / workspace buffers
  DevBuf d_in, d_off, d_out, d_mask, d_status, d_binom;
  HostBuf z_in, z_out, z_aux;           // zero-copy staging of small host-resident calls
  PipeSlot pipe[kPipeSlots];
  std::map<std::pair<uint32_t, uint32_t>, std::unique_ptr<EncodePlan>> enc_plans;
  std::map<std::pair<uint32_t, uint32_t>, std::unique_ptr<DecodePlan>> dec_plans;
  // Message of the last failing call on this context (fec_ctx_last_error): callers whose
  // threads migrate between the failing call and the read (Go goroutines) cannot rely on the
  // thread-local fec_hip_last_error.  Own lock: readable while a call holds `mu`.
  std::mutex err_mu;
  std::string last_error;
  // fec_decode_loss_hint: expected share of groups with lost data in device-resident decode
  // calls (< 0: unknown, treated as dense).
  double decode_need_share = -1.0;
  // per-stream record-offset workspaces of the device-resident decodes (stream_workspace)
  std::vector<std::unique_ptr<StreamWorkspace>> stream_ws;
  uint64_t ws_clock = 0;

  ~FECEncoderCtx() {
    DeviceGuard g(device);
    if (!stream_ws.empty()) {  // caller streams may still run decodes that read them
      (void)hipDeviceSynchronize();
      stream_ws.clear();
    }
    if (stream) (void)hipStreamSynchronize(stream);
    for (auto& p : pipe)
      if (p.s) (void)hipStreamSynchronize(p.s);
    d_in.release();
    d_off.release();
    d_out.release();
    d_mask.release();
    d_status.release();
    d_binom.release();
    z_in.release();
    z_out.release();
    z_aux.release();
    for (auto& p : pipe) {
      p.in.release();
      p.par.release();
      p.mask.release();
      p.status.release();
      p.rec.release();
      p.h_in.release();
      p.h_par.release();
      p.h_mask.release();
      if (p.s) (void)hipStreamDestroy(p.s);
    }
    enc_plans.clear();
    dec_plans.clear();
    if (stream) (void)hipStreamDestroy(stream);
  }
};

namespace {

// The first kernel launched on a device loads the library's code object there (all kernels of
// fec_kernels.hip at once), and the resident encoder's first call allocates its page-locked
// ring: together ~26 ms that otherwise land on the first fec_encode_batch of the process — the
// first repair packet of the first QUIC stream (batcher_latency legacy_raw: max delay 25.8-27.5
// ms without, 11.5-12.2 ms with the code object loaded here).  Done once per device, at the
// first context; failures are left to the calls that follow (they report them).
void warm_device_once(int device, hipStream_t s) {
  constexpr int kMaxWarm = 64;
  static std::once_flag once[kMaxWarm];
  if (device < 0 || device >= kMaxWarm || std::getenv("QUICFEC_NO_WARMUP") != nullptr) return;
  std::call_once(once[device], [&] {
    uint8_t* p = nullptr;
    if (hipMalloc(&p, 256) == hipSuccess) {
      if (qfec::launch_fill_splitmix(p, 256, 0, 0, s) == hipSuccess) (void)hipStreamSynchronize(s);
      (void)hipFree(p);
    }
    (void)hipGetLastError();
    qfec::coalesce_prepare(device);
  });
}

FECEncoderCtx* make_ctx(double redundancy, uint32_t max_groups, int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
    (void)hipGetLastError();
    set_error("fec_encoder_new: no HIP device available");
    return nullptr;
  }
  if (device < 0) {
    if (hipGetDevice(&device) != hipSuccess) device = 0;
  }
  if (device >= n) {
    set_error("fec_encoder_new: device %d out of range (%d devices)", device, n);
    return nullptr;
  }
  DeviceGuard g(device);
  if (!g.ok) {
    set_error("fec_encoder_new: hipSetDevice(%d) failed", device);
    return nullptr;
  }
  auto* ctx = new FECEncoderCtx();
  // fec_xor_simd.cpp:540-541 defaults
  ctx->redundancy = (redundancy > 0 && redundancy <= 1.0) ? redundancy : 0.10;
  ctx->max_groups = max_groups > 0 ? max_groups : 1024;
  ctx->device = device;
  const hipError_t e = hipStreamCreateWithFlags(&ctx->stream, hipStreamDefault);
  if (e != hipSuccess) {
    set_error("fec_encoder_new: hipStreamCreate: %s", hipGetErrorString(e));
    ctx->stream = nullptr;
    delete ctx;
    return nullptr;
  }
  warm_device_once(device, ctx->stream);
  return ctx;
}

int get_encode_plan(FECEncoderCtx* ctx, uint32_t k, uint32_t r, const void** tables) {
  if (r == 1) {  // the XOR row alone needs no coefficients, so any number of packets works
    *tables = nullptr;
    return k > 0 ? FEC_OK : FEC_ERR_RANGE;
  }
  auto key = std::make_pair(k, r);
  auto it = ctx->enc_plans.find(key);
  if (it == ctx->enc_plans.end()) {
    std::vector<uint8_t> M;
    if (!qfec::parity_matrix(k, r, M)) {
      set_error("encode: unsupported k=%u r=%u (need k>0, r>0, k+r<=256)", k, r);
      return FEC_ERR_RANGE;
    }
    auto plan = std::make_unique<EncodePlan>();
    if (r > 1) {
      std::vector<qfec::CoefEntry> tab(size_t(r - 1) * k);
      for (uint32_t i = 1; i < r; ++i)
        for (uint32_t j = 0; j < k; ++j) tab[(i - 1) * k + j] = qfec::make_entry(M[i * k + j]);
      QFEC_HIP(plan->tables.ensure(tab.size() * sizeof(qfec::CoefEntry)));
      QFEC_HIP(hipMemcpy(plan->tables.ptr, tab.data(), tab.size() * sizeof(qfec::CoefEntry),
                         hipMemcpyHostToDevice));
    }
    it = ctx->enc_plans.emplace(key, std::move(plan)).first;
  }
  *tables = it->second->tables.ptr;
  return FEC_OK;
}

int get_decode_plan(FECEncoderCtx* ctx, uint32_t k, uint32_t r, DecodePlan** out) {
  auto key = std::make_pair(k, r);
  auto it = ctx->dec_plans.find(key);
  if (it == ctx->dec_plans.end()) {
    auto plan = std::make_unique<DecodePlan>();
    if (k + r > qfec::kMaxDecodeShards || !qfec::parity_matrix(k, r, plan->M)) {
      set_error("decode: unsupported k=%u r=%u (need k+r<=64)", k, r);
      return FEC_ERR_RANGE;
    }
    // Dense codebook when it fits the cap; otherwise records are built per call for the
    // patterns present (build_sparse_plan).
    plan->dense = qfec::codebook_layout(k, r, kCodebookCap, plan->layout);
    if (plan->dense) {
      std::vector<uint8_t> book;
      if (!qfec::build_codebook(plan->layout, plan->M, book)) {
        set_error("decode: singular recovery submatrix for k=%u r=%u", k, r);
        return FEC_ERR_RANGE;
      }
      QFEC_HIP(plan->codebook.ensure(book.size()));
      QFEC_HIP(hipMemcpy(plan->codebook.ptr, book.data(), book.size(), hipMemcpyHostToDevice));
    }
    if (!ctx->d_binom.ptr) {
      QFEC_HIP(ctx->d_binom.ensure(sizeof(qfec::binom().c)));
      QFEC_HIP(hipMemcpy(ctx->d_binom.ptr, qfec::binom().c, sizeof(qfec::binom().c),
                         hipMemcpyHostToDevice));
    }
    it = ctx->dec_plans.emplace(key, std::move(plan)).first;
  }
  *out = it->second.get();
  return FEC_OK;
}

hipStream_t pick_stream(FECEncoderCtx* ctx, void* stream) {
  return stream ? static_cast<hipStream_t>(stream) : ctx->stream;
}

// Device-resident encode, contiguous layout.  Caller holds ctx->mu and the device.
int encode_dev_locked(FECEncoderCtx* ctx, const uint8_t* d_data, const void* d_offsets,
                      qfec::OffsetKind ok, uint64_t G, uint32_t k, uint32_t r, uint32_t P,
                      uint8_t* d_parity, hipStream_t s) {
  const void* tables = nullptr;
  int rc = get_encode_plan(ctx, k, r, &tables);
  if (rc != FEC_OK) return rc;
  qfec::EncodeLaunch a;
  a.data = d_data;
  a.offsets = d_offsets;
  a.off_kind = ok;
  a.parity = d_parity;
  a.groups = G;
  a.k = k;
  a.r = r;
  a.P = P;
  a.tables = tables;
  QFEC_HIP(qfec::launch_encode(a, s));
  return FEC_OK;
}

// Record-offset workspace of device-resident decodes, one buffer per caller stream: calls
// on one stream run in stream order, so the next call on it may reuse the buffer while the
// previous call's kernels are still queued; decodes in flight on different streams never
// share one (the context-wide buffer they used to share could be overwritten by the next
// call's classify before the previous call's decode read it).  A buffer grows only after
// its stream has drained; the least recently used of kMaxStreamWorkspaces is dropped after
// a device synchronize.  (A per-call stream-ordered allocation, hipMallocAsync/hipFreeAsync,
// handed out memory that a queued decode on the same stream was still reading:
// tools/batcher_latency.cpp decode mode, ~20% of k=10 r=2 groups wrong.)  Caller holds
// ctx->mu.
constexpr size_t kMaxStreamWorkspaces = 16;

hipError_t find_stream_ws(FECEncoderCtx* ctx, hipStream_t s, StreamWorkspace** out);

hipError_t stream_workspace(FECEncoderCtx* ctx, hipStream_t s, size_t bytes, void** out) {
  StreamWorkspace* w = nullptr;
  const hipError_t fe = find_stream_ws(ctx, s, &w);
  if (fe != hipSuccess) return fe;
  if (bytes > w->buf.cap) {
    if (w->buf.ptr) {
      const hipError_t e = hipStreamSynchronize(s);  // queued calls may still read the old one
      if (e != hipSuccess) return e;
    }
    const hipError_t e = w->buf.ensure(bytes);
    if (e != hipSuccess) return e;
  }
  *out = w->buf.ptr;
  return hipSuccess;
}

// The recover_runs workspace of caller stream s and the first look-back epoch of a call of G
// groups.  Epochs are never reused while the buffer lives (words of earlier launches on this
// stream cannot match); the buffer is zeroed when allocated and when the epochs wrap.
hipError_t runs_workspace(FECEncoderCtx* ctx, hipStream_t s, uint64_t G, void** out, uint32_t* epoch) {
  StreamWorkspace* w = nullptr;
  hipError_t e = find_stream_ws(ctx, s, &w);
  if (e != hipSuccess) return e;
  const uint64_t bytes = qfec::runs_workspace_bytes(G);
  const uint32_t n = qfec::runs_launches(G);
  if (bytes > w->runs.cap) {
    if (w->runs.ptr && (e = hipStreamSynchronize(s)) != hipSuccess) return e;
    if ((e = w->runs.ensure(bytes)) != hipSuccess) return e;
    w->epoch = 0;
    if ((e = hipMemsetAsync(w->runs.ptr, 0, w->runs.cap, s)) != hipSuccess) return e;
  } else if (w->epoch + n >= (1u << 30)) {
    w->epoch = 0;
    if ((e = hipMemsetAsync(w->runs.ptr, 0, w->runs.cap, s)) != hipSuccess) return e;
  }
  *out = w->runs.ptr;
  *epoch = w->epoch + 1;
  w->epoch += n;
  return hipSuccess;
}

hipError_t find_stream_ws(FECEncoderCtx* ctx, hipStream_t s, StreamWorkspace** out) {
  StreamWorkspace* w = nullptr;
  for (auto& e : ctx->stream_ws)
    if (e->s == s) {
      w = e.get();
      break;
    }
  if (!w) {
    if (ctx->stream_ws.size() >= kMaxStreamWorkspaces) {
      auto lru = std::min_element(ctx->stream_ws.begin(), ctx->stream_ws.end(),
                                  [](const auto& x, const auto& y) { return x->last_use < y->last_use; });
      const hipError_t e = hipDeviceSynchronize();  // its stream may be gone: drain everything
      if (e != hipSuccess) return e;
      ctx->stream_ws.erase(lru);
    }
    ctx->stream_ws.push_back(std::make_unique<StreamWorkspace>());
    w = ctx->stream_ws.back().get();
    w->s = s;
  }
  w->last_use = ++ctx->ws_clock;
  *out = w;
  return hipSuccess;
}

int decode_dev_locked(FECEncoderCtx* ctx, uint8_t* d_data, const uint8_t* d_parity,
                      const uint64_t* d_masks, uint64_t G, uint32_t k, uint32_t r, uint32_t P,
                      uint8_t* d_status, hipStream_t s, DevBuf* rec = nullptr,
                      uint8_t* d_out = nullptr, double need_share = -1.0, bool compact_out = false,
                      uint32_t* row_start = nullptr, uint64_t* row_total = nullptr) {
  DecodePlan* plan = nullptr;
  int rc = get_decode_plan(ctx, k, r, &plan);
  if (rc != FEC_OK) return rc;
  qfec::DecodeLaunch a;
  a.data = d_data;
  a.parity = d_parity;
  a.masks = d_masks;
  a.rec_off = nullptr;
  a.out = d_out;
  a.compact_out = compact_out;
  a.status = d_status;
  a.codebook = plan->codebook.as<uint8_t>();
  a.binom = ctx->d_binom.as<uint64_t>();
  std::memset(&a.meta, 0, sizeof(a.meta));
  for (uint32_t e = 1; e <= 32; ++e) {
    a.meta.base[e] = plan->layout.level_base[e];
    a.meta.stride[e] = plan->layout.level_stride[e];
    a.meta.count_r[e] = qfec::binom().c[r][e];
  }
  a.groups = G;
  a.k = k;
  a.r = r;
  a.P = P;
  a.rec_ready = !plan->dense;
  if (plan->dense && qfec::decode_compact_tables(a)) {
    // the form reads bare coefficient bytes: the compact book of the same patterns
    if (!plan->cbook.ptr) {
      std::vector<uint8_t> book;
      if (!qfec::codebook_layout(k, r, kCodebookCap, plan->clayout, /*compact=*/true) ||
          !qfec::build_codebook(plan->clayout, plan->M, book)) {
        set_error("decode: compact codebook failed for k=%u r=%u", k, r);
        return FEC_ERR_RANGE;
      }
      QFEC_HIP(plan->cbook.ensure(book.size()));
      QFEC_HIP(hipMemcpy(plan->cbook.ptr, book.data(), book.size(), hipMemcpyHostToDevice));
    }
    a.compact_tables = true;
    a.codebook = plan->cbook.as<uint8_t>();
    for (uint32_t e = 1; e <= 32; ++e) {
      a.meta.base[e] = plan->clayout.level_base[e];
      a.meta.stride[e] = plan->clayout.level_stride[e];
    }
  }
  // Groups per wave of the mask-addressed form: the scan form when the caller knows that
  // few groups need a rebuild (need_share, from a host scan of the masks); device-resident
  // callers get one wave per group (the test library's TestKnob::kDecodeScan overrides it).
  if (need_share < 0.0) need_share = ctx->decode_need_share;
  if (need_share >= 0.0 && need_share < qfec::kDecodeScanMaxShare) a.scan = qfec::kDecodeScanGroups;
  a.scan = static_cast<uint32_t>(qfec::test_knob(qfec::TestKnob::kDecodeScan, a.scan));
  if (row_start != nullptr) {
    // packed rows: only the mask-addressed (inline-classify) forms place rows by row_start,
    // which they read from rec_off
    if (!plan->dense || qfec::decode_needs_rec_off(a)) {
      set_error("packed recover: no mask-addressed form for k=%u r=%u P=%u (use fec_recover_batch_rs_dev)", k, r, P);
      return FEC_ERR_RANGE;
    }
    // Sparse loss (the scan form's share): one launch, recover_runs --
    // each workgroup finds its rows' place by decoupled look-back and writes them as one run
    // (C5: 0.229-0.235 vs 0.242-0.268 ms for the slot rows; profiles/r04_probe_runs_*.txt).
    // Dense loss keeps the prefix launches + decode_fused (the runs form rebuilds a workgroup's
    // groups wave by wave: 2.7-2.8 vs 2.2-2.45 ms at C3).  The test library's
    // TestKnob::kPackedRuns forces it on (1) or off (0).
    const long runs_env = qfec::test_knob(qfec::TestKnob::kPackedRuns, -1);
    if (runs_env != 0 && (runs_env == 1 || a.scan == qfec::kDecodeScanGroups) && qfec::runs_supported(k, r, P)) {
      qfec::RunsLaunch ra{};
      ra.data = d_data;
      ra.parity = d_parity;
      ra.masks = d_masks;
      ra.groups = G;
      ra.k = k;
      ra.r = r;
      ra.P = P;
      ra.codebook = a.codebook;
      ra.meta = a.meta;
      ra.out = d_out;
      ra.row_start = row_start;
      ra.total = row_total;
      ra.status = d_status;
      QFEC_HIP(runs_workspace(ctx, s, G, &ra.workspace, &ra.epoch));
      QFEC_HIP(qfec::launch_recover_runs(ra, s));
      return FEC_OK;
    }
    a.rec_off = row_start;
    a.packed_rows = true;
    // the form exists: now the row starts (two small launches ahead of the recover; the block
    // sums use the stream's workspace, which this path does not otherwise take)
    void* ws = nullptr;
    QFEC_HIP(stream_workspace(ctx, s, qfec::rows_prefix_workspace_bytes(G), &ws));
    QFEC_HIP(qfec::launch_rows_prefix(d_masks, G, k, r, row_start, static_cast<uint32_t*>(ws), row_total, s));
  }
  // Workspace: the caller's slot buffer (pipeline slots: private stream, calls serialised
  // by the context lock), else one private to this call.
  if (row_start == nullptr && (!plan->dense || qfec::decode_needs_rec_off(a))) {
    if (rec) {
      QFEC_HIP(rec->ensure(G * sizeof(uint32_t)));
      a.rec_off = rec->as<uint32_t>();
    } else {
      void* ws = nullptr;
      QFEC_HIP(stream_workspace(ctx, s, G * sizeof(uint32_t), &ws));
      a.rec_off = static_cast<uint32_t*>(ws);
    }
  }
  std::vector<uint8_t> book, st;
  std::vector<uint32_t> ro;
  if (!plan->dense) {
    // Sparse plan: the masks come to the host (after the stream's earlier work), records
    // are built for the patterns present, and the call completes synchronously.
    std::vector<uint64_t> hm(G);
    QFEC_HIP(hipStreamSynchronize(s));
    QFEC_HIP(hipMemcpy(hm.data(), d_masks, G * 8, hipMemcpyDefault));
    if (!qfec::build_sparse_plan(k, r, plan->M, hm.data(), G, qfec::kRecNone, qfec::kRecBad, book, ro, st)) {
      set_error("decode: sparse plan failed for k=%u r=%u", k, r);
      return FEC_ERR_RANGE;
    }
    QFEC_HIP(plan->sparse_book.ensure(book.size() + 32));
    if (!book.empty())
      QFEC_HIP(hipMemcpyAsync(plan->sparse_book.ptr, book.data(), book.size(), hipMemcpyHostToDevice, s));
    QFEC_HIP(hipMemcpyAsync(a.rec_off, ro.data(), G * 4, hipMemcpyHostToDevice, s));
    if (d_status) QFEC_HIP(hipMemcpyAsync(d_status, st.data(), G, hipMemcpyDefault, s));
    a.codebook = plan->sparse_book.as<uint8_t>();
  }
  QFEC_HIP(qfec::launch_decode(a, s));
  // sparse: the records (and the host vectors above) are reused / freed after this call
  if (!plan->dense) QFEC_HIP(hipStreamSynchronize(s));
  return FEC_OK;
}

// A pipelined call that fails part-way returns only after its slots' streams have drained:
// earlier chunks' copies still read the caller's buffers and write its outputs.
struct PipeDrain {
  FECEncoderCtx* ctx;
  bool done = false;
  ~PipeDrain() {
    if (done) return;
    for (auto& p : ctx->pipe)
      if (p.s) (void)hipStreamSynchronize(p.s);
    (void)hipGetLastError();
  }
};

int ensure_pipe(FECEncoderCtx* ctx) {
  for (auto& p : ctx->pipe)
    if (!p.s) QFEC_HIP(hipStreamCreateWithFlags(&p.s, hipStreamNonBlocking));
  return FEC_OK;
}

// Host-resident batches: chunks of ~64 MB of data flow H2D -> kernel -> D2H, chunk c on
// pipeline slot c % 3, so the copy engines (H2D and D2H run on separate DMA engines) and
// the kernels of neighbouring chunks overlap.  Page-locked host buffers (fec_alloc_slab)
// make the copies asynchronous; pageable ones still work, with less overlap.
int encode_host_pipelined(FECEncoderCtx* ctx, const uint8_t* data, uint64_t G, uint32_t k, uint32_t r,
                          uint32_t P, uint8_t* parity_out) {
  int rc = ensure_pipe(ctx);
  if (rc != FEC_OK) return rc;
  PipeDrain drain{ctx};
  const uint64_t in_g = uint64_t(k) * P, out_g = uint64_t(r) * P;
  uint64_t cg = pipe_chunk_bytes() / in_g;
  cg = cg == 0 ? 1 : (cg > G ? G : cg);
  for (auto& p : ctx->pipe) {
    QFEC_HIP(p.in.ensure(cg * in_g));
    QFEC_HIP(p.par.ensure(cg * out_g));
  }
  uint64_t c = 0;
  for (uint64_t g0 = 0; g0 < G; g0 += cg, ++c) {
    PipeSlot& sl = ctx->pipe[c % kPipeSlots];
    const uint64_t n = (G - g0 < cg) ? G - g0 : cg;
    QFEC_HIP(hipMemcpyAsync(sl.in.ptr, data + g0 * in_g, n * in_g, hipMemcpyHostToDevice, sl.s));
    rc = encode_dev_locked(ctx, sl.in.as<uint8_t>(), nullptr, qfec::OffsetKind::kNone, n, k, r, P,
                           sl.par.as<uint8_t>(), sl.s);
    if (rc != FEC_OK) return rc;
    QFEC_HIP(hipMemcpyAsync(parity_out + g0 * out_g, sl.par.ptr, n * out_g, hipMemcpyDeviceToHost, sl.s));
  }
  for (auto& p : ctx->pipe) QFEC_HIP(hipStreamSynchronize(p.s));
  drain.done = true;
  return FEC_OK;
}

int decode_host_pipelined(FECEncoderCtx* ctx, uint8_t* data, const uint8_t* parity, const uint64_t* masks,
                          uint64_t G, uint32_t k, uint32_t r, uint32_t P, uint8_t* status_out) {
  int rc = ensure_pipe(ctx);
  if (rc != FEC_OK) return rc;
  PipeDrain drain{ctx};
  const uint64_t in_g = uint64_t(k) * P, par_g = uint64_t(r) * P;
  uint64_t cg = pipe_chunk_bytes() / in_g;
  cg = cg == 0 ? 1 : (cg > G ? G : cg);
  for (auto& p : ctx->pipe) {
    QFEC_HIP(p.in.ensure(cg * in_g));
    QFEC_HIP(p.par.ensure(cg * par_g));
    QFEC_HIP(p.mask.ensure(cg * 8));
    QFEC_HIP(p.status.ensure(cg));
  }
  // Page-locked data: the kernel stores the rebuilt shards straight into host memory
  // (zero-copy PCIe writes of ~e*P bytes per group) instead of a D2H of the whole chunk.
  uint8_t* host_dev = nullptr;
  if (classify_ptr(data) == Mem::kPinned) {
    hipPointerAttribute_t attr;
    std::memset(&attr, 0, sizeof(attr));
    if (hipPointerGetAttributes(&attr, data) == hipSuccess && attr.devicePointer)
      host_dev = static_cast<uint8_t*>(attr.devicePointer);
    else
      (void)hipGetLastError();
  }
  uint64_t c = 0;
  for (uint64_t g0 = 0; g0 < G; g0 += cg, ++c) {
    PipeSlot& sl = ctx->pipe[c % kPipeSlots];
    const uint64_t n = (G - g0 < cg) ? G - g0 : cg;
    QFEC_HIP(hipMemcpyAsync(sl.in.ptr, data + g0 * in_g, n * in_g, hipMemcpyHostToDevice, sl.s));
    QFEC_HIP(hipMemcpyAsync(sl.par.ptr, parity + g0 * par_g, n * par_g, hipMemcpyHostToDevice, sl.s));
    QFEC_HIP(hipMemcpyAsync(sl.mask.ptr, masks + g0, n * 8, hipMemcpyHostToDevice, sl.s));
    rc = decode_dev_locked(ctx, sl.in.as<uint8_t>(), sl.par.as<uint8_t>(), sl.mask.as<uint64_t>(), n, k, r, P,
                           sl.status.as<uint8_t>(), sl.s, &sl.rec, host_dev ? host_dev + g0 * in_g : nullptr);
    if (rc != FEC_OK) return rc;
    if (!host_dev)
      QFEC_HIP(hipMemcpyAsync(data + g0 * in_g, sl.in.ptr, n * in_g, hipMemcpyDeviceToHost, sl.s));
    QFEC_HIP(hipMemcpyAsync(status_out + g0, sl.status.ptr, n, hipMemcpyDeviceToHost, sl.s));
  }
  for (auto& p : ctx->pipe) QFEC_HIP(hipStreamSynchronize(p.s));
  drain.done = true;
  return FEC_OK;
}

// Host-resident decode when few groups lost data shards (e.g. the satellite profile, iid
// loss p = 0.01: ~11% of k=10 r=3 groups): only those groups cross PCIe.  Per chunk, host
// threads gather the groups' data and parity into page-locked staging, the chunk goes
// H2D -> decode -> D2H on its pipeline slot, and the rebuilt packets are scattered back
// into `data`.  Slot c % 3's previous chunk is scattered before its staging is refilled,
// so the CPU gather of one chunk overlaps the copies and kernels of the two before it.
// `need` lists the groups with lost data that are recoverable (status 0); everything
// else needs no device work.
int decode_host_compacted(FECEncoderCtx* ctx, uint8_t* data, const uint8_t* parity, const uint64_t* masks,
                          const std::vector<uint64_t>& need, uint32_t k, uint32_t r, uint32_t P) {
  int rc = ensure_pipe(ctx);
  if (rc != FEC_OK) return rc;
  PipeDrain drain{ctx};
  const uint64_t N = need.size();
  const uint64_t in_g = uint64_t(k) * P, par_g = uint64_t(r) * P;
  uint64_t cg = pipe_chunk_bytes() / in_g;
  cg = cg == 0 ? 1 : (cg > N ? N : cg);
  for (auto& p : ctx->pipe) {
    QFEC_HIP(p.in.ensure(cg * in_g));
    QFEC_HIP(p.par.ensure(cg * par_g));
    QFEC_HIP(p.mask.ensure(cg * 8));
    QFEC_HIP(p.h_in.ensure(cg * in_g));
    QFEC_HIP(p.h_par.ensure(cg * par_g));
    QFEC_HIP(p.h_mask.ensure(cg * 8));
    p.h_groups.clear();
  }
  const uint64_t kmask = (1ull << k) - 1;
  // Rebuilt packets of the slot's last chunk: D2H landed in h_in; copy the erased ones out.
  auto scatter = [&](PipeSlot& sl) -> int {
    if (sl.h_groups.empty()) return FEC_OK;
    QFEC_HIP(hipStreamSynchronize(sl.s));
    const uint8_t* src = sl.h_in.as<uint8_t>();
    const uint64_t* gl = sl.h_groups.data();
    parallel_for(sl.h_groups.size(), 512, [&](uint64_t b, uint64_t e) {
      for (uint64_t i = b; i < e; ++i) {
        const uint64_t g = gl[i];
        for (uint64_t lost = masks[g] & kmask; lost; lost &= lost - 1) {
          const uint32_t j = static_cast<uint32_t>(__builtin_ctzll(lost));
          std::memcpy(data + g * in_g + uint64_t(j) * P, src + i * in_g + uint64_t(j) * P, P);
        }
      }
    });
    sl.h_groups.clear();
    return FEC_OK;
  };
  uint64_t c = 0;
  for (uint64_t i0 = 0; i0 < N; i0 += cg, ++c) {
    PipeSlot& sl = ctx->pipe[c % kPipeSlots];
    rc = scatter(sl);
    if (rc != FEC_OK) return rc;
    const uint64_t n = (N - i0 < cg) ? N - i0 : cg;
    const uint64_t* gl = need.data() + i0;
    uint8_t* hi = sl.h_in.as<uint8_t>();
    uint8_t* hp = sl.h_par.as<uint8_t>();
    uint64_t* hm = sl.h_mask.as<uint64_t>();
    parallel_for(n, 512, [&](uint64_t b, uint64_t e) {
      for (uint64_t i = b; i < e; ++i) {
        const uint64_t g = gl[i];
        std::memcpy(hi + i * in_g, data + g * in_g, in_g);
        std::memcpy(hp + i * par_g, parity + g * par_g, par_g);
        hm[i] = masks[g];
      }
    });
    sl.h_groups.assign(gl, gl + n);
    QFEC_HIP(hipMemcpyAsync(sl.in.ptr, hi, n * in_g, hipMemcpyHostToDevice, sl.s));
    QFEC_HIP(hipMemcpyAsync(sl.par.ptr, hp, n * par_g, hipMemcpyHostToDevice, sl.s));
    QFEC_HIP(hipMemcpyAsync(sl.mask.ptr, hm, n * 8, hipMemcpyHostToDevice, sl.s));
    rc = decode_dev_locked(ctx, sl.in.as<uint8_t>(), sl.par.as<uint8_t>(), sl.mask.as<uint64_t>(), n, k, r, P,
                           nullptr, sl.s, &sl.rec);
    if (rc != FEC_OK) return rc;
    QFEC_HIP(hipMemcpyAsync(hi, sl.in.ptr, n * in_g, hipMemcpyDeviceToHost, sl.s));
  }
  for (auto& p : ctx->pipe) {
    rc = scatter(p);
    if (rc != FEC_OK) return rc;
  }
  drain.done = true;
  return FEC_OK;
}

// Zero-copy view of a host buffer for a kernel: its own device address when page-locked,
// else the staging buffer `stage` (grown to `bytes`, filled from `host` when `fill`).
// `*staged` says which.
int zc_view(HostBuf& stage, const void* host, Mem m, void* dev, uint64_t bytes, bool fill, uint8_t** out,
            bool* staged) {
  if (m == Mem::kPinned && dev) {
    *out = static_cast<uint8_t*>(dev);
    *staged = false;
    return FEC_OK;
  }
  QFEC_HIP(stage.ensure(bytes));
  if (fill) std::memcpy(stage.ptr, host, bytes);
  *out = stage.dev_as<uint8_t>();
  *staged = true;
  return FEC_OK;
}

// Small host-resident encode, zero-copy (see small_call_bytes).  Caller holds ctx->mu.
int encode_host_zero_copy(FECEncoderCtx* ctx, const uint8_t* data, Mem dmem, void* ddev, uint64_t G, uint32_t k,
                          uint32_t r, uint32_t P, uint8_t* parity_out, Mem omem, void* odev) {
  const uint64_t in_bytes = G * k * uint64_t(P), out_bytes = G * r * uint64_t(P);
  uint8_t *src = nullptr, *dst = nullptr;
  bool in_staged = false, out_staged = false;
  int rc = zc_view(ctx->z_in, data, dmem, ddev, in_bytes, true, &src, &in_staged);
  if (rc == FEC_OK) rc = zc_view(ctx->z_out, parity_out, omem, odev, out_bytes, false, &dst, &out_staged);
  if (rc == FEC_OK) rc = encode_dev_locked(ctx, src, nullptr, qfec::OffsetKind::kNone, G, k, r, P, dst, ctx->stream);
  if (rc != FEC_OK) return rc;
  QFEC_HIP(wait_stream(ctx->stream));
  if (out_staged) std::memcpy(parity_out, ctx->z_out.ptr, out_bytes);
  return FEC_OK;
}

// Small host-resident decode, zero-copy: survivors are read and rebuilt shards written in
// place through PCIe.  Statuses come from the caller's host scan.  Caller holds ctx->mu.
int decode_host_zero_copy(FECEncoderCtx* ctx, uint8_t* data, Mem dmem, void* ddev, const uint8_t* parity, Mem pmem,
                          void* pdev, const uint64_t* masks, uint64_t G, uint32_t k, uint32_t r, uint32_t P,
                          double need_share) {
  const uint64_t in_g = uint64_t(k) * P;
  uint8_t *d = nullptr, *p = nullptr;
  bool d_staged = false, p_staged = false;
  int rc = zc_view(ctx->z_in, data, dmem, ddev, G * in_g, true, &d, &d_staged);
  if (rc == FEC_OK) rc = zc_view(ctx->z_out, parity, pmem, pdev, G * r * uint64_t(P), true, &p, &p_staged);
  if (rc != FEC_OK) return rc;
  QFEC_HIP(ctx->z_aux.ensure(G * 8));
  std::memcpy(ctx->z_aux.ptr, masks, G * 8);
  rc = decode_dev_locked(ctx, d, p, ctx->z_aux.dev_as<uint64_t>(), G, k, r, P, nullptr, ctx->stream, nullptr,
                         nullptr, need_share);
  if (rc != FEC_OK) return rc;
  QFEC_HIP(wait_stream(ctx->stream));
  if (d_staged) {  // only erased data packets changed (unrecoverable groups: untouched bytes)
    const uint64_t kmask = (1ull << k) - 1;
    const uint8_t* z = ctx->z_in.as<uint8_t>();
    for (uint64_t g = 0; g < G; ++g)
      for (uint64_t lost = masks[g] & kmask; lost; lost &= lost - 1) {
        const uint64_t o = g * in_g + uint64_t(__builtin_ctzll(lost)) * P;
        std::memcpy(data + o, z + o, P);
      }
  }
  return FEC_OK;
}

// Process-wide context used by the context-free xor_packets_* entry points.
FECEncoderCtx* default_ctx() {
  static std::once_flag once;
  static FECEncoderCtx* ctx = nullptr;
  std::call_once(once, [] { ctx = make_ctx(0.10, 1024, -1); });
  return ctx;
}

void xor_packets_gpu(const uint8_t* packets[], size_t n, size_t packet_size, uint8_t* repair) {
  g_last_error.clear();  // void return: callers read fec_hip_last_error() to detect failure
  if (n == 0 || packet_size == 0) return;  // fec_xor_simd.cpp:417-419
  if (!packets || !repair) {
    set_error("xor_packets: NULL argument");
    return;
  }
  if (packet_size > 0xFFFFFFFFull || n > 0xFFFFFFFFull) {
    set_error("xor_packets: size out of range");
    return;
  }
  FECEncoderCtx* ctx = default_ctx();
  if (!ctx) return;
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard dg(ctx->device);
  const uint32_t P = static_cast<uint32_t>(packet_size);
  if ((n + 1) * uint64_t(packet_size) <= small_call_bytes(false)) {
    // Host packets: gather them into page-locked staging and run zero-copy.
    bool host = classify_ptr(repair) != Mem::kDevice;
    for (size_t p = 0; p < n && host; ++p) host = classify_ptr(packets[p]) != Mem::kDevice;
    if (host) {
      if (ctx->z_in.ensure(n * packet_size) != hipSuccess || ctx->z_out.ensure(packet_size) != hipSuccess) {
        set_error("xor_packets: page-locked staging allocation failed");
        return;
      }
      for (size_t p = 0; p < n; ++p) std::memcpy(ctx->z_in.as<uint8_t>() + p * packet_size, packets[p], packet_size);
      if (encode_dev_locked(ctx, ctx->z_in.dev_as<uint8_t>(), nullptr, qfec::OffsetKind::kNone, 1,
                            static_cast<uint32_t>(n), 1, P, ctx->z_out.dev_as<uint8_t>(), ctx->stream) != FEC_OK)
        return;
      if (wait_stream(ctx->stream) != hipSuccess) {
        set_error("xor_packets: kernel failed");
        return;
      }
      std::memcpy(repair, ctx->z_out.ptr, packet_size);
      return;
    }
  }
  // Stage the packets contiguously (k = n, one group, r = 1).
  if (ctx->d_in.ensure(n * packet_size) != hipSuccess || ctx->d_out.ensure(packet_size) != hipSuccess) {
    set_error("xor_packets: device allocation failed");
    return;
  }
  for (size_t p = 0; p < n; ++p) {
    if (hipMemcpyAsync(ctx->d_in.as<uint8_t>() + p * packet_size, packets[p], packet_size,
                       hipMemcpyDefault, ctx->stream) != hipSuccess) {
      set_error("xor_packets: H2D copy failed");
      return;
    }
  }
  if (encode_dev_locked(ctx, ctx->d_in.as<uint8_t>(), nullptr, qfec::OffsetKind::kNone, 1,
                        static_cast<uint32_t>(n), 1, P, ctx->d_out.as<uint8_t>(),
                        ctx->stream) != FEC_OK)
    return;
  if (hipMemcpyAsync(repair, ctx->d_out.ptr, packet_size, hipMemcpyDefault, ctx->stream) != hipSuccess ||
      hipStreamSynchronize(ctx->stream) != hipSuccess) {
    set_error("xor_packets: D2H copy failed");
  }
}

// Non-zero codes copy the thread's message into the context (fec_ctx_last_error).
int record_ctx_error(FECEncoderCtx* ctx, int rc) {
  if (rc != FEC_OK && ctx != nullptr) {
    std::lock_guard<std::mutex> lk(ctx->err_mu);
    ctx->last_error = g_last_error.empty() ? "error code " + std::to_string(rc) : g_last_error;
  }
  return rc;
}

}  // namespace

// =====================================================================================
// Reference ABI (include/fec_xor_simd.h)
// =====================================================================================

QFEC_EXPORT FECEncoderCtx* fec_encoder_new(double redundancy, uint32_t max_groups) {
  return make_ctx(redundancy, max_groups, -1);
}

QFEC_EXPORT void fec_encoder_free(FECEncoderCtx* ctx) { delete ctx; }

QFEC_EXPORT void* fec_alloc_slab(size_t size) {
  const size_t aligned = (size + 63) & ~size_t(63);  // fec_xor_simd.cpp:471
  void* p = nullptr;
  const hipError_t e = hipHostMalloc(&p, aligned == 0 ? 64 : aligned, hipHostMallocDefault);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    set_error("fec_alloc_slab(%zu): %s", size, hipGetErrorString(e));
    return nullptr;
  }
  pinned_register(p, aligned == 0 ? 64 : aligned);
  return p;
}

namespace {

// NUMA-placed slabs (fec_alloc_slab_numa): mmap'd, mbind'd, then registered with HIP.
// fec_free_slab looks pointers up here to undo exactly what was done.
struct NumaSlab {
  size_t len;
  bool registered;
};
std::mutex g_numa_mu;
std::map<void*, NumaSlab> g_numa_slabs;

}  // namespace

QFEC_EXPORT void* fec_alloc_slab_numa(size_t size, int numa_node) {
  if (numa_node < 0) return fec_alloc_slab(size);
  const size_t page = static_cast<size_t>(sysconf(_SC_PAGESIZE));
  const size_t len = ((size == 0 ? 1 : size) + page - 1) / page * page;
  void* p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
  if (p == MAP_FAILED) {
    set_error("fec_alloc_slab_numa(%zu): mmap: %s", size, std::strerror(errno));
    return nullptr;
  }
  // Bind before the first touch so every page is allocated on the node (fec_xor_simd.cpp:
  // 497-502 binds with MPOL_MF_MOVE and ignores failure; so does this -- e.g. a node the
  // machine does not have leaves the default policy).  The range is page-aligned, which
  // mbind requires.
  constexpr int kMaxNodes = 1024;
  unsigned long mask[kMaxNodes / (8 * sizeof(unsigned long))] = {};
  if (numa_node < kMaxNodes) {
    mask[numa_node / (8 * sizeof(unsigned long))] |= 1ul << (numa_node % (8 * sizeof(unsigned long)));
    constexpr int kMpolBind = 2, kMpolMfMove = 1 << 1;
    (void)syscall(SYS_mbind, p, len, kMpolBind, mask, static_cast<unsigned long>(kMaxNodes + 1), kMpolMfMove);
  }
  // Page-lock for DMA / zero-copy kernel access; pinning faults the pages in under the
  // policy above.  Without a GPU the memory stays pageable (the reference's behaviour).
  bool registered = false;
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) == hipSuccess && ndev > 0)
    registered = hipHostRegister(p, len, hipHostRegisterDefault) == hipSuccess;
  (void)hipGetLastError();
  if (registered) pinned_register(p, len);
  std::lock_guard<std::mutex> lk(g_numa_mu);
  g_numa_slabs[p] = NumaSlab{len, registered};
  return p;
}

QFEC_EXPORT void* fec_alloc_repair_buffer(size_t size) { return fec_alloc_slab(size); }

QFEC_EXPORT void fec_free_slab(void* ptr) {
  if (!ptr) return;
  pinned_unregister(ptr);
  {
    std::lock_guard<std::mutex> lk(g_numa_mu);
    auto it = g_numa_slabs.find(ptr);
    if (it != g_numa_slabs.end()) {
      if (it->second.registered) (void)hipHostUnregister(ptr);
      (void)munmap(ptr, it->second.len);
      g_numa_slabs.erase(it);
      return;
    }
  }
  (void)hipHostFree(ptr);
}

QFEC_EXPORT void fec_free_repair_buffer(void* ptr) { fec_free_slab(ptr); }

// What fec_coalesce.cpp borrows (fec_internal.hpp).
namespace qfec {

HostMem classify_host_pointer(const void* p, void** dev) {
  switch (classify_ptr(p, dev)) {
    case Mem::kDevice:
      return HostMem::kDevice;
    case Mem::kPinned:
      return HostMem::kPinned;
    default:
      return HostMem::kPageable;
  }
}

int encode_addr_batch(FECEncoderCtx* ctx, const uint64_t* d_addr, uint64_t G, uint32_t k, uint32_t r, uint32_t P,
                      uint8_t* d_parity, hipStream_t s) {
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard dg(ctx->device);
  if (!dg.ok) {
    set_error("fec_encode_batch: cannot bind device %d", ctx->device);
    return FEC_ERR_NODEV;
  }
  return encode_dev_locked(ctx, nullptr, d_addr, OffsetKind::kAddr, G, k, r, P, d_parity, s);
}

void set_last_error(const char* msg) { g_last_error = msg ? msg : ""; }

}  // namespace qfec

static int fec_encode_batch_impl(FECEncoderCtx* ctx, const uint8_t* slab, const uint32_t* offsets,
                                 uint32_t num_groups, uint32_t packet_size, uint8_t* repair_out) {
  // fec_xor_simd.cpp:564-570, same order
  if (ctx == nullptr || slab == nullptr || offsets == nullptr || repair_out == nullptr) return -1;
  if (num_groups == 0 || packet_size == 0) return 0;
  // Small host-resident calls -- the reference's one group per call from each stream's own
  // context -- share launches with every other context's (fec_coalesce.cpp).
  int crc = 0;
  if (qfec::coalesce_legacy_encode(ctx->device, slab, offsets, num_groups, packet_size, repair_out, &crc, ctx->stream))
    return crc;
  constexpr uint32_t kPackets = 10;  // fec_xor_simd.cpp:580
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard dg(ctx->device);
  if (!dg.ok) {
    set_error("fec_encode_batch: cannot bind device %d", ctx->device);
    return FEC_ERR_NODEV;
  }
  const uint64_t noff = uint64_t(num_groups) * kPackets;
  const uint64_t P = packet_size;
  void *slab_dev = nullptr, *out_dev = nullptr;
  const Mem slab_mem = classify_ptr(slab, &slab_dev);
  const Mem off_mem = classify_ptr(offsets);
  const Mem out_mem = classify_ptr(repair_out, &out_dev);
  hipStream_t s = ctx->stream;

  const uint8_t* d_slab = slab;
  const uint32_t* d_offsets = offsets;
  if (slab_mem != Mem::kDevice || off_mem != Mem::kDevice) {
    // Host offsets: read them here to size the slab window.
    std::vector<uint32_t> host_off;
    const uint32_t* hoff = offsets;
    if (off_mem == Mem::kDevice) {
      host_off.resize(noff);
      QFEC_HIP(hipMemcpy(host_off.data(), offsets, noff * 4, hipMemcpyDeviceToHost));
      hoff = host_off.data();
    }
    uint32_t lo = 0xFFFFFFFFu, hi = 0;
    for (uint64_t i = 0; i < noff; ++i) {
      lo = hoff[i] < lo ? hoff[i] : lo;
      hi = hoff[i] > hi ? hoff[i] : hi;
    }
    const uint64_t span = uint64_t(hi) + P - lo;
    const uint64_t small = small_call_bytes(slab_mem == Mem::kPinned && out_mem == Mem::kPinned);
    if (slab_mem != Mem::kDevice && out_mem != Mem::kDevice && (noff + num_groups) * P <= small &&
        (slab_mem == Mem::kPinned || span <= small)) {
      // Small call, zero-copy: offsets (rebased to the staged window unless the slab is
      // page-locked) and the slab window in page-locked memory, read by the kernel over PCIe.
      QFEC_HIP(ctx->z_aux.ensure(noff * 4));
      uint32_t* zo = ctx->z_aux.as<uint32_t>();
      const uint8_t* zs = static_cast<const uint8_t*>(slab_dev);
      if (slab_mem == Mem::kPinned && zs) {
        std::memcpy(zo, hoff, noff * 4);
      } else {
        QFEC_HIP(ctx->z_in.ensure(span));
        std::memcpy(ctx->z_in.ptr, slab + lo, span);
        for (uint64_t i = 0; i < noff; ++i) zo[i] = hoff[i] - lo;
        zs = ctx->z_in.dev_as<uint8_t>();
      }
      uint8_t* zr = nullptr;
      bool out_staged = false;
      int rc = zc_view(ctx->z_out, repair_out, out_mem, out_dev, uint64_t(num_groups) * P, false, &zr, &out_staged);
      if (rc == FEC_OK)
        rc = encode_dev_locked(ctx, zs, ctx->z_aux.dev_as<uint32_t>(), qfec::OffsetKind::kU32, num_groups, kPackets,
                               1, packet_size, zr, s);
      if (rc != FEC_OK) return rc;
      QFEC_HIP(wait_stream(s));
      if (out_staged) std::memcpy(repair_out, ctx->z_out.ptr, uint64_t(num_groups) * P);
      return 0;
    }
    if (slab_mem == Mem::kDevice) {
      if (off_mem != Mem::kDevice) {
        QFEC_HIP(ctx->d_off.ensure(noff * 4));
        QFEC_HIP(hipMemcpyAsync(ctx->d_off.ptr, hoff, noff * 4, hipMemcpyHostToDevice, s));
        d_offsets = ctx->d_off.as<uint32_t>();
      }
    } else {
      // Copy the window [lo, hi + P) of the host slab; rebase offsets to it.
      std::vector<uint32_t> rebased(noff);
      for (uint64_t i = 0; i < noff; ++i) rebased[i] = hoff[i] - lo;
      QFEC_HIP(ctx->d_in.ensure(span));
      QFEC_HIP(ctx->d_off.ensure(noff * 4));
      QFEC_HIP(hipMemcpyAsync(ctx->d_in.ptr, slab + lo, span, hipMemcpyHostToDevice, s));
      QFEC_HIP(hipMemcpyAsync(ctx->d_off.ptr, rebased.data(), noff * 4, hipMemcpyHostToDevice, s));
      QFEC_HIP(hipStreamSynchronize(s));  // `rebased` dies at scope end
      d_slab = ctx->d_in.as<uint8_t>();
      d_offsets = ctx->d_off.as<uint32_t>();
    }
  }
  uint8_t* d_repair = repair_out;
  if (out_mem != Mem::kDevice) {
    QFEC_HIP(ctx->d_out.ensure(uint64_t(num_groups) * P));
    d_repair = ctx->d_out.as<uint8_t>();
  }
  const int rc = encode_dev_locked(ctx, d_slab, d_offsets, qfec::OffsetKind::kU32, num_groups,
                                   kPackets, 1, packet_size, d_repair, s);
  if (rc != FEC_OK) return rc;
  if (out_mem != Mem::kDevice)
    QFEC_HIP(hipMemcpyAsync(repair_out, d_repair, uint64_t(num_groups) * P, hipMemcpyDeviceToHost, s));
  QFEC_HIP(hipStreamSynchronize(s));
  return 0;
}

QFEC_EXPORT int fec_encode_batch(FECEncoderCtx* ctx, const uint8_t* slab, const uint32_t* offsets,
                                 uint32_t num_groups, uint32_t packet_size, uint8_t* repair_out) {
  g_last_error.clear();
  return record_ctx_error(ctx, fec_encode_batch_impl(ctx, slab, offsets, num_groups, packet_size, repair_out));
}

QFEC_EXPORT xor_impl_fn fec_select_xor_impl(void) { return xor_packets_gpu; }

QFEC_EXPORT void xor_packets_scalar(const uint8_t* packets[], size_t n, size_t packet_size,
                                    uint8_t* repair) {
  xor_packets_gpu(packets, n, packet_size, repair);
}
QFEC_EXPORT void xor_packets_avx2(const uint8_t* packets[], size_t n, size_t packet_size,
                                  uint8_t* repair) {
  xor_packets_gpu(packets, n, packet_size, repair);
}
QFEC_EXPORT void xor_packets_avx512(const uint8_t* packets[], size_t n, size_t packet_size,
                                    uint8_t* repair) {
  xor_packets_gpu(packets, n, packet_size, repair);
}
QFEC_EXPORT void xor_packets_neon(const uint8_t* packets[], size_t n, size_t packet_size,
                                  uint8_t* repair) {
  xor_packets_gpu(packets, n, packet_size, repair);
}

// =====================================================================================
// Batch GF(2^8) API (include/fec_hip.h)
// =====================================================================================

QFEC_EXPORT int fec_hip_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

QFEC_EXPORT const char* fec_hip_last_error(void) { return g_last_error.c_str(); }

QFEC_EXPORT size_t fec_ctx_last_error(FECEncoderCtx* ctx, char* buf, size_t buflen) {
  if (!ctx) return 0;
  std::lock_guard<std::mutex> lk(ctx->err_mu);
  if (buf && buflen > 0) {
    const size_t n = ctx->last_error.size() < buflen - 1 ? ctx->last_error.size() : buflen - 1;
    std::memcpy(buf, ctx->last_error.data(), n);
    buf[n] = '\0';
  }
  return ctx->last_error.size();
}

QFEC_EXPORT FECEncoderCtx* fec_encoder_new_device(double redundancy, uint32_t max_groups, int device) {
  if (device < 0) {
    set_error("fec_encoder_new_device: negative device");
    return nullptr;
  }
  return make_ctx(redundancy, max_groups, device);
}

QFEC_EXPORT int fec_encoder_device(const FECEncoderCtx* ctx) { return ctx ? ctx->device : -1; }

extern "C" const char qfec_src_hash[];  // src_hash.o, generated by src_hash.py at build time

QFEC_EXPORT const char* fec_hip_version(void) {
  static const std::string v = std::string("libfec_hip 0.2 gfx950 src=") + qfec_src_hash;
  return v.c_str();
}

QFEC_EXPORT int fec_parity_matrix(uint32_t k, uint32_t r, uint8_t* out) {
  if (!out) return FEC_ERR_NULL;
  std::vector<uint8_t> M;
  if (!qfec::parity_matrix(k, r, M)) return FEC_ERR_RANGE;
  std::memcpy(out, M.data(), M.size());
  return FEC_OK;
}

namespace {

int check_shape(uint64_t G, uint32_t k, uint32_t r, uint32_t P, bool decode) {
  if (k == 0 || r == 0 || k + r > (decode ? qfec::kMaxDecodeShards : 256u)) {
    set_error("unsupported k=%u r=%u", k, r);
    return FEC_ERR_RANGE;
  }
  if (P == 0 && G != 0) {
    set_error("packet_size must be > 0");
    return FEC_ERR_RANGE;
  }
  return FEC_OK;
}

}  // namespace

static int fec_encode_batch_rs_impl(FECEncoderCtx* ctx, const uint8_t* data, const uint64_t* offsets,
                                    uint64_t G, uint32_t k, uint32_t r, uint32_t P, uint8_t* parity_out) {
  if (!ctx || !data || !parity_out) return FEC_ERR_NULL;
  int rc = check_shape(G, k, r, P, false);
  if (rc != FEC_OK) return rc;
  if (G == 0) return FEC_OK;
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard dg(ctx->device);
  if (!dg.ok) return FEC_ERR_NODEV;
  hipStream_t s = ctx->stream;
  const uint64_t nin = G * k;
  const uint64_t out_bytes = G * r * uint64_t(P);
  void *ddev = nullptr, *odev = nullptr;
  const Mem dmem = classify_ptr(data, &ddev);
  const Mem omem = classify_ptr(parity_out, &odev);
  if (!offsets && dmem != Mem::kDevice && omem != Mem::kDevice) {
    if (nin * P + out_bytes <= small_call_bytes(dmem == Mem::kPinned && omem == Mem::kPinned))
      return encode_host_zero_copy(ctx, data, dmem, ddev, G, k, r, P, parity_out, omem, odev);
    return encode_host_pipelined(ctx, data, G, k, r, P, parity_out);
  }
  const uint8_t* d_data = data;
  const void* d_off = nullptr;
  qfec::OffsetKind ok = qfec::OffsetKind::kNone;
  std::vector<uint64_t> rebased;
  if (offsets) {
    ok = qfec::OffsetKind::kU64;
    const Mem offmem = classify_ptr(offsets);
    std::vector<uint64_t> host_off;
    const uint64_t* hoff = offsets;
    if (offmem == Mem::kDevice) {
      host_off.resize(nin);
      QFEC_HIP(hipMemcpy(host_off.data(), offsets, nin * 8, hipMemcpyDeviceToHost));
      hoff = host_off.data();
    }
    uint64_t lo = ~0ull, hi = 0;
    for (uint64_t i = 0; i < nin; ++i) {
      lo = hoff[i] < lo ? hoff[i] : lo;
      hi = hoff[i] > hi ? hoff[i] : hi;
    }
    if (dmem == Mem::kDevice) {
      if (offmem != Mem::kDevice) {
        QFEC_HIP(ctx->d_off.ensure(nin * 8));
        QFEC_HIP(hipMemcpyAsync(ctx->d_off.ptr, hoff, nin * 8, hipMemcpyHostToDevice, s));
        QFEC_HIP(hipStreamSynchronize(s));
        d_off = ctx->d_off.ptr;
      } else {
        d_off = offsets;
      }
    } else {
      const uint64_t span = hi + P - lo;
      rebased.resize(nin);
      for (uint64_t i = 0; i < nin; ++i) rebased[i] = hoff[i] - lo;
      QFEC_HIP(ctx->d_in.ensure(span));
      QFEC_HIP(ctx->d_off.ensure(nin * 8));
      QFEC_HIP(hipMemcpyAsync(ctx->d_in.ptr, data + lo, span, hipMemcpyHostToDevice, s));
      QFEC_HIP(hipMemcpyAsync(ctx->d_off.ptr, rebased.data(), nin * 8, hipMemcpyHostToDevice, s));
      d_data = ctx->d_in.as<uint8_t>();
      d_off = ctx->d_off.ptr;
    }
  } else {
    if (dmem != Mem::kDevice) {
      QFEC_HIP(ctx->d_in.ensure(nin * P));
      QFEC_HIP(hipMemcpyAsync(ctx->d_in.ptr, data, nin * P, hipMemcpyHostToDevice, s));
      d_data = ctx->d_in.as<uint8_t>();
    }
  }
  uint8_t* d_par = parity_out;
  if (omem != Mem::kDevice) {
    QFEC_HIP(ctx->d_out.ensure(out_bytes));
    d_par = ctx->d_out.as<uint8_t>();
  }
  rc = encode_dev_locked(ctx, d_data, d_off, ok, G, k, r, P, d_par, s);
  if (rc != FEC_OK) return rc;
  if (omem != Mem::kDevice)
    QFEC_HIP(hipMemcpyAsync(parity_out, d_par, out_bytes, hipMemcpyDeviceToHost, s));
  QFEC_HIP(hipStreamSynchronize(s));
  return FEC_OK;
}

QFEC_EXPORT int fec_encode_batch_rs(FECEncoderCtx* ctx, const uint8_t* data, const uint64_t* offsets,
                                    uint64_t G, uint32_t k, uint32_t r, uint32_t P, uint8_t* parity_out) {
  g_last_error.clear();
  return record_ctx_error(ctx, fec_encode_batch_rs_impl(ctx, data, offsets, G, k, r, P, parity_out));
}

static int fec_decode_batch_rs_impl(FECEncoderCtx* ctx, uint8_t* data, const uint8_t* parity,
                                    const uint64_t* masks, uint64_t G, uint32_t k, uint32_t r,
                                    uint32_t P, uint8_t* status_out, uint64_t* unrecoverable_out) {
  if (!ctx || !data || !parity || !masks) return FEC_ERR_NULL;
  int rc = check_shape(G, k, r, P, true);
  if (rc != FEC_OK) return rc;
  if (unrecoverable_out) *unrecoverable_out = 0;
  if (G == 0) return FEC_OK;
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard dg(ctx->device);
  if (!dg.ok) return FEC_ERR_NODEV;
  hipStream_t s = ctx->stream;
  const uint64_t data_bytes = G * k * uint64_t(P);
  const uint64_t par_bytes = G * r * uint64_t(P);
  void *ddev = nullptr, *pdev = nullptr;
  const Mem dmem = classify_ptr(data, &ddev), pmem = classify_ptr(parity, &pdev), mmem = classify_ptr(masks);
  if (dmem != Mem::kDevice && pmem != Mem::kDevice && mmem != Mem::kDevice &&
      (!status_out || classify_ptr(status_out) != Mem::kDevice)) {
    std::vector<uint8_t> st_local;
    uint8_t* st = status_out;
    if (!st) {
      st_local.resize(G);
      st = st_local.data();
    }
    // Which groups need work: lost data shards, and no more than the surviving parity rows
    // (the classify rule, fec_kernels.hip); status is known on the host from the masks.
    const uint64_t kmask = (1ull << k) - 1, rmask = (r >= 64) ? ~0ull : ((1ull << r) - 1);
    std::vector<uint64_t> need;
    uint64_t bad = 0;
    for (uint64_t g = 0; g < G; ++g) {
      const uint64_t m = masks[g];
      const uint32_t e = static_cast<uint32_t>(__builtin_popcountll(m & kmask));
      const uint32_t alive = r - static_cast<uint32_t>(__builtin_popcountll((m >> k) & rmask));
      const bool unrec = e > 0 && e > alive;
      bad += unrec;
      if (e > 0 && !unrec) need.push_back(g);
    }
    const bool small = data_bytes + par_bytes <= small_call_bytes(dmem == Mem::kPinned && pmem == Mem::kPinned);
    if (small || need.size() * kCompactMaxShare <= G) {
      // few groups to rebuild: move only those (statuses from the host scan); a small call
      // runs zero-copy
      for (uint64_t g = 0; g < G; ++g) {
        const uint64_t m = masks[g];
        const uint32_t e = static_cast<uint32_t>(__builtin_popcountll(m & kmask));
        st[g] = (e > 0 && e > r - static_cast<uint32_t>(__builtin_popcountll((m >> k) & rmask))) ? 1 : 0;
      }
      if (!need.empty())
        rc = small ? decode_host_zero_copy(ctx, data, dmem, ddev, parity, pmem, pdev, masks, G, k, r, P,
                                           double(need.size()) / double(G))
                   : decode_host_compacted(ctx, data, parity, masks, need, k, r, P);
    } else {
      rc = decode_host_pipelined(ctx, data, parity, masks, G, k, r, P, st);
    }
    if (rc != FEC_OK) return rc;
    if (unrecoverable_out) *unrecoverable_out = bad;
    return FEC_OK;
  }
  uint8_t* d_data = data;
  const uint8_t* d_par = parity;
  const uint64_t* d_masks = masks;
  if (dmem != Mem::kDevice) {
    QFEC_HIP(ctx->d_in.ensure(data_bytes));
    QFEC_HIP(hipMemcpyAsync(ctx->d_in.ptr, data, data_bytes, hipMemcpyHostToDevice, s));
    d_data = ctx->d_in.as<uint8_t>();
  }
  if (pmem != Mem::kDevice) {
    QFEC_HIP(ctx->d_out.ensure(par_bytes));
    QFEC_HIP(hipMemcpyAsync(ctx->d_out.ptr, parity, par_bytes, hipMemcpyHostToDevice, s));
    d_par = ctx->d_out.as<uint8_t>();
  }
  if (mmem != Mem::kDevice) {
    QFEC_HIP(ctx->d_mask.ensure(G * 8));
    QFEC_HIP(hipMemcpyAsync(ctx->d_mask.ptr, masks, G * 8, hipMemcpyHostToDevice, s));
    d_masks = ctx->d_mask.as<uint64_t>();
  }
  QFEC_HIP(ctx->d_status.ensure(G));
  rc = decode_dev_locked(ctx, d_data, d_par, d_masks, G, k, r, P, ctx->d_status.as<uint8_t>(), s);
  if (rc != FEC_OK) return rc;
  if (dmem != Mem::kDevice)
    QFEC_HIP(hipMemcpyAsync(data, d_data, data_bytes, hipMemcpyDeviceToHost, s));
  std::vector<uint8_t> st(G);
  QFEC_HIP(hipMemcpyAsync(st.data(), ctx->d_status.ptr, G, hipMemcpyDeviceToHost, s));
  QFEC_HIP(hipStreamSynchronize(s));
  uint64_t bad = 0;
  for (uint64_t g = 0; g < G; ++g) bad += st[g] != 0;
  if (status_out) std::memcpy(status_out, st.data(), G);
  if (unrecoverable_out) *unrecoverable_out = bad;
  return FEC_OK;
}

QFEC_EXPORT int fec_decode_batch_rs(FECEncoderCtx* ctx, uint8_t* data, const uint8_t* parity,
                                    const uint64_t* masks, uint64_t G, uint32_t k, uint32_t r,
                                    uint32_t P, uint8_t* status_out, uint64_t* unrecoverable_out) {
  g_last_error.clear();
  return record_ctx_error(ctx, fec_decode_batch_rs_impl(ctx, data, parity, masks, G, k, r, P, status_out, unrecoverable_out));
}

static int fec_encode_batch_rs_dev_impl(FECEncoderCtx* ctx, const uint8_t* d_data, uint64_t G,
                                        uint32_t k, uint32_t r, uint32_t P, uint8_t* d_parity,
                                        void* stream) {
  if (!ctx || !d_data || !d_parity) return FEC_ERR_NULL;
  int rc = check_shape(G, k, r, P, false);
  if (rc != FEC_OK) return rc;
  if (G == 0) return FEC_OK;
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard dg(ctx->device);
  if (!dg.ok) return FEC_ERR_NODEV;
  return encode_dev_locked(ctx, d_data, nullptr, qfec::OffsetKind::kNone, G, k, r, P, d_parity,
                           pick_stream(ctx, stream));
}

QFEC_EXPORT int fec_encode_batch_rs_dev(FECEncoderCtx* ctx, const uint8_t* d_data, uint64_t G,
                                        uint32_t k, uint32_t r, uint32_t P, uint8_t* d_parity,
                                        void* stream) {
  g_last_error.clear();
  return record_ctx_error(ctx, fec_encode_batch_rs_dev_impl(ctx, d_data, G, k, r, P, d_parity, stream));
}

static int fec_decode_batch_rs_dev_impl(FECEncoderCtx* ctx, uint8_t* d_data, const uint8_t* d_parity,
                                        const uint64_t* d_masks, uint64_t G, uint32_t k, uint32_t r,
                                        uint32_t P, uint8_t* d_status, void* stream) {
  if (!ctx || !d_data || !d_parity || !d_masks) return FEC_ERR_NULL;
  int rc = check_shape(G, k, r, P, true);
  if (rc != FEC_OK) return rc;
  if (G == 0) return FEC_OK;
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard dg(ctx->device);
  if (!dg.ok) return FEC_ERR_NODEV;
  return decode_dev_locked(ctx, d_data, d_parity, d_masks, G, k, r, P, d_status,
                           pick_stream(ctx, stream));
}

QFEC_EXPORT int fec_decode_batch_rs_dev(FECEncoderCtx* ctx, uint8_t* d_data, const uint8_t* d_parity,
                                        const uint64_t* d_masks, uint64_t G, uint32_t k, uint32_t r,
                                        uint32_t P, uint8_t* d_status, void* stream) {
  g_last_error.clear();
  return record_ctx_error(ctx, fec_decode_batch_rs_dev_impl(ctx, d_data, d_parity, d_masks, G, k, r, P, d_status, stream));
}

static int fec_recover_batch_rs_dev_impl(FECEncoderCtx* ctx, const uint8_t* d_data, const uint8_t* d_parity,
                                         const uint64_t* d_masks, uint64_t G, uint32_t k, uint32_t r, uint32_t P,
                                         uint8_t* d_rebuilt, uint8_t* d_status, void* stream) {
  if (!ctx || !d_data || !d_parity || !d_masks || !d_rebuilt) return FEC_ERR_NULL;
  int rc = check_shape(G, k, r, P, true);
  if (rc != FEC_OK) return rc;
  if (G == 0) return FEC_OK;
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard dg(ctx->device);
  if (!dg.ok) return FEC_ERR_NODEV;
  // the kernels only read `data` when the output is compact
  return decode_dev_locked(ctx, const_cast<uint8_t*>(d_data), d_parity, d_masks, G, k, r, P, d_status,
                           pick_stream(ctx, stream), nullptr, d_rebuilt, -1.0, /*compact_out=*/true);
}

static int fec_recover_batch_rs_dev_packed_impl(FECEncoderCtx* ctx, const uint8_t* d_data, const uint8_t* d_parity,
                                                const uint64_t* d_masks, uint64_t G, uint32_t k, uint32_t r,
                                                uint32_t P, uint8_t* d_rebuilt, uint32_t* d_row_start,
                                                uint64_t* d_total, uint8_t* d_status, void* stream) {
  if (!ctx || !d_data || !d_parity || !d_masks || !d_rebuilt || !d_row_start) return FEC_ERR_NULL;
  int rc = check_shape(G, k, r, P, true);
  if (rc != FEC_OK) return rc;
  if (G * r >= (1ull << 32)) {
    set_error("packed recover: %llu groups x %u rows exceed 32-bit row indices", static_cast<unsigned long long>(G), r);
    return FEC_ERR_RANGE;
  }
  if (G == 0) {
    if (d_total) {
      std::lock_guard<std::mutex> lk(ctx->mu);
      DeviceGuard dg(ctx->device);
      if (!dg.ok) return FEC_ERR_NODEV;
      QFEC_HIP(hipMemsetAsync(d_total, 0, sizeof(uint64_t), pick_stream(ctx, stream)));
    }
    return FEC_OK;
  }
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard dg(ctx->device);
  if (!dg.ok) return FEC_ERR_NODEV;
  // decode_dev_locked checks the form first and only then launches the row prefix, so an
  // unsupported shape returns FEC_ERR_RANGE with d_row_start / d_total untouched
  return decode_dev_locked(ctx, const_cast<uint8_t*>(d_data), d_parity, d_masks, G, k, r, P, d_status,
                           pick_stream(ctx, stream), nullptr, d_rebuilt, -1.0, /*compact_out=*/true, d_row_start,
                           d_total);
}

QFEC_EXPORT int fec_recover_batch_rs_dev_packed(FECEncoderCtx* ctx, const uint8_t* d_data, const uint8_t* d_parity,
                                                const uint64_t* d_masks, uint64_t G, uint32_t k, uint32_t r,
                                                uint32_t P, uint8_t* d_rebuilt, uint32_t* d_row_start,
                                                uint64_t* d_total, uint8_t* d_status, void* stream) {
  g_last_error.clear();
  return record_ctx_error(ctx, fec_recover_batch_rs_dev_packed_impl(ctx, d_data, d_parity, d_masks, G, k, r, P, d_rebuilt,
                                                                    d_row_start, d_total, d_status, stream));
}

QFEC_EXPORT int fec_recover_batch_rs_dev(FECEncoderCtx* ctx, const uint8_t* d_data, const uint8_t* d_parity,
                                         const uint64_t* d_masks, uint64_t G, uint32_t k, uint32_t r, uint32_t P,
                                         uint8_t* d_rebuilt, uint8_t* d_status, void* stream) {
  g_last_error.clear();
  return record_ctx_error(ctx, fec_recover_batch_rs_dev_impl(ctx, d_data, d_parity, d_masks, G, k, r, P, d_rebuilt,
                                                             d_status, stream));
}

static int fec_decode_prepare_impl(FECEncoderCtx* ctx, uint32_t k, uint32_t r, uint64_t* bytes_out) {
  if (!ctx) return FEC_ERR_NULL;
  int rc = check_shape(1, k, r, 1, true);
  if (rc != FEC_OK) return rc;
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard dg(ctx->device);
  if (!dg.ok) return FEC_ERR_NODEV;
  DecodePlan* plan = nullptr;
  rc = get_decode_plan(ctx, k, r, &plan);
  if (rc != FEC_OK) return rc;
  if (bytes_out) *bytes_out = plan->dense ? plan->layout.total_bytes : 0;  // 0: sparse per-call plans
  return FEC_OK;
}

QFEC_EXPORT int fec_decode_prepare(FECEncoderCtx* ctx, uint32_t k, uint32_t r, uint64_t* bytes_out) {
  g_last_error.clear();
  return record_ctx_error(ctx, fec_decode_prepare_impl(ctx, k, r, bytes_out));
}

static int fec_fill_random_dev_impl(FECEncoderCtx* ctx, uint8_t* d_dst, uint64_t nbytes, uint64_t seed,
                                    uint64_t byte_offset, void* stream) {
  if (!ctx || !d_dst) return FEC_ERR_NULL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard dg(ctx->device);
  if (!dg.ok) return FEC_ERR_NODEV;
  QFEC_HIP(qfec::launch_fill_splitmix(d_dst, nbytes, seed, byte_offset, pick_stream(ctx, stream)));
  return FEC_OK;
}

QFEC_EXPORT int fec_fill_random_dev(FECEncoderCtx* ctx, uint8_t* d_dst, uint64_t nbytes, uint64_t seed,
                                    uint64_t byte_offset, void* stream) {
  g_last_error.clear();
  return record_ctx_error(ctx, fec_fill_random_dev_impl(ctx, d_dst, nbytes, seed, byte_offset, stream));
}

static int fec_copy_dev_impl(FECEncoderCtx* ctx, const uint8_t* d_src, uint8_t* d_dst, uint64_t nbytes,
                             void* stream) {
  if (!ctx || !d_src || !d_dst) return FEC_ERR_NULL;
  if (nbytes % 16 || reinterpret_cast<uintptr_t>(d_src) % 16 || reinterpret_cast<uintptr_t>(d_dst) % 16)
  {
    set_error("fec_copy_dev: size and addresses must be multiples of 16");
    return FEC_ERR_RANGE;
  }
  std::lock_guard<std::mutex> lk(ctx->mu);
  DeviceGuard dg(ctx->device);
  if (!dg.ok) return FEC_ERR_NODEV;
  QFEC_HIP(qfec::launch_copy_words(d_src, d_dst, nbytes, pick_stream(ctx, stream)));
  return FEC_OK;
}

QFEC_EXPORT int fec_copy_dev(FECEncoderCtx* ctx, const uint8_t* d_src, uint8_t* d_dst, uint64_t nbytes,
                             void* stream) {
  g_last_error.clear();
  return record_ctx_error(ctx, fec_copy_dev_impl(ctx, d_src, d_dst, nbytes, stream));
}

QFEC_EXPORT int fec_decode_loss_hint(FECEncoderCtx* ctx, double share) {
  if (!ctx) return FEC_ERR_NULL;
  std::lock_guard<std::mutex> lk(ctx->mu);
  ctx->decode_need_share = share >= 0.0 && share <= 1.0 ? share : -1.0;
  return FEC_OK;
}

QFEC_EXPORT int fec_synchronize(FECEncoderCtx* ctx) {
  if (!ctx) return FEC_ERR_NULL;
  DeviceGuard dg(ctx->device);
  QFEC_HIP(hipStreamSynchronize(ctx->stream));
  return FEC_OK;
}

// ---------------------------------------------------------------------------------
// Device groups: one host batch sharded over several GPUs.  Groups
// are independent, so shard i of n takes the contiguous range [G*i/n, G*(i+1)/n) and
// runs on its own context (device, streams, staging) from its own host thread; there is
// no exchange between devices.
// ---------------------------------------------------------------------------------
struct FECDeviceGroup {
  std::vector<FECEncoderCtx*> ctxs;
  ~FECDeviceGroup() {
    for (auto* c : ctxs) delete c;
  }
};

namespace {

// Run f(i, g0, n) for every shard, shard 0 on the calling thread; the first failing
// shard's code and message become the caller's.
template <class F>
int for_each_shard(FECDeviceGroup* grp, uint64_t G, F&& f) {
  const uint64_t n = grp->ctxs.size();
  std::vector<int> rc(n, FEC_OK);
  std::vector<std::string> msg(n);
  auto run = [&](uint64_t i) {
    const uint64_t g0 = G * i / n, g1 = G * (i + 1) / n;
    if (g1 > g0) rc[i] = f(i, g0, g1 - g0);
    if (rc[i] != FEC_OK) msg[i] = g_last_error;
  };
  std::vector<std::thread> th;
  for (uint64_t i = 1; i < n; ++i) th.emplace_back(run, i);
  run(0);
  for (auto& t : th) t.join();
  for (uint64_t i = 0; i < n; ++i)
    if (rc[i] != FEC_OK) {
      g_last_error = "shard " + std::to_string(i) + " (device " + std::to_string(grp->ctxs[i]->device) +
                     "): " + msg[i];
      return rc[i];
    }
  return FEC_OK;
}

bool any_device_ptr(std::initializer_list<const void*> ps) {
  for (const void* p : ps)
    if (p && classify_ptr(p) == Mem::kDevice) return true;
  return false;
}

}  // namespace

QFEC_EXPORT FECDeviceGroup* fec_group_new(const int* devices, int ndevices) {
  const int n = fec_hip_device_count();
  if (n <= 0) {
    set_error("fec_group_new: no HIP device available");
    return nullptr;
  }
  std::vector<int> devs;
  if (!devices || ndevices <= 0) {
    for (int d = 0; d < n; ++d) devs.push_back(d);
  } else {
    for (int i = 0; i < ndevices; ++i) {
      if (devices[i] < 0 || devices[i] >= n) {
        set_error("fec_group_new: device %d out of range (%d devices)", devices[i], n);
        return nullptr;
      }
      devs.push_back(devices[i]);
    }
  }
  auto* grp = new FECDeviceGroup();
  for (int d : devs) {
    FECEncoderCtx* c = make_ctx(0.10, 1024, d);
    if (!c) {
      delete grp;
      return nullptr;
    }
    grp->ctxs.push_back(c);
  }
  return grp;
}

QFEC_EXPORT void fec_group_free(FECDeviceGroup* grp) { delete grp; }

QFEC_EXPORT int fec_group_size(const FECDeviceGroup* grp) { return grp ? static_cast<int>(grp->ctxs.size()) : 0; }

QFEC_EXPORT FECEncoderCtx* fec_group_context(FECDeviceGroup* grp, int i) {
  if (!grp || i < 0 || i >= static_cast<int>(grp->ctxs.size())) return nullptr;
  return grp->ctxs[i];
}

QFEC_EXPORT int fec_group_encode_batch_rs(FECDeviceGroup* grp, const uint8_t* data, uint64_t G, uint32_t k,
                                          uint32_t r, uint32_t P, uint8_t* parity_out) {
  if (!grp || !data || !parity_out) return FEC_ERR_NULL;
  int rc = check_shape(G, k, r, P, false);
  if (rc != FEC_OK) return rc;
  if (G == 0) return FEC_OK;
  if (any_device_ptr({data, parity_out})) {
    set_error("fec_group_encode_batch_rs: host buffers only (device buffers belong to one context)");
    return FEC_ERR_RANGE;
  }
  return for_each_shard(grp, G, [&](uint64_t i, uint64_t g0, uint64_t n) {
    return fec_encode_batch_rs(grp->ctxs[i], data + g0 * k * uint64_t(P), nullptr, n, k, r, P,
                               parity_out + g0 * r * uint64_t(P));
  });
}

QFEC_EXPORT int fec_group_decode_batch_rs(FECDeviceGroup* grp, uint8_t* data, const uint8_t* parity,
                                          const uint64_t* masks, uint64_t G, uint32_t k, uint32_t r,
                                          uint32_t P, uint8_t* status_out, uint64_t* unrecoverable_out) {
  if (!grp || !data || !parity || !masks) return FEC_ERR_NULL;
  int rc = check_shape(G, k, r, P, true);
  if (rc != FEC_OK) return rc;
  if (unrecoverable_out) *unrecoverable_out = 0;
  if (G == 0) return FEC_OK;
  if (any_device_ptr({data, parity, masks, status_out})) {
    set_error("fec_group_decode_batch_rs: host buffers only (device buffers belong to one context)");
    return FEC_ERR_RANGE;
  }
  std::vector<uint64_t> bad(grp->ctxs.size(), 0);
  rc = for_each_shard(grp, G, [&](uint64_t i, uint64_t g0, uint64_t n) {
    return fec_decode_batch_rs(grp->ctxs[i], data + g0 * k * uint64_t(P), parity + g0 * r * uint64_t(P),
                               masks + g0, n, k, r, P, status_out ? status_out + g0 : nullptr, &bad[i]);
  });
  if (rc != FEC_OK) return rc;
  if (unrecoverable_out)
    for (uint64_t b : bad) *unrecoverable_out += b;
  return FEC_OK;
}
