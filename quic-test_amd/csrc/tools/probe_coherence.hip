// probe_coherence — does a kernel read what the CPU wrote into page-locked host memory since
// an earlier kernel read the same addresses?  For each way of page-locking: fill a small host
// buffer with value v, launch a kernel that copies it to device memory (plain loads, so the
// lines may be cached on the GPU), synchronize, repeat with v + 1, and count the words the
// kernel saw stale.  Prints the allocation flags hipPointerGetAttributes reports.
// Development probe; not part of the library.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                                  \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) {                                                                       \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
      std::exit(1);                                                                               \
    }                                                                                             \
  } while (0)

__global__ void copy_in(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}

// Keeps the stream busy for ~`cycles` without touching memory, so the next launch is queued
// behind a running kernel (as the batcher's flusher queues a batch behind the previous one).
__global__ void spin(uint64_t cycles, uint32_t* sink) {
  const uint64_t t0 = clock64();
  while (clock64() - t0 < cycles) {
  }
  if (threadIdx.x == 9999) sink[0] = 1;
}

static int g_queued = 0;  // 1: each copy_in is queued behind a spin kernel

static void run(const char* name, uint32_t* host, uint32_t n, hipStream_t s, uint32_t* dev_out) {
  void* dptr = nullptr;
  if (hipHostGetDevicePointer(&dptr, host, 0) != hipSuccess) {
    (void)hipGetLastError();
    dptr = host;
  }
  hipPointerAttribute_t attr{};
  (void)hipPointerGetAttributes(&attr, host);
  std::vector<uint32_t> back(n);
  long stale = 0;
  for (uint32_t round = 0; round < 50; ++round) {
    for (uint32_t i = 0; i < n; ++i) host[i] = round * 1000003u + i;
    if (g_queued) hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s, 200000ull, dev_out + n);
    hipLaunchKernelGGL(copy_in, dim3((n + 255) / 256), dim3(256), 0, s, static_cast<const uint32_t*>(dptr), dev_out, n);
    CHECK(hipStreamSynchronize(s));
    CHECK(hipMemcpy(back.data(), dev_out, n * 4, hipMemcpyDeviceToHost));
    for (uint32_t i = 0; i < n; ++i) stale += back[i] != round * 1000003u + i;
  }
  std::printf("{\"alloc\": \"%s\", \"queued_behind_kernel\": %d, \"allocationFlags\": \"0x%x\", \"stale_words\": %ld, "
              "\"of\": %lu}\n", name, g_queued, attr.allocationFlags, stale, 50ul * n);
  std::fflush(stdout);
}

// The other direction: a kernel writes the host buffer (plain or non-temporal stores), the
// host waits on an event recorded behind it (as the batcher's flusher does), then reads.
__global__ void fill_out(uint32_t* __restrict__ dst, uint32_t n, uint32_t v, int nt) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (nt) __builtin_nontemporal_store(v + i, dst + i);
  else dst[i] = v + i;
}

static void run_write(const char* name, uint32_t* host, uint32_t n, hipStream_t s, int nt, unsigned ev_flags) {
  void* dptr = nullptr;
  if (hipHostGetDevicePointer(&dptr, host, 0) != hipSuccess) {
    (void)hipGetLastError();
    dptr = host;
  }
  hipEvent_t ev;
  CHECK(hipEventCreateWithFlags(&ev, ev_flags));
  long stale = 0;
  for (uint32_t round = 0; round < 50; ++round) {
    hipLaunchKernelGGL(fill_out, dim3((n + 255) / 256), dim3(256), 0, s, static_cast<uint32_t*>(dptr), n,
                       round * 1000003u, nt);
    CHECK(hipEventRecord(ev, s));
    CHECK(hipEventSynchronize(ev));
    for (uint32_t i = 0; i < n; ++i) stale += host[i] != round * 1000003u + i;
  }
  CHECK(hipEventDestroy(ev));
  std::printf("{\"alloc\": \"%s\", \"gpu_writes\": \"%s\", \"event_flags\": \"0x%x\", \"stale_words\": %ld, \"of\": %lu}\n",
              name, nt ? "nt" : "plain", ev_flags, stale, 50ul * n);
  std::fflush(stdout);
}

int main() {
  const uint32_t n = 16384;  // 64 KB: stays in the GPU's caches between launches
  hipStream_t s;
  CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  uint32_t* dev_out;
  CHECK(hipMalloc(&dev_out, n * 4 + 64));
  for (unsigned fl : {hipHostMallocDefault, hipHostMallocCoherent})
    for (int nt = 0; nt < 2; ++nt)
      for (unsigned ef : {unsigned(hipEventDisableTiming), unsigned(hipEventDisableTiming | hipEventReleaseToSystem)}) {
        uint32_t* h = nullptr;
        CHECK(hipHostMalloc(&h, n * 4, fl));
        run_write(fl ? "hipHostMalloc(Coherent)" : "hipHostMalloc(Default)", h, n, s, nt, ef);
        CHECK(hipHostFree(h));
      }
  for (g_queued = 0; g_queued < 2; ++g_queued) {
  struct A {
    const char* name;
    unsigned flags;
  };
  for (A a : {A{"hipHostMalloc(Default)", hipHostMallocDefault}, A{"hipHostMalloc(Coherent)", hipHostMallocCoherent},
              A{"hipHostMalloc(NonCoherent)", hipHostMallocNonCoherent},
              A{"hipHostMalloc(Mapped|Coherent)", hipHostMallocMapped | hipHostMallocCoherent}}) {
    uint32_t* h = nullptr;
    CHECK(hipHostMalloc(&h, n * 4, a.flags));
    run(a.name, h, n, s, dev_out);
    CHECK(hipHostFree(h));
  }
  for (A a : {A{"hipHostRegister(Default)", hipHostRegisterDefault}, A{"hipHostRegister(Mapped)", hipHostRegisterMapped}}) {
    uint32_t* h = static_cast<uint32_t*>(std::aligned_alloc(4096, n * 4));
    CHECK(hipHostRegister(h, n * 4, a.flags));
    run(a.name, h, n, s, dev_out);
    CHECK(hipHostUnregister(h));
    std::free(h);
  }
  }
  return 0;
}
