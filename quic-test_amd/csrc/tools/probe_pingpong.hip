// probe_pingpong.hip — host <-> device round-trip latency through page-locked host memory, the
// floor under the resident legacy encoder (fec_coalesce.cpp).  Not part of the library.
//
// One resident workgroup polls a host word (system-coherent loads), and answers each new value
// by storing it to a second host word (system-scope release); the host writes the first word
// and spins on the second.  Variants: the answer after 0 / 1 / 2 extra dependent host-memory
// reads (the resident encoder reads packet addresses, then packets), with and without a
// system-scope fence before the answer, with an s_sleep between polls or not.  Every instance
// leaves after max_iters polls or when the host stores the stop value.
//
//   probe_pingpong [rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e_ = (x);                                                        \
    if (e_ != hipSuccess) {                                                     \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));              \
      std::exit(2);                                                             \
    }                                                                           \
  } while (0)

constexpr uint64_t kStop = ~0ull;

__device__ __forceinline__ uint64_t vload(const uint64_t* p) { return *reinterpret_cast<const volatile uint64_t*>(p); }

// MODE bit 0: fence (system release) before the answer; bit 1: s_sleep between polls.
// CHAIN: dependent host reads between seeing the ping and answering it.
template <int MODE, int CHAIN>
__global__ __launch_bounds__(64) void pong(const uint64_t* ping, uint64_t* pongw, const uint64_t* chain,
                                           uint32_t max_iters) {
  uint64_t last = 0;
  for (uint32_t it = 0; it < max_iters; ++it) {
    const uint64_t v = vload(ping);
    if (v == kStop) break;
    if (v == last) {
      if constexpr ((MODE & 2) != 0) __builtin_amdgcn_s_sleep(8);
      continue;
    }
    last = v;
    uint64_t x = v;
    if constexpr (CHAIN >= 1) x += vload(chain + (x & 7));
    if constexpr (CHAIN >= 2) x += vload(chain + 8 + (x & 7));
    if constexpr ((MODE & 1) != 0) __threadfence_system();
    const uint64_t ans = x == 0x123456789ABCull ? v + 1 : v;  // waits for the chain's reads
    if (threadIdx.x == 0) __hip_atomic_store(pongw, ans, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// The resident encoder's work step alone: on each ping, lanes [0, cols) load their 16-B column
// of NPK packets of P bytes (contiguous, host memory), XOR them and store the result to host
// memory, fence, answer.  FLAT: through generic pointers (as the encoder does) or global ones.
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
template <int NPK, bool FLAT>
__global__ __launch_bounds__(128) void pong_work(const uint64_t* ping, uint64_t* pongw, const uint8_t* pk, uint8_t* out,
                                                 uint32_t P, uint32_t cols, uint32_t max_iters) {
  __shared__ uint64_t s_v;
  __shared__ uint32_t s_stop;
  uint64_t last = 0;
  for (uint32_t it = 0; it < max_iters; ++it) {
    if (threadIdx.x == 0) {
      uint64_t v;
      do {
        v = vload(ping);
      } while (v == last && ++it < max_iters);
      s_v = v;
      s_stop = v == kStop || it >= max_iters;
    }
    __syncthreads();
    const uint64_t v = s_v;
    if (s_stop) break;
    last = v;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    if (threadIdx.x < cols) {
      const uint32_t o = threadIdx.x * 16u;
      u32x4 acc = {0, 0, 0, 0};
#pragma unroll
      for (int j = 0; j < NPK; ++j) {
        const uint8_t* src = pk + size_t(j) * P + o;
        if constexpr (FLAT) {
          const uint64_t a = reinterpret_cast<uint64_t>(src);
          acc ^= *reinterpret_cast<const u32x4*>(reinterpret_cast<const uint8_t*>(a));
        } else {
          typedef const __attribute__((address_space(1))) u32x4* gptr;
          acc ^= *(gptr)(reinterpret_cast<uintptr_t>(src));
        }
      }
      *reinterpret_cast<u32x4*>(out + o) = acc;
    }
    __threadfence_system();
    __syncthreads();
    if (threadIdx.x == 0) __hip_atomic_store(pongw, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <int NPK, bool FLAT>
void run_work(const char* name, uint64_t* hping, uint64_t* hpong, uint64_t* dping, uint64_t* dpong, const uint8_t* dpk,
              uint8_t* dout, int rounds) {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  *hping = 0;
  *hpong = 0;
  hipLaunchKernelGGL((pong_work<NPK, FLAT>), dim3(1), dim3(128), 0, s, dping, dpong, dpk, dout, 1200u, 75u, 1u << 26);
  CK(hipGetLastError());
  std::vector<double> us;
  for (int i = 1; i <= rounds; ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    __atomic_store_n(hping, uint64_t(i), __ATOMIC_RELEASE);
    while (__atomic_load_n(hpong, __ATOMIC_ACQUIRE) != uint64_t(i)) {
      __builtin_ia32_pause();
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
        std::fprintf(stderr, "%s: no answer\n", name);
        __atomic_store_n(hping, kStop, __ATOMIC_RELEASE);
        CK(hipStreamSynchronize(s));
        std::exit(1);
      }
    }
    us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  __atomic_store_n(hping, kStop, __ATOMIC_RELEASE);
  CK(hipStreamSynchronize(s));
  CK(hipStreamDestroy(s));
  std::sort(us.begin(), us.end());
  std::printf("{\"probe\": \"pong_work\", \"variant\": \"%s\", \"rounds\": %d, \"us\": {\"p10\": %.2f, \"p50\": %.2f, "
              "\"p90\": %.2f}}\n", name, rounds, us[us.size() / 10], us[us.size() / 2], us[us.size() * 9 / 10]);
  std::fflush(stdout);
}

template <int MODE, int CHAIN>
void run(const char* name, uint64_t* hping, uint64_t* hpong, uint64_t* dping, uint64_t* dpong, uint64_t* dchain,
         int rounds) {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  *hping = 0;
  *hpong = 0;
  hipLaunchKernelGGL((pong<MODE, CHAIN>), dim3(1), dim3(64), 0, s, dping, dpong, dchain, 1u << 26);
  CK(hipGetLastError());
  std::vector<double> us;
  for (int i = 1; i <= rounds; ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    __atomic_store_n(hping, uint64_t(i), __ATOMIC_RELEASE);
    const auto deadline = t0 + std::chrono::seconds(2);
    while (__atomic_load_n(hpong, __ATOMIC_ACQUIRE) != uint64_t(i)) {
      __builtin_ia32_pause();
      if (std::chrono::steady_clock::now() > deadline) {
        std::fprintf(stderr, "%s: no answer to round %d\n", name, i);
        __atomic_store_n(hping, kStop, __ATOMIC_RELEASE);
        CK(hipStreamSynchronize(s));
        std::exit(1);
      }
    }
    us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  __atomic_store_n(hping, kStop, __ATOMIC_RELEASE);
  CK(hipStreamSynchronize(s));
  CK(hipStreamDestroy(s));
  std::sort(us.begin(), us.end());
  std::printf("{\"probe\": \"pingpong\", \"variant\": \"%s\", \"rounds\": %d, \"us\": {\"p10\": %.2f, \"p50\": %.2f, "
              "\"p90\": %.2f, \"p99\": %.2f}}\n",
              name, rounds, us[us.size() / 10], us[us.size() / 2], us[us.size() * 9 / 10], us[us.size() * 99 / 100]);
  std::fflush(stdout);
}

// Host-side cost of classifying a pointer (what every legacy call does for its slab, offsets and
// repair buffer): hipPointerGetAttributes on page-locked, pageable and device memory.
void ptr_attr_cost() {
  void* pinned = nullptr;
  void* dev = nullptr;
  CK(hipHostMalloc(&pinned, 1 << 20, hipHostMallocDefault));
  CK(hipMalloc(&dev, 1 << 20));
  std::vector<uint8_t> pageable(1 << 20);
  const void* ptrs[3] = {pinned, pageable.data(), dev};
  const char* names[3] = {"pinned", "pageable", "device"};
  for (int k = 0; k < 3; ++k) {
    const int n = 200000;
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < n; ++i) {
      hipPointerAttribute_t a;
      if (hipPointerGetAttributes(&a, static_cast<const uint8_t*>(ptrs[k]) + (i & 1023)) != hipSuccess) (void)hipGetLastError();
    }
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / n;
    std::printf("{\"probe\": \"hipPointerGetAttributes\", \"memory\": \"%s\", \"us_per_call\": %.3f}\n", names[k], us);
  }
  CK(hipHostFree(pinned));
  CK(hipFree(dev));
}

int main(int argc, char** argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 20000;
  ptr_attr_cost();
  for (int coherent = 1; coherent >= 0; --coherent) {
    uint64_t* h = nullptr;
    const unsigned flags = coherent ? (hipHostMallocCoherent | hipHostMallocMapped) : hipHostMallocDefault;
    CK(hipHostMalloc(reinterpret_cast<void**>(&h), 4096, flags));
    for (int i = 0; i < 512; ++i) h[i] = 0;
    uint64_t* d = nullptr;
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0));
    uint64_t *hping = h, *hpong = h + 64, *hchain = h + 128;
    uint64_t *dping = d, *dpong = d + 64, *dchain = d + 128;
    (void)hchain;
    std::printf("{\"probe\": \"pingpong\", \"host_memory\": \"%s\"}\n", coherent ? "coherent" : "default");
    run<0, 0>(coherent ? "coh plain" : "def plain", hping, hpong, dping, dpong, dchain, rounds);
    run<2, 0>(coherent ? "coh sleep" : "def sleep", hping, hpong, dping, dpong, dchain, rounds);
    run<1, 0>(coherent ? "coh fence" : "def fence", hping, hpong, dping, dpong, dchain, rounds);
    run<1, 1>(coherent ? "coh fence+1read" : "def fence+1read", hping, hpong, dping, dpong, dchain, rounds);
    run<1, 2>(coherent ? "coh fence+2reads" : "def fence+2reads", hping, hpong, dping, dpong, dchain, rounds);
    // the work step: 10 (or 1) packets of 1200 B from page-locked memory of each kind
    uint8_t *hp = nullptr, *dp = nullptr;
    CK(hipHostMalloc(reinterpret_cast<void**>(&hp), 10 * 1200 + 2048, flags));
    for (int i = 0; i < 10 * 1200 + 2048; ++i) hp[i] = uint8_t(i * 7);
    CK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dp), hp, 0));
    run_work<10, true>(coherent ? "coh 10pk flat" : "def 10pk flat", hping, hpong, dping, dpong, dp, dp + 12000, rounds);
    run_work<10, false>(coherent ? "coh 10pk global" : "def 10pk global", hping, hpong, dping, dpong, dp, dp + 12000, rounds);
    run_work<1, false>(coherent ? "coh 1pk global" : "def 1pk global", hping, hpong, dping, dpong, dp, dp + 12000, rounds);
    CK(hipHostFree(hp));
    CK(hipHostFree(h));
  }
  return 0;
}
