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
    CK(hipHostFree(h));
  }
  return 0;
}
