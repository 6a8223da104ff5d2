// probe_vram_host.hip — development probe: can the host write device memory directly (through
// the PCIe BAR), and how fast does a device poll see it?  For the resident legacy encoder: the
// packets and the slot header written by the host into VRAM would make the server's poll and
// packet loads local instead of two PCIe read round trips.  For each allocation kind:
//   * whether hipPointerGetAttributes reports a host-usable pointer;
//   * host store bandwidth for 12 KB (memcpy into the mapping), median of many;
//   * a ping-pong: host writes a 12-KB payload + a flag word into VRAM, a persistent one-wave
//     kernel polls the flag in VRAM (uncached loads), reads the payload, XORs it, writes the
//     result + a done word into page-locked host memory; the host waits for done.
// Not part of the library.  Run under `timeout`: an allocation kind the host cannot touch ends
// the probe with a fault on the host side, before any kernel is launched for it.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::printf("{\"error\": \"%s: %s\"}\n", #x, hipGetErrorString(e_));                   \
      std::fflush(stdout);                                                                   \
      std::exit(2);                                                                          \
    }                                                                                        \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kPayload = 12000;  // ten 1200-B packets

// One wave: poll flag (VRAM, uncached) for round r, XOR the payload's 10 packets column-wise,
// write 1200 B + done (host, write-through).  Leaves after `rounds` rounds or ~2 s idle.
__global__ void server(const uint8_t* vram, const volatile uint64_t* flag, uint8_t* host_out, uint64_t* host_done,
                       uint32_t rounds) {
  const uint32_t lane = threadIdx.x;
  for (uint32_t r = 1; r <= rounds; ++r) {
    uint64_t spins = 0;
    while (__hip_atomic_load(const_cast<uint64_t*>(flag), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != r) {
      if (++spins > (1ull << 26)) return;
    }
    for (uint32_t c = lane; c < 75; c += 64) {
      u32x4 acc = {0u, 0u, 0u, 0u};
      u32x4 v[10];
#pragma unroll
      for (int j = 0; j < 10; ++j)
        v[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(vram + j * 1200 + c * 16));
#pragma unroll
      for (int j = 0; j < 10; ++j) acc ^= v[j];
      *reinterpret_cast<volatile u32x4*>(host_out + c * 16) = acc;
    }
    __builtin_amdgcn_s_waitcnt(0x0F70);
    __builtin_amdgcn_wave_barrier();
    if (lane == 0) __hip_atomic_store(host_done, static_cast<uint64_t>(r), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

static void run(const char* kind, uint8_t* dptr, uint8_t* hptr) {
  std::printf("{\"kind\": \"%s\", \"host_ptr\": \"%p\", \"dev_ptr\": \"%p\"}\n", kind, (void*)hptr, (void*)dptr);
  std::fflush(stdout);
  std::vector<uint8_t> src(kPayload + 64);
  for (size_t i = 0; i < src.size(); ++i) src[i] = uint8_t(i * 7 + 1);
  // host store bandwidth into the mapping
  std::vector<double> wus;
  for (int i = 0; i < 2000; ++i) {
    const auto t0 = std::chrono::steady_clock::now();
    std::memcpy(hptr + 64, src.data(), kPayload);
    std::atomic_thread_fence(std::memory_order_seq_cst);
    wus.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
  }
  std::sort(wus.begin(), wus.end());
  // ping-pong
  uint8_t* hout;
  uint64_t* hdone;
  CK(hipHostMalloc(reinterpret_cast<void**>(&hout), 4096, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipHostMalloc(reinterpret_cast<void**>(&hdone), 64, hipHostMallocCoherent | hipHostMallocMapped));
  *reinterpret_cast<volatile uint64_t*>(hdone) = 0;
  volatile uint64_t* hflag = reinterpret_cast<volatile uint64_t*>(hptr);
  *hflag = 0;
  std::atomic_thread_fence(std::memory_order_seq_cst);
  const uint32_t rounds = 5000;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipLaunchKernelGGL(server, dim3(1), dim3(64), 0, s, dptr + 64, reinterpret_cast<const volatile uint64_t*>(dptr), hout,
                     hdone, rounds);
  CK(hipGetLastError());
  std::vector<double> us;
  uint32_t bad = 0;
  for (uint32_t r = 1; r <= rounds; ++r) {
    src[0] = uint8_t(r);
    const auto t0 = std::chrono::steady_clock::now();
    std::memcpy(hptr + 64, src.data(), kPayload);
    std::atomic_thread_fence(std::memory_order_release);
    *hflag = r;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    const auto t_lim = t0 + std::chrono::seconds(2);
    while (*reinterpret_cast<volatile uint64_t*>(hdone) != r) {
      if (std::chrono::steady_clock::now() > t_lim) {
        std::printf("{\"kind\": \"%s\", \"timeout_round\": %u}\n", kind, r);
        std::fflush(stdout);
        CK(hipStreamSynchronize(s));
        return;
      }
    }
    us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
    // check the first 16 bytes of the XOR
    uint8_t want[16] = {};
    for (int j = 0; j < 10; ++j)
      for (int b = 0; b < 16; ++b) want[b] ^= src[j * 1200 + b];
    if (std::memcmp(want, hout, 16) != 0) ++bad;
  }
  CK(hipStreamSynchronize(s));
  std::sort(us.begin(), us.end());
  std::printf("{\"kind\": \"%s\", \"host_write_12KB_us\": {\"p50\": %.2f, \"p90\": %.2f}, \"pingpong_us\": {\"p10\": %.2f, "
              "\"p50\": %.2f, \"p90\": %.2f, \"p99\": %.2f}, \"wrong\": %u, \"rounds\": %u}\n",
              kind, wus[wus.size() / 2], wus[wus.size() * 9 / 10], us[us.size() / 10], us[us.size() / 2],
              us[us.size() * 9 / 10], us[us.size() * 99 / 100], bad, rounds);
  std::fflush(stdout);
  CK(hipStreamDestroy(s));
  CK(hipHostFree(hout));
  CK(hipHostFree(hdone));
}

int main(int argc, char** argv) {
  const std::string which = argc > 1 ? argv[1] : "all";
  const size_t bytes = 1 << 20;
  if (which == "all" || which == "host") {  // baseline: page-locked host memory (today's slab)
    void* h;
    CK(hipHostMalloc(&h, bytes, hipHostMallocCoherent | hipHostMallocMapped));
    void* d;
    CK(hipHostGetDevicePointer(&d, h, 0));
    run("host_coherent", static_cast<uint8_t*>(d), static_cast<uint8_t*>(h));
  }
  if (which == "all" || which == "finegrained") {
    void* d = nullptr;
    CK(hipExtMallocWithFlags(&d, bytes, hipDeviceMallocFinegrained));
    hipPointerAttribute_t a;
    std::memset(&a, 0, sizeof(a));
    CK(hipPointerGetAttributes(&a, d));
    std::printf("{\"kind\": \"finegrained_vram\", \"type\": %d, \"hostPointer\": \"%p\", \"devicePointer\": \"%p\"}\n",
                int(a.type), a.hostPointer, a.devicePointer);
    std::fflush(stdout);
    if (a.hostPointer != nullptr) run("finegrained_vram", static_cast<uint8_t*>(d), static_cast<uint8_t*>(a.hostPointer));
  }
  if (which == "finegrained_direct") {  // the device pointer dereferenced on the host (large BAR, SVM)
    void* d = nullptr;
    CK(hipExtMallocWithFlags(&d, bytes, hipDeviceMallocFinegrained));
    run("finegrained_vram_direct", static_cast<uint8_t*>(d), static_cast<uint8_t*>(d));
  }
  if (which == "uncached_direct") {
    void* d = nullptr;
    CK(hipExtMallocWithFlags(&d, bytes, hipDeviceMallocUncached));
    run("uncached_vram_direct", static_cast<uint8_t*>(d), static_cast<uint8_t*>(d));
  }
  return 0;
}
