// exit_path_test.cpp — the legacy call site's process exit makes no HIP call from libfec_hip.so
// (fec_coalesce.cpp shutdown_all), and a resident encoder that never serves
// poisons itself instead of hanging later calls (fec_coalesce.cpp Resident::encode).
//
// The program makes legacy fec_encode_batch calls the way the reference's Go wrapper does
// (fec_cgo.go:64/76/138: page-locked slab and repair buffer from the library's allocators, one
// group of ten packets per call), checks every repair row against the XOR on the CPU, and then
// returns from main with its encoders alive, like a Go process exiting.  It defines the HIP
// runtime functions the library calls at teardown itself (the executable's definitions take
// precedence for libfec_hip.so's references; each forwards to the runtime's through
// dlsym(RTLD_NEXT)), and counts the calls that come FROM libfec_hip.so (dladdr of the return
// address) after an atexit hook registered behind the library's has run.
//
//   exit_path_test [resident|coalescer|pageable|nolaunch] [calls]
//   -> one JSON line at exit: {"mode", "calls", "repairs_ok", "first_rc", "calls_after_exit", "names"}
// Built by quic-test_amd/csrc/Makefile (target tests); run by tests/test_gpu_coalesce.py.
#include <dlfcn.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "fec_hip.h"

namespace {

std::atomic<bool> g_exiting{false};
std::atomic<int> g_after{0};
std::mutex g_mu;
std::string g_names;
std::string g_mode = "resident";
int g_calls = 0, g_first_rc = 0;
bool g_ok = true;

bool from_library(void* ret) {
  Dl_info info;
  return dladdr(ret, &info) != 0 && info.dli_fname != nullptr && std::strstr(info.dli_fname, "libfec_hip") != nullptr;
}

void note(const char* name, void* ret) {
  if (!g_exiting.load(std::memory_order_acquire) || !from_library(ret)) return;
  g_after.fetch_add(1);
  std::lock_guard<std::mutex> lk(g_mu);
  if (g_names.find(name) == std::string::npos) g_names += std::string(g_names.empty() ? "" : ",") + name;
}

template <class F>
F real(const char* name) {
  return reinterpret_cast<F>(dlsym(RTLD_NEXT, name));
}

void mark_exit() { g_exiting.store(true, std::memory_order_release); }

void report() {
  std::printf("{\"mode\": \"%s\", \"calls\": %d, \"repairs_ok\": %s, \"first_rc\": %d, \"calls_after_exit\": %d, "
              "\"names\": \"%s\"}\n",
              g_mode.c_str(), g_calls, g_ok ? "true" : "false", g_first_rc, g_after.load(), g_names.c_str());
  std::fflush(stdout);
}

}  // namespace

// ---- the runtime entry points the library's teardown paths used to call ----
#define QFEC_WRAP1(NAME, T1)                                                   \
  extern "C" hipError_t NAME(T1 a) {                                           \
    note(#NAME, __builtin_return_address(0));                                  \
    static auto f = real<hipError_t (*)(T1)>(#NAME);                           \
    return f(a);                                                               \
  }
QFEC_WRAP1(hipStreamSynchronize, hipStream_t)
QFEC_WRAP1(hipStreamDestroy, hipStream_t)
QFEC_WRAP1(hipEventDestroy, hipEvent_t)
QFEC_WRAP1(hipEventSynchronize, hipEvent_t)
QFEC_WRAP1(hipHostFree, void*)
QFEC_WRAP1(hipFree, void*)
QFEC_WRAP1(hipSetDevice, int)
QFEC_WRAP1(hipGetDevice, int*)
#undef QFEC_WRAP1
extern "C" hipError_t hipDeviceSynchronize(void) {
  note("hipDeviceSynchronize", __builtin_return_address(0));
  static auto f = real<hipError_t (*)(void)>("hipDeviceSynchronize");
  return f();
}

int main(int argc, char** argv) {
  std::atexit(report);  // first registered: runs last
  if (argc > 1) g_mode = argv[1];
  const int calls = argc > 2 ? std::atoi(argv[2]) : 200;
  if (g_mode == "coalescer") setenv("QUICFEC_RESIDENT", "0", 1);
  if (g_mode == "nolaunch") {
    setenv("QUICFEC_RESIDENT_TEST_NOLAUNCH", "1", 1);
    setenv("QUICFEC_RESIDENT_DEADLINE_MS", "200", 1);
  }
  FECEncoderCtx* ctx = fec_encoder_new(0.10, 1024);
  if (!ctx) {
    std::printf("{\"skip\": \"no GPU\"}\n");
    return 0;
  }
  constexpr uint32_t P = 1200, K = 10;
  const bool pageable = g_mode == "pageable";
  uint8_t* slab = static_cast<uint8_t*>(pageable ? std::malloc(K * P) : fec_alloc_slab(K * P));
  uint8_t* repair = static_cast<uint8_t*>(pageable ? std::malloc(P) : fec_alloc_repair_buffer(P));
  uint32_t offsets[K];
  for (uint32_t j = 0; j < K; ++j) offsets[j] = j * P;
  uint64_t x = 0x5EED0000u;
  std::vector<uint8_t> want(P);
  for (int c = 0; c < calls; ++c) {
    for (uint32_t i = 0; i < K * P; ++i) {
      x = x * 6364136223846793005ull + 1442695040888963407ull;
      slab[i] = static_cast<uint8_t>(x >> 56);
    }
    std::fill(want.begin(), want.end(), 0);
    for (uint32_t j = 0; j < K; ++j)
      for (uint32_t i = 0; i < P; ++i) want[i] ^= slab[offsets[j] + i];
    std::memset(repair, 0, P);
    const int rc = fec_encode_batch(ctx, slab, offsets, 1, P, repair);
    if (c == 0) g_first_rc = rc;
    if (g_mode == "nolaunch" && c == 0) {
      // the never-serving instance: this call fails (bounded by the deadline), nothing hangs
      if (rc == 0) g_ok = false;
      ++g_calls;
      continue;
    }
    if (rc != 0 || std::memcmp(repair, want.data(), P) != 0) g_ok = false;
    ++g_calls;
  }
  std::atexit(mark_exit);  // registered after the library's shutdown_all: runs before it
  return 0;               // encoders, slab and repair buffer stay alive (a Go process exiting)
}
