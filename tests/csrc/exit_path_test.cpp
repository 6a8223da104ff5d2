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
// The mixed modes cycle through shapes on both sides of the VRAM ring's inline bounds (1..8
// groups, P 16..2048, odd P, scattered offsets) over page-locked and pageable slabs and repair
// buffers; the *hostring modes keep the resident ring in page-locked host memory
// (QUICFEC_RESIDENT_VRAM=0: the ring kind is fixed per process).
//
// The ring's tag checks (fec_kernels.hpp server_tag):
//  * tear: QUICFEC_RESIDENT_TEST_TEAR -- every inline call stores one chunk's tagged high half
//    first and its low half ~100 us after the slot's header (a write-combined 16-B store evicted
//    in two pieces), and every addressed call of several groups stores its later groups' address
//    words ~100 us after the header.  The server must retry such a slot (resident_bad_slots > 0)
//    and never serve it from the stale half or word.
//  * epoch / epoch_hostring: a tag epoch of 2 laps (QUICFEC_RESIDENT_TEST_EPOCH) with the tear
//    hook: slots 0, 5, 10, ... take 8-group addressed calls on even laps and one-group inline
//    calls on odd laps, so an 8-group call's later address words from two laps back carry the
//    current tag unless the epoch scrub zeroed them -- and the late stores make the server read
//    those words before the new ones land.
//  * poison_mt: 8 threads with a context each make one-group calls; the Resident's 601st call
//    fails as if its deadline had passed (QUICFEC_RESIDENT_TEST_FAIL_AT).  Every call of every thread --
//    that one and the ones in flight when the Resident went out of service included -- must
//    return 0 with the right row (served, or run on the coalescer path).
//
//  * cycles_mt: 4 threads with a context each make one-group calls in bursts of 8 with a 2-ms
//    pause after each (QUICFEC_RESIDENT_IDLE_US=300), so resident instances leave and are
//    relaunched many times while other threads' calls are in flight -- with several serving
//    classes (QUICFEC_RESIDENT_SERVERS) every class must resume from its own progress mark.
//
// Every mode honours QUICFEC_RESIDENT_SERVERS from the environment (serving workgroups).
//
//   exit_path_test [resident|hostring|coalescer|pageable|nolaunch|mixed|mixed_hostring|tear|
//                   epoch|epoch_hostring|poison_mt|cycles_mt] [calls]
//   -> one JSON line at exit: {"mode", "calls", "repairs_ok", "first_rc", "calls_after_exit", "names",
//                              "resident_calls", "resident_inline", "resident_vram", "bad_slots", "scrubs",
//                              "resident_launches", "resident_servers"}
// Built by quic-test_amd/csrc/Makefile (target tests); run by tests/test_gpu_coalesce.py.
#include <dlfcn.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
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
unsigned long long g_resident_calls = 0, g_resident_inline = 0, g_resident_vram = 0, g_bad = 0, g_scrubs = 0;
unsigned long long g_launches = 0, g_servers = 0;
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
              "\"names\": \"%s\", \"resident_calls\": %llu, \"resident_inline\": %llu, \"resident_vram\": %llu, "
              "\"bad_slots\": %llu, \"scrubs\": %llu, \"resident_launches\": %llu, \"resident_servers\": %llu}\n",
              g_mode.c_str(), g_calls, g_ok ? "true" : "false", g_first_rc, g_after.load(), g_names.c_str(), g_resident_calls,
              g_resident_inline, g_resident_vram, g_bad, g_scrubs, g_launches, g_servers);
  std::fflush(stdout);
}

// The library's counters into the report.
void take_stats() {
  FECCoalesceStats st{};
  fec_coalesce_stats_sized(&st, sizeof(st), 0);
  g_resident_calls = st.resident_calls;
  g_resident_inline = st.resident_inline;
  g_resident_vram = st.resident_vram;
  g_bad = st.resident_bad_slots;
  g_scrubs = st.resident_scrubs;
  g_launches = st.resident_launches;
  g_servers = st.resident_servers;
}

// One thread of poison_mt / cycles_mt: `calls` one-group calls of 10 x 1200 B on a context of its
// own, every row checked against the XOR; pause_every > 0: a 2-ms pause after every that many
// calls.  Returns false on any failure.
bool call_thread(int t, int calls, int pause_every) {
  constexpr uint32_t K = 10, P = 1200;
  FECEncoderCtx* ctx = fec_encoder_new(0.10, 1024);
  if (!ctx) return false;
  uint8_t* slab = static_cast<uint8_t*>(fec_alloc_slab(K * P));
  uint8_t* rep = static_cast<uint8_t*>(fec_alloc_repair_buffer(P));
  uint32_t offsets[K];
  for (uint32_t j = 0; j < K; ++j) offsets[j] = j * P;
  uint64_t x = 0x5EED0100u + uint64_t(t);
  std::vector<uint8_t> want(P);
  bool ok = true;
  for (int c = 0; c < calls; ++c) {
    for (uint32_t i = 0; i < K * P; i += 8) {
      x = x * 6364136223846793005ull + 1442695040888963407ull;
      std::memcpy(slab + i, &x, 8);
    }
    std::fill(want.begin(), want.end(), 0);
    for (uint32_t j = 0; j < K; ++j)
      for (uint32_t i = 0; i < P; ++i) want[i] ^= slab[j * P + i];
    const int rc = fec_encode_batch(ctx, slab, offsets, 1, P, rep);
    if (rc != 0 || std::memcmp(rep, want.data(), P) != 0) ok = false;
    if (pause_every > 0 && (c + 1) % pause_every == 0) std::this_thread::sleep_for(std::chrono::milliseconds(2));
  }
  return ok;  // the context and buffers stay alive (a Go process exiting)
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
  const bool mixed = g_mode.rfind("mixed", 0) == 0;
  if (g_mode == "coalescer") setenv("QUICFEC_RESIDENT", "0", 1);
  if (g_mode == "hostring" || g_mode == "mixed_hostring") setenv("QUICFEC_RESIDENT_VRAM", "0", 1);
  if (g_mode == "nolaunch") {
    setenv("QUICFEC_RESIDENT_TEST_NOLAUNCH", "1", 1);
    setenv("QUICFEC_RESIDENT_DEADLINE_MS", "200", 1);
  }
  const bool tear = g_mode == "tear", epoch = g_mode.rfind("epoch", 0) == 0;
  if (tear || epoch) setenv("QUICFEC_RESIDENT_TEST_TEAR", "1", 1);
  if (epoch) setenv("QUICFEC_RESIDENT_TEST_EPOCH", "2", 1);
  // epoch: call c must take seq c (slot c % 1024, lap c / 1024) whatever the serving classes
  if (epoch) setenv("QUICFEC_RESIDENT_SPREAD", "1", 1);
  if (g_mode == "epoch_hostring") setenv("QUICFEC_RESIDENT_VRAM", "0", 1);
  if (g_mode == "poison_mt" || g_mode == "cycles_mt") {
    const bool cycles = g_mode == "cycles_mt";
    if (cycles) setenv("QUICFEC_RESIDENT_IDLE_US", "300", 1);
    else setenv("QUICFEC_RESIDENT_TEST_FAIL_AT", "600", 1);
    const int threads = cycles ? 4 : 8;
    std::vector<std::thread> th;
    std::vector<char> ok(threads, 0);
    for (int t = 0; t < threads; ++t)
      th.emplace_back([t, calls, threads, cycles, &ok] { ok[t] = call_thread(t, calls / threads, cycles ? 8 : 0) ? 1 : 0; });
    for (auto& x : th) x.join();
    for (int t = 0; t < threads; ++t) g_ok = g_ok && ok[t] != 0;
    g_calls = calls / threads * threads;
    take_stats();
    std::atexit(mark_exit);
    return 0;
  }
  FECEncoderCtx* ctx = fec_encoder_new(0.10, 1024);
  if (!ctx) {
    std::printf("{\"skip\": \"no GPU\"}\n");
    return 0;
  }
  constexpr uint32_t K = 10, kMaxG = 8, kMaxP = 2048, kSlab = kMaxG * K * kMaxP + 4096;
  // mixed: shapes on both sides of the inline bounds (<= 4 groups, P % 4 == 0, P <= 1536)
  static const uint32_t kShapes[][2] = {{1, 1200}, {4, 1536}, {2, 16}, {3, 100}, {1, 1201}, {5, 1200},
                                        {8, 1500}, {1, 2048}, {4, 20}, {2, 1538}, {1, 1500}, {6, 333}};
  // tear: every inline shape, plus addressed calls of several groups from the page-locked slab
  static const uint32_t kTearShapes[][2] = {{1, 1200}, {4, 1536}, {2, 16}, {3, 100}, {1, 1500}, {4, 20},
                                            {2, 1224}, {5, 1200}, {8, 1500}, {3, 1201}};
  const bool pageable = g_mode == "pageable";
  uint8_t* slab_pin = static_cast<uint8_t*>(fec_alloc_slab(kSlab));
  uint8_t* rep_pin = static_cast<uint8_t*>(fec_alloc_repair_buffer(kMaxG * kMaxP));
  uint8_t* slab_pg = static_cast<uint8_t*>(std::malloc(kSlab));
  uint8_t* rep_pg = static_cast<uint8_t*>(std::malloc(kMaxG * kMaxP));
  uint32_t offsets[kMaxG * K];
  uint64_t x = 0x5EED0000u;
  auto rnd = [&x] {
    x = x * 6364136223846793005ull + 1442695040888963407ull;
    return static_cast<uint32_t>(x >> 33);
  };
  std::vector<uint8_t> want(kMaxG * kMaxP);
  for (int c = 0; c < calls; ++c) {
    uint32_t G = mixed ? kShapes[c % 12][0] : 1, P = mixed ? kShapes[c % 12][1] : 1200;
    if (tear) G = kTearShapes[c % 10][0], P = kTearShapes[c % 10][1];
    // epoch: call c goes to slot c % 1024 on lap c / 1024 (one thread, one Resident)
    if (epoch) G = ((c % 1024) % 5 == 0 && (c / 1024) % 2 == 0) ? 8 : 1, P = 1200;
    const bool scattered = mixed || tear || epoch;
    uint8_t* slab = (mixed ? (c / 12) % 2 == 1 : tear ? (G <= 4 && P % 4 == 0 && P <= 1536 && (c / 10) % 2 == 1) : pageable) ? slab_pg : slab_pin;
    uint8_t* repair = (mixed ? (c / 24) % 2 == 1 : tear ? (c / 20) % 2 == 1 : pageable) ? rep_pg : rep_pin;
    for (uint32_t i = 0; i < G * K; ++i) offsets[i] = scattered ? rnd() % (kSlab - P + 1) : i * P;
    if (epoch || tear) {
      // fresh bytes where this call's packets are (a stale address or half reads other bytes)
      for (uint32_t i = 0; i < G * K; ++i)
        for (uint32_t b = 0; b < P; b += 4) {
          const uint32_t v = rnd();
          std::memcpy(slab + offsets[i] + b, &v, std::min<uint32_t>(4, P - b));
        }
    } else {
      for (uint32_t i = 0; i < kSlab; i += 4) {
        const uint32_t v = rnd();
        std::memcpy(slab + i, &v, 4);
      }
    }
    std::fill(want.begin(), want.end(), 0);
    for (uint32_t g = 0; g < G; ++g)
      for (uint32_t j = 0; j < K; ++j)
        for (uint32_t i = 0; i < P; ++i) want[g * P + i] ^= slab[offsets[g * K + j] + i];
    std::memset(repair, 0xEE, G * P);
    const int rc = fec_encode_batch(ctx, slab, offsets, G, P, repair);
    if (c == 0) g_first_rc = rc;
    if (g_mode == "nolaunch" && c == 0) {
      // the never-serving instance: this call fails (bounded by the deadline), nothing hangs
      if (rc == 0) g_ok = false;
      ++g_calls;
      continue;
    }
    if (rc != 0 || std::memcmp(repair, want.data(), size_t(G) * P) != 0) g_ok = false;
    ++g_calls;
  }
  take_stats();
  std::atexit(mark_exit);  // registered after the library's shutdown_all: runs before it
  return 0;               // encoders, slabs and repair buffers stay alive (a Go process exiting)
}
