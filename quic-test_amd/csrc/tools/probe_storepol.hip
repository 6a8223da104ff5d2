// probe_storepol.hip — the C2 encode's memory pattern under each cache policy of its loads and
// its staged row stores (round 6).  Not part of the library.
//
// MI355X_MICROARCH.md (the fence / policy table): plain, sc0 and nt stores KEEP the written line in
// the XCD's L2, sc1 and sc0 sc1 stores DROP it; sc1 / nt loads bypass L1 only.  The encode writes
// 3.6 GB once and never reads it back, so its parity lines only take L2 room from the 12 GB read
// stream.  This probe times a memory-only replica of encode_v16<10,3>'s staged form -- workgroup =
// 4 whole groups of 10 x 1200 B, lane = one 16-B column, 10 loads, the XOR (no GF rows: the
// arithmetic is free at this size), the 3 rows staged in LDS and stored by
// consecutive lanes as one 14.4-KB run, 2 workgroups per CU -- with each store policy (plain, nt,
// sc1, sc0 sc1, nt sc1) x load policy (plain, nt), interleaved over rounds in one process, next to
// the product kernel itself (fec_encode_batch_rs_dev) and the 16-B copy (fec_copy_dev).
//
//   probe_storepol [groups=1000000] [rounds=5] [reps=10]  ->  one JSON line per (variant, round)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "fec_hip.h"

namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));

constexpr uint32_t K = 10, R = 3, P = 1200, CPP = P / 16, TILE = 4;
constexpr uint32_t BS = 320;  // TILE * CPP = 300 lanes, 5 waves

enum Store { kPlain = 0, kNt = 1, kSc1 = 2, kSc0Sc1 = 3, kNtSc1 = 4 };

template <int ST>
__device__ __forceinline__ void store16(uint8_t* p, u32x4 v) {
  if constexpr (ST == kPlain) *reinterpret_cast<u32x4u*>(p) = v;
  else if constexpr (ST == kNt) __builtin_nontemporal_store(v, reinterpret_cast<u32x4u*>(p));
  else if constexpr (ST == kSc1) __asm__ volatile("global_store_dwordx4 %0, %1, off sc1" : : "v"(p), "v"(v) : "memory");
  else if constexpr (ST == kSc0Sc1) __asm__ volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(p), "v"(v) : "memory");
  else __asm__ volatile("global_store_dwordx4 %0, %1, off nt sc1" : : "v"(p), "v"(v) : "memory");
}

template <bool NTL>
__device__ __forceinline__ u32x4 load16(const uint8_t* p) {
  if constexpr (NTL) return __builtin_nontemporal_load(reinterpret_cast<const u32x4u*>(p));
  else return *reinterpret_cast<const u32x4u*>(p);
}

template <int ST, bool NTL>
__global__ __launch_bounds__(BS) void enc_replica(const uint8_t* __restrict__ data, uint8_t* __restrict__ parity,
                                                  uint64_t groups) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];  // >= TILE * R * P; sized for 2 per CU
  const uint32_t lane = threadIdx.x, gl = lane / CPP, col = lane - gl * CPP;
  const uint64_t g0 = uint64_t(blockIdx.x) * TILE;
  const uint64_t g = g0 + gl;
  if (gl < TILE && g < groups) {
    const uint8_t* src = data + g * K * P + col * 16u;
    u32x4 d[K];
#pragma unroll
    for (uint32_t j = 0; j < K; ++j) d[j] = load16<NTL>(src + j * P);
    u32x4 a = d[0];
#pragma unroll
    for (uint32_t j = 1; j < K; ++j) a ^= d[j];
#pragma unroll
    for (uint32_t i = 0; i < R; ++i) {
      *reinterpret_cast<u32x4*>(lds + (gl * R + i) * P + col * 16u) = a;
      a = a.yzwx;
    }
  }
  __syncthreads();
  const uint64_t ng = groups - g0 < TILE ? groups - g0 : TILE;
  const uint32_t bytes = static_cast<uint32_t>(ng * R * P);
  uint8_t* dst = parity + g0 * R * P;
  for (uint32_t o = lane * 16u; o < bytes; o += BS * 16u) store16<ST>(dst + o, *reinterpret_cast<const u32x4*>(lds + o));
}

#define CK(x)                                                                                   \
  do {                                                                                          \
    hipError_t e_ = (x);                                                                        \
    if (e_ != hipSuccess) {                                                                     \
      std::printf("{\"error\": \"%s\", \"line\": %d}\n", hipGetErrorString(e_), __LINE__);     \
      std::exit(1);                                                                             \
    }                                                                                           \
  } while (0)

}  // namespace

int main(int argc, char** argv) {
  const uint64_t G = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1000000;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 5;
  const int reps = argc > 3 ? std::atoi(argv[3]) : 10;
  if (fec_hip_device_count() <= 0) {
    std::printf("{\"error\": \"no GPU\"}\n");
    return 1;
  }
  CK(hipSetDevice(0));
  FECEncoderCtx* ctx = fec_encoder_new_device(0.3, 1024, 0);
  if (!ctx) return 1;
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  uint8_t *data = nullptr, *par = nullptr, *ref = nullptr;
  const size_t db = G * K * P, pb = G * R * P;
  CK(hipMalloc(&data, db));
  CK(hipMalloc(&par, pb));
  CK(hipMalloc(&ref, pb));
  if (fec_fill_random_dev(ctx, data, db, 0x5EED5701ull, 0, st) != 0) return 1;
  CK(hipStreamSynchronize(st));
  // 2 workgroups per CU: 160 KiB of LDS per CU
  const uint32_t smem = 64u * 1024u;
  const uint32_t blocks = static_cast<uint32_t>((G + TILE - 1) / TILE);
  struct Var {
    const char* name;
    std::function<void()> run;
    double bytes;
  };
  std::vector<Var> vars;
#define V(ST, NTL, NAME) \
  vars.push_back({NAME, [&] { hipLaunchKernelGGL((enc_replica<ST, NTL>), dim3(blocks), dim3(BS), smem, st, data, par, G); }, double(db + pb)})
  V(kPlain, false, "replica store plain, load plain");
  V(kNt, false, "replica store nt, load plain");
  V(kSc1, false, "replica store sc1, load plain");
  V(kSc0Sc1, false, "replica store sc0 sc1, load plain");
  V(kNtSc1, false, "replica store nt sc1, load plain");
  V(kNt, true, "replica store nt, load nt");
  V(kSc1, true, "replica store sc1, load nt");
#undef V
  vars.push_back({"product encode_v16<10,3> (fec_encode_batch_rs_dev)",
                  [&] { (void)fec_encode_batch_rs_dev(ctx, data, G, K, R, P, ref, st); }, double(db + pb)});
  vars.push_back({"16-B copy (fec_copy_dev), 3.6 GB", [&] { (void)fec_copy_dev(ctx, data, ref, pb, st); },
                  2.0 * double(pb)});
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  // check once: the replica's XOR row 0 equals the product's parity row 0
  {
    vars[1].run();
    vars[7].run();
    CK(hipStreamSynchronize(st));
    std::vector<uint8_t> a(P), b(P);
    bool ok = true;
    for (uint64_t g : {uint64_t(0), G / 2, G - 1}) {
      CK(hipMemcpy(a.data(), par + g * R * P, P, hipMemcpyDeviceToHost));
      CK(hipMemcpy(b.data(), ref + g * R * P, P, hipMemcpyDeviceToHost));
      ok = ok && a == b;
    }
    std::printf("{\"check_row0_equal_product\": %s}\n", ok ? "true" : "false");
  }
  for (int rd = 0; rd < rounds; ++rd)
    for (auto& v : vars) {
      v.run();
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < reps; ++i) v.run();
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      const double per = ms / reps;
      std::printf("{\"round\": %d, \"variant\": \"%s\", \"ms\": %.4f, \"TBps\": %.3f}\n", rd, v.name, per,
                  v.bytes / (per * 1e-3) / 1e12);
      std::fflush(stdout);
    }
  CK(hipFree(data));
  CK(hipFree(par));
  CK(hipFree(ref));
  fec_encoder_free(ctx);
  return 0;
}
