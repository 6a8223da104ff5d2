// probe_glds — does an LDS-DMA (global_load_lds_dwordx4) read stream beat 16-B register
// loads on this box?  Reads a 12 GB buffer (the C2 encode's input) with each form, plain
// and non-temporal, and prints the rate.  Development probe; not part of the library.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                           \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// register loads: every lane 4 x 16 B in flight per iteration, grid-stride
template <bool NT>
__global__ __launch_bounds__(256) void read_reg(const u32x4* __restrict__ in, uint32_t* __restrict__ out,
                                                uint64_t n) {
  const uint64_t stride = uint64_t(gridDim.x) * 256;
  uint32_t acc = 0;
  uint64_t t = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  for (; t + 3 * stride < n; t += 4 * stride) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = NT ? __builtin_nontemporal_load(in + t + u * stride) : in[t + u * stride];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; t < n; t += stride) {
    const u32x4 v = in[t];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x9E3779B9u) out[0] = acc;
}

// LDS-DMA: each wave streams 1-KiB pieces (one glds instruction each) into its own ring of
// SLOTS pieces, keeping INFLIGHT of them outstanding; the bytes are folded from LDS once at
// the end so the loads are not dead.  CONTIG: block b streams its own contiguous range
// instead of the chip sweeping one window.
template <int N>
__device__ __forceinline__ void wait_vm() {
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (N == 1) asm volatile("s_waitcnt vmcnt(1)" ::: "memory");
  if constexpr (N == 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
  if constexpr (N == 3) asm volatile("s_waitcnt vmcnt(3)" ::: "memory");
  if constexpr (N == 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  if constexpr (N == 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  if constexpr (N == 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  if constexpr (N == 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  if constexpr (N == 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
}

__device__ __forceinline__ void glds16(const uint8_t* src, void* lds, int aux_nt) {
  if (aux_nt)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src),
                                     (__attribute__((address_space(3))) void*)(lds), 16, 0, 2);
  else
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src),
                                     (__attribute__((address_space(3))) void*)(lds), 16, 0, 0);
}

template <int AUX, int INFLIGHT, int WAVES, bool CONTIG>
__global__ __launch_bounds__(WAVES * 64) void read_glds(const uint8_t* __restrict__ in, uint32_t* __restrict__ out,
                                                        uint64_t pieces) {
  constexpr int SLOTS = 16;
  __shared__ __attribute__((aligned(16))) uint8_t ring[WAVES][SLOTS][1024];
  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  uint64_t p, end, step;
  if (CONTIG) {
    const uint64_t per = (pieces + gridDim.x - 1) / gridDim.x;
    const uint64_t b0 = uint64_t(blockIdx.x) * per;
    p = b0 + wave;
    end = b0 + per < pieces ? b0 + per : pieces;
    step = WAVES;
  } else {
    p = uint64_t(blockIdx.x) * WAVES + wave;
    end = pieces;
    step = uint64_t(gridDim.x) * WAVES;
  }
  int slot = 0;
  for (; p < end; p += step) {
    glds16(in + p * 1024 + lane * 16, &ring[wave][slot][0], AUX);
    slot = (slot + 1) % SLOTS;
    wait_vm<INFLIGHT>();
  }
  wait_vm<0>();
  const uint32_t v = reinterpret_cast<const uint32_t*>(&ring[wave][0][0])[lane];
  if (v == 0x9E3779B9u) out[1] = v;
}

// Register loads with the glds kernel's piece order and a fixed burst of B pieces per wave.
template <int B>
__global__ __launch_bounds__(256) void read_reg_pieces(const uint8_t* __restrict__ in, uint32_t* __restrict__ out,
                                                       uint64_t pieces) {
  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const uint64_t step = uint64_t(gridDim.x) * 4;
  uint32_t acc = 0;
  uint64_t p = uint64_t(blockIdx.x) * 4 + wave;
  for (; p + (B - 1) * step < pieces; p += B * step) {
    u32x4 v[B];
#pragma unroll
    for (int u = 0; u < B; ++u)
      v[u] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(in + (p + u * step) * 1024 + lane * 16));
#pragma unroll
    for (int u = 0; u < B; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x9E3779B9u) out[2] = acc;
}

// Encode-shaped traffic with no arithmetic: per 10 pieces read by glds (nt), write 3 pieces
// (16-B nt stores of LDS bytes) to out3 -- 12 GB in, 3.6 GB out.
template <int INFLIGHT>
__global__ __launch_bounds__(256) void rw_glds(const uint8_t* __restrict__ in, uint8_t* __restrict__ outp,
                                               uint64_t units) {  // unit = 10 pieces in, 3 out
  constexpr int SLOTS = 16;
  __shared__ __attribute__((aligned(16))) uint8_t ring[4][SLOTS][1024];
  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const uint64_t step = uint64_t(gridDim.x) * 4;
  int slot = 0;
  for (uint64_t u = uint64_t(blockIdx.x) * 4 + wave; u < units; u += step) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
      glds16(in + (u * 10 + i) * 1024 + lane * 16, &ring[wave][(slot + i) % SLOTS][0], 1);
      if (i >= INFLIGHT) wait_vm<INFLIGHT>();
    }
    wait_vm<0>();
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const u32x4 a = *reinterpret_cast<const u32x4*>(&ring[wave][(slot + i) % SLOTS][lane * 16]);
      const u32x4 b = *reinterpret_cast<const u32x4*>(&ring[wave][(slot + i + 3) % SLOTS][lane * 16]);
      __builtin_nontemporal_store(a ^ b, reinterpret_cast<u32x4*>(outp + (u * 3 + i) * 1024 + lane * 16));
    }
    slot = (slot + 10) % SLOTS;
  }
}

// Encode-shaped traffic, pipelined: a wave streams units of 10 pieces into a 2-unit ring
// (unit u+1 in flight while unit u is consumed) and writes 3 pieces per unit.  VMCNT counts
// the stores too, so the wait after issuing unit u+1 also covers unit u-1's stores.
template <int WAVES, bool NTS, int NTL = 1>
__global__ __launch_bounds__(WAVES * 64) void rw2_glds(const uint8_t* __restrict__ in, uint8_t* __restrict__ outp,
                                                       uint64_t units) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[WAVES][20][1024];
  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const uint64_t step = uint64_t(gridDim.x) * WAVES;
  uint64_t u = uint64_t(blockIdx.x) * WAVES + wave;
  if (u >= units) return;
#pragma unroll
  for (int i = 0; i < 10; ++i) glds16(in + (u * 10 + i) * 1024 + lane * 16, &ring[wave][i][0], NTL);
  int cur = 0;
  for (; u < units; u += step) {
    const uint64_t nu = u + step;
    if (nu < units) {
#pragma unroll
      for (int i = 0; i < 10; ++i) glds16(in + (nu * 10 + i) * 1024 + lane * 16, &ring[wave][(1 - cur) * 10 + i][0], NTL);
      wait_vm<10>();  // wait_vm has no 10: emitted below
    } else {
      wait_vm<0>();
    }
    u32x4 acc[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) acc[i] = *reinterpret_cast<const u32x4*>(&ring[wave][cur * 10 + i][lane * 16]);
#pragma unroll
    for (int j = 3; j < 10; ++j) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(&ring[wave][cur * 10 + j][lane * 16]);
      acc[j % 3] ^= v;
    }
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      u32x4* dst = reinterpret_cast<u32x4*>(outp + (u * 3 + i) * 1024 + lane * 16);
      if (NTS) __builtin_nontemporal_store(acc[i], dst); else *dst = acc[i];
    }
    cur = 1 - cur;
  }
}

// C4-shaped traffic (k=20 r=5, 80/20 read/write): a wave streams units of
// KP pieces by LDS-DMA into a 2-unit ring (unit u+1 in flight while u is folded) and stores RP
// pieces per unit (nt).  One wave per workgroup so the ring (2 * KP KiB) fits beside others.
template <int KP, int RP, int NTL>
__global__ __launch_bounds__(64) void rw2_glds_kr(const uint8_t* __restrict__ in, uint8_t* __restrict__ outp,
                                                  uint64_t units) {
  __shared__ __attribute__((aligned(16))) uint8_t ring[2 * KP][1024];
  const int lane = threadIdx.x;
  const uint64_t step = uint64_t(gridDim.x);
  uint64_t u = blockIdx.x;
  if (u >= units) return;
#pragma unroll
  for (int i = 0; i < KP; ++i) glds16(in + (u * KP + i) * 1024 + lane * 16, &ring[i][0], NTL);
  int cur = 0;
  for (; u < units; u += step) {
    const uint64_t nu = u + step;
    if (nu < units) {
#pragma unroll
      for (int i = 0; i < KP; ++i) glds16(in + (nu * KP + i) * 1024 + lane * 16, &ring[(1 - cur) * KP + i][0], NTL);
      asm volatile("s_waitcnt vmcnt(%0)" ::"n"(KP) : "memory");
    } else {
      wait_vm<0>();
    }
    u32x4 acc[RP];
#pragma unroll
    for (int i = 0; i < RP; ++i) acc[i] = *reinterpret_cast<const u32x4*>(&ring[cur * KP + i][lane * 16]);
#pragma unroll
    for (int j = RP; j < KP; ++j) acc[j % RP] ^= *reinterpret_cast<const u32x4*>(&ring[cur * KP + j][lane * 16]);
#pragma unroll
    for (int i = 0; i < RP; ++i)
      __builtin_nontemporal_store(acc[i], reinterpret_cast<u32x4*>(outp + (u * RP + i) * 1024 + lane * 16));
    cur = 1 - cur;
  }
}

// The same C4-shaped traffic with register loads (KP pieces in flight per wave, then RP stores).
template <int KP, int RP>
__global__ __launch_bounds__(256) void rw_reg_kr(const uint8_t* __restrict__ in, uint8_t* __restrict__ outp, uint64_t units) {
  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const uint64_t step = uint64_t(gridDim.x) * 4;
  for (uint64_t u = uint64_t(blockIdx.x) * 4 + wave; u < units; u += step) {
    u32x4 v[KP];
#pragma unroll
    for (int j = 0; j < KP; ++j) v[j] = *reinterpret_cast<const u32x4*>(in + (u * KP + j) * 1024 + lane * 16);
    u32x4 acc[RP];
#pragma unroll
    for (int i = 0; i < RP; ++i) acc[i] = v[i];
#pragma unroll
    for (int j = RP; j < KP; ++j) acc[j % RP] ^= v[j];
#pragma unroll
    for (int i = 0; i < RP; ++i)
      __builtin_nontemporal_store(acc[i], reinterpret_cast<u32x4*>(outp + (u * RP + i) * 1024 + lane * 16));
  }
}

// The same traffic with register loads: a wave loads a unit's 10 pieces, folds, stores 3.
template <int WAVES, bool NTL>
__global__ __launch_bounds__(WAVES * 64) void rw_reg(const uint8_t* __restrict__ in, uint8_t* __restrict__ outp,
                                                     uint64_t units) {
  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const uint64_t step = uint64_t(gridDim.x) * WAVES;
  for (uint64_t u = uint64_t(blockIdx.x) * WAVES + wave; u < units; u += step) {
    u32x4 v[10];
#pragma unroll
    for (int j = 0; j < 10; ++j) {
      const u32x4* src = reinterpret_cast<const u32x4*>(in + (u * 10 + j) * 1024 + lane * 16);
      v[j] = NTL ? __builtin_nontemporal_load(src) : *src;
    }
    u32x4 acc[3] = {v[0], v[1], v[2]};
#pragma unroll
    for (int j = 3; j < 10; ++j) acc[j % 3] ^= v[j];
#pragma unroll
    for (int i = 0; i < 3; ++i)
      __builtin_nontemporal_store(acc[i], reinterpret_cast<u32x4*>(outp + (u * 3 + i) * 1024 + lane * 16));
  }
}

__global__ __launch_bounds__(256) void write16(u32x4* __restrict__ out, uint64_t n) {
  const uint64_t t = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (t < n) __builtin_nontemporal_store(u32x4{1u, 2u, 3u, uint32_t(t)}, out + t);
}

__global__ __launch_bounds__(256) void copy16(const u32x4* __restrict__ in, u32x4* __restrict__ out, uint64_t n) {
  const uint64_t t = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (t < n) out[t] = in[t];
}

int main(int argc, char** argv) {
  const uint64_t bytes = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 12000000000ull;
  const int reps = 10;
  uint8_t* buf;
  uint32_t* out;
  CHECK(hipMalloc(&buf, bytes));
  CHECK(hipMalloc(&out, 64));
  CHECK(hipMemset(buf, 0x5A, bytes));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  const uint64_t n16 = bytes / 16, pieces = bytes / 1024;
  auto time = [&](const char* name, auto fn) {
    fn();
    CHECK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int i = 0; i < reps; ++i) {
      CHECK(hipEventRecord(e0));
      fn();
      CHECK(hipEventRecord(e1));
      CHECK(hipEventSynchronize(e1));
      float t;
      CHECK(hipEventElapsedTime(&t, e0, e1));
      ms.push_back(t);
    }
    std::sort(ms.begin(), ms.end());
    std::printf("%-28s %8.4f ms  %7.1f GB/s\n", name, ms[reps / 2], bytes / (ms[reps / 2] * 1e-3) / 1e9);
    std::fflush(stdout);
  };
  time("reg x16/CU", [&] { read_reg<false><<<cus * 16, 256>>>((const u32x4*)buf, out, n16); });
  time("reg nt x16/CU", [&] { read_reg<true><<<cus * 16, 256>>>((const u32x4*)buf, out, n16); });
  uint8_t* outp;
  const uint64_t units = pieces / 10;
  CHECK(hipMalloc(&outp, units * 3 * 1024));
  time("glds x1 if4 (reads)", [&] { read_glds<2, 4, 4, false><<<cus, 256>>>(buf, out, pieces); });
  std::printf("-- 12 GB read + 3.6 GB written; GB/s column = 12 GB / t; x1.3 for total\n");
  time("copy16 6GB->6GB (R=W)", [&] { copy16<<<(pieces * 32 + 255) / 256, 256>>>((const u32x4*)buf, (u32x4*)(buf + bytes / 2), pieces * 32); });
  time("write 3.6GB nt only", [&] { write16<<<(units * 192 + 255) / 256, 256>>>((u32x4*)outp, units * 192); });
  time("rw2 4w x1 nt", [&] { rw2_glds<4, true><<<cus, 256>>>(buf, outp, units); });
  time("rw2 4w x1 nt, loads default", [&] { rw2_glds<4, true, 0><<<cus, 256>>>(buf, outp, units); });
  time("rw reg 4w x4", [&] { rw_reg<4, false><<<cus * 4, 256>>>(buf, outp, units); });
  time("rw reg 4w x8", [&] { rw_reg<4, false><<<cus * 8, 256>>>(buf, outp, units); });
  time("rw reg 5w x2", [&] { rw_reg<5, false><<<cus * 2, 320>>>(buf, outp, units); });
  time("rw reg nt 4w x4", [&] { rw_reg<4, true><<<cus * 4, 256>>>(buf, outp, units); });
  time("rw reg nt 4w x8", [&] { rw_reg<4, true><<<cus * 8, 256>>>(buf, outp, units); });
  time("rw reg 4w x16", [&] { rw_reg<4, false><<<cus * 16, 256>>>(buf, outp, units); });
  CHECK(hipFree(outp));
  // C4's mix (k=20 r=5): 24 GB read, 6 GB written when the buffer is 24 GB (argv[1] = 24000000000)
  {
    const uint64_t u20 = pieces / 20;
    CHECK(hipMalloc(&outp, u20 * 5 * 1024));
    std::printf("-- C4 mix: %.1f GB read + %.1f GB written; GB/s column = read bytes / t\n", u20 * 20 * 1024 / 1e9,
                u20 * 5 * 1024 / 1e9);
    time("c4 glds 1w x4/CU nt", [&] { rw2_glds_kr<20, 5, 1><<<cus * 4, 64>>>(buf, outp, u20); });
    time("c4 glds 1w x3/CU nt", [&] { rw2_glds_kr<20, 5, 1><<<cus * 3, 64>>>(buf, outp, u20); });
    time("c4 glds 1w x4/CU", [&] { rw2_glds_kr<20, 5, 0><<<cus * 4, 64>>>(buf, outp, u20); });
    time("c4 reg 4w x2", [&] { rw_reg_kr<20, 5><<<cus * 2, 256>>>(buf, outp, u20); });
    time("c4 reg 4w x3", [&] { rw_reg_kr<20, 5><<<cus * 3, 256>>>(buf, outp, u20); });
    time("c4 reg 4w x4", [&] { rw_reg_kr<20, 5><<<cus * 4, 256>>>(buf, outp, u20); });
    CHECK(hipFree(outp));
  }
  CHECK(hipFree(buf));
  CHECK(hipFree(out));
  return 0;
}
