// probe_encode.hip — development probe: HBM ceilings and encode-kernel variants,
// interleaved in one process (cdna_hip_programming.md §5.4 rule 24).  Not part of the
// library.  Build: make -C quic-test_amd/csrc probe ; run: quic-test_amd/lib/probe_encode
#include "../fec_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "../gf256.hpp"

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                    \
    }                                                                                  \
  } while (0)

namespace qfec {
namespace {

__global__ __launch_bounds__(256) void copy16(const u32x4* __restrict__ in, u32x4* __restrict__ out, uint64_t n) {
  const uint64_t t = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  if (t < n) out[t] = in[t];
}

__global__ __launch_bounds__(256) void read16(const u32x4* __restrict__ in, uint32_t* __restrict__ out, uint64_t n) {
  const uint64_t t = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  u32x4 a = {0u, 0u, 0u, 0u};
  for (uint64_t i = t; i < n; i += uint64_t(gridDim.x) * 256) a ^= in[i];
  const uint32_t v = a.x ^ a.y ^ a.z ^ a.w;
  if (v == 0x12345678u) out[t] = v;  // practically never: keeps the loads alive
}

// Encode access pattern with XOR only (no GF arithmetic): memory ceiling of the layout.
template <int K, int R>
__global__ __launch_bounds__(256) void enc_mem(const uint8_t* __restrict__ data, uint8_t* __restrict__ parity,
                                               uint32_t nthreads, uint32_t cpp, uint32_t P) {
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
  if (t >= nthreads) return;
  const uint32_t g = t / cpp, col = t - g * cpp;
  const uint8_t* src = data + uint64_t(g) * K * P + col * 16u;
  u32x4 d[K];
#pragma unroll
  for (int j = 0; j < K; ++j) d[j] = *reinterpret_cast<const u32x4*>(src + uint64_t(j) * P);
  u32x4 a = d[0];
#pragma unroll
  for (int j = 1; j < K; ++j) a ^= d[j];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    *reinterpret_cast<u32x4*>(parity + (uint64_t(g) * R + i) * P + col * 16u) = a;
    a = a.yzwx;
  }
}

// Each lane reads NR 16-byte pieces at wave-row stride STRIDE (bytes) and writes NW.
// STRIDE = 1024: every wave row is one aligned KiB; STRIDE = 1200: the encode layout.
template <int NR, int NW, int STRIDE, int POL, int BS>
__global__ __launch_bounds__(BS) void rw_pattern(const uint8_t* __restrict__ in, uint8_t* __restrict__ out,
                                                 uint32_t nthreads, uint32_t cpp) {
  const uint32_t t = blockIdx.x * BS + threadIdx.x;
  if (t >= nthreads) return;
  const uint32_t g = t / cpp, col = t - g * cpp;
  const uint8_t* src = in + uint64_t(g) * NR * STRIDE + col * 16u;
  u32x4 d[NR];
#pragma unroll
  for (int j = 0; j < NR; ++j) d[j] = ld16<POL>(src + uint64_t(j) * STRIDE);
  u32x4 a = d[0];
#pragma unroll
  for (int j = 1; j < NR; ++j) a ^= d[j];
#pragma unroll
  for (int i = 0; i < NW; ++i) {
    st16<POL>(out + (uint64_t(g) * NW + i) * STRIDE + col * 16u, a);
    a = a.yzwx;
  }
}

// Block = T whole groups (k=10, r=3, P=1200 fixed here): lanes [0, T*75) own (group, column),
// the rest idle.  Tile start = T*12000 B, 128-B aligned for T % 4 == 0.
template <int T, int POL>
__global__ __launch_bounds__(((T * 75 + 63) / 64) * 64) void enc_blk(const uint8_t* __restrict__ data,
                                                                   uint8_t* __restrict__ parity, uint32_t groups,
                                                                   const Tab* __restrict__ tabs) {
  constexpr int K = 10, R = 3, P = 1200, CPP = 75;
  const uint32_t lane = threadIdx.x;
  if (lane >= T * CPP) return;
  const uint32_t gl = lane / CPP, col = lane - gl * CPP;
  const uint64_t g = uint64_t(blockIdx.x) * T + gl;
  if (g >= groups) return;
  const uint8_t* src = data + g * K * P + col * 16u;
  u32x4 d[K];
#pragma unroll
  for (int j = 0; j < K; ++j) d[j] = ld16<POL>(src + j * P);
  u32x4 acc[R];
#pragma unroll
  for (int i = 0; i < R; ++i) acc[i] = d[0];
#pragma unroll
  for (int j = 1; j < K; ++j) {
    Sel s;
    prep(d[j], s);
    acc[0] ^= d[j];
#pragma unroll
    for (int i = 1; i < R; ++i) mac(acc[i], s, tabs[(i - 1) * K + j]);
  }
#pragma unroll
  for (int i = 0; i < R; ++i) st16<POL>(parity + (g * R + i) * P + col * 16u, acc[i]);
}

// Memory-pattern probe: enc_xcd<4> with every packet / parity row base rounded down to a
// 128-B line (LA: loads, SA: stores).  Results are garbage when rounded; timing only.
template <bool LA, bool SA, bool NS = false>
__global__ __launch_bounds__(320) void enc_align(const uint8_t* __restrict__ data, uint8_t* __restrict__ parity,
                                                 uint32_t groups, const Tab* __restrict__ tabs) {
  extern __shared__ __attribute__((aligned(16))) uint8_t cap_lds[];
  if (groups == 0xFFFFFFFFu) cap_lds[threadIdx.x] = 0;
  constexpr int T = 4, K = 10, R = 3, P = 1200, CPP = 75;
  const uint32_t nb = gridDim.x, b = blockIdx.x;
  const uint32_t per = nb / 8;
  const uint32_t tile = (b < per * 8) ? (b % 8) * per + b / 8 : b;
  const uint32_t lane = threadIdx.x;
  if (lane >= T * CPP) return;
  const uint32_t gl = lane / CPP, col = lane - gl * CPP;
  const uint64_t g = uint64_t(tile) * T + gl;
  if (g >= groups) return;
  u32x4 d[K];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    uint64_t pb = (g * K + j) * P;
    if (LA) pb &= ~uint64_t(127);
    d[j] = ld16<0>(data + pb + col * 16u);
  }
  u32x4 acc[R];
#pragma unroll
  for (int i = 0; i < R; ++i) acc[i] = d[0];
#pragma unroll
  for (int j = 1; j < K; ++j) {
    Sel s;
    prep(d[j], s);
    acc[0] ^= d[j];
#pragma unroll
    for (int i = 1; i < R; ++i) mac(acc[i], s, tabs[(i - 1) * K + j]);
  }
  if (NS && (acc[0].x != 0x9E3779B9u || acc[R - 1].w != 0x7F4A7C15u)) return;  // reads only
#pragma unroll
  for (int i = 0; i < R; ++i) {
    uint64_t pb = (g * R + i) * P;
    if (SA) pb &= ~uint64_t(127);
    st16<2>(parity + pb + col * 16u, acc[i]);
  }
}

// enc_blk with an XCD-aware tile order: blocks b and b+8 share an XCD (round-robin
// dispatch), so tile = (b % 8) * (nblocks / 8) + b / 8 gives each XCD one contiguous
// eighth of the data.
template <int T, int POL>
__global__ __launch_bounds__(((T * 75 + 63) / 64) * 64) void enc_xcd(const uint8_t* __restrict__ data,
                                                                   uint8_t* __restrict__ parity, uint32_t groups,
                                                                   const Tab* __restrict__ tabs) {
  extern __shared__ __attribute__((aligned(16))) uint8_t cap_lds[];
  if (groups == 0xFFFFFFFFu) cap_lds[threadIdx.x] = 0;
  constexpr int K = 10, R = 3, P = 1200, CPP = 75;
  const uint32_t nb = gridDim.x, b = blockIdx.x;
  const uint32_t per = nb / 8;
  const uint32_t tile = (b < per * 8) ? (b % 8) * per + b / 8 : b;
  const uint32_t lane = threadIdx.x;
  if (lane >= T * CPP) return;
  const uint32_t gl = lane / CPP, col = lane - gl * CPP;
  const uint64_t g = uint64_t(tile) * T + gl;
  if (g >= groups) return;
  const uint8_t* src = data + g * K * P + col * 16u;
  u32x4 d[K];
#pragma unroll
  for (int j = 0; j < K; ++j) d[j] = ld16<POL>(src + j * P);
  u32x4 acc[R];
#pragma unroll
  for (int i = 0; i < R; ++i) acc[i] = d[0];
#pragma unroll
  for (int j = 1; j < K; ++j) {
    Sel s;
    prep(d[j], s);
    acc[0] ^= d[j];
#pragma unroll
    for (int i = 1; i < R; ++i) mac(acc[i], s, tabs[(i - 1) * K + j]);
  }
#pragma unroll
  for (int i = 0; i < R; ++i) st16<POL>(parity + (g * R + i) * P + col * 16u, acc[i]);
}

// Two groups per lane: a workgroup owns 2T whole groups, lane (gl, col) computes column col
// of groups 2gl and 2gl+1 (the second group's loads issued with the first's), so each lane
// has 2K loads in flight and stores 2R rows at once: half the waves for the same bytes in
// flight, and the writes leave in bursts twice as large.  XCD-aware tile order; R = 1 or 3.
template <int T, int R, int POL>
__global__ __launch_bounds__(((T * 75 + 63) / 64) * 64) void enc_2g(const uint8_t* __restrict__ data,
                                                                  uint8_t* __restrict__ parity, uint32_t groups,
                                                                  const Tab* __restrict__ tabs) {
  extern __shared__ __attribute__((aligned(16))) uint8_t cap_lds[];
  if (groups == 0xFFFFFFFFu) cap_lds[threadIdx.x] = 0;
  constexpr int K = 10, P = 1200, CPP = 75;
  const uint32_t nb = gridDim.x, b = blockIdx.x;
  const uint32_t per = nb / 8;
  const uint32_t tile = (b < per * 8) ? (b % 8) * per + b / 8 : b;
  const uint32_t lane = threadIdx.x;
  if (lane >= T * CPP) return;
  const uint32_t gl = lane / CPP, col = lane - gl * CPP;
  const uint64_t g0 = uint64_t(tile) * (2 * T) + 2 * gl;
  if (g0 >= groups) return;
  const bool two = g0 + 1 < groups;
  const uint8_t* src = data + g0 * K * P + col * 16u;
  u32x4 d[2][K];
#pragma unroll
  for (int j = 0; j < K; ++j) d[0][j] = ld16<POL>(src + j * P);
#pragma unroll
  for (int j = 0; j < K; ++j) d[1][j] = two ? ld16<POL>(src + (K + j) * P) : d[0][j];
  u32x4 acc[2][R];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int i = 0; i < R; ++i) acc[h][i] = d[h][0];
#pragma unroll
    for (int j = 1; j < K; ++j) {
      acc[h][0] ^= d[h][j];
      if constexpr (R > 1) {
        Sel s;
        prep(d[h][j], s);
#pragma unroll
        for (int i = 1; i < R; ++i) mac(acc[h][i], s, tabs[(i - 1) * K + j]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < R; ++i) st16<POL>(parity + (g0 * R + i) * P + col * 16u, acc[0][i]);
  if (two) {
#pragma unroll
    for (int i = 0; i < R; ++i) st16<POL>(parity + ((g0 + 1) * R + i) * P + col * 16u, acc[1][i]);
  }
}

// enc_blk as a persistent grid: each workgroup walks tiles blockIdx.x, +gridDim.x, ...
template <int T, int POL>
__global__ __launch_bounds__(((T * 75 + 63) / 64) * 64) void enc_persist(const uint8_t* __restrict__ data,
                                                                       uint8_t* __restrict__ parity, uint32_t groups,
                                                                       const Tab* __restrict__ tabs) {
  constexpr int K = 10, R = 3, P = 1200, CPP = 75;
  const uint32_t lane = threadIdx.x;
  if (lane >= T * CPP) return;
  const uint32_t gl = lane / CPP, col = lane - gl * CPP;
  const uint32_t ntiles = (groups + T - 1) / T;
  for (uint32_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const uint64_t g = uint64_t(tile) * T + gl;
    if (g >= groups) break;
    const uint8_t* src = data + g * K * P + col * 16u;
    u32x4 d[K];
#pragma unroll
    for (int j = 0; j < K; ++j) d[j] = ld16<POL>(src + j * P);
    u32x4 acc[R];
#pragma unroll
    for (int i = 0; i < R; ++i) acc[i] = d[0];
#pragma unroll
    for (int j = 1; j < K; ++j) {
      Sel s;
      prep(d[j], s);
      acc[0] ^= d[j];
#pragma unroll
      for (int i = 1; i < R; ++i) mac(acc[i], s, tabs[(i - 1) * K + j]);
    }
#pragma unroll
    for (int i = 0; i < R; ++i) st16<POL>(parity + (g * R + i) * P + col * 16u, acc[i]);
  }
}

// LDS-staged: block = 4 groups (48000 B, 128-B aligned tile).  Aligned 1 KiB wave-row loads
// into LDS, barrier, each lane reads its column of the 10 packets from LDS.
template <int POL>
__global__ __launch_bounds__(320) void enc_lds(const uint8_t* __restrict__ data, uint8_t* __restrict__ parity,
                                               uint32_t groups, const Tab* __restrict__ tabs) {
  constexpr int K = 10, R = 3, P = 1200, CPP = 75, T = 4, TILE = T * K * P;  // 48000
  __shared__ __attribute__((aligned(16))) uint8_t lds[TILE];
  const uint32_t tid = threadIdx.x;
  const uint64_t g0 = uint64_t(blockIdx.x) * T;
  const uint8_t* tile = data + g0 * K * P;
  const uint32_t nbytes = (g0 + T <= groups ? T : uint32_t(groups - g0)) * K * P;
  // 3000 16-B pieces, 320 lanes -> 10 rounds (last partial)
#pragma unroll
  for (int q = 0; q < 10; ++q) {
    const uint32_t off = (q * 320 + tid) * 16u;
    if (off < nbytes) *reinterpret_cast<u32x4*>(lds + off) = ld16<POL>(tile + off);
  }
  __syncthreads();
  if (tid >= T * CPP) return;
  const uint32_t gl = tid / CPP, col = tid - gl * CPP;
  if (g0 + gl >= groups) return;
  const uint8_t* src = lds + gl * K * P + col * 16u;
  u32x4 d[K];
#pragma unroll
  for (int j = 0; j < K; ++j) d[j] = *reinterpret_cast<const u32x4*>(src + j * P);
  u32x4 acc[R];
#pragma unroll
  for (int i = 0; i < R; ++i) acc[i] = d[0];
#pragma unroll
  for (int j = 1; j < K; ++j) {
    Sel s;
    prep(d[j], s);
    acc[0] ^= d[j];
#pragma unroll
    for (int i = 1; i < R; ++i) mac(acc[i], s, tabs[(i - 1) * K + j]);
  }
  const uint64_t g = g0 + gl;
#pragma unroll
  for (int i = 0; i < R; ++i) st16<POL>(parity + (g * R + i) * P + col * 16u, acc[i]);
}

// Persistent, software-pipelined LDS staging: workgroup = 320 lanes, tile = 4 groups
// (48000 B, 128-B aligned).  Tile t+1 is loaded with aligned, fully coalesced 16-B pieces
// into registers while tile t is computed from LDS; then registers -> LDS.
template <int POL>
__global__ __launch_bounds__(320) void enc_lds2(const uint8_t* __restrict__ data, uint8_t* __restrict__ parity,
                                                uint32_t groups, const Tab* __restrict__ tabs) {
  constexpr int K = 10, R = 3, P = 1200, CPP = 75, T = 4, TILE = T * K * P, NT = 320;
  constexpr int QN = (TILE / 16 + NT - 1) / NT;  // 10 pieces per lane (last round partial)
  __shared__ __attribute__((aligned(16))) uint8_t lds[TILE];
  const uint32_t tid = threadIdx.x;
  const uint32_t ntiles = (groups + T - 1) / T;
  uint32_t tile = blockIdx.x;
  if (tile >= ntiles) return;
  auto pieces_of = [&](uint32_t t) -> uint32_t {
    const uint32_t g0 = t * T;
    const uint32_t gn = (groups - g0 < uint32_t(T)) ? groups - g0 : uint32_t(T);
    return gn * (K * P / 16);
  };
  // Piece indices are clamped to the tile's last piece: surplus lanes load and store that
  // piece again (same bytes, same LDS address), so no lane needs a branch.
  u32x4 reg[QN];
  {
    const uint8_t* src = data + uint64_t(tile) * TILE;
    const uint32_t last = pieces_of(tile) - 1;
#pragma unroll
    for (int q = 0; q < QN; ++q) reg[q] = ld16<0>(src + min(q * NT + tid, last) * 16u);
  }
  const uint32_t gl = tid / CPP, col = tid - gl * CPP;
  for (; tile < ntiles; tile += gridDim.x) {
    const uint32_t last = pieces_of(tile) - 1;
#pragma unroll
    for (int q = 0; q < QN; ++q) *reinterpret_cast<u32x4*>(lds + min(q * NT + tid, last) * 16u) = reg[q];
    __syncthreads();
    const uint32_t next = tile + gridDim.x;
    if (next < ntiles) {
      const uint8_t* src = data + uint64_t(next) * TILE;
      const uint32_t nl = pieces_of(next) - 1;
#pragma unroll
      for (int q = 0; q < QN; ++q) reg[q] = ld16<0>(src + min(q * NT + tid, nl) * 16u);
    }
    const uint64_t g = uint64_t(tile) * T + gl;
    if (tid < uint32_t(T * CPP) && g < groups) {
      const uint8_t* s = lds + gl * (K * P) + col * 16u;
      u32x4 acc[R];
      const u32x4 d0 = *reinterpret_cast<const u32x4*>(s);
#pragma unroll
      for (int i = 0; i < R; ++i) acc[i] = d0;
#pragma unroll
      for (int j = 1; j < K; ++j) {
        const u32x4 dj = *reinterpret_cast<const u32x4*>(s + j * P);
        Sel sl;
        prep(dj, sl);
        acc[0] ^= dj;
#pragma unroll
        for (int i = 1; i < R; ++i) mac(acc[i], sl, tabs[(i - 1) * K + j]);
      }
#pragma unroll
      for (int i = 0; i < R; ++i) st16<POL>(parity + (g * R + i) * P + col * 16u, acc[i]);
    }
    __syncthreads();
  }
}

// Pure reads: NR aligned 1 KiB wave rows per lane, one-shot grid; a store only on a
// practically impossible value keeps the loads alive.
template <int NR>
__global__ __launch_bounds__(256) void read_nr(const uint8_t* __restrict__ in, uint32_t* __restrict__ out,
                                               uint32_t nthreads) {
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
  if (t >= nthreads) return;
  const uint32_t w = t >> 6, l = t & 63;
  const uint8_t* src = in + uint64_t(w) * NR * 1024 + l * 16u;
  u32x4 a = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int j = 0; j < NR; ++j) a ^= *reinterpret_cast<const u32x4*>(src + j * 1024);
  if ((a.x ^ a.y ^ a.z ^ a.w) == 0x9E3779B9u) out[t] = a.x;
}

// Ideal 10:3 stream: every lane reads one 16-B piece of a 12 GB stream; 3 of every 10 waves
// also write one piece of a 3.6 GB stream.
__global__ __launch_bounds__(256) void mix_stream(const u32x4* __restrict__ in, u32x4* __restrict__ out,
                                                  uint32_t nthreads) {
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
  if (t >= nthreads) return;
  const u32x4 v = in[t];
  const uint32_t w = t >> 6;
  if (w % 10 < 3) out[(w / 10 * 3 + w % 10) * 64 + (t & 63)] = v;
}

__device__ __forceinline__ uint32_t swap_pair(uint32_t v) {
  // quad_perm [1,0,3,2]: exchange with the neighbouring lane
  return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);
}

// Block = T whole groups, two lanes per column: lane half h owns packets [5h, 5h+5).
// Partials are combined with a DPP lane swap; h=0 stores rows 0,1 and h=1 stores row 2.
template <int T, int POL>
__global__ __launch_bounds__(((2 * T * 75 + 63) / 64) * 64) void enc_pair(const uint8_t* __restrict__ data,
                                                                        uint8_t* __restrict__ parity, uint32_t groups,
                                                                        const Tab* __restrict__ tabs) {
  constexpr int K = 10, H = 5, R = 3, P = 1200, CPP = 75;
  const uint32_t lane = threadIdx.x;
  const uint32_t p = lane >> 1, h = lane & 1;
  const bool live = p < uint32_t(T * CPP);
  const uint32_t gl = live ? p / CPP : 0, col = live ? p - gl * CPP : 0;
  const uint64_t g = uint64_t(blockIdx.x) * T + gl;
  const bool ok = live && g < groups;
  const uint8_t* src = data + (ok ? g : 0) * K * P + col * 16u + h * (H * P);
  u32x4 d[H];
#pragma unroll
  for (int j = 0; j < H; ++j) d[j] = ok ? ld16<POL>(src + j * P) : u32x4{0u, 0u, 0u, 0u};
  u32x4 acc[R];
  acc[0] = acc[1] = acc[2] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
  for (int j = 0; j < H; ++j) {
    Sel s;
    prep(d[j], s);
    acc[0] ^= d[j];
#pragma unroll
    for (int i = 1; i < R; ++i) {
      // column 0 has coefficient 1, whose tables are the identity: no special case
      const Tab& ta = tabs[(i - 1) * K + j];
      const Tab& tb = tabs[(i - 1) * K + H + j];
      Tab t;
      t.t0lo = h ? tb.t0lo : ta.t0lo;
      t.t0hi = h ? tb.t0hi : ta.t0hi;
      t.t1lo = h ? tb.t1lo : ta.t1lo;
      t.t1hi = h ? tb.t1hi : ta.t1hi;
      t.t2 = h ? tb.t2 : ta.t2;
      mac(acc[i], s, t);
    }
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    acc[i].x ^= swap_pair(acc[i].x);
    acc[i].y ^= swap_pair(acc[i].y);
    acc[i].z ^= swap_pair(acc[i].z);
    acc[i].w ^= swap_pair(acc[i].w);
  }
  if (!ok) return;
  uint8_t* dst = parity + g * R * P + col * 16u;
  if (h == 0) {
    st16<POL>(dst, acc[0]);
    st16<POL>(dst + P, acc[1]);
  } else {
    st16<POL>(dst + 2 * P, acc[2]);
  }
}

}  // namespace
}  // namespace qfec

using namespace qfec;

int main(int argc, char** argv) {
  const uint32_t k = 10, r = 3, P = argc > 4 ? std::atoi(argv[4]) : 1200;
  const uint64_t G = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1000000;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 7;
  const uint64_t nd = G * k * P, np = G * r * P;
  uint8_t *data, *par, *scratch;
  CK(hipMalloc(&data, nd));
  CK(hipMalloc(&par, np));
  CK(hipMalloc(&scratch, nd));
  CK(launch_fill_splitmix(data, nd, 0x5EED0002, 0, nullptr));
  std::vector<uint8_t> M;
  parity_matrix(k, r, M);
  std::vector<CoefEntry> tab;
  for (uint32_t i = 1; i < r; ++i)
    for (uint32_t j = 0; j < k; ++j) tab.push_back(make_entry(M[i * k + j]));
  Tab* dtab;
  CK(hipMalloc(&dtab, tab.size() * 32));
  CK(hipMemcpy(dtab, tab.data(), tab.size() * 32, hipMemcpyHostToDevice));
  const uint32_t cpp = P / 16, nth = uint32_t(G * cpp), blocks = (nth + 255) / 256;
  const uint64_t enc_bytes = (k + r) * uint64_t(P) * G;

  struct Var {
    std::string name;
    uint64_t bytes;
    std::function<void()> run;
    std::vector<float> ms;
  };
  std::vector<Var> vars;
  const uint64_t ncopy = (enc_bytes / 2) / 16;
  vars.push_back({"copy16 (R=W)", ncopy * 32, [&] { copy16<<<(ncopy + 255) / 256, 256>>>((const u32x4*)data, (u32x4*)scratch, ncopy); }, {}});
  const uint64_t nread = nd / 16;
  vars.push_back({"read16 (12GB)", nd, [&] { read16<<<256 * 16, 256>>>((const u32x4*)data, (uint32_t*)scratch, nread); }, {}});
  vars.push_back({"enc_mem<10,3> xor-only", enc_bytes, [&] { enc_mem<10, 3><<<blocks, 256>>>(data, par, nth, cpp, P); }, {}});
#define ENC(POL)                                                                                          \
  vars.push_back({"encode_v16 POL=" #POL, enc_bytes, [&] {                                               \
                    encode_v16<10, 3, 0, true, POL><<<blocks, 256>>>(data, nullptr, par, 0, nth, cpp, P, k, r, 0, dtab, 0u, G, 0u); \
                  }, {}});
  ENC(0)
  ENC(2)
  // read/write mixes on aligned (1024) vs encode (1200) rows
  const uint32_t cpp64 = 64;  // 1 KiB rows: 64 lanes of 16 B
#define RW(NR, NW, ST, POL, BS)                                                                    \
  {                                                                                                \
    const uint64_t grp = nd / (uint64_t(NR) * ST);                                                 \
    const uint32_t cp = ST / 16;                                                                   \
    const uint32_t n = uint32_t(grp * cp);                                                         \
    vars.push_back({"rw<" #NR "," #NW "," #ST ",pol" #POL ",bs" #BS ">", grp * (NR + NW) * uint64_t(ST), [=] { \
                      rw_pattern<NR, NW, ST, POL, BS><<<(n + BS - 1) / BS, BS>>>(data, scratch, n, cp);   \
                    }, {}});                                                                       \
  }
  (void)cpp64;
  RW(10, 3, 1200, 2, 256)
  RW(10, 3, 1024, 2, 256)
#define BLK(T, POL)                                                                                   \
  vars.push_back({"enc_blk<T=" #T ",pol" #POL ">", enc_bytes, [&] {                                   \
                    enc_blk<T, POL><<<uint32_t((G + T - 1) / T), ((T * 75 + 63) / 64) * 64>>>(data, par, uint32_t(G), dtab); \
                  }, {}});
  BLK(4, 0)
  BLK(4, 2)
  BLK(8, 2)
  BLK(12, 2)
#define PAIR(T, POL)                                                                                  \
  vars.push_back({"enc_pair<T=" #T ",pol" #POL ">", enc_bytes, [&] {                                  \
                    enc_pair<T, POL><<<uint32_t((G + T - 1) / T), ((2 * T * 75 + 63) / 64) * 64>>>(data, par, uint32_t(G), dtab); \
                  }, {}});
  // occupancy caps on the production-shaped kernel via dynamic LDS: blocks per CU <= 160K / smem
  for (int smem : {40 * 1024, 53 * 1024, 80 * 1024, 81 * 1024}) {
    vars.push_back({"enc_blk<4> cap " + std::to_string(160 * 1024 / smem) + "/CU smem" + std::to_string(smem / 1024), enc_bytes, [=] {
                      enc_blk<4, 2><<<uint32_t((G + 3) / 4), 320, smem>>>(data, par, uint32_t(G), dtab);
                    }, {}});
  }
  for (int smem : {0, 81 * 1024 / 2 + 16, 80 * 1024}) {
    vars.push_back({"enc_xcd<4> smem" + std::to_string(smem / 1024), enc_bytes, [=] {
                      enc_xcd<4, 2><<<uint32_t((G + 3) / 4), 320, smem>>>(data, par, uint32_t(G), dtab);
                    }, {}});
  }
  // two groups per lane (enc_2g): 2 x 4 groups per 5-wave workgroup at 1 / 2 / 3 workgroups per CU
  for (int per_cu : {1, 2, 3, 4}) {
    const uint32_t smem = per_cu >= 4 ? 0u : 160u * 1024u / (per_cu + 1) + 16u;
    vars.push_back({"enc_2g<4,3> x" + std::to_string(per_cu), enc_bytes, [=] {
                      enc_2g<4, 3, 2><<<uint32_t((G + 7) / 8), 320, smem>>>(data, par, uint32_t(G), dtab);
                    }, {}});
  }
  // XOR row only (r = 1): the production kernel at its r = 1 default vs two groups per lane
  {
    const uint64_t xor_bytes = (k + 1) * uint64_t(P) * G;
    EncodeLaunch e1;
    e1.data = data;
    e1.offsets = nullptr;
    e1.off_kind = OffsetKind::kNone;
    e1.parity = scratch;
    e1.groups = G;
    e1.k = k;
    e1.r = 1;
    e1.P = P;
    e1.tables = nullptr;
    vars.push_back({"xor prod r1", xor_bytes, [=] { CK(launch_encode(e1, nullptr)); }, {}});
    for (int per_cu : {1, 2, 3, 4}) {
      const uint32_t smem = per_cu >= 4 ? 0u : 160u * 1024u / (per_cu + 1) + 16u;
      vars.push_back({"xor_2g r1 x" + std::to_string(per_cu), xor_bytes, [=] {
                        enc_2g<4, 1, 2><<<uint32_t((G + 7) / 8), 320, smem>>>(data, scratch, uint32_t(G), dtab);
                      }, {}});
    }
  }
  {
    const uint32_t smem = 160 * 1024 / 3 + 16;  // 2 workgroups (10 waves) per CU
    vars.push_back({"algn ld0 st0", enc_bytes, [=] { enc_align<false, false><<<uint32_t((G + 3) / 4), 320, smem>>>(data, par, uint32_t(G), dtab); }, {}});
    vars.push_back({"algn ld1 st0", enc_bytes, [=] { enc_align<true, false><<<uint32_t((G + 3) / 4), 320, smem>>>(data, par, uint32_t(G), dtab); }, {}});
    vars.push_back({"algn ld0 st1", enc_bytes, [=] { enc_align<false, true><<<uint32_t((G + 3) / 4), 320, smem>>>(data, par, uint32_t(G), dtab); }, {}});
    vars.push_back({"algn reads only", nd, [=] { enc_align<false, false, true><<<uint32_t((G + 3) / 4), 320, smem>>>(data, par, uint32_t(G), dtab); }, {}});
    vars.push_back({"algn reads only uncapped", nd, [=] { enc_align<false, false, true><<<uint32_t((G + 3) / 4), 320, 0>>>(data, par, uint32_t(G), dtab); }, {}});
    vars.push_back({"algn ld1 st1", enc_bytes, [=] { enc_align<true, true><<<uint32_t((G + 3) / 4), 320, smem>>>(data, par, uint32_t(G), dtab); }, {}});
  }
  for (int per_cu : {1}) {
    const uint32_t ntl = uint32_t((G + 3) / 4);
    const uint32_t grid = std::min<uint32_t>(ntl, 256u * per_cu);
    vars.push_back({"enc_lds2 nt x" + std::to_string(per_cu), enc_bytes, [=] {
                      enc_lds2<2><<<grid, 320>>>(data, par, uint32_t(G), dtab);
                    }, {}});
  }
  {
    EncodeLaunch el;
    el.data = data;
    el.offsets = nullptr;
    el.off_kind = OffsetKind::kNone;
    el.parity = par;
    el.groups = G;
    el.k = k;
    el.r = r;
    el.P = P;
    el.tables = dtab;
    vars.push_back({"enc prod launch_encode", enc_bytes, [=] { CK(launch_encode(el, nullptr)); }, {}});
    for (int w : {5, 10, 15, 20, 40}) {
      EncodeLaunch e2 = el;
      e2.waves_per_cu = w;
      vars.push_back({"enc prod nt-load cap" + std::to_string(w), enc_bytes, [=] {
                        CK((run_encode_v16<10, 3, 0, true, kNtStore | kNtLoad>(e2, 0, nullptr)));
                      }, {}});
    }
    for (int w : {6, 8, 10, 12, 16, 20}) {
      EncodeLaunch e2 = el;
      e2.waves_per_cu = w;
      vars.push_back({"enc prod cap" + std::to_string(w), enc_bytes, [=] { CK(launch_encode(e2, nullptr)); }, {}});
    }
  }
#define LDSV(POL)                                                                                    \
  vars.push_back({"enc_lds<pol" #POL ">", enc_bytes, [&] {                                            \
                    enc_lds<POL><<<uint32_t((G + 3) / 4), 320>>>(data, par, uint32_t(G), dtab);          \
                  }, {}});
#define RNR(NR)                                                                                       \
  {                                                                                                   \
    const uint32_t n = uint32_t(nd / (uint64_t(NR) * 1024) * 64);                                     \
    vars.push_back({"read_nr<" #NR ">", uint64_t(n) / 64 * NR * 1024, [=] {                           \
                      read_nr<NR><<<(n + 255) / 256, 256>>>(data, (uint32_t*)scratch, n);             \
                    }, {}});                                                                          \
  }
  RNR(1)
  RNR(2)
  RNR(4)
  RNR(10)
  {
    const uint32_t n = uint32_t(nd / 16);
    vars.push_back({"mix_stream 10:3", nd + nd * 3 / 10, [=] {
                      mix_stream<<<(n + 255) / 256, 256>>>((const u32x4*)data, (u32x4*)scratch, n);
                    }, {}});
  }
  if (argc > 3) {  // keep only the variants whose name contains one of the '|'-separated filters
    const std::string f = argv[3];
    std::vector<Var> keep;
    for (auto& v : vars) {
      size_t p0 = 0;
      bool hit = false;
      while (p0 <= f.size()) {
        const size_t p1 = std::min(f.find('|', p0), f.size());
        if (p1 > p0 && v.name.find(f.substr(p0, p1 - p0)) != std::string::npos) hit = true;
        p0 = p1 + 1;
      }
      if (hit) keep.push_back(v);
    }
    vars.swap(keep);
  }
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (auto& v : vars) v.run();  // warm
  CK(hipDeviceSynchronize());
  for (int rd = 0; rd < rounds; ++rd)
    for (auto& v : vars) {
      CK(hipEventRecord(a));
      v.run();
      CK(hipEventRecord(b));
      CK(hipEventSynchronize(b));
      float ms;
      CK(hipEventElapsedTime(&ms, a, b));
      v.ms.push_back(ms);
    }
  // every encode variant must reproduce the production kernel's parity bytes
  {
    std::vector<uint8_t> ref(np), got(np);
    encode_v16<10, 3, 0, true, 0><<<blocks, 256>>>(data, nullptr, par, 0, nth, cpp, P, k, r, 0, dtab, 0u, G, 0u);
    CK(hipMemcpy(ref.data(), par, np, hipMemcpyDeviceToHost));
    for (auto& v : vars) {
      if (v.name.rfind("enc", 0) != 0 || v.name.rfind("enc_mem", 0) == 0) continue;
      CK(hipMemset(par, 0, np));
      v.run();
      CK(hipMemcpy(got.data(), par, np, hipMemcpyDeviceToHost));
      std::printf("check %-22s %s\n", v.name.c_str(), got == ref ? "OK" : "MISMATCH");
    }
  }
  {  // the r = 1 variants against the production XOR kernel
    const uint64_t nx = G * uint64_t(P);
    std::vector<uint8_t> ref, got(nx);
    for (auto& v : vars) {
      if (v.name.rfind("xor", 0) != 0) continue;
      CK(hipMemset(scratch, 0, nx));
      v.run();
      CK(hipMemcpy(got.data(), scratch, nx, hipMemcpyDeviceToHost));
      if (ref.empty()) ref = got;
      std::printf("check %-22s %s\n", v.name.c_str(), got == ref ? "OK" : "MISMATCH");
    }
  }
  std::printf("%-28s %10s %10s %10s\n", "variant", "med_ms", "min_ms", "GB/s(med)");
  for (auto& v : vars) {
    std::sort(v.ms.begin(), v.ms.end());
    const float med = v.ms[v.ms.size() / 2];
    std::printf("%-28s %10.4f %10.4f %10.1f\n", v.name.c_str(), med, v.ms[0], v.bytes / (med * 1e-3) / 1e9);
  }
  return 0;
}
