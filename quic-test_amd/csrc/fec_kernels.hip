// fec_kernels.hip — gfx950 (MI355X, CDNA4) kernels of libfec_hip.
//
// Hot path (SURVEY.md §8(a) a1/a4 and the new GF rows): batched systematic erasure
// encode and decode of QUIC packet groups.  Byte-field arithmetic, HBM-bound: no MFMA.
//
//  * encode_v16<K,R,...>: one lane per 16-byte column of one group (flat over all groups,
//    so a wave covers 64 consecutive columns and its loads are 1 KiB coalesced rows).
//    A lane loads its column of all K data packets (K dwordx4 loads in flight), XORs them
//    into parity row 0 (the reference XOR, fec_xor_simd.cpp:411-427) and multiplies them
//    into rows 1..R-1 with v_perm_b32 table lookups (3 per dword per coefficient, tables
//    in SGPRs via scalar loads), then stores R dwordx4.
//  * classify: one lane per group, erasure mask -> codebook record (rank of the erased
//    data set and of the parity rows used), status byte.
//  * decode_v16<K,MAXE>: one wave per group, so the record (survivor list + tables) is
//    wave-uniform and lives in SGPRs; lanes walk the group's 16-byte columns.
//  * *_bytes: packets shorter than 16 B (one lane per byte), same tables.
//
// Any packet size P >= 16 and any packet alignment run on the vector kernels: the last
// 16-byte column of a packet is shifted back to [P - 16, P) (it overlaps the column before
// it; both lanes compute the same bytes and store the same values), and loads / stores of
// 16 B at any byte address are legal on gfx950 (unaligned global access, which the
// compiler also assumes for amdhsa).  GF arithmetic is byte-wise with one coefficient per
// packet, so a column's position inside its packet never changes its arithmetic.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>
#include <type_traits>

#include "bitslice.hpp"
#include "coef_tables.hpp"
#include "fec_kernels.hpp"
#include "fec_knobs.hpp"

// Forms only the probes (tools/probe_*.hip, built with -DQUICFEC_PROBE_FORMS) select: the
// library's own choice never reaches them, so the product library does not carry them.
#ifdef QUICFEC_PROBE_FORMS
#define QFEC_PROBE_ONLY(...) (__VA_ARGS__)
#else
#define QFEC_PROBE_ONLY(...) hipErrorNotSupported
#endif

namespace qfec {
namespace {

struct Tab {
  uint32_t t0lo, t0hi, t1lo, t1hi, t2, coef, p0, p1;
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
// Byte-aligned views for packet memory (any P, any packet address): same dwordx4 / dword
// instructions as the aligned types.
typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t u32u __attribute__((aligned(1)));

// Memory policy bits of the streaming kernels.
constexpr int kNtLoad = 1;        // non-temporal loads (data read once)
constexpr int kNtStore = 2;       // non-temporal stores
constexpr int kNoCoefBranch = 4;  // decode: multiply by every coefficient, no 0/1 branches
// decode_fused: coefficient tables through LDS.  A record-addressed wave reads e*K 32-B
// table entries of its group's record.  For large codebooks (k=20 r=5: 53,130 records,
// 143 MB) the records miss the scalar cache, and one scalar load per coefficient — a few
// in flight at a time — stalls the wave for several memory round trips per group.  With
// this bit the wave fetches its rows with vector loads issued next to its survivor loads
// (one round trip) and reads them from a per-wave LDS slice.
constexpr int kLdsTabs = 64;
// decode_fused / decode_wave: the m-th rebuilt shard of group g (erased data shards in
// ascending order) goes to out + (g * r + m) * P -- one contiguous run of rebuilt packets
// per group, groups back to back, like encode's parity rows -- instead of its place among
// the group's data shards (fec_recover_batch_rs_dev).  Measured at k=10 r=3, 2 erasures:
// 2.32 vs 2.47 ms in place (profiles/r02_probe_decode_compact_out.txt).
constexpr int kCompactOut = 1024;
// decode_fused with kLdsTabs: the record holds bare coefficient bytes (compact codebook,
// gf256.hpp) and the wave computes each coefficient's tables into its LDS slice
// (coef_tables.hpp) instead of copying 32-byte table entries in: k=20 r=5 records shrink
// from up to 3.3 KB to 256 B, the whole codebook from 143 MB to 12 MB.
constexpr int kCoefBytes = 2048;
// encode_v16: coefficients taken two at a time, so every 3-input XOR (v_bitop3) folds two
// new table products into the accumulator: 6 v_perm + 3 v_bitop3 per pair of coefficients
// and dword instead of 6 v_perm + 2 v_bitop3 + 2 v_xor, and one v_bitop3 per pair on the
// XOR row instead of two v_xor.
constexpr int kPairMac = 4096;
// encode_v16 / encode_bits (tiled, P % 16 == 0, every row of the code in this launch): the
// workgroup's parity rows -- one contiguous window of tile * R * P bytes in HBM -- are staged in
// the LDS the launch already reserves for its occupancy cap and stored by consecutive lanes as
// consecutive 16-B pieces, so only the window's two end lines are partial.  Stored by the lanes
// that computed them, a 1200-B row starts 48 B into a 128-B line and one store instruction
// covers the end of one group's row and the start of another's: each row's edge lines leave as
// pieces of different instructions (PMC writes 1.046x algorithmic at k=10 r=3, 1.053x at k=20
// r=5).
constexpr int kStageRows = 8192;
constexpr int kEncodeStageDefault = 1;  // on: C2 encode 2.753 -> 2.659 ms, C4 5.578 -> 5.520 (profiles/r05a)

template <int POL>
__device__ __forceinline__ u32x4 ld16(const uint8_t* p) {
  if constexpr ((POL & kNtLoad) != 0) return __builtin_nontemporal_load(reinterpret_cast<const u32x4u*>(p));
  else return *reinterpret_cast<const u32x4u*>(p);
}

template <int POL>
__device__ __forceinline__ void st16(uint8_t* p, u32x4 v) {
  if constexpr ((POL & kNtStore) != 0) __builtin_nontemporal_store(v, reinterpret_cast<u32x4u*>(p));
  else *reinterpret_cast<u32x4u*>(p) = v;
}

__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Selector bytes for the three pieces of every byte of a dword.
struct Sel {
  uint32_t s0[4], s1[4], s2[4];
};

__device__ __forceinline__ void prep(const u32x4& x, Sel& s) {
  const uint32_t w[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    s.s0[q] = w[q] & 0x07070707u;
    s.s1[q] = (w[q] >> 3) & 0x07070707u;
    s.s2[q] = (w[q] >> 6) & 0x03030303u;
  }
}

// GF(2^8) product of four bytes with the table's constant.
__device__ __forceinline__ uint32_t gmul(uint32_t s0, uint32_t s1, uint32_t s2, const Tab& t) {
  return xor3(__builtin_amdgcn_perm(t.t0hi, t.t0lo, s0), __builtin_amdgcn_perm(t.t1hi, t.t1lo, s1),
              __builtin_amdgcn_perm(t.t2, t.t2, s2));
}

__device__ __forceinline__ void mac(u32x4& acc, const Sel& s, const Tab& t) {
  acc.x ^= gmul(s.s0[0], s.s1[0], s.s2[0], t);
  acc.y ^= gmul(s.s0[1], s.s1[1], s.s2[1], t);
  acc.z ^= gmul(s.s0[2], s.s1[2], s.s2[2], t);
  acc.w ^= gmul(s.s0[3], s.s1[3], s.s2[3], t);
}

__device__ __forceinline__ void xor_into(u32x4& acc, const u32x4& x) { acc ^= x; }

// acc ^= a*ta ^ b*tb (two coefficients, see kPairMac)
__device__ __forceinline__ uint32_t mac2_dword(uint32_t acc, uint32_t sa0, uint32_t sa1, uint32_t sa2, const Tab& ta,
                                               uint32_t sb0, uint32_t sb1, uint32_t sb2, const Tab& tb) {
  const uint32_t a0 = __builtin_amdgcn_perm(ta.t0hi, ta.t0lo, sa0);
  const uint32_t a1 = __builtin_amdgcn_perm(ta.t1hi, ta.t1lo, sa1);
  const uint32_t a2 = __builtin_amdgcn_perm(ta.t2, ta.t2, sa2);
  const uint32_t b0 = __builtin_amdgcn_perm(tb.t0hi, tb.t0lo, sb0);
  const uint32_t b1 = __builtin_amdgcn_perm(tb.t1hi, tb.t1lo, sb1);
  const uint32_t b2 = __builtin_amdgcn_perm(tb.t2, tb.t2, sb2);
  return xor3(xor3(xor3(acc, a0, a1), a2, b0), b1, b2);
}

__device__ __forceinline__ void mac2(u32x4& acc, const Sel& a, const Tab& ta, const Sel& b, const Tab& tb) {
  acc.x = mac2_dword(acc.x, a.s0[0], a.s1[0], a.s2[0], ta, b.s0[0], b.s1[0], b.s2[0], tb);
  acc.y = mac2_dword(acc.y, a.s0[1], a.s1[1], a.s2[1], ta, b.s0[1], b.s1[1], b.s2[1], tb);
  acc.z = mac2_dword(acc.z, a.s0[2], a.s1[2], a.s2[2], ta, b.s0[2], b.s1[2], b.s2[2], tb);
  acc.w = mac2_dword(acc.w, a.s0[3], a.s1[3], a.s2[3], ta, b.s0[3], b.s1[3], b.s2[3], tb);
}

__device__ __forceinline__ void xor2_into(u32x4& acc, const u32x4& x, const u32x4& y) {
  acc.x = xor3(acc.x, x.x, y.x);
  acc.y = xor3(acc.y, x.y, y.y);
  acc.z = xor3(acc.z, x.z, y.z);
  acc.w = xor3(acc.w, x.w, y.w);
}

__device__ __forceinline__ uint8_t gmul_byte(uint32_t x, const Tab& t) {
  return static_cast<uint8_t>(gmul(x & 7u, (x >> 3) & 7u, (x >> 6) & 3u, t));
}

// XCD-aware order of the workgroups' tiles.  Workgroups are dealt round-robin to the 8
// XCDs (b and b + 8 share one; MI355X_MICROARCH.md "Workgroup dispatch"), so mapping
// b -> (b % 8) * (n / 8) + b / 8 hands every XCD one contiguous eighth of the batch
// instead of every eighth tile.  Placement only changes speed, never results (any
// bijection of tiles is correct).  Measured +4..8% on encode (tools/probe_encode.hip).
__device__ __forceinline__ uint32_t xcd_tile(uint32_t b, uint32_t n) {
  const uint32_t per = n >> 3;
  return b < (per << 3) ? (b & 7u) * per + (b >> 3) : b;
}

// Tile of a decode workgroup by the launch's `swz`: bit 0 the XCD-aware order (xcd_tile),
// bit 1 the groups from last to first.
__device__ __forceinline__ uint32_t decode_block(uint32_t swz) {
  const uint32_t b = (swz & 2u) ? gridDim.x - 1u - blockIdx.x : blockIdx.x;
  return (swz & 1u) ? xcd_tile(b, gridDim.x) : b;
}

// Byte offset of 16-byte column `col` inside a packet of P >= 16 bytes: the last column
// is shifted back to end at P (see the header).
__device__ __forceinline__ uint32_t col_off16(uint32_t col, uint32_t P) {
  const uint32_t o = col * 16u;
  return o + 16u <= P ? o : P - 16u;
}

template <int OFF>
__device__ __forceinline__ const uint8_t* packet_ptr(const uint8_t* data, const void* offsets,
                                                     uint64_t g, uint32_t k, uint32_t j, uint32_t P) {
  if constexpr (OFF == 0) {
    return data + (g * k + j) * static_cast<uint64_t>(P);
  } else if constexpr (OFF == 1) {
    return data + static_cast<const uint32_t*>(offsets)[g * k + j];
  } else if constexpr (OFF == 2) {
    return data + static_cast<const uint64_t*>(offsets)[g * k + j];
  } else {  // absolute packet addresses (OffsetKind::kAddr)
    return reinterpret_cast<const uint8_t*>(static_cast<const uint64_t*>(offsets)[g * k + j]);
  }
}

// kStageRows: after the workgroup's barrier, its staged window (bytes, a multiple of 16) leaves
// LDS as consecutive 16-B pieces from consecutive lanes.
template <int POL>
__device__ __forceinline__ void stage_rows_out(const uint8_t* lds, uint8_t* dst, uint32_t bytes) {
  __syncthreads();
  for (uint32_t o = threadIdx.x * 16u; o < bytes; o += blockDim.x * 16u)
    st16<POL>(dst + o, *reinterpret_cast<const u32x4*>(lds + o));
}

// ---------------------------------------------------------------------------------
// Encode, 16-byte columns.  K > 0: compile-time group size, all K loads issued before
// the arithmetic.  K == 0: runtime k, loop.  Rows [row0, row0 + R) of the parity; when
// FIRST (row0 == 0) row 0 is the plain XOR.  Column 0 of every row is 1 by construction.
// ---------------------------------------------------------------------------------
//
// Columns per packet cpp = ceil(P / 16); column c covers bytes [min(16c, P - 16), +16).
// Thread -> (group, column) mapping, two forms:
//  * tiled (tile > 0): a workgroup owns `tile` whole groups (lanes [0, tile*cpp), the rest
//    idle).  The workgroup's data window then starts and ends on group boundaries, so no
//    cache line is split between workgroups (which sit on different XCDs, each with its
//    own L2) and every line is fetched from HBM once.  Measured +2..4% over flat at
//    k=10/1200 B (tools/probe_encode.hip).
//  * flat (tile == 0): one lane per column over all groups (packet sizes > 512 columns).
template <int K, int R, int OFF, bool FIRST, int POL = 0>
__global__ __launch_bounds__(512) void encode_v16(const uint8_t* __restrict__ data,
                                                  const void* __restrict__ offsets,
                                                  uint8_t* __restrict__ parity, uint64_t g_first,
                                                  uint32_t nthreads, uint32_t cpp, uint32_t P,
                                                  uint32_t k_rt, uint32_t r_total, uint32_t row0,
                                                  const Tab* __restrict__ tabs, uint32_t tile,
                                                  uint64_t groups, uint32_t never) {
  // Dynamic LDS is only an occupancy cap (occupancy_cap_lds).  It is declared and
  // referenced so that every HIP runtime honours the launch's dynamic LDS size; `never`
  // is always 0.
  extern __shared__ __attribute__((aligned(16))) uint8_t occupancy_lds[];
  if (never) occupancy_lds[threadIdx.x] = 0;
  // kStageRows: the rows through LDS (the launcher sizes the dynamic LDS for the window)
  const bool stage = (POL & kStageRows) != 0 && tile > 0 && (P & 15u) == 0 && row0 == 0 && r_total == static_cast<uint32_t>(R);
  uint32_t gl, col, gtile = 0, glocal = 0;
  bool active = true;
  if (tile > 0) {
    const uint32_t lane = threadIdx.x;
    gl = lane / cpp;
    col = lane - gl * cpp;
    glocal = gl;
    active = gl < tile;
    gtile = xcd_tile(blockIdx.x, gridDim.x) * tile;
    gl += gtile;
    active = active && gl < groups;
  } else {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    active = t < nthreads;
    gl = t / cpp;
    col = t - gl * cpp;
  }
  // (staged: an idle lane stays for the workgroup's barrier)
  if (!active && !stage) return;
  const uint64_t g = g_first + gl;
  const uint32_t k = K > 0 ? static_cast<uint32_t>(K) : k_rt;
  const size_t coff = col_off16(col, P);

  u32x4 acc[R];
  if (active) {
  if constexpr (K > 0) {
    u32x4 d[K];
#pragma unroll
    for (int j = 0; j < K; ++j) d[j] = ld16<POL>(packet_ptr<OFF>(data, offsets, g, K, j, P) + coff);
#pragma unroll
    for (int i = 0; i < R; ++i) acc[i] = d[0];
    // kPairMac: coefficients j = 1..K-1 two at a time; an odd one left over takes the
    // single-coefficient loop below (jstart)
    constexpr bool kPair = (POL & kPairMac) != 0 && !(FIRST && R == 1);
    constexpr int kPairs = kPair ? (K - 1) / 2 : 0;
#pragma unroll
    for (int pj = 0; pj < kPairs; ++pj) {
      const int j = 1 + 2 * pj;
      Sel sa, sb;
      prep(d[j], sa);
      prep(d[j + 1], sb);
#pragma unroll
      for (int i = 0; i < R; ++i) {
        if (FIRST && i == 0) {
          xor2_into(acc[0], d[j], d[j + 1]);
        } else {
          const uint32_t row = row0 + static_cast<uint32_t>(i);
          mac2(acc[i], sa, tabs[(row - 1) * K + j], sb, tabs[(row - 1) * K + j + 1]);
        }
      }
    }
    constexpr int jstart = 1 + 2 * kPairs;
#pragma unroll
    for (int j = jstart; j < K; ++j) {
      if constexpr (FIRST && R == 1) {
        xor_into(acc[0], d[j]);
      } else {
        Sel s;
        prep(d[j], s);
#pragma unroll
        for (int i = 0; i < R; ++i) {
          if (FIRST && i == 0) {
            xor_into(acc[0], d[j]);
          } else {
            const uint32_t row = row0 + static_cast<uint32_t>(i);
            mac(acc[i], s, tabs[(row - 1) * K + j]);
          }
        }
      }
    }
  } else {
    const u32x4 d0 = ld16<POL>(packet_ptr<OFF>(data, offsets, g, k, 0, P) + coff);
#pragma unroll
    for (int i = 0; i < R; ++i) acc[i] = d0;
#pragma unroll 4
    for (uint32_t j = 1; j < k; ++j) {
      const u32x4 x = ld16<POL>(packet_ptr<OFF>(data, offsets, g, k, j, P) + coff);
      Sel s;
      prep(x, s);
#pragma unroll
      for (int i = 0; i < R; ++i) {
        if (FIRST && i == 0) {
          xor_into(acc[0], x);
        } else {
          const uint32_t row = row0 + static_cast<uint32_t>(i);
          mac(acc[i], s, tabs[(row - 1) * k + j]);
        }
      }
    }
  }
  }
  if (!stage) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      st16<POL>(parity + (g * r_total + row0 + static_cast<uint32_t>(i)) * static_cast<uint64_t>(P) + coff, acc[i]);
    }
    return;
  }
  // staged: the tile's rows (tile groups x R rows, back to back as in HBM) into LDS, then out
  if (active) {
#pragma unroll
    for (int i = 0; i < R; ++i)
      *reinterpret_cast<u32x4*>(occupancy_lds + (glocal * R + static_cast<uint32_t>(i)) * P + coff) = acc[i];
  }
  stage_rows_out<POL>(occupancy_lds, parity + (g_first + gtile) * R * static_cast<uint64_t>(P),
                      static_cast<uint32_t>((groups - gtile < tile ? groups - gtile : tile) * R * P));
}

// ---------------------------------------------------------------------------------
// Encode, bit-sliced (bitslice.hpp): the code's coefficients compiled in, no tables.
// A lane owns one 16-byte column of two groups: group gl and group gl + tile of its
// workgroup's 2 * tile groups.  The 32 bytes a lane transposes need not be neighbours —
// every byte of packet j is multiplied by the same coefficient in every group — so each load
// instruction of a wave reads 64 consecutive columns exactly as encode_v16 does.  A second
// group past the end repeats the first and is not stored.  All R rows, device-contiguous
// packets.  Measured alternatives (profiles/r03_ab_bits_*.jsonl): a 32-byte chunk of one packet
// per lane (two column runs per instruction) 10% slower at k=10 r=3; adjacent groups, or wave
// pairs over one run of columns, the same as this form; non-temporal loads no better.
// ---------------------------------------------------------------------------------
template <int K, int R, int W, int POL>
__global__ __launch_bounds__(512) void encode_bits(const uint8_t* __restrict__ data,
                                                   uint8_t* __restrict__ parity, uint64_t g_first,
                                                   uint32_t cpp, uint32_t P, uint32_t tile,
                                                   uint64_t groups, uint32_t never) {
  extern __shared__ __attribute__((aligned(16))) uint8_t occupancy_lds[];
  if (never) occupancy_lds[threadIdx.x] = 0;
  // kStageRows: the workgroup's 2 * tile groups' rows through LDS (the launcher sizes it)
  const bool stage = (POL & kStageRows) != 0 && (P & 15u) == 0;
  const uint32_t lane = threadIdx.x;
  const uint32_t glocal = lane / cpp;
  const uint32_t c = lane - glocal * cpp;
  const uint32_t gtile = xcd_tile(blockIdx.x, gridDim.x) * (2 * tile);
  const uint32_t gl = gtile + glocal;
  const bool active = glocal < tile && gl < groups;
  // (staged: an idle lane stays for the workgroup's barrier)
  if (!active && !stage) return;
  const bool second = gl + tile < groups;
  const uint64_t g = g_first + gl, g2 = second ? g + tile : g;
  const uint32_t o = col_off16(c, P);
  uint32_t out[R][8];
  if (active) {
    const uint8_t* base = data + g * K * static_cast<uint64_t>(P) + o;
    const uint8_t* base2 = data + g2 * K * static_cast<uint64_t>(P) + o;
    auto load = [&](int j, uint32_t(&x)[8]) {
      const u32x4 a = ld16<POL>(base + static_cast<uint64_t>(j) * P), b = ld16<POL>(base2 + static_cast<uint64_t>(j) * P);
      x[0] = a.x, x[1] = a.y, x[2] = a.z, x[3] = a.w;
      x[4] = b.x, x[5] = b.y, x[6] = b.z, x[7] = b.w;
    };
    bs::encode_stream<K, R, W>(load, out);
  }
  if (!stage) {
#pragma unroll
    for (int i = 0; i < R; ++i)
      st16<POL>(parity + (g * R + i) * static_cast<uint64_t>(P) + o, u32x4{out[i][0], out[i][1], out[i][2], out[i][3]});
    if (second) {
#pragma unroll
      for (int i = 0; i < R; ++i)
        st16<POL>(parity + (g2 * R + i) * static_cast<uint64_t>(P) + o, u32x4{out[i][4], out[i][5], out[i][6], out[i][7]});
    }
    return;
  }
  if (active) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      *reinterpret_cast<u32x4*>(occupancy_lds + (glocal * R + static_cast<uint32_t>(i)) * P + o) =
          u32x4{out[i][0], out[i][1], out[i][2], out[i][3]};
      if (second)
        *reinterpret_cast<u32x4*>(occupancy_lds + ((glocal + tile) * R + static_cast<uint32_t>(i)) * P + o) =
            u32x4{out[i][4], out[i][5], out[i][6], out[i][7]};
    }
  }
  stage_rows_out<POL>(occupancy_lds, parity + (g_first + gtile) * R * static_cast<uint64_t>(P),
                      static_cast<uint32_t>((groups - gtile < 2 * tile ? groups - gtile : 2 * tile) * R * P));
}

// Encode, one lane per byte (any size / alignment).  All r rows.
template <int OFF>
__global__ __launch_bounds__(256) void encode_bytes(const uint8_t* __restrict__ data,
                                                    const void* __restrict__ offsets,
                                                    uint8_t* __restrict__ parity, uint64_t g_first,
                                                    uint32_t nthreads, uint32_t P, uint32_t k,
                                                    uint32_t r, const Tab* __restrict__ tabs) {
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
  if (t >= nthreads) return;
  const uint32_t gl = t / P;
  const uint32_t b = t - gl * P;
  const uint64_t g = g_first + gl;
  for (uint32_t i = 0; i < r; ++i) {
    uint32_t acc = 0;
    for (uint32_t j = 0; j < k; ++j) {
      const uint32_t x = packet_ptr<OFF>(data, offsets, g, k, j, P)[b];
      acc ^= (i == 0 || j == 0) ? x : gmul_byte(x, tabs[(i - 1) * k + j]);
    }
    parity[(g * r + i) * static_cast<uint64_t>(P) + b] = static_cast<uint8_t>(acc);
  }
}

// ---------------------------------------------------------------------------------
// Decode
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void classify(const uint64_t* __restrict__ masks, uint64_t groups,
                                                uint32_t k, uint32_t r,
                                                const uint64_t* __restrict__ binom, LevelMeta meta,
                                                uint32_t* __restrict__ rec_off,
                                                uint8_t* __restrict__ status) {
  const uint64_t g = static_cast<uint64_t>(blockIdx.x) * 256u + threadIdx.x;
  if (g >= groups) return;
  const uint64_t m = masks[g];
  const uint64_t kmask = k >= 64 ? ~0ull : ((1ull << k) - 1);
  const uint64_t rmask = r >= 64 ? ~0ull : ((1ull << r) - 1);
  uint64_t dm = m & kmask;
  const uint64_t pm = (k >= 64) ? 0 : ((m >> k) & rmask);
  const uint32_t e = __popcll(dm);
  uint32_t rec = kRecNone;
  uint8_t st = 0;
  if (e > 0) {
    const uint32_t alive = r - __popcll(pm);
    if (e > alive) {
      rec = kRecBad;
      st = 1;
    } else {
      uint64_t rank_e = 0, rank_r = 0;
      for (uint32_t t = 0; dm; ++t) {
        const uint32_t j = __ffsll(static_cast<unsigned long long>(dm)) - 1;
        rank_e += binom[j * 65 + t + 1];
        dm &= dm - 1;
      }
      uint64_t sp = ~pm & rmask;
      for (uint32_t t = 0; t < e; ++t) {
        const uint32_t i = __ffsll(static_cast<unsigned long long>(sp)) - 1;
        rank_r += binom[i * 65 + t + 1];
        sp &= sp - 1;
      }
      const uint64_t idx = rank_e * meta.count_r[e] + rank_r;
      rec = static_cast<uint32_t>((meta.base[e] + idx * meta.stride[e]) >> 5);
    }
  }
  rec_off[g] = rec;
  if (status) status[g] = st;
}

// C(n, t) for t = 1..3 without the table (the mask-addressed decode ranks inline; its
// shapes have r <= 3, so e <= 3).  n < t gives 0 like the table.
__device__ __forceinline__ uint64_t choose_small(uint32_t n, uint32_t t) {
  const uint64_t a = n, b = n - 1u, c = n - 2u;
  return t == 1u ? a : t == 2u ? (a * b) >> 1 : (a * b * c) / 6u;
}

// Per-wave LDS slice of N coefficient entries (decode_fused with kLdsTabs; 4 waves per
// workgroup).  Only instantiated by the kernels that use it.
template <int N>
__device__ __forceinline__ Tab* wave_tabs_lds() {
  __shared__ __attribute__((aligned(16))) Tab t[4 * N];
  return t + (threadIdx.x >> 6) * N;
}

// f(std::integral_constant<int, n>) for a wave-uniform n in [1, N]: one straight-line body
// per row count.
template <int N, typename F>
__device__ __forceinline__ void for_row_count(uint32_t n, F& f) {
  if constexpr (N >= 1) {
    if (n == static_cast<uint32_t>(N)) {
      f(std::integral_constant<int, N>{});
      return;
    }
    for_row_count<N - 1>(n, f);
  }
}

// Codebook levels e = 1..3 for the inline classify of the mask-addressed decode.
struct RankMeta {
  uint64_t base[4], stride[4], count_r[4];
};

__device__ __forceinline__ uint32_t rec_byte(const uint32_t* __restrict__ w, uint32_t i) {
  return (w[i >> 2] >> (8u * (i & 3u))) & 0xFFu;
}

// NW-dword (NW = 4: 16 B, NW = 1: 4 B) load/store of one lane's piece.
template <int NW, int POL>
__device__ __forceinline__ void ldw(const uint8_t* p, uint32_t (&v)[NW]) {
  if constexpr (NW == 4) {
    const u32x4 t = ld16<POL>(p);
    v[0] = t.x;
    v[1] = t.y;
    v[2] = t.z;
    v[3] = t.w;
  } else {
    v[0] = *reinterpret_cast<const u32u*>(p);
  }
}

template <int NW, int POL>
__device__ __forceinline__ void stw(uint8_t* p, const uint32_t (&v)[NW]) {
  if constexpr (NW == 4) {
    st16<POL>(p, u32x4{v[0], v[1], v[2], v[3]});
  } else {
    if constexpr ((POL & kNtStore) != 0) __builtin_nontemporal_store(v[0], reinterpret_cast<u32u*>(p));
    else *reinterpret_cast<u32u*>(p) = v[0];
  }
}

// Rebuild rows [m0, m0 + MAXE) of one group's record at byte offset `off` of every
// packet, NW dwords per lane.  The record (survivors, tables) is wave-uniform: SGPRs.
template <int K, int MAXE, int POL, int NW>
__device__ __forceinline__ void decode_piece(const uint32_t* __restrict__ rw, const Tab* __restrict__ tabs,
                                             const uint8_t* __restrict__ dg, const uint8_t* __restrict__ pg,
                                             uint8_t* __restrict__ og, uint32_t k, uint32_t P, uint32_t off,
                                             uint32_t e, uint32_t m0, bool xor_only) {
  auto src_of = [&](uint32_t s) {
    const uint32_t sid = rec_byte(rw, s);
    return sid < k ? dg + sid * static_cast<uint64_t>(P) : pg + (sid - k) * static_cast<uint64_t>(P);
  };
  // Runtime k: survivors in batches of kBatch loads in flight (slots past k re-load
  // survivor 0, a valid address, and are not used).
  constexpr uint32_t kBatch = 8;
  if (xor_only) {  // single data loss rebuilt from parity row 0: the reference XOR
    uint32_t acc[NW] = {};
    for (uint32_t s0 = 0; s0 < k; s0 += kBatch) {
      uint32_t v[kBatch][NW];
#pragma unroll
      for (uint32_t b = 0; b < kBatch; ++b) ldw<NW, POL>(src_of(s0 + b < k ? s0 + b : 0) + off, v[b]);
#pragma unroll
      for (uint32_t b = 0; b < kBatch; ++b)
        if (s0 + b < k)
#pragma unroll
          for (int q = 0; q < NW; ++q) acc[q] ^= v[b][q];
    }
    stw<NW, POL>(og + ((POL & kCompactOut) != 0 ? 0u : rec_byte(rw, 64)) * static_cast<uint64_t>(P) + off, acc);
    return;
  }
  uint32_t acc[MAXE][NW];
#pragma unroll
  for (int m = 0; m < MAXE; ++m)
#pragma unroll
    for (int q = 0; q < NW; ++q) acc[m][q] = 0;
  auto consume = [&](const uint32_t (&v)[NW], uint32_t s, uint32_t kk) {
    uint32_t s0[NW], s1[NW], s2[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      s0[q] = v[q] & 0x07070707u;
      s1[q] = (v[q] >> 3) & 0x07070707u;
      s2[q] = (v[q] >> 6) & 0x03030303u;
    }
#pragma unroll
    for (int m = 0; m < MAXE; ++m) {
      if (m0 + m < e) {
        const Tab& t = tabs[(m0 + m) * kk + s];
        if constexpr ((POL & kNoCoefBranch) != 0) {
          // coefficient 0 / 1 tables are the zero / identity maps: no branch on the value
#pragma unroll
          for (int q = 0; q < NW; ++q) acc[m][q] ^= gmul(s0[q], s1[q], s2[q], t);
        } else if (t.coef == 1u) {
#pragma unroll
          for (int q = 0; q < NW; ++q) acc[m][q] ^= v[q];
        } else if (t.coef != 0u) {
#pragma unroll
          for (int q = 0; q < NW; ++q) acc[m][q] ^= gmul(s0[q], s1[q], s2[q], t);
        }
      }
    }
  };
  if constexpr (K > 0) {
    uint32_t x[K][NW];
#pragma unroll
    for (int s = 0; s < K; ++s) {
      const uint32_t sid = rec_byte(rw, s);
      const uint8_t* src = sid < K ? dg + sid * static_cast<uint64_t>(P) : pg + (sid - K) * static_cast<uint64_t>(P);
      ldw<NW, POL>(src + off, x[s]);
    }
#pragma unroll
    for (int s = 0; s < K; ++s) consume(x[s], s, K);
  } else {
    for (uint32_t s0 = 0; s0 < k; s0 += kBatch) {
      uint32_t v[kBatch][NW];
#pragma unroll
      for (uint32_t b = 0; b < kBatch; ++b) ldw<NW, POL>(src_of(s0 + b < k ? s0 + b : 0) + off, v[b]);
#pragma unroll
      for (uint32_t b = 0; b < kBatch; ++b)
        if (s0 + b < k) consume(v[b], s0 + b, k);
    }
  }
#pragma unroll
  for (int m = 0; m < MAXE; ++m) {
    if (m0 + m < e) {
      // in place: at the erased shard; compact (kCompactOut): row m0 + m of the group's run
      const uint32_t eid = (POL & kCompactOut) != 0 ? m0 + m : rec_byte(rw, 64 + m0 + m);
      stw<NW, POL>(og + eid * static_cast<uint64_t>(P) + off, acc[m]);
    }
  }
}

// decode_wave with the main (16 B/lane) and tail (4 B/lane) passes fused: each lane holds
// NM 16-byte pieces and NT 4-byte pieces of every survivor, so every coefficient table is
// loaded (scalar) and branched on once per wave instead of once per pass.  Packet sizes
// with NM = P / 1024 and NT = ceil((P % 1024) / 256) matching the instantiation.  Tail
// pieces past the packet end are shifted back to [P - 4, P) (same bytes, same values as
// the lane that owns them), so every lane loads and stores and no packet size needs a
// mask; P >= 4.
//
// DIRECT: the survivor and erased shard ids come from the group's erasure mask (scalar bit
// scans) instead of the record header, so the survivor loads depend on one scalar load
// (the mask) rather than two in a chain (rec_off, then the record); the record is then
// read only for its coefficient tables, behind the data loads.  Same ids in the same order
// as the record (gf256.hpp build_record: surviving data ascending, then the e lowest
// surviving parity rows; erased data ascending).
//
// INLINE (mask-addressed only, e <= 3): the kernel classifies its group itself — status
// byte, colex ranks of the erased data set and of the parity rows used, record offset,
// exactly as `classify` does — so no classify launch (and no rec_off round trip through
// HBM) precedes it.  One launch per decode call instead of two.
//
// SCAN > 0 (mask-addressed inline forms): one wave per SCAN consecutive groups (see the
// kernel).
//
// One group of decode_fused (below): `m` is the group's erasure mask (DIRECT forms; wave-
// uniform), `lane` the lane in the wave.
template <int K, int MAXE, int POL, int NM, int NT, bool DIRECT, bool INLINE>
__device__ __forceinline__ void fused_group(uint64_t gw, uint64_t m, uint32_t lane, const uint8_t* __restrict__ data,
                                            const uint8_t* __restrict__ parity,
                                            const uint32_t* __restrict__ rec_off,
                                            const uint8_t* __restrict__ codebook, uint32_t P, uint32_t r,
                                            uint32_t m0, uint8_t* __restrict__ out, const RankMeta& rm,
                                            uint8_t* __restrict__ status) {
  constexpr int NW = 4 * NM + NT;  // dwords per lane and survivor
  constexpr uint64_t kmask = (1ull << K) - 1;
  uint64_t rec_byte_off;
  if constexpr (INLINE) {
    uint64_t dm = m & kmask;
    const uint64_t rmask = (1ull << r) - 1;
    const uint64_t pm = (m >> K) & rmask;
    const uint32_t ne = static_cast<uint32_t>(__popcll(dm));
    const bool bad = ne > r - static_cast<uint32_t>(__popcll(pm));
    if (status != nullptr && lane == 0) status[gw] = bad ? 1 : 0;
    if (ne == 0 || bad) return;
    uint64_t rank_e = 0, rank_r = 0;
    for (uint32_t t = 0; dm; ++t) {
      rank_e += choose_small(static_cast<uint32_t>(__builtin_ctzll(dm)), t + 1u);
      dm &= dm - 1;
    }
    uint64_t sp = ~pm & rmask;
    for (uint32_t t = 0; t < ne; ++t) {
      rank_r += choose_small(static_cast<uint32_t>(__builtin_ctzll(sp)), t + 1u);
      sp &= sp - 1;
    }
    rec_byte_off = rm.base[ne] + (rank_e * rm.count_r[ne] + rank_r) * rm.stride[ne];
  } else {
    const uint32_t rec = __builtin_amdgcn_readfirstlane(rec_off[gw]);
    if (rec >= kRecBad) return;
    rec_byte_off = static_cast<uint64_t>(rec) * 32u;
  }
  const uint8_t* recp = codebook + rec_byte_off;
  const uint32_t* rw = reinterpret_cast<const uint32_t*>(recp);
  uint32_t e;
  bool xor_only;
  // DIRECT: survivor ids (ascending bits of `surv`) and erased ids (bits of `lost`).
  uint64_t surv = 0, lost = 0;
  if constexpr (DIRECT) {
    lost = m & kmask;
    e = static_cast<uint32_t>(__popcll(lost));
    uint64_t alive = ~(m >> K) & ((r >= 64 ? 0ull : (1ull << r)) - 1);
    xor_only = e == 1 && (alive & 1u);
    uint64_t rsel = 0;
    for (uint32_t t = 0; t < e; ++t) {
      rsel |= alive & (~alive + 1);
      alive &= alive - 1;
    }
    surv = (~lost & kmask) | (rsel << K);
  } else {
    e = rw[24] & 0xFFu;
    xor_only = ((rw[24] >> 8) & 0xFFu) != 0;
  }
  if (m0 >= e) return;
  const Tab* tabs = reinterpret_cast<const Tab*>(recp + 128);
  const uint8_t* dg = data + gw * K * static_cast<uint64_t>(P);
  const uint8_t* pg = parity + gw * r * static_cast<uint64_t>(P);
  uint8_t* og = out + gw * K * static_cast<uint64_t>(P);
  const uint32_t main_end = NM * 1024u;
  uint32_t toff[NT > 0 ? NT : 1];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    toff[t] = main_end + t * 256u + lane * 4u;
    if (toff[t] + 4u > P) toff[t] = P - 4u;
  }
  auto load = [&](const uint8_t* base, uint32_t (&v)[NW]) {
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      const u32x4 t = ld16<POL>(base + i * 1024u + lane * 16u);
      v[4 * i] = t.x;
      v[4 * i + 1] = t.y;
      v[4 * i + 2] = t.z;
      v[4 * i + 3] = t.w;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if constexpr ((POL & kNtLoad) != 0) v[4 * NM + t] = __builtin_nontemporal_load(reinterpret_cast<const u32u*>(base + toff[t]));
      else v[4 * NM + t] = *reinterpret_cast<const u32u*>(base + toff[t]);
    }
  };
  auto store = [&](uint8_t* base, const uint32_t (&v)[NW]) {
#pragma unroll
    for (int i = 0; i < NM; ++i) st16<POL>(base + i * 1024u + lane * 16u, u32x4{v[4 * i], v[4 * i + 1], v[4 * i + 2], v[4 * i + 3]});
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if constexpr ((POL & kNtStore) != 0) __builtin_nontemporal_store(v[4 * NM + t], reinterpret_cast<u32u*>(base + toff[t]));
      else *reinterpret_cast<u32u*>(base + toff[t]) = v[4 * NM + t];
    }
  };
  auto shard = [&](uint32_t sid) {
    return sid < K ? dg + sid * static_cast<uint64_t>(P) : pg + (sid - K) * static_cast<uint64_t>(P);
  };
  // Survivor slot s -> shard id, and erased slot m -> data shard id.
  uint32_t sid[K];
#pragma unroll
  for (int s = 0; s < K; ++s) {
    if constexpr (DIRECT) {
      sid[s] = static_cast<uint32_t>(__builtin_ctzll(surv));
      surv &= surv - 1;
    } else {
      sid[s] = rec_byte(rw, s);
    }
  }
  // destination of rebuilt row m (erased data shard `erased(m)`)
  auto dest = [&](uint32_t m, uint32_t eid) -> uint8_t* {
    if constexpr ((POL & kCompactOut) != 0) {
      // packed rows (fec_recover_batch_rs_dev_packed): the group's first row from its prefix
      // sum, passed in rec_off, which the inline-classify forms do not otherwise read
      uint64_t row = gw * r + m;
      if constexpr (INLINE) {
        if (rec_off != nullptr) row = static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(rec_off[gw])) + m;
      }
      return out + row * static_cast<uint64_t>(P);
    } else {
      return og + eid * static_cast<uint64_t>(P);
    }
  };
  auto erased = [&](uint32_t m) -> uint32_t {
    if constexpr (DIRECT) {
      uint64_t x = lost;
      for (uint32_t t = 0; t < m; ++t) x &= x - 1;
      return static_cast<uint32_t>(__builtin_ctzll(x));
    } else {
      return rec_byte(rw, 64 + m);
    }
  };
  if (xor_only) {  // single data loss rebuilt from parity row 0: the reference XOR
    uint32_t acc[NW] = {};
#pragma unroll
    for (int s = 0; s < K; ++s) {
      uint32_t v[NW];
      load(shard(sid[s]), v);
#pragma unroll
      for (int q = 0; q < NW; ++q) acc[q] ^= v[q];
    }
    store(dest(0, erased(0)), acc);
    return;
  }
  // kLdsTabs: the wave's coefficient rows [m0, m0 + MAXE) come in with vector loads issued
  // next to the survivor loads and are read back from LDS, instead of one scalar load per
  // coefficient (records of large codebooks miss the scalar cache; see kLdsTabs).
  constexpr bool kLds = (POL & kLdsTabs) != 0;
  constexpr int kTabPieces = MAXE * K * 2;  // 16-B pieces of MAXE rows of K entries
  constexpr int kTabIter = kLds ? (kTabPieces + 63) / 64 : 1;
  const uint32_t tab_pieces = (e - m0 < MAXE ? e - m0 : MAXE) * K * 2u;
  // the slice holds kTabIter whole wave-loads (16 B per lane), so no load writes past it
  constexpr int kSliceTabs = kTabIter * 64 / 2;
  // kCoefBytes: coefficient (m, s) of this pass is byte m * K + s after the compact record's
  // header; lane i loads coefficient i (+ 64 j) now, ahead of the survivor loads, and builds
  // its tables into the LDS slice once the survivor loads are in flight (below).
  constexpr int kCoefIter = (MAXE * K + 63) / 64;
  uint32_t coef[kCoefIter];
  if constexpr (kLds && (POL & kCoefBytes) != 0) {
    const uint8_t* cb = recp + 128 + m0 * K;
    const uint32_t ncoef = tab_pieces / 2u;
#pragma unroll
    for (int j = 0; j < kCoefIter; ++j) {
      const uint32_t i = lane + 64u * j;
      coef[j] = i < ncoef ? cb[i] : 0u;
    }
  } else if constexpr (kLds) {
    // direct-to-LDS loads (global_load_lds_dwordx4: LDS address = wave base + lane * 16, no
    // VGPR destination); pieces past the rows re-read the last piece into unused slots
    const uint8_t* src = reinterpret_cast<const uint8_t*>(tabs + m0 * K);
    uint8_t* dst = reinterpret_cast<uint8_t*>(wave_tabs_lds<kSliceTabs>());
#pragma unroll
    for (int i = 0; i < kTabIter; ++i) {
      uint32_t idx = lane + 64u * i;
      if (idx >= tab_pieces) idx = tab_pieces - 1u;
      __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + idx * 16u),
                                       (__attribute__((address_space(3))) void*)(dst + i * 1024), 16, 0, 0);
    }
  }
  // kLds: survivors stream through a window of kWin loads in flight (survivor s + kWin is
  // loaded as survivor s is consumed), so K = 20 needs a third of the data VGPRs: 114 VGPRs,
  // 4 waves per SIMD at 1200 B (window 10: 153, 3 waves; 5-erasure decode 4.73 vs 4.28-4.50
  // TB/s, profiles/r01_probe_decode_window.txt).  The first window is in flight with the
  // table loads.
  constexpr bool kWinPath = kLds;
  constexpr int kWinW = 6;
  constexpr int kWin = kWinPath ? (K < kWinW ? K : kWinW) : K;
  uint32_t x[K][NW];
#pragma unroll
  for (int s = 0; s < kWin; ++s) load(shard(sid[s]), x[s]);
  if constexpr (kLds && (POL & kCoefBytes) != 0) {
    Tab* lt = wave_tabs_lds<kSliceTabs>();
    const uint32_t ncoef = tab_pieces / 2u;
#pragma unroll
    for (int j = 0; j < kCoefIter; ++j) {
      const uint32_t i = lane + 64u * j;
      if (i < ncoef) {
        const TabWords w = tab_words(coef[j]);
        lt[i] = Tab{w.t0lo, w.t0hi, w.t1lo, w.t1hi, w.t2, coef[j], 0u, 0u};
      }
    }
  }
  const Tab* rt = tabs + m0 * K;  // rows of this pass: entry (m, s) at rt[m * K + s]
  if constexpr (kWinPath) {
    const Tab* lt = rt;
    if constexpr (kLds) {
      // Wait for every load so far (vmcnt(0): the compiler may order the survivor loads
      // around the LDS loads, so no counted wait), then keep LDS reads below the wait.
      __builtin_amdgcn_s_waitcnt(0x0F70);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      lt = wave_tabs_lds<kSliceTabs>();
    }
    // Straight-line body per row count NR (no branch on the row index or the coefficient:
    // table values are VGPRs here, and the 0 / 1 entries are the zero / identity maps).
    auto rebuild = [&](auto nr_c) __attribute__((always_inline)) {
      constexpr int NR = decltype(nr_c)::value;
      uint32_t acc[NR][NW];
#pragma unroll
      for (int m = 0; m < NR; ++m)
#pragma unroll
        for (int q = 0; q < NW; ++q) acc[m][q] = 0;
#pragma unroll
      for (int s = 0; s < K; ++s) {
        // survivor s's selectors, table reads and the next window load stay in its
        // iteration (the compiler otherwise hoists them all: 472 VGPRs + AGPRs, one wave
        // per SIMD)
#pragma unroll
        for (int q = 0; q < NW; ++q) __asm__ volatile("" : "+v"(x[s][q]));
        __builtin_amdgcn_sched_barrier(0);
        if (s + kWin < K) load(shard(sid[s + kWin]), x[s + kWin]);  // folded when unrolled
        uint32_t s0[NW], s1[NW], s2[NW];
#pragma unroll
        for (int q = 0; q < NW; ++q) {
          s0[q] = x[s][q] & 0x07070707u;
          s1[q] = (x[s][q] >> 3) & 0x07070707u;
          s2[q] = (x[s][q] >> 6) & 0x03030303u;
        }
#pragma unroll
        for (int m = 0; m < NR; ++m) {
          const Tab t = lt[m * K + s];
#pragma unroll
          for (int q = 0; q < NW; ++q) {
            acc[m][q] ^= gmul(s0[q], s1[q], s2[q], t);
            // pin the accumulation order: reassociating the K-term XOR chains into trees
            // keeps every survivor's products live at once (spills)
            __asm__ volatile("" : "+v"(acc[m][q]));
          }
        }
      }
#pragma unroll
      for (int m = 0; m < NR; ++m) store(dest(m0 + m, erased(m0 + m)), acc[m]);
    };
    for_row_count<MAXE>(e - m0 < MAXE ? e - m0 : MAXE, rebuild);
    return;
  } else {
#pragma unroll
    for (int s = kWin; s < K; ++s) load(shard(sid[s]), x[s]);
  }
  uint32_t acc[MAXE][NW];
#pragma unroll
  for (int m = 0; m < MAXE; ++m)
#pragma unroll
    for (int q = 0; q < NW; ++q) acc[m][q] = 0;
#pragma unroll
  for (int s = 0; s < K; ++s) {
    uint32_t s0[NW], s1[NW], s2[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      s0[q] = x[s][q] & 0x07070707u;
      s1[q] = (x[s][q] >> 3) & 0x07070707u;
      s2[q] = (x[s][q] >> 6) & 0x03030303u;
    }
#pragma unroll
    for (int m = 0; m < MAXE; ++m) {
      if (m0 + m < e) {
        const Tab& t = rt[m * K + s];
        if (t.coef == 1u) {
#pragma unroll
          for (int q = 0; q < NW; ++q) acc[m][q] ^= x[s][q];
        } else if (t.coef != 0u) {
#pragma unroll
          for (int q = 0; q < NW; ++q) acc[m][q] ^= gmul(s0[q], s1[q], s2[q], t);
        }
      }
    }
  }
#pragma unroll
  for (int m = 0; m < MAXE; ++m)
    if (m0 + m < e) store(dest(m0 + m, erased(m0 + m)), acc[m]);
}

template <int K, int MAXE, int POL, int NM, int NT, bool DIRECT = false, bool INLINE = DIRECT, int SCAN = 0>
__global__ __launch_bounds__(256) void decode_fused(const uint8_t* __restrict__ data,
                                                    const uint8_t* __restrict__ parity,
                                                    const uint32_t* __restrict__ rec_off,
                                                    const uint8_t* __restrict__ codebook,
                                                    uint64_t groups, uint32_t P, uint32_t r, uint32_t m0,
                                                    uint8_t* __restrict__ out, uint32_t never, uint32_t swz,
                                                    const uint64_t* __restrict__ masks, RankMeta rm,
                                                    uint8_t* __restrict__ status) {
  static_assert(!INLINE || (DIRECT && MAXE <= 3), "inline classify: mask-addressed forms with r <= 3");
  static_assert(SCAN == 0 || (DIRECT && INLINE && (SCAN <= 64 || SCAN % 256 == 0)),
                "scan: mask-addressed inline forms, <= 64 groups per wave or whole 256-group rows per block");
  extern __shared__ __attribute__((aligned(16))) uint8_t occupancy_lds[];  // see encode_v16
  if (never) occupancy_lds[threadIdx.x] = 0;
  const uint64_t wv = static_cast<uint64_t>(decode_block(swz)) * 4u +
                      static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(threadIdx.x >> 6));
  const uint32_t lane = threadIdx.x & 63u;
  if constexpr (SCAN > 64) {
    // Segment form: the block's 4 waves check SCAN groups (one mask per thread and row of
    // 256), write every status byte, compact the groups to rebuild into LDS in group order
    // and share them out round robin, so every wave of the block gets the same number of
    // groups (+-1) whatever the loss pattern; a block's groups sit within SCAN * (k + r)
    // packets of each other.
    constexpr int J = SCAN / 256;
    __shared__ uint64_t seg_mask[SCAN];
    __shared__ uint16_t seg_idx[SCAN];
    __shared__ uint32_t seg_cnt[J * 4];
    const uint64_t g0 = static_cast<uint64_t>(decode_block(swz)) * SCAN;
    if (g0 >= groups) return;
    const uint32_t wave = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(threadIdx.x >> 6));
    constexpr uint64_t kmask = (1ull << K) - 1;
    uint64_t mv[J], bal[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      const uint64_t g = g0 + j * 256u + threadIdx.x;
      bool need = false;
      mv[j] = 0;
      if (g < groups) {
        mv[j] = masks[g];
        const uint32_t ne = static_cast<uint32_t>(__popcll(mv[j] & kmask));
        const bool bad = ne > r - static_cast<uint32_t>(__popcll((mv[j] >> K) & ((1ull << r) - 1)));
        if (status != nullptr) status[g] = bad ? 1 : 0;
        need = ne > 0 && !bad;
      }
      bal[j] = __ballot(need);
      if (lane == 0) seg_cnt[j * 4 + wave] = static_cast<uint32_t>(__popcll(bal[j]));
    }
    __syncthreads();
    uint32_t total = 0, off[J];
#pragma unroll
    for (int c = 0; c < J * 4; ++c) {
      if (static_cast<uint32_t>(c % 4) == wave) off[c / 4] = total;
      total += seg_cnt[c];
    }
    const uint64_t below = (1ull << lane) - 1;
#pragma unroll
    for (int j = 0; j < J; ++j) {
      if ((bal[j] >> lane) & 1u) {
        const uint32_t pos = off[j] + static_cast<uint32_t>(__popcll(bal[j] & below));
        seg_mask[pos] = mv[j];
        seg_idx[pos] = static_cast<uint16_t>(j * 256u + threadIdx.x);
      }
    }
    __syncthreads();
    for (uint32_t i = wave; i < total; i += 4u) {
      const uint64_t mi = seg_mask[i];
      const uint64_t m = (static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(mi >> 32))) << 32) |
                         __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(mi));
      const uint32_t gl = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(seg_idx[i]));
      fused_group<K, MAXE, POL, NM, NT, DIRECT, INLINE>(g0 + gl, m, lane, data, parity, rec_off, codebook, P, r, m0,
                                                        out, rm, nullptr);
    }
  } else if constexpr (SCAN == 0) {
    if (wv >= groups) return;
    const uint64_t m = DIRECT ? masks[wv] : 0;
    fused_group<K, MAXE, POL, NM, NT, DIRECT, INLINE>(wv, m, lane, data, parity, rec_off, codebook, P, r, m0, out, rm,
                                                      status);
  } else {
    // SCAN groups per wave: lanes 0..SCAN-1 read the masks with one vector load and write
    // the status bytes; the groups with lost, recoverable data shards (a ballot) are then
    // rebuilt one after another by the whole wave.  Sparse loss (C5: ~10% of groups) costs
    // one wave per SCAN groups instead of one per group.
    const uint64_t g0 = wv * SCAN;
    if (g0 >= groups) return;
    uint64_t mv = 0;
    bool need = false;
    if (lane < static_cast<uint32_t>(SCAN) && g0 + lane < groups) {
      mv = masks[g0 + lane];
      constexpr uint64_t kmask = (1ull << K) - 1;
      const uint32_t ne = static_cast<uint32_t>(__popcll(mv & kmask));
      const bool bad = ne > r - static_cast<uint32_t>(__popcll((mv >> K) & ((1ull << r) - 1)));
      if (status != nullptr) status[g0 + lane] = bad ? 1 : 0;
      need = ne > 0 && !bad;
    }
    uint64_t work = __ballot(need);
    while (work) {
      const uint32_t b = static_cast<uint32_t>(__builtin_ctzll(work));
      work &= work - 1;
      const uint64_t m = (static_cast<uint64_t>(__builtin_amdgcn_readlane(static_cast<uint32_t>(mv >> 32), b)) << 32) |
                         __builtin_amdgcn_readlane(static_cast<uint32_t>(mv), b);
      fused_group<K, MAXE, POL, NM, NT, DIRECT, INLINE>(g0 + b, m, lane, data, parity, rec_off, codebook, P, r, m0,
                                                        out, rm, nullptr);
    }
  }

}

// ---------------------------------------------------------------------------------
// Packed recover in one launch: recover_runs (fec_recover_batch_rs_dev_packed; DESIGN.md §5,
// round 4).  The reference decoder hands rebuilt packets back as separate buffers
// (decoder.go:16-22 `Recovered`, listed at :195-207); the packed list puts all of a batch's rebuilt packets back
// to back, group g's from row row_start[g] (exclusive prefix sum of the rows every group
// rebuilds: its lost data shards when recoverable, else 0).
//
// A workgroup owns a tile of consecutive groups (one erasure mask per thread), so all of
// their rebuilt rows form ONE contiguous run of the packed list:
//  1. every thread classifies its group (status byte; rows), the block scans the rows and
//     lists the groups to rebuild in LDS, in group order;
//  2. wave 0 finds the run's first row by decoupled look-back over the blocks before it
//     (blocks take their tile from an atomic ticket, so every block one waits on has
//     started and publishes its own row count before it waits on anything) and publishes
//     its inclusive prefix; row_start[g] is written for every group.  No prefix launches;
//  3. the 4 waves rebuild the listed groups (mask-addressed, exactly decode_fused's INLINE
//     arithmetic) into an LDS image of the run; rows past the image's capacity (dense loss)
//     are stored straight to HBM;
//  4. the block copies the image out with 16-B stores by consecutive threads, so the run
//     leaves as whole 128-B lines except at its two ends -- instead of every 1.2-KB row being
//     stored by its own wave with partial lines at both ends.
// Look-back words: epoch (bits 34..63) | flag (bits 32..33: kRunAgg, kRunIncl) | rows.  The
// epoch is the launch's, so words left by earlier launches never match (no reset launch).
// ---------------------------------------------------------------------------------
constexpr uint64_t kRunAgg = 1ull << 32;
constexpr uint64_t kRunIncl = 2ull << 32;
constexpr uint32_t kRunEpochShift = 34;

// One group's rebuild in two stages, so a wave can have the next group's survivor loads in flight
// while it computes and stores this one (kRunPipe): runs_load issues the survivor loads and finds
// the record, runs_compute forms the rows.  Same survivor choice, record and arithmetic as
// fused_group's DIRECT + INLINE path (survivors: the surviving data shards ascending, then the e
// lowest surviving parity rows; record from the colex ranks).
struct RunMeta {
  const Tab* tabs;
  uint32_t e;
  bool xor_only;
};

template <int K, int R, int NM, int NT, int POL>
__device__ __forceinline__ RunMeta runs_load(uint64_t g, uint64_t m, uint32_t lane, const uint8_t* __restrict__ data,
                                             const uint8_t* __restrict__ parity, const uint8_t* __restrict__ codebook,
                                             const RankMeta& rm, uint32_t P, const uint32_t (&toff)[NT > 0 ? NT : 1],
                                             uint32_t (&x)[K][4 * NM + NT]) {
  constexpr uint64_t kmask = (1ull << K) - 1;
  constexpr uint64_t rmask = (1ull << R) - 1;
  const uint64_t lost = m & kmask;
  const uint32_t e = static_cast<uint32_t>(__popcll(lost));
  const uint64_t pm = (m >> K) & rmask;
  uint64_t rank_e = 0, rank_r = 0, rsel = 0;
  {
    uint64_t dm = lost;
    for (uint32_t t = 0; dm; ++t) {
      rank_e += choose_small(static_cast<uint32_t>(__builtin_ctzll(dm)), t + 1u);
      dm &= dm - 1;
    }
    uint64_t sp = ~pm & rmask;
    for (uint32_t t = 0; t < e; ++t) {
      const uint32_t bit = static_cast<uint32_t>(__builtin_ctzll(sp));
      rank_r += choose_small(bit, t + 1u);
      rsel |= 1ull << bit;
      sp &= sp - 1;
    }
  }
  RunMeta mt;
  mt.e = e;
  mt.xor_only = e == 1 && (pm & 1u) == 0;
  mt.tabs = reinterpret_cast<const Tab*>(codebook + rm.base[e] + (rank_e * rm.count_r[e] + rank_r) * rm.stride[e] + 128);
  uint64_t surv = (~lost & kmask) | (rsel << K);
  const uint8_t* dg = data + g * K * static_cast<uint64_t>(P);
  const uint8_t* pg = parity + g * R * static_cast<uint64_t>(P);
#pragma unroll
  for (int s = 0; s < K; ++s) {
    const uint32_t sid = static_cast<uint32_t>(__builtin_ctzll(surv));
    surv &= surv - 1;
    const uint8_t* src = sid < K ? dg + sid * static_cast<uint64_t>(P) : pg + (sid - K) * static_cast<uint64_t>(P);
#pragma unroll
    for (int i = 0; i < NM; ++i) {
      const u32x4 t = ld16<POL>(src + i * 1024u + lane * 16u);
      x[s][4 * i] = t.x;
      x[s][4 * i + 1] = t.y;
      x[s][4 * i + 2] = t.z;
      x[s][4 * i + 3] = t.w;
    }
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      if constexpr ((POL & kNtLoad) != 0) x[s][4 * NM + t] = __builtin_nontemporal_load(reinterpret_cast<const u32u*>(src + toff[t]));
      else x[s][4 * NM + t] = *reinterpret_cast<const u32u*>(src + toff[t]);
    }
  }
  return mt;
}

template <int K, int R, int NM, int NT>
__device__ __forceinline__ void runs_compute(const RunMeta& mt, uint32_t (&x)[K][4 * NM + NT], uint32_t (&acc)[R][4 * NM + NT]) {
  constexpr int NW = 4 * NM + NT;
#pragma unroll
  for (int mm = 0; mm < R; ++mm)
#pragma unroll
    for (int q = 0; q < NW; ++q) acc[mm][q] = 0;
  if (mt.xor_only) {  // single data loss rebuilt from parity row 0: the reference XOR
#pragma unroll
    for (int s = 0; s < K; ++s)
#pragma unroll
      for (int q = 0; q < NW; ++q) acc[0][q] ^= x[s][q];
    return;
  }
#pragma unroll
  for (int s = 0; s < K; ++s) {
    // survivor s's selectors stay in its iteration (left alone, LLVM hoists every survivor's
    // selectors ahead of the arithmetic: 160 VGPRs, 3 waves per SIMD; see decode_fused kLdsTabs)
#pragma unroll
    for (int q = 0; q < NW; ++q) __asm__ volatile("" : "+v"(x[s][q]));
    uint32_t s0[NW], s1[NW], s2[NW];
#pragma unroll
    for (int q = 0; q < NW; ++q) {
      s0[q] = x[s][q] & 0x07070707u;
      s1[q] = (x[s][q] >> 3) & 0x07070707u;
      s2[q] = (x[s][q] >> 6) & 0x03030303u;
    }
#pragma unroll
    for (int mm = 0; mm < R; ++mm) {
      if (static_cast<uint32_t>(mm) < mt.e) {
        const Tab& t = mt.tabs[mm * K + s];
        if (t.coef == 1u) {
#pragma unroll
          for (int q = 0; q < NW; ++q) acc[mm][q] ^= x[s][q];
        } else if (t.coef != 0u) {
#pragma unroll
          for (int q = 0; q < NW; ++q) acc[mm][q] ^= gmul(s0[q], s1[q], s2[q], t);
        }
      }
    }
  }
}

// recover_runs: the wave's groups one after another (default), or with the next group's survivor
// loads issued before this group's arithmetic and stores (probe form).
constexpr int kRunPipe = 16384;
// recover_runs (probe form): the run image leaves by plain stores while rows past the image keep
// the POL's store policy.
constexpr int kRunImgPlain = 32768;

// stage_bytes: dynamic LDS of the run image (0: every row straight to HBM).  The image is used
// only when P % 16 == 0 and `out` is 16-B aligned (the launcher passes 0 otherwise), so row
// starts in the image and in HBM are 16-B aligned alike.
// base_in (nullable): rows before this launch (chunked launches: the previous chunk's total).
// POL: kNtLoad for the survivor loads, kNtStore for the row stores.  WAVES: waves per workgroup;
// TG: groups per workgroup (<= 64 * WAVES: the first TG threads classify one group each).
// flags bit 0 (probes only): no row stores at all.
template <int K, int R, int NM, int NT, int POL, int WAVES, int TG = 64 * WAVES>
__global__ __launch_bounds__(64 * WAVES) void recover_runs(const uint8_t* __restrict__ data,
                                                    const uint8_t* __restrict__ parity,
                                                    const uint64_t* __restrict__ masks, uint64_t groups,
                                                    uint32_t P, const uint8_t* __restrict__ codebook, RankMeta rm,
                                                    uint8_t* __restrict__ out, uint32_t* __restrict__ row_start,
                                                    uint8_t* __restrict__ status, uint64_t* __restrict__ lb,
                                                    uint32_t* __restrict__ ticket, uint32_t epoch,
                                                    uint32_t stage_bytes, const uint64_t* __restrict__ base_in,
                                                    uint64_t* __restrict__ total_out, uint64_t* __restrict__ total_user,
                                                    uint32_t flags) {
  static_assert(R <= 3, "mask-addressed shapes: r <= 3");
  static_assert(TG <= 64 * WAVES && (TG % 64 == 0 || TG < 64), "one classifying thread per group");
  constexpr uint32_t kTile = TG;
  constexpr uint32_t kScanWaves = TG >= 64 ? TG / 64 : 1;
  constexpr int NW = 4 * NM + NT;
  constexpr uint64_t kmask = (1ull << K) - 1;
  constexpr uint64_t rmask = (1ull << R) - 1;
  extern __shared__ __attribute__((aligned(16))) uint8_t run_image[];
  __shared__ uint64_t s_mask[kTile];
  __shared__ uint32_t s_item[kTile];  // (local group << 16) | first row in the run
  __shared__ uint32_t s_wrows[kScanWaves], s_wwork[kScanWaves];
  __shared__ uint32_t s_tile, s_first;
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  const uint32_t wave = static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(tid >> 6));
  if (tid == 0) {
    const uint32_t t = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // every ticket of this launch is taken: the counter starts from 0 for the next launch
    // (which the stream orders after this one)
    if (t == gridDim.x - 1u) __hip_atomic_store(ticket, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_tile = t;
  }
  __syncthreads();
  const uint32_t tile = s_tile;
  const uint64_t g = static_cast<uint64_t>(tile) * kTile + tid;
  uint64_t m = 0;
  uint32_t rows = 0;
  if (tid < kTile && g < groups) {
    m = masks[g];
    const uint32_t ne = static_cast<uint32_t>(__popcll(m & kmask));
    const bool bad = ne > R - static_cast<uint32_t>(__popcll((m >> K) & rmask));
    if (status != nullptr) status[g] = bad ? 1 : 0;
    rows = ne > 0 && !bad ? ne : 0u;
  }
  uint32_t incl = rows;
#pragma unroll
  for (uint32_t d = 1; d < 64; d <<= 1) {
    const uint32_t v = __shfl_up(incl, d, 64);
    if (lane >= d) incl += v;
  }
  const uint64_t need = __ballot(rows != 0u);
  if (wave < kScanWaves) {
    if (lane == 63u) s_wrows[wave] = incl;
    if (lane == 0u) s_wwork[wave] = static_cast<uint32_t>(__popcll(need));
  }
  __syncthreads();
  uint32_t wrow = 0, witem = 0, A = 0, nwork = 0;
#pragma unroll
  for (uint32_t w = 0; w < kScanWaves; ++w) {
    if (w < wave) {
      wrow += s_wrows[w];
      witem += s_wwork[w];
    }
    A += s_wrows[w];
    nwork += s_wwork[w];
  }
  const uint32_t lrow = wrow + incl - rows;  // the group's first row inside the run
  if (rows != 0u) {
    const uint32_t i = witem + static_cast<uint32_t>(__popcll(need & ((1ull << lane) - 1)));
    s_mask[i] = m;
    s_item[i] = (tid << 16) | lrow;
  }
  // The run's first row (wave 0): decoupled look-back over the tiles before this one.
  auto find_first = [&]() {
    const uint64_t tag = static_cast<uint64_t>(epoch) << kRunEpochShift;
    const uint32_t base = base_in != nullptr ? static_cast<uint32_t>(*base_in) : 0u;
    uint32_t excl = 0;
    if (tile == 0) {
      excl = base;  // published with its row count below
    } else {
      int64_t pos = static_cast<int64_t>(tile) - 1;
      for (;;) {
        const int64_t idx = pos - static_cast<int64_t>(lane);
        uint64_t s = tag | kRunIncl | base;  // "before tile 0": the rows before this launch
        if (idx >= 0) {
          for (;;) {
            s = __hip_atomic_load(&lb[idx], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if ((s >> kRunEpochShift) == epoch && (s & (kRunAgg | kRunIncl)) != 0) break;
            __builtin_amdgcn_s_sleep(1);
          }
        }
        const uint64_t inc = __ballot((s & kRunIncl) != 0);
        const uint32_t stop = inc ? static_cast<uint32_t>(__builtin_ctzll(inc)) : 64u;
        uint32_t v = lane <= stop ? static_cast<uint32_t>(s) : 0u;
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
        excl += v;
        if (inc) break;
        pos -= 64;
      }
      if (lane == 0) __hip_atomic_store(&lb[tile], tag | kRunIncl | (excl + A), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (lane == 0) {
      s_first = excl;
      if (tile == gridDim.x - 1u) {
        if (total_out != nullptr) *total_out = static_cast<uint64_t>(excl) + A;
        if (total_user != nullptr) *total_user = static_cast<uint64_t>(excl) + A;
      }
    }
  };
  // Publish this tile's row count at once (successors look back through it), then find the run's
  // first row: before the rebuild when some rows go straight to HBM (they need their place), after
  // it when every row fits the LDS image -- the look-back's wait then hides behind the rebuild.
  const uint32_t cap_rows = stage_bytes / P;
  const bool defer = (flags & 1u) == 0 && A <= cap_rows;
  // (tile 0 knows its first row already: the rows before this launch)
  if (wave == 0 && lane == 0) {
    const uint64_t tag = static_cast<uint64_t>(epoch) << kRunEpochShift;
    const uint64_t w = tile == 0 ? tag | kRunIncl | ((base_in != nullptr ? static_cast<uint32_t>(*base_in) : 0u) + A)
                                 : tag | kRunAgg | A;
    __hip_atomic_store(&lb[tile], w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (!defer && wave == 0) find_first();
  __syncthreads();
  uint32_t toff[NT > 0 ? NT : 1];
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    toff[t] = NM * 1024u + t * 256u + lane * 4u;
    if (toff[t] + 4u > P) toff[t] = P - 4u;
  }
  auto item_of = [&](uint32_t i, uint64_t& gi, uint64_t& mw, uint32_t& r0) {
    const uint64_t mi = s_mask[i];
    mw = (static_cast<uint64_t>(__builtin_amdgcn_readfirstlane(static_cast<uint32_t>(mi >> 32))) << 32) |
         __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(mi));
    const uint32_t item = __builtin_amdgcn_readfirstlane(s_item[i]);
    gi = static_cast<uint64_t>(tile) * kTile + (item >> 16);
    r0 = item & 0xFFFFu;
  };
  constexpr bool kPipe = (POL & kRunPipe) != 0;
  uint32_t xn[kPipe ? K : 1][kPipe ? NW : 1];  // kRunPipe: the next group's survivors, loads in flight
  RunMeta mn{};
  if constexpr (kPipe) {
    if (wave < nwork) {
      uint64_t gi, mw;
      uint32_t r0;
      item_of(wave, gi, mw, r0);
      mn = runs_load<K, R, NM, NT, POL>(gi, mw, lane, data, parity, codebook, rm, P, toff, xn);
    }
  }
  for (uint32_t i = wave; i < nwork; i += WAVES) {
    uint64_t gi, mw;
    uint32_t r0;
    item_of(i, gi, mw, r0);
    uint32_t acc[R][NW];
    uint32_t e;
    if constexpr (kPipe) {
      uint32_t x[K][NW];
#pragma unroll
      for (int s2 = 0; s2 < K; ++s2)
#pragma unroll
        for (int q = 0; q < NW; ++q) x[s2][q] = xn[s2][q];
      const RunMeta mt = mn;
      if (i + WAVES < nwork) {
        uint64_t gn, mwn;
        uint32_t rn;
        item_of(i + WAVES, gn, mwn, rn);
        mn = runs_load<K, R, NM, NT, POL>(gn, mwn, lane, data, parity, codebook, rm, P, toff, xn);
      }
      runs_compute<K, R, NM, NT>(mt, x, acc);
      e = mt.e;
    } else {
      uint32_t x[K][NW];
      const RunMeta mt = runs_load<K, R, NM, NT, POL>(gi, mw, lane, data, parity, codebook, rm, P, toff, x);
      runs_compute<K, R, NM, NT>(mt, x, acc);
      e = mt.xor_only ? 1u : mt.e;
    }
    if (flags & 1u) continue;  // probe: reads and arithmetic only
#pragma unroll
    for (int mm = 0; mm < R; ++mm) {
      if (static_cast<uint32_t>(mm) < e) {
        const uint32_t row = r0 + mm;
        if (row < cap_rows) {  // into the run image (16-B aligned rows: see stage_bytes)
          uint8_t* dst = run_image + row * P;
#pragma unroll
          for (int q = 0; q < NM; ++q)
            *reinterpret_cast<u32x4*>(dst + q * 1024u + lane * 16u) =
                u32x4{acc[mm][4 * q], acc[mm][4 * q + 1], acc[mm][4 * q + 2], acc[mm][4 * q + 3]};
#pragma unroll
          for (int t = 0; t < NT; ++t) *reinterpret_cast<uint32_t*>(dst + toff[t]) = acc[mm][4 * NM + t];
        } else {  // past the image (never when defer): straight to the row's place
          uint8_t* dst = out + (static_cast<uint64_t>(s_first) + row) * P;
#pragma unroll
          for (int q = 0; q < NM; ++q)
            st16<POL>(dst + q * 1024u + lane * 16u,
                      u32x4{acc[mm][4 * q], acc[mm][4 * q + 1], acc[mm][4 * q + 2], acc[mm][4 * q + 3]});
#pragma unroll
          for (int t = 0; t < NT; ++t) {
            if constexpr ((POL & kNtStore) != 0) __builtin_nontemporal_store(acc[mm][4 * NM + t], reinterpret_cast<u32u*>(dst + toff[t]));
            else *reinterpret_cast<u32u*>(dst + toff[t]) = acc[mm][4 * NM + t];
          }
        }
      }
    }
  }
  if (defer) {
    __syncthreads();  // (the image is complete, too)
    if (wave == 0) find_first();
  }
  __syncthreads();
  const uint32_t first = s_first;
  if (tid < kTile && g < groups) row_start[g] = first + lrow;
  const uint32_t staged = (flags & 1u) ? 0u : (A < cap_rows ? A : cap_rows);
  if (staged == 0u) return;
  // the image leaves in 16-B pieces by consecutive threads: whole lines but at the run's ends
  uint8_t* run = out + static_cast<uint64_t>(first) * P;
  const uint32_t n16 = staged * P / 16u;
  constexpr int kImgPol = (POL & kRunImgPlain) != 0 ? (POL & ~kNtStore) : POL;
  for (uint32_t c = tid; c < n16; c += 64u * WAVES)
    st16<kImgPol>(run + c * 16u, *reinterpret_cast<const u32x4*>(run_image + c * 16u));
}

// Packed recover rows: row_start[g] = exclusive prefix sum over groups of the number of rows a
// group rebuilds (its lost data shards when recoverable, else 0).  Block sums of kRowsPerBlock
// groups first; then every block of rows_write adds up the sums of the blocks before it itself
// (at most kRowsDirectBlocks of them: two launches in all), or, past that, a one-block scan of
// the sums runs in between.  rocprof at C5 (1M groups): the first form with 4096-group blocks
// took 23 us in three launches (rows_write 11.5, block sums 6.9, one-block scan 4.9).
constexpr uint32_t kRowsPerThread = 4;
// thread_rows loads the masks as one u64x4 and the scans add rows[0..3]
static_assert(kRowsPerThread == 4, "thread_rows and the rows_* kernels are written for 4 groups per thread");
constexpr uint32_t kRowsPerBlock = 256 * kRowsPerThread;
constexpr uint32_t kRowsDirectBlocks = 4096;

__device__ __forceinline__ uint32_t rebuilt_rows(uint64_t m, uint32_t k, uint32_t r) {
  const uint64_t kmask = k >= 64 ? ~0ull : (1ull << k) - 1;
  const uint32_t ne = static_cast<uint32_t>(__popcll(m & kmask));
  const uint32_t pl = static_cast<uint32_t>(__popcll((m >> k) & ((1ull << r) - 1)));
  return ne > 0 && ne + pl <= r ? ne : 0u;
}

// Inclusive scan of one value per thread over a 256-thread block (LDS, 8 steps).
__device__ __forceinline__ uint32_t block_inclusive_scan(uint32_t v, uint32_t* lds) {
  const uint32_t t = threadIdx.x;
  lds[t] = v;
  __syncthreads();
  for (uint32_t d = 1; d < 256; d <<= 1) {
    const uint32_t add = t >= d ? lds[t - d] : 0u;
    __syncthreads();
    lds[t] += add;
    __syncthreads();
  }
  return lds[t];
}

// Sum of one value per thread over a 256-thread block (wave reduction, then 4 partials).
__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t* lds) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if ((threadIdx.x & 63u) == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  const uint32_t total = lds[0] + lds[1] + lds[2] + lds[3];
  __syncthreads();
  return total;
}

// The rows of a thread's kRowsPerThread consecutive groups (one 32-B load of their masks when
// they are all in range).
__device__ __forceinline__ void thread_rows(const uint64_t* __restrict__ masks, uint64_t groups, uint64_t g0,
                                            uint32_t k, uint32_t r, uint32_t (&rows)[kRowsPerThread]) {
  if (g0 + kRowsPerThread <= groups) {
    typedef uint64_t u64x4 __attribute__((ext_vector_type(4), aligned(8)));  // masks may be 8-B aligned
    const u64x4 m = *reinterpret_cast<const u64x4*>(masks + g0);
    rows[0] = rebuilt_rows(m.x, k, r);
    rows[1] = rebuilt_rows(m.y, k, r);
    rows[2] = rebuilt_rows(m.z, k, r);
    rows[3] = rebuilt_rows(m.w, k, r);
  } else {
    for (uint32_t i = 0; i < kRowsPerThread; ++i) rows[i] = g0 + i < groups ? rebuilt_rows(masks[g0 + i], k, r) : 0u;
  }
}

__global__ __launch_bounds__(256) void rows_block_sums(const uint64_t* __restrict__ masks, uint64_t groups, uint32_t k,
                                                       uint32_t r, uint32_t* __restrict__ block_sums) {
  __shared__ uint32_t lds[4];
  const uint64_t g0 = static_cast<uint64_t>(blockIdx.x) * kRowsPerBlock + threadIdx.x * kRowsPerThread;
  uint32_t rows[kRowsPerThread];
  thread_rows(masks, groups, g0, k, r, rows);
  const uint32_t total = block_sum(rows[0] + rows[1] + rows[2] + rows[3], lds);
  if (threadIdx.x == 0) block_sums[blockIdx.x] = total;
}

// One block: block_sums[0, nb) -> exclusive prefix sums, in place; *total = the sum.
__global__ __launch_bounds__(256) void rows_scan_blocks(uint32_t* __restrict__ block_sums, uint32_t nb,
                                                        uint64_t* __restrict__ total) {
  __shared__ uint32_t lds[256];
  uint32_t carry = 0;
  for (uint32_t b0 = 0; b0 < nb; b0 += 256) {
    const uint32_t i = b0 + threadIdx.x;
    const uint32_t v = i < nb ? block_sums[i] : 0u;
    const uint32_t incl = block_inclusive_scan(v, lds);
    if (i < nb) block_sums[i] = carry + incl - v;
    carry += lds[255];
    __syncthreads();
  }
  if (threadIdx.x == 0 && total != nullptr) *total = carry;
}

// DIRECT: block_sums holds the blocks' own sums; each block adds up those before it (and the
// last block writes the total).  Else block_sums holds exclusive offsets (rows_scan_blocks).
template <bool DIRECT>
__global__ __launch_bounds__(256) void rows_write(const uint64_t* __restrict__ masks, uint64_t groups, uint32_t k,
                                                  uint32_t r, const uint32_t* __restrict__ block_sums,
                                                  uint32_t* __restrict__ row_start, uint64_t* __restrict__ total) {
  __shared__ uint32_t lds[256];
  uint32_t base;
  if constexpr (DIRECT) {
    uint32_t part = 0;
    for (uint32_t b = threadIdx.x; b < blockIdx.x; b += 256) part += block_sums[b];
    base = block_sum(part, lds);
  } else {
    base = block_sums[blockIdx.x];
  }
  const uint64_t g0 = static_cast<uint64_t>(blockIdx.x) * kRowsPerBlock + threadIdx.x * kRowsPerThread;
  uint32_t rows[kRowsPerThread];
  thread_rows(masks, groups, g0, k, r, rows);
  const uint32_t sum = rows[0] + rows[1] + rows[2] + rows[3];
  const uint32_t incl = block_inclusive_scan(sum, lds);
  uint32_t at = base + incl - sum;
  for (uint32_t i = 0; i < kRowsPerThread; ++i) {
    if (g0 + i < groups) row_start[g0 + i] = at;
    at += rows[i];
  }
  if constexpr (DIRECT) {
    if (total != nullptr && blockIdx.x == gridDim.x - 1 && threadIdx.x == 255) *total = base + incl;
  }
}

// One wave per group, so the record is wave-uniform (SGPRs).  A packet is covered by
// whole 1 KiB passes of 16 B per lane, then the remainder (< 1 KiB) by 256 B passes of
// 4 B per lane: at 1200 B that is 64 + 44 busy lanes instead of 64 + 11 lanes doing
// 16-B work, i.e. 5 instead of 8 dword slots of VALU per lane and survivor.  Tail pieces
// past the packet end are shifted back to [P - 4, P) (duplicates of a neighbour's bytes,
// same values), so any P >= 4 works and no lane branches on the packet end.
template <int K, int MAXE, int POL = 0>
__global__ __launch_bounds__(256) void decode_wave(uint8_t* __restrict__ data,
                                                   const uint8_t* __restrict__ parity,
                                                   const uint32_t* __restrict__ rec_off,
                                                   const uint8_t* __restrict__ codebook,
                                                   uint64_t groups, uint32_t P, uint32_t k_rt, uint32_t r,
                                                   uint32_t m0, uint8_t* __restrict__ out, uint32_t never,
                                                   uint32_t swz, uint32_t lds_slice) {
  // Dynamic LDS: an occupancy cap, or (kLdsTabs) 4 per-wave slices of `lds_slice` bytes
  // holding the wave's coefficient rows (see kLdsTabs and decode_fused).
  extern __shared__ __attribute__((aligned(16))) uint8_t occupancy_lds[];
  if (never) occupancy_lds[threadIdx.x] = 0;
  const uint64_t gw = static_cast<uint64_t>(decode_block(swz)) * 4u +
                      static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(threadIdx.x >> 6));
  if (gw >= groups) return;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t rec = __builtin_amdgcn_readfirstlane(rec_off[gw]);
  if (rec >= kRecBad) return;
  const uint32_t k = K > 0 ? static_cast<uint32_t>(K) : k_rt;
  const uint8_t* recp = codebook + static_cast<uint64_t>(rec) * 32u;
  const uint32_t* rw = reinterpret_cast<const uint32_t*>(recp);
  const uint32_t e = rw[24] & 0xFFu;
  const bool xor_only = ((rw[24] >> 8) & 0xFFu) != 0;
  if (m0 >= e) return;
  const Tab* tabs = reinterpret_cast<const Tab*>(recp + 128);
  if constexpr ((POL & kLdsTabs) != 0) {
    if (!xor_only) {
      // rows [m0, m0 + min(e - m0, MAXE)) of the record into this wave's slice, by
      // direct-to-LDS loads (LDS address = wave base + lane * 16); every pass over the
      // packet then reads them from LDS instead of re-reading them through the scalar cache
      const uint32_t pieces = (e - m0 < MAXE ? e - m0 : MAXE) * k * 2u;
      const uint8_t* src = reinterpret_cast<const uint8_t*>(tabs + m0 * k);
      uint8_t* slice = occupancy_lds + (threadIdx.x >> 6) * lds_slice;
      for (uint32_t i = 0; i * 64u < pieces; ++i) {
        uint32_t idx = lane + 64u * i;
        if (idx >= pieces) idx = pieces - 1u;  // slots past the rows: unused, inside the slice
        __builtin_amdgcn_global_load_lds(reinterpret_cast<const void*>(src + idx * 16u),
                                         (__attribute__((address_space(3))) void*)(slice + i * 1024u), 16, 0, 0);
      }
      __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      // decode_piece indexes rows from m0
      tabs = reinterpret_cast<const Tab*>(slice) - static_cast<ptrdiff_t>(m0) * k;
    }
  }
  const uint8_t* dg = data + gw * k * static_cast<uint64_t>(P);
  const uint8_t* pg = parity + gw * r * static_cast<uint64_t>(P);
  uint8_t* og = out + gw * ((POL & kCompactOut) != 0 ? r : k) * static_cast<uint64_t>(P);
  const uint32_t main_end = P & ~1023u;
  for (uint32_t base = 0; base < main_end; base += 1024u)
    decode_piece<K, MAXE, POL, 4>(rw, tabs, dg, pg, og, k, P, base + lane * 16u, e, m0, xor_only);
  for (uint32_t base = main_end; base < P; base += 256u) {
    const uint32_t off = base + lane * 4u;
    decode_piece<K, MAXE, POL, 1>(rw, tabs, dg, pg, og, k, P, off + 4u <= P ? off : P - 4u, e, m0, xor_only);
  }
}

// One wave per group.  K > 0: compile-time k (survivor loads all issued first).
// MAXE: rows rebuilt per pass (rows [m0, m0 + MAXE) of the record's e).
template <int K, int MAXE, int POL = 0>
__global__ __launch_bounds__(256) void decode_v16(uint8_t* __restrict__ data,
                                                  const uint8_t* __restrict__ parity,
                                                  const uint32_t* __restrict__ rec_off,
                                                  const uint8_t* __restrict__ codebook,
                                                  uint64_t groups, uint32_t cpp, uint32_t P,
                                                  uint32_t k_rt, uint32_t r, uint32_t m0) {
  const uint64_t gw = static_cast<uint64_t>(blockIdx.x) * 4u +
                      static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(threadIdx.x >> 6));
  if (gw >= groups) return;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t rec = __builtin_amdgcn_readfirstlane(rec_off[gw]);
  if (rec >= kRecBad) return;
  const uint32_t k = K > 0 ? static_cast<uint32_t>(K) : k_rt;
  const uint8_t* recp = codebook + static_cast<uint64_t>(rec) * 32u;
  const uint32_t* rw = reinterpret_cast<const uint32_t*>(recp);
  const uint32_t e = rw[24] & 0xFFu;
  const bool xor_only = ((rw[24] >> 8) & 0xFFu) != 0;
  if (m0 >= e) return;
  const Tab* tabs = reinterpret_cast<const Tab*>(recp + 128);
  uint8_t* dg = data + gw * k * static_cast<uint64_t>(P);
  const uint8_t* pg = parity + gw * r * static_cast<uint64_t>(P);

  for (uint32_t col = lane; col < cpp; col += 64u) {
    const size_t coff = col_off16(col, P);
    if (xor_only) {  // single data loss rebuilt from parity row 0: the reference XOR
      u32x4 acc = {0u, 0u, 0u, 0u};
      for (uint32_t s = 0; s < k; ++s) {
        const uint32_t sid = rec_byte(rw, s);
        const uint8_t* src = sid < k ? dg + sid * static_cast<uint64_t>(P) : pg + (sid - k) * static_cast<uint64_t>(P);
        acc ^= ld16<POL>(src + coff);
      }
      st16<POL>(dg + rec_byte(rw, 64) * static_cast<uint64_t>(P) + coff, acc);
      continue;
    }
    u32x4 acc[MAXE];
#pragma unroll
    for (int m = 0; m < MAXE; ++m) acc[m] = u32x4{0u, 0u, 0u, 0u};
    if constexpr (K > 0) {
      u32x4 x[K];
#pragma unroll
      for (int s = 0; s < K; ++s) {
        const uint32_t sid = rec_byte(rw, s);
        const uint8_t* src = sid < k ? dg + sid * static_cast<uint64_t>(P) : pg + (sid - k) * static_cast<uint64_t>(P);
        x[s] = ld16<POL>(src + coff);
      }
#pragma unroll
      for (int s = 0; s < K; ++s) {
        Sel sl;
        prep(x[s], sl);
#pragma unroll
        for (int m = 0; m < MAXE; ++m) {
          if (m0 + m < e) {
            const Tab& t = tabs[(m0 + m) * K + s];
            if (t.coef == 1u) xor_into(acc[m], x[s]);
            else if (t.coef != 0u) mac(acc[m], sl, t);
          }
        }
      }
    } else {
#pragma unroll 2
      for (uint32_t s = 0; s < k; ++s) {
        const uint32_t sid = rec_byte(rw, s);
        const uint8_t* src = sid < k ? dg + sid * static_cast<uint64_t>(P) : pg + (sid - k) * static_cast<uint64_t>(P);
        const u32x4 xv = ld16<POL>(src + coff);
        Sel sl;
        prep(xv, sl);
#pragma unroll
        for (int m = 0; m < MAXE; ++m) {
          if (m0 + m < e) {
            const Tab& t = tabs[(m0 + m) * k + s];
            if (t.coef == 1u) xor_into(acc[m], xv);
            else if (t.coef != 0u) mac(acc[m], sl, t);
          }
        }
      }
    }
#pragma unroll
    for (int m = 0; m < MAXE; ++m) {
      if (m0 + m < e) {
        const uint32_t eid = rec_byte(rw, 64 + m0 + m);
        st16<POL>(dg + eid * static_cast<uint64_t>(P) + coff, acc[m]);
      }
    }
  }
}

// Tiled decode: a workgroup owns `tile` whole groups and one lane owns one 16-byte column
// of one group (all lanes busy, like encode_v16's tiled form).  A wave may then hold two
// groups with different erasure patterns, so each lane reads its own record (header and
// tables through the vector cache; lanes of one group read the same lines) and runs the
// multiply for every coefficient, 0 and 1 included (their tables are the zero / identity
// maps): no lane-divergent branches except the row count e.  The library's form for
// packets of <= 256 B, where one group per wave would leave most lanes idle (k=10 r=3,
// 2 erasures: 64 B 3.4 vs 0.72 TB/s, 256 B 4.6 vs 3.7; profiles/r01_probe_decode_small.txt).
template <int K, int MAXE, int POL = 0>
__global__ __launch_bounds__(512) void decode_tiled(const uint8_t* __restrict__ data,
                                                    const uint8_t* __restrict__ parity,
                                                    const uint32_t* __restrict__ rec_off,
                                                    const uint8_t* __restrict__ codebook,
                                                    uint64_t groups, uint32_t cpp, uint32_t P,
                                                    uint32_t r, uint32_t tile, uint8_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x;
  uint32_t gl = lane / cpp;
  const uint32_t col = lane - gl * cpp;
  if (gl >= tile) return;
  gl += blockIdx.x * tile;
  if (gl >= groups) return;
  const uint64_t g = gl;
  const uint32_t rec = rec_off[g];
  if (rec >= kRecBad) return;
  const uint8_t* recp = codebook + static_cast<uint64_t>(rec) * 32u;
  const uint32_t* rw = reinterpret_cast<const uint32_t*>(recp);
  const uint32_t e = rw[24] & 0xFFu;
  const Tab* tabs = reinterpret_cast<const Tab*>(recp + 128);
  const uint8_t* dg = data + g * K * static_cast<uint64_t>(P);
  const uint8_t* pg = parity + g * r * static_cast<uint64_t>(P);
  // in place: the erased shard's slot; kCompactOut: row m of the group's run (g*r + m)*P
  uint8_t* og = out + g * ((POL & kCompactOut) != 0 ? r : K) * static_cast<uint64_t>(P);
  const size_t coff = col_off16(col, P);
  uint32_t sw[(K + 3) / 4];
#pragma unroll
  for (int q = 0; q < (K + 3) / 4; ++q) sw[q] = rw[q];
  u32x4 x[K];
#pragma unroll
  for (int s = 0; s < K; ++s) {
    const uint32_t sid = (sw[s >> 2] >> (8 * (s & 3))) & 0xFFu;
    const uint8_t* src = sid < K ? dg + sid * static_cast<uint64_t>(P) : pg + (sid - K) * static_cast<uint64_t>(P);
    x[s] = ld16<POL>(src + coff);
  }
  u32x4 acc[MAXE];
#pragma unroll
  for (int m = 0; m < MAXE; ++m) acc[m] = u32x4{0u, 0u, 0u, 0u};
#pragma unroll
  for (int s = 0; s < K; ++s) {
    Sel sl;
    prep(x[s], sl);
#pragma unroll
    for (int m = 0; m < MAXE; ++m) {
      if (static_cast<uint32_t>(m) < e) mac(acc[m], sl, tabs[m * K + s]);
    }
  }
  const uint32_t ew = rw[16];  // erased ids E_0..E_3 (bytes 64..67)
#pragma unroll
  for (int m = 0; m < MAXE; ++m) {
    if (static_cast<uint32_t>(m) < e) {
      const uint32_t eid = (POL & kCompactOut) != 0 ? static_cast<uint32_t>(m)
                           : m < 4                     ? (ew >> (8 * m)) & 0xFFu
                                                       : rec_byte(rw, 64 + m);
      st16<POL>(og + eid * static_cast<uint64_t>(P) + coff, acc[m]);
    }
  }
}

// Decode, one lane per byte (packets shorter than 16 B).
__global__ __launch_bounds__(256) void decode_bytes(const uint8_t* __restrict__ data,
                                                    const uint8_t* __restrict__ parity,
                                                    const uint32_t* __restrict__ rec_off,
                                                    const uint8_t* __restrict__ codebook,
                                                    uint64_t g_first, uint32_t nthreads, uint32_t P,
                                                    uint32_t k, uint32_t r, uint8_t* __restrict__ out,
                                                    uint32_t compact) {
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
  if (t >= nthreads) return;
  const uint32_t gl = t / P;
  const uint32_t b = t - gl * P;
  const uint64_t g = g_first + gl;
  const uint32_t rec = rec_off[g];
  if (rec >= kRecBad) return;
  const uint8_t* recp = codebook + static_cast<uint64_t>(rec) * 32u;
  const uint32_t e = recp[96];
  const Tab* tabs = reinterpret_cast<const Tab*>(recp + 128);
  const uint8_t* dg = data + g * k * static_cast<uint64_t>(P);
  const uint8_t* pg = parity + g * r * static_cast<uint64_t>(P);
  for (uint32_t m = 0; m < e; ++m) {
    uint32_t acc = 0;
    for (uint32_t s = 0; s < k; ++s) {
      const uint32_t sid = recp[s];
      const uint32_t x = sid < k ? dg[sid * static_cast<uint64_t>(P) + b] : pg[(sid - k) * static_cast<uint64_t>(P) + b];
      acc ^= gmul_byte(x, tabs[m * k + s]);
    }
    // Erased shards are never survivors, so writing here cannot feed a later read.
    const uint64_t slot = compact ? g * r + m : g * k + recp[64 + m];
    out[slot * static_cast<uint64_t>(P) + b] = static_cast<uint8_t>(acc);
  }
}

// ---------------------------------------------------------------------------------
// Synthetic data: counter-based splitmix64 (oracle_fill_splitmix restates it on the CPU).
// ---------------------------------------------------------------------------------
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void fill_words(uint8_t* __restrict__ dst, uint32_t n16,
                                                  uint64_t seed, uint64_t word0) {
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
  if (t >= n16) return;
  const uint64_t w = word0 + 2ull * t;
  const uint64_t a = mix64(seed + (w + 1) * 0x9E3779B97F4A7C15ull);
  const uint64_t b = mix64(seed + (w + 2) * 0x9E3779B97F4A7C15ull);
  reinterpret_cast<uint4*>(dst)[t] =
      make_uint4(static_cast<uint32_t>(a), static_cast<uint32_t>(a >> 32), static_cast<uint32_t>(b),
                 static_cast<uint32_t>(b >> 32));
}

__global__ __launch_bounds__(256) void fill_bytes(uint8_t* __restrict__ dst, uint32_t n, uint64_t seed,
                                                  uint64_t pos0) {
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
  if (t >= n) return;
  const uint64_t pos = pos0 + t;
  const uint64_t w = mix64(seed + (pos / 8 + 1) * 0x9E3779B97F4A7C15ull);
  dst[t] = static_cast<uint8_t>(w >> (8 * (pos % 8)));
}

// Box calibration: a plain 16-B-per-lane copy, the same access pattern as the encode's loads
// and stores without the arithmetic; bench.py reports the kernels against its rate.
__global__ __launch_bounds__(256) void copy_words(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                  uint32_t n16) {
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
  if (t < n16) dst[t] = src[t];
}

// Resident legacy encoder (fec_kernels.hpp ServerSlot): workgroups of 16 waves, one per serving
// class (below).  One poll
// is one round trip over PCIe: 128 lanes read the first two 64-B lines of each of the next 16
// slots (the header words and the first group's 10 packet addresses, 16 B a lane: 32 line reads
// in all -- reading every word of 64 slots separately took 5 us a poll, 2x a round trip); a
// slot is complete when every one of those words carries its lap tag, and the run of complete
// slots from the next expected seq is served (slots in order).  Then every thread takes work
// items (one 16-B column of one group: its 10 packets loaded, XORed -- the reference's row 0,
// fec_xor_simd.cpp:411-427 -- and stored to the repair row), the workgroup fences its stores
// at system scope and the slots' done words are stored (release).  Every wave leaves together:
// at the host's stop flag, after idle_ticks without work, after life_ticks, and in any case
// after kServerMaxPolls polls.
constexpr uint32_t kServerThreads = 1024;
constexpr uint32_t kServerMaxPolls = 1u << 22;
constexpr uint32_t kServerHeadWords = 16;  // words of a slot read by the poll: out, shape, addr[0..13]

__device__ __forceinline__ void sys_store_release(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// System-coherent (uncached) access for the words the host polls: program order with the
// system-coherent stores before them, and vmcnt(0) in between, is the ordering.
__device__ __forceinline__ void sys_store_relaxed(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// 16 bytes to host memory at any address, written system-coherent (sc0 sc1: write-through, no
// cache keeps a copy), so legacy_server's vmcnt(0) after its repair-row stores means the rows
// are in host memory before it stores the done words (no release fence;
// profiles/r03_resident_store_ab.txt).  That is the gfx94x / gfx95x ISA's meaning of sc0 sc1,
// not the HIP memory model's guarantee: a build for another target stops here.
#if defined(__HIP_DEVICE_COMPILE__) && !defined(__gfx950__) && !defined(__gfx942__)
#error "legacy_server assumes gfx94x/gfx95x sc0 sc1 stores are write-through (sys_store_16b)"
#endif
// Written as the instruction itself: a volatile store compiles to the same instruction but is
// followed by s_waitcnt vmcnt(0), one PCIe acknowledgement per store before the thread goes on
// (the VRAM ring's stamps: 1.7 us a batch spent there).  The server's own vmcnt(0) before its
// done words is the one wait the rows need; the "memory" clobber keeps the compiler's memory
// operations on their side of it, and an extra outstanding store only makes the compiler's own
// vmcnt waits (in-order completion on gfx9) stricter.
__device__ __forceinline__ void sys_store_16b(uint8_t* p, u32x4 v) {
  __asm__ volatile("global_store_dwordx4 %0, %1, off sc0 sc1" : : "v"(p), "v"(v) : "memory");
}

typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

// The server's workgroup barrier: every value it publishes between its waves is in LDS, so the
// fences are LDS-only (s_waitcnt lgkmcnt(0) + s_barrier).  __syncthreads' workgroup fence also
// waits vmcnt(0) -- the PCIe acknowledgement of every repair-row store, which an inline batch
// does not need (its rows carry lap words) and an addressed batch waits for explicitly.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// 16 bytes of host memory as they are now (system-coherent load, no cache).
__device__ __forceinline__ u64x2 sys_load_16(const uint64_t* p) {
  return *reinterpret_cast<const volatile __attribute__((address_space(1))) u64x2*>(reinterpret_cast<uintptr_t>(p));
}

// The VRAM ring (inl != nullptr, fec_kernels.hpp kServerInline): the poll reads the slots from
// device memory -- local, not a PCIe round trip -- and an inline slot's work item is one 16-B
// chunk column (g, c): its 10 chunks loaded from the slot's data area (or, at the head of the
// run, from the poll's prefetch), the tags of both 8-B halves of each checked, the 12 payload
// bytes XORed and stored with the tag in both halves as chunk (g, c) of the slot's output
// staging.  A half whose tag is not yet this slot's (the host's stores through the BAR landed
// in another order, or a 16-B store arrived as two pieces) marks the slot bad: the run is served
// up to the first bad slot and the poll comes back for the rest.  The host takes an inline
// slot's rows by their tags, so its done word needs no acknowledgement of the row stores: a
// batch of inline slots only waits for them when it also holds an addressed slot (or scrubs a
// slot at an epoch boundary, fec_kernels.hpp server_tag).
//
// Serving classes (fec_kernels.hpp kServerMaxClasses): workgroup c of `classes` serves the seqs
// of class c (seq % classes == c) and steps through them `classes` apart; its poll, run, done
// words and progress mark are its class's alone.  The workgroups share only the ServerCoord
// words (uncached device memory, read with the poll): an idle flag each, and the leave word any
// of them sets when it leaves on its own (the stop word, the life bound, its poll bound) or finds
// every class idle -- so an instance leaves as a whole, and the last workgroup out stores the
// exited word the host relaunches on.
__global__ __launch_bounds__(kServerThreads) void legacy_server(ServerSlot* __restrict__ ring,
                                                                uint8_t* __restrict__ inl,
                                                                uint64_t* __restrict__ done,
                                                                ServerControl* __restrict__ ctl,
                                                                ServerCoord* __restrict__ coord, uint32_t classes,
                                                                uint64_t gen, uint64_t idle_ticks, uint64_t slow_ticks,
                                                                uint64_t life_ticks, uint64_t* __restrict__ stamps,
                                                                uint32_t epoch) {
  __shared__ uint64_t s_next;
  __shared__ uint32_t s_n, s_exit, s_stop, s_ack, s_told, s_slow;
  __shared__ uint64_t s_idle[kServerMaxClasses];
  __shared__ uint32_t s_first[kServerPoll + 1];  // work items before slot i of the run
  __shared__ uint32_t s_P[kServerPoll], s_cpp[kServerPoll], s_inl[kServerPoll], s_bad[kServerPoll];
  __shared__ uint64_t s_head[kServerPoll][kServerHeadWords];  // out, shape, addr[0..13] (tagged)
  const uint32_t K = classes, cls = blockIdx.x;
  // the shared words are read by every 8th poll (an instance leaves within 8 polls of the word)
  constexpr uint32_t kCoordEvery = 7u;
  if (cls != 0) stamps = nullptr;  // class 0's stamps only
  // VRAM ring: every poll also reads the first 16 KB of the next slot's inline data area, one
  // 16-B chunk a thread, in flight with the header loads -- an inline slot found complete at
  // the head of the run then takes its chunks from here instead of a second dependent round
  // trip to memory (1 group of P <= 1224: 10 * ceil(P / 12) chunks <= 1024).  Read before the
  // slot is known complete: the chunks' lap words decide, as for any chunk.
  __shared__ u32x4 s_pre[kServerThreads];
  const uint32_t tid = threadIdx.x, lane = tid & 63u;
  uint64_t t0 = 0, t_last = 0;  // thread 0 only
  uint64_t n_bad = 0, n_scrub = 0;  // thread 0 only: the diagnostic counters, continued from the last instance's
  bool was_idle = false;            // thread 0 only: this class's idle flag as last published
  if (tid == 0) {
    // the class's first unserved seq: its progress mark (the first instance's marks are 0, so
    // rounded up into the class)
    const uint64_t p = *reinterpret_cast<const volatile uint64_t*>(&ctl->progress[cls]);
    s_next = p + (cls + K - static_cast<uint32_t>(p % K)) % K;
    t0 = t_last = static_cast<uint64_t>(wall_clock64());
    s_told = 0;
    for (uint32_t c = 0; c < kServerMaxClasses; ++c) s_idle[c] = 0;
    n_bad = *reinterpret_cast<const volatile uint64_t*>(&ctl->bad_slots[cls]);
    n_scrub = *reinterpret_cast<const volatile uint64_t*>(&ctl->scrubs[cls]);
  }
  lds_barrier();
  // Diagnostic stamps (stamps != nullptr; the test library's TestKnob::kResidentStamps): thread 0's wall clock at the
  // phases of each served batch, into a ring of 256 records of 8 words in host memory that no
  // other code reads; never part of a result.
  uint64_t st_batches = 0, st_polls = 0, st_t[7] = {};
  for (uint32_t it = 0; it < kServerMaxPolls; ++it) {
    const uint64_t next = s_next;
    if (stamps != nullptr && tid == 0) st_t[0] = static_cast<uint64_t>(wall_clock64());
    // the poll: the first two lines of each of the next kServerPoll slots, 16 B a lane, and the
    // host's stop word, all in one round trip
    u32x4 pre = {0u, 0u, 0u, 0u};
    if (inl != nullptr)
      pre = __builtin_nontemporal_load(reinterpret_cast<const __attribute__((address_space(1))) u32x4*>(
          reinterpret_cast<uintptr_t>(inl + static_cast<uint64_t>(next % kServerSlots) * kInlineSlotBytes) + tid * 16u));
    constexpr uint32_t kPollLanes = kServerPoll * kServerHeadWords / 2;
    if (tid < kPollLanes) {
      const uint32_t i = tid / (kServerHeadWords / 2), piece = tid % (kServerHeadWords / 2);
      const u64x2 v = sys_load_16(reinterpret_cast<const uint64_t*>(ring + (next + uint64_t(i) * K) % kServerSlots) + 2 * piece);
      s_head[i][2 * piece] = v.x;
      s_head[i][2 * piece + 1] = v.y;
    } else if (tid == kPollLanes) {
      // with the ring in VRAM the stop word (host memory) would make every poll a PCIe round
      // trip again: every 16th poll reads it (the idle and life bounds hold regardless)
      s_stop = (inl == nullptr || (it & 15u) == 0) ? (*reinterpret_cast<const volatile uint64_t*>(&ctl->stop) != 0 ? 1u : 0u)
                                                   : 0u;
    } else if (coord != nullptr && (it & kCoordEvery) == 0 && tid == kPollLanes + 1) {
      s_told = sys_load_16(&coord->leave).x == gen ? 1u : 0u;
    } else if (coord != nullptr && (it & kCoordEvery) == 0 && tid >= kPollLanes + 2 &&
               tid < kPollLanes + 2 + kServerMaxClasses / 2) {
      const uint32_t q = tid - (kPollLanes + 2);
      const u64x2 v = sys_load_16(&coord->idle[2 * q]);
      s_idle[2 * q] = v.x;
      s_idle[2 * q + 1] = v.y;
    }
    s_pre[tid] = pre;
    lds_barrier();
    if (tid < 64) {
      const uint64_t seq = next + uint64_t(lane) * K;
      const uint64_t tag = server_tag(seq, epoch);
      bool ok = lane < kServerPoll;
      bool inline_slot = false;
      if (ok) {
        // out, shape and (unless the packets are inline) the first group's 10 addresses (words 0 .. 11)
        inline_slot = inl != nullptr && (s_head[lane][1] & kServerInline) != 0;
        const uint32_t nw = inline_slot ? 2u : 2u + kServerPackets;
#pragma unroll
        for (uint32_t w = 0; w < 2 + kServerPackets; ++w) ok = ok && (w >= nw || (s_head[lane][w] >> kServerTagShift) == tag);
        s_bad[lane] = 0;
      }
      const uint64_t bal = __ballot(ok);
      const uint32_t n = ~bal == 0 ? 64u : static_cast<uint32_t>(__builtin_ctzll(~bal));
      const uint64_t addressed = __ballot(lane < n && !inline_slot);  // rows straight to the caller
      uint32_t work = 0;
      if (lane < n) {
        const uint64_t sh = s_head[lane][1];
        const uint32_t P = static_cast<uint32_t>(sh & 0xFFFFu), G = static_cast<uint32_t>((sh >> 16) & 0xFFu);
        const uint32_t cpp = inline_slot ? (P + kInlinePayload - 1u) / kInlinePayload : (P + 15u) / 16u;
        s_P[lane] = P;
        s_cpp[lane] = cpp;
        s_inl[lane] = inline_slot ? 1u : 0u;
        // (an inline shape past the data area is never written by the host: nothing is read for it)
        work = inline_slot && (G > kInlineMaxGroups || P > kInlineMaxP) ? 0u : G * cpp;
      }
      uint32_t incl = work;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const uint32_t y = __shfl_up(incl, d, 64);
        if (lane >= static_cast<uint32_t>(d)) incl += y;
      }
      if (lane < kServerPoll) s_first[lane + 1] = incl;
      if (lane == 0) {
        s_first[0] = 0;
        const uint64_t now = static_cast<uint64_t>(wall_clock64());
        if (n > 0) t_last = now;
        const bool stop = s_stop != 0;
        s_n = n;
        s_ack = addressed != 0 ? 1u : 0u;
        const bool idle = n == 0 && now - t_last > idle_ticks;
        // (class 0, where the host puts a lone caller's calls, never polls slowly)
        s_slow = cls != 0 && n == 0 && now - t_last > slow_ticks ? 1u : 0u;
        bool leave = stop || now - t0 > life_ticks || it + 1 == kServerMaxPolls;
        if (coord == nullptr) {
          leave = leave || idle;
        } else {
          // every class idle (this one now, the others by their published flags), or told to leave
          const bool all_idle = server_all_idle(idle, s_idle, K, cls, gen);
          if (idle != was_idle) {
            sys_store_relaxed(&coord->idle[cls], idle ? gen : 0);
            was_idle = idle;
          }
          if ((leave || all_idle) && s_told == 0) sys_store_relaxed(&coord->leave, gen);
          leave = leave || all_idle || s_told != 0;
        }
        s_exit = leave ? 1u : 0u;
      }
    }
    lds_barrier();
    const uint32_t n = s_n;
    const bool leave = s_exit != 0;
    if (stamps != nullptr && tid == 0) {
      st_t[1] = static_cast<uint64_t>(wall_clock64());
      ++st_polls;
    }
    if (n > 0) {
      // the packets (and any later groups' addresses) as the host wrote them before the words above
      // The caller's packets as the host wrote them before its slot (the L2 may hold an older
      // copy of the same lines from an earlier call).  Cached loads after this acquire: reading
      // the packets system-coherent instead (sc0 sc1, no fence) made every 16-B load its own
      // PCIe read and the work step 2.8x slower (12.6 vs 4.5 us a batch).
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      if (stamps != nullptr && tid == 0) st_t[2] = st_t[6] = static_cast<uint64_t>(wall_clock64());  // (a bad slot: no item)
      const uint32_t total = s_first[n];
      for (uint32_t w = tid; w < total; w += kServerThreads) {
        uint32_t i = 0;
        while (s_first[i + 1] <= w) ++i;
        const uint32_t local = w - s_first[i];
        const uint32_t cpp = s_cpp[i], P = s_P[i];
        const uint32_t g = local / cpp, col = local - g * cpp;
        const uint64_t seq = next + uint64_t(i) * K;
        if (s_inl[i] != 0) {
          const uint32_t c0 = g * kServerPackets * cpp + col;  // chunk (g, 0, col)
          u32x4 v[kServerPackets];
          if (i == 0 && (g + 1) * kServerPackets * cpp <= kServerThreads) {
            // the head of the run: the poll brought its chunks
#pragma unroll
            for (uint32_t j = 0; j < kServerPackets; ++j) v[j] = s_pre[c0 + j * cpp];
          } else {
            const uint8_t* src = inl + static_cast<uint64_t>(seq % kServerSlots) * kInlineSlotBytes + c0 * 16u;
#pragma unroll
            for (uint32_t j = 0; j < kServerPackets; ++j)
              v[j] = *reinterpret_cast<const __attribute__((address_space(1))) u32x4*>(
                  reinterpret_cast<uintptr_t>(src + static_cast<uint64_t>(j) * cpp * 16u));
#pragma unroll
            for (uint32_t j = 0; j < kServerPackets; ++j) __asm__ volatile("" : "+v"(v[j]));
          }
          // both 8-B halves of every chunk carry this lap's tag in their top two bytes
          const uint32_t tag = server_tag(seq, epoch);
          bool fresh = true;
          u32x4 acc = v[0];
#pragma unroll
          for (uint32_t j = 0; j < kServerPackets; ++j) fresh = fresh && (v[j].y >> 16) == tag && (v[j].w >> 16) == tag;
#pragma unroll
          for (uint32_t j = 1; j < kServerPackets; ++j) acc ^= v[j];
          if (!fresh) {
            s_bad[i] = 1u;
            continue;
          }
          if (stamps != nullptr && tid == 0 && w == 0) st_t[6] = static_cast<uint64_t>(wall_clock64());
          // tagged rows, whole 16-B pieces side by side: a wave's stores cover whole lines (three
          // 32-bit stores per 12 bytes, each writing every third word of a line, took 31 us a
          // call instead of 6.9: every batch was found only by the poll that also read the stop
          // word from host memory -- the partial-line writes and the done word behind them left
          // the device only when a read to the host pushed them; profiles/r04_vram_store_forms.txt)
          sys_store_16b(reinterpret_cast<uint8_t*>(s_head[i][0] & kServerAddrMask) + (static_cast<uint64_t>(g) * cpp + col) * 16u,
                        u32x4{acc.x, (acc.y & 0xFFFFu) | (tag << 16), acc.z, (acc.w & 0xFFFFu) | (tag << 16)});
          continue;
        }
        const uint32_t coff = col * 16u + 16u <= P ? col * 16u : P - 16u;
        uint64_t ad[kServerPackets];
        if (g == 0) {
#pragma unroll
          for (uint32_t j = 0; j < kServerPackets; ++j) ad[j] = s_head[i][2 + j];
        } else {
          // written by the host before the slot's first group and header, seen complete above;
          // relaxed system-scope loads (uncached, all ten in flight: volatile loads were each
          // followed by a full wait, one PCIe round trip apiece)
          const uint64_t* src = ring[seq % kServerSlots].addr + g * kServerPackets;
#pragma unroll
          for (uint32_t j = 0; j < kServerPackets; ++j)
            ad[j] = __hip_atomic_load(reinterpret_cast<const __attribute__((address_space(1))) uint64_t*>(
                                          reinterpret_cast<uintptr_t>(src + j)),
                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          // tagged like the header: in a VRAM ring the host's stores through the BAR carry no
          // order, and a word of the previous lap marks the slot bad (served by a later poll)
          const uint64_t tag = server_tag(seq, epoch);
          bool fresh = true;
#pragma unroll
          for (uint32_t j = 0; j < kServerPackets; ++j) fresh = fresh && (ad[j] >> kServerTagShift) == tag;
          if (!fresh) {
            s_bad[i] = 1u;
            continue;
          }
        }
        // All ten packet loads in flight at once, as global (address space 1) loads: the addresses
        // come from integers, so plain pointers compile to flat loads, which count on lgkmcnt too
        // and were issued two at a time with a full wait between pairs -- five dependent PCIe
        // round trips, ~8 us of a ~12-us call (the server's stamps, DESIGN_HISTORY.md §8c round 4).
        u32x4 v[kServerPackets];
#pragma unroll
        for (uint32_t j = 0; j < kServerPackets; ++j)
          v[j] = *reinterpret_cast<const __attribute__((address_space(1))) u32x4u*>((ad[j] & kServerAddrMask) + coff);
#pragma unroll
        for (uint32_t j = 0; j < kServerPackets; ++j) __asm__ volatile("" : "+v"(v[j]));  // no load sunk into the XOR
        u32x4 acc = v[0];
#pragma unroll
        for (uint32_t j = 1; j < kServerPackets; ++j) acc ^= v[j];
        if (stamps != nullptr && tid == 0 && w == 0) {  // thread 0's packet loads have returned
          __asm__ volatile("" : "+v"(acc));
          st_t[6] = static_cast<uint64_t>(wall_clock64());
        }
        uint8_t* dst = reinterpret_cast<uint8_t*>(s_head[i][0] & kServerAddrMask) + static_cast<uint64_t>(g) * P + coff;
        sys_store_16b(dst, acc);
      }
      if (stamps != nullptr && tid == 0) st_t[3] = static_cast<uint64_t>(wall_clock64());
      // The repair rows were stored system-coherent (no cache to write back): wait until every
      // one of this thread's stores is acknowledged, then the workgroup's barrier, then the done
      // words -- no release fence.  Same box, alternating (profiles/r03_resident_store_ab.txt):
      // one caller 8.0 vs 10.9 us a call, 16 callers 550k vs 330k calls/s against plain stores
      // and a system release fence (its L2 write-back 1.7-2.9 us a batch).  Not for a batch of
      // inline slots only: their rows carry lap words, and their done words only say the slot
      // was consumed (its loads have returned).
      if (s_ack != 0) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
      if (stamps != nullptr && tid == 0) st_t[4] = static_cast<uint64_t>(wall_clock64());
      lds_barrier();
      // the run up to its first slot with a word not yet landed (n when every word had)
      uint32_t n_ok = n;
      bool scrub = false;
      for (uint32_t k = 0; k < n; ++k) {
        if (s_bad[k] != 0) {
          n_ok = k;
          break;
        }
        scrub = scrub || server_scrub_after(next + uint64_t(k) * K, epoch);
      }
      if (tid == 0 && n_ok < n) sys_store_relaxed(&ctl->bad_slots[cls], ++n_bad);
      if (scrub) {
        // The last lap of an epoch (fec_kernels.hpp server_tag): zero the served slot's words and
        // inline data area before its done word, so no word of this epoch can match a tag of the
        // next.  Its next occupant writes only after it has seen the done word.
        constexpr uint32_t kSlotPieces = sizeof(ServerSlot) / 16u;
        const uint32_t pieces = kSlotPieces + (inl != nullptr ? kInlineSlotBytes / 16u : 0u);
        for (uint32_t k = 0; k < n_ok; ++k) {
          const uint64_t seq = next + uint64_t(k) * K;
          if (!server_scrub_after(seq, epoch)) continue;
          uint8_t* slot = reinterpret_cast<uint8_t*>(ring + seq % kServerSlots);
          uint8_t* area = inl != nullptr ? inl + (seq % kServerSlots) * kInlineSlotBytes : nullptr;
          for (uint32_t c = tid; c < pieces; c += kServerThreads)
            sys_store_16b(c < kSlotPieces ? slot + c * 16u : area + (c - kSlotPieces) * 16u, u32x4{0u, 0u, 0u, 0u});
          if (tid == 0) ++n_scrub;
        }
        __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): every zero in place before the done words
        lds_barrier();
        if (tid == 0) sys_store_relaxed(&ctl->scrubs[cls], n_scrub);
      }
      if (tid < n_ok) {
        const uint64_t seq = next + uint64_t(tid) * K;
        sys_store_relaxed(&done[seq % kServerSlots], seq + 1);
      }
      if (tid == 0) {
        s_next = next + uint64_t(n_ok) * K;
        sys_store_relaxed(&ctl->progress[cls], next + uint64_t(n_ok) * K);
      }
      if (stamps != nullptr && tid == 0) {
        st_t[5] = static_cast<uint64_t>(wall_clock64());
        uint64_t* rec = stamps + (st_batches % 256) * 8;
        rec[0] = st_t[1] - st_t[0];  // the poll that found the run
        rec[1] = st_t[2] - st_t[1];  // decision + acquire fence
        rec[2] = st_t[6] - st_t[2];  // thread 0's first work item: its 10 packet loads
        rec[3] = st_t[3] - st_t[6];  // its store (and any further items)
        rec[4] = st_t[5] - st_t[3];  // stores acknowledged + barrier + done stores
        rec[5] = n;
        rec[6] = st_polls;           // polls since the previous batch, this one included
        __threadfence_system();
        sys_store_release(&rec[7], ++st_batches);
        st_polls = 0;
      }
    } else if (!leave) {
      // a class other than 0 without work for slow_ticks polls every ~5 us instead of every ~1.5
      // (the host gives a lone caller's calls to class 0, whose polls other classes' polls slow down)
      if (s_slow != 0)
        __builtin_amdgcn_s_sleep(127);
      else
        __builtin_amdgcn_s_sleep(8);
    }
    lds_barrier();
    if (leave) break;
  }
  if (tid == 0) {
    sys_store_release(&ctl->progress[cls], s_next);
    bool last = true;
    if (coord != nullptr) {
      // count this workgroup out of instance gen (the word still holds the previous instance's
      // count until the first of this one's); at most `classes` contenders, so the loop ends
      uint64_t v = __hip_atomic_load(&coord->exits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM), nv = 0;
      do {
        nv = server_exits_next(v, gen);
      } while (!__hip_atomic_compare_exchange_strong(&coord->exits, &v, nv, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED,
                                                      __HIP_MEMORY_SCOPE_SYSTEM));
      last = server_exits_last(nv, K);
    }
    if (last) sys_store_release(&ctl->exited, gen);
  }
}

constexpr uint32_t kMaxThreadsPerLaunch = 1u << 30;
// Wave-per-group decode launches: 256-thread workgroups, so at most 2^22 of them keep the
// grid's work-item count (blocks * 256) inside 32 bits with room to spare.
constexpr uint64_t kMaxWaveBlocks = kMaxThreadsPerLaunch / 256u;
// Blocks per wave-per-group decode launch: kMaxWaveBlocks (the test library's
// TestKnob::kMaxWaveBlocks forces the chunked launches, which otherwise start only past 16.7M
// groups).
uint64_t max_wave_blocks() {
  const long n = test_knob(TestKnob::kMaxWaveBlocks, 0);
  return n > 0 && static_cast<uint64_t>(n) < kMaxWaveBlocks ? static_cast<uint64_t>(n) : kMaxWaveBlocks;
}
constexpr uint32_t kVecMinP = 16;  // shorter packets take the byte kernels

inline uint32_t blocks_for(uint64_t n) { return static_cast<uint32_t>((n + 255) / 256); }

}  // namespace

// ---------------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------------
namespace {

// A test-library switch (fec_knobs.hpp) as an int; `def` in the product library.
int knob(TestKnob k, int def) { return static_cast<int>(test_knob(k, def)); }

// XCD-aware group order for a decode kernel: at k=10 r=3 measured +10% for decode_fused and
// -1%..+5% for decode_wave over two boxes (tools/probe_decode.hip; tunable per kernel).
uint32_t decode_swizzle(const DecodeLaunch& a, int tuned) {
  return static_cast<uint32_t>(a.xcd_swizzle >= 0 ? a.xcd_swizzle : tuned);
}


// Groups per workgroup for the tiled mapping: the fewest idle lanes (workgroup = whole
// waves), preferring tiles whose byte size is a multiple of 128 (tile starts stay
// cache-line aligned).  0 = use the flat mapping (columns per packet > 512).
uint32_t pick_tile(uint32_t cpp, uint32_t k, uint32_t P) {
  if (cpp == 0 || cpp > 512) return 0;
  const uint32_t tmax = 512 / cpp;
  uint32_t best = 1;
  double best_score = 1e9;
  for (uint32_t t = 1; t <= tmax; ++t) {
    const uint32_t lanes = t * cpp, bs = (lanes + 63) / 64 * 64;
    double score = double(bs - lanes) / bs;
    if ((uint64_t(t) * k * P) % 128 != 0) score += 0.05;
    if (bs < 256) score += 0.02;
    if (score < best_score - 1e-9) {
      best_score = score;
      best = t;
    }
  }
  return best;
}

// Groups per workgroup of the tiled encodes (encode_bits: per half): pick_tile (the test
// library's TestKnob::kEncodeTile overrides it when the tile fits 512 lanes).
uint32_t encode_tile(const EncodeLaunch& a) {
  const uint32_t cpp = (a.P + 15u) / 16u;
  const int tile_env = knob(TestKnob::kEncodeTile, 0);
  return tile_env > 0 && cpp > 0 && uint32_t(tile_env) * cpp <= 512 ? uint32_t(tile_env) : pick_tile(cpp, a.k, a.P);
}

// POL: parity is written once and not re-read by this kernel (non-temporal stores).
template <int K, int R, int OFF, bool FIRST, int POL = kNtStore>
hipError_t run_encode_v16(const EncodeLaunch& a, uint32_t row0, hipStream_t s) {
  const uint32_t cpp = (a.P + 15u) / 16u;
  const uint32_t tile = encode_tile(a);
  const uint64_t gchunk = kMaxThreadsPerLaunch / cpp;
  for (uint64_t g0 = 0; g0 < a.groups; g0 += gchunk) {
    const uint64_t gn = (a.groups - g0 < gchunk) ? a.groups - g0 : gchunk;
    const uint32_t n = static_cast<uint32_t>(gn * cpp);
    if (tile > 0) {
      const uint32_t bs = (tile * cpp + 63) / 64 * 64;
      const uint32_t blocks = static_cast<uint32_t>((gn + tile - 1) / tile);
      // Workgroups per CU: the compile-time-k kernels with few table rows stream best at 2;
      // with r >= 4 rows of table arithmetic per load the kernel is VALU-bound and wants more
      // waves: k=20 r=5 at 4 workgroups 5.22-5.40 ms, 3: 5.35-5.50, uncapped 5.22-5.59
      // (profiles/r02_ab_encode_blocks_c4.txt, two boxes).  The runtime-k loop runs uncapped.
      // The XOR-only kernel (r = 1, the reference's computation) streams best at ~15 waves per
      // CU: k=10 at 1200 B (5-wave workgroups) 2.30 ms at 3 workgroups vs 2.39 at 2 and 2.36 at
      // 4; at 1400 B (7-wave workgroups) 2 (14 waves) beats 3 (21) by 1.7%
      // (profiles/r02_ab_encode_blocks_r1.txt, r02_ab_encode_blocks_r2.txt).
      constexpr int kDefBlocks = K == 0 ? 0 : (R >= 4 ? kEncodeBlocksPerCU + 2 : kEncodeBlocksPerCU);
      const int blocks_env = knob(TestKnob::kEncodeBlocks, -1);
      const int blocks_per_cu = blocks_env >= 0 ? blocks_env : kDefBlocks;
      const bool xor_waves = K > 0 && FIRST && R == 1 && blocks_env < 0;
      const int waves = a.waves_per_cu ? a.waves_per_cu
                                       : knob(TestKnob::kEncodeWaves, xor_waves ? kEncodeXorWavesPerCU
                                                                                : blocks_per_cu * static_cast<int>(bs / 64));
      uint32_t smem = occupancy_cap_lds(waves, bs / 64);
      if constexpr ((POL & kStageRows) != 0) smem = std::max<uint32_t>(smem, tile * R * a.P);
      hipLaunchKernelGGL((encode_v16<K, R, OFF, FIRST, POL>), dim3(blocks), dim3(bs), smem, s, a.data,
                         a.offsets, a.parity, g0, n, cpp, a.P, a.k, a.r, row0,
                         static_cast<const Tab*>(a.tables), tile, gn, 0u);
    } else {
      hipLaunchKernelGGL((encode_v16<K, R, OFF, FIRST, POL>), dim3(blocks_for(n)), dim3(256), 0, s, a.data,
                         a.offsets, a.parity, g0, n, cpp, a.P, a.k, a.r, row0,
                         static_cast<const Tab*>(a.tables), 0u, gn, 0u);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

template <int K, int R, int W, int POL = kNtStore>
hipError_t run_encode_bits(const EncodeLaunch& a, hipStream_t s) {
  const uint32_t cpp = (a.P + 15u) / 16u;
  const uint32_t tile = encode_tile(a);
  if (tile == 0) return hipErrorInvalidValue;  // callers route P > 8,192 elsewhere
  const uint32_t bs = (tile * cpp + 63) / 64 * 64;
  const uint64_t gchunk = max_wave_blocks() * 2 * tile;
  for (uint64_t g0 = 0; g0 < a.groups; g0 += gchunk) {
    const uint64_t gn = (a.groups - g0 < gchunk) ? a.groups - g0 : gchunk;
    const uint32_t blocks = static_cast<uint32_t>((gn + 2 * tile - 1) / (2 * tile));
    // Unstaged: uncapped (k=20 r=5 at 12 / 18 / 24 waves per CU within 0.2%, 3 waves per SIMD by
    // VGPRs).  Staged rows (kStageRows): 2 workgroups per CU, 5.163 vs 5.246 ms uncapped on two
    // boxes (scripts/sweep_encode_tiles.py, profiles/r05h, r05i).
    constexpr int kDefWaves = (POL & kStageRows) != 0 ? 10 : 0;
    const int waves = a.waves_per_cu ? a.waves_per_cu : knob(TestKnob::kEncodeWaves, kDefWaves);
    uint32_t smem = occupancy_cap_lds(waves, bs / 64);
    if constexpr ((POL & kStageRows) != 0) smem = std::max<uint32_t>(smem, 2 * tile * R * a.P);
    hipLaunchKernelGGL((encode_bits<K, R, W, POL>), dim3(blocks), dim3(bs), smem, s, a.data, a.parity, g0, cpp, a.P,
                       tile, gn, 0u);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// Bit-sliced encode for a compile-time shape where it is faster than the tables (r >= 4: the
// table form is VALU-bound there); the test library's TestKnob::kEncodeBits forces it on (1,
// every compiled shape) or off (0).
bool use_encode_bits(uint32_t r) {
  const int mode = knob(TestKnob::kEncodeBits, -1);
  return mode == 1 || (mode < 0 && r >= 4);
}

// kStageRows for a launch whose workgroup window (groups_per_block * r * P bytes) fits the LDS a
// workgroup may take (the test library's TestKnob::kEncodeStage: 1 on, 0 off).
bool use_stage_rows(const EncodeLaunch& a, uint32_t groups_per_block) {
  const int mode = knob(TestKnob::kEncodeStage, kEncodeStageDefault);
  return mode == 1 && a.P % 16 == 0 && uint64_t(groups_per_block) * a.r * a.P <= 64u * 1024u;
}

template <int OFF>
hipError_t run_encode_generic(const EncodeLaunch& a, hipStream_t s) {
  if (a.P < kVecMinP) {
    const uint64_t gchunk = kMaxThreadsPerLaunch / a.P;
    for (uint64_t g0 = 0; g0 < a.groups; g0 += gchunk) {
      const uint64_t gn = (a.groups - g0 < gchunk) ? a.groups - g0 : gchunk;
      const uint32_t n = static_cast<uint32_t>(gn * a.P);
      hipLaunchKernelGGL(encode_bytes<OFF>, dim3(blocks_for(n)), dim3(256), 0, s, a.data, a.offsets,
                         a.parity, g0, n, a.P, a.k, a.r, static_cast<const Tab*>(a.tables));
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  // Runtime k: passes of up to 8 parity rows; the first pass owns the XOR row.
  for (uint32_t row0 = 0; row0 < a.r; row0 += 8) {
    const uint32_t rows = (a.r - row0 < 8) ? a.r - row0 : 8;
    hipError_t e = hipSuccess;
#define QFEC_PASS(RR)                                                            \
  case RR:                                                                       \
    e = row0 == 0 ? run_encode_v16<0, RR, OFF, true>(a, row0, s)                 \
                  : run_encode_v16<0, RR, OFF, false>(a, row0, s);               \
    break;
    switch (rows) {
      QFEC_PASS(1)
      QFEC_PASS(2)
      QFEC_PASS(3)
      QFEC_PASS(4)
      QFEC_PASS(5)
      QFEC_PASS(6)
      QFEC_PASS(7)
      QFEC_PASS(8)
      default:
        return hipErrorInvalidValue;
    }
#undef QFEC_PASS
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// A compile-time encode in its staged form (kStageRows) where the workgroup's window fits
// (use_stage_rows), else with POL's direct stores.
template <int K, int R, int OFF, int POL = kNtStore>
hipError_t run_encode_v16_staged(const EncodeLaunch& a, hipStream_t s) {
  if (use_stage_rows(a, encode_tile(a))) return run_encode_v16<K, R, OFF, true, POL | kStageRows>(a, 0, s);
  return run_encode_v16<K, R, OFF, true, POL>(a, 0, s);
}

}  // namespace

hipError_t launch_encode(const EncodeLaunch& a, hipStream_t s) {
  if (a.groups == 0) return hipSuccess;
  if (a.P >= kVecMinP) {
    if (a.off_kind == OffsetKind::kNone) {
      // The paired-coefficient arithmetic (kPairMac): +0.9% at k=20 r=5 (5.53 vs 5.58 ms),
      // +1.0% at k=10 r=3 (2.65 vs 2.68 ms), same box, alternating runs
      // (profiles/r02_ab_encode_pair.txt).  Staged rows keep the default cache policy, NT stores
      // with cached loads (C2 2.590 ms vs 2.606-2.702, C4 4.991 vs 5.062-5.345 for the other
      // three; profiles/r05k/sweep_mempol.jsonl).
      // Bit-sliced form (bitslice.hpp) while a workgroup holds whole groups.  k=20 r=5 (VALU-
      // bound with the tables): 5.24-5.41 vs 5.37-5.54 ms over six boxes; k=10 r=3 (HBM-bound
      // with the tables) 2.74-2.76 vs 2.63-2.66 ms, so not chosen there.  4 packets in flight per
      // lane (2: 5.70 ms, 8: 5.28, 20: 5.91-6.03; profiles/r03_ab_bits.txt).
      if (a.P <= 8192 && use_encode_bits(a.r)) {
        const bool stg = use_stage_rows(a, 2 * encode_tile(a));
        if (a.k == 20 && a.r == 5)
          return stg ? run_encode_bits<20, 5, 4, kNtStore | kStageRows>(a, s) : run_encode_bits<20, 5, 4>(a, s);
        if (a.k == 10 && a.r == 3) return stg ? run_encode_bits<10, 3, 4, kNtStore | kStageRows>(a, s) : run_encode_bits<10, 3, 4>(a, s);
      }
      if (a.k == 10 && a.r == 3) return run_encode_v16_staged<10, 3, 0, kNtStore | kPairMac>(a, s);
      // staged rows measured per shape (scripts/ab_stage_rows.py, profiles/r05k): k=10 r=1 level
      // (2.383 vs 2.378 ms), k=10 r=2 -1.5% (2.537 vs 2.575), k=4 r=2 +8.9% (1.351 vs 1.241): the
      // XOR row and k=4 keep their direct stores
      if (a.k == 10 && a.r == 1) return run_encode_v16<10, 1, 0, true>(a, 0, s);
      if (a.k == 20 && a.r == 5) return run_encode_v16<20, 5, 0, true, kNtStore | kPairMac>(a, 0, s);
      if (a.k == 4 && a.r == 2) return run_encode_v16<4, 2, 0, true>(a, 0, s);
      // k=10 r=2 (the campaign's 20% FEC rate): compile-time k (2.50 vs 2.56 ms for the runtime-k
      // loop, profiles/r02_ab_encode_r1r2_defaults.txt)
      if (a.k == 10 && a.r == 2) return run_encode_v16_staged<10, 2, 0, kNtStore | kPairMac>(a, s);
    } else if (a.off_kind == OffsetKind::kU32) {
      if (a.k == 10 && a.r == 1) return run_encode_v16<10, 1, 1, true>(a, 0, s);
    } else if (a.off_kind == OffsetKind::kAddr) {
      if (a.k == 10 && a.r == 1) return run_encode_v16<10, 1, 3, true>(a, 0, s);
    }
  }
  switch (a.off_kind) {
    case OffsetKind::kNone:
      return run_encode_generic<0>(a, s);
    case OffsetKind::kU32:
      return run_encode_generic<1>(a, s);
    case OffsetKind::kU64:
      return run_encode_generic<2>(a, s);
    default:
      return run_encode_generic<3>(a, s);
  }
}

namespace {

template <int K, int MAXE>
hipError_t run_decode_v16(const DecodeLaunch& a, hipStream_t s) {
  const uint32_t cpp = (a.P + 15u) / 16u;
  const uint32_t passes = (a.r + MAXE - 1) / MAXE;  // e <= r
  for (uint32_t p = 0; p < passes; ++p) {
    const uint32_t m0 = p * MAXE;
    const uint64_t blocks = (a.groups + 3) / 4;
    const uint64_t max_blocks = max_wave_blocks();
    for (uint64_t b0 = 0; b0 < blocks; b0 += max_blocks) {
      const uint64_t bn = (blocks - b0 < max_blocks) ? blocks - b0 : max_blocks;
      const uint64_t g0 = b0 * 4;
      const uint64_t gn = (a.groups - g0 < bn * 4) ? a.groups - g0 : bn * 4;
      hipLaunchKernelGGL((decode_v16<K, MAXE>), dim3(static_cast<uint32_t>(bn)), dim3(256), 0, s,
                         a.data + g0 * a.k * static_cast<uint64_t>(a.P),
                         a.parity + g0 * a.r * static_cast<uint64_t>(a.P), a.rec_off ? a.rec_off + g0 : nullptr, a.codebook,
                         gn, cpp, a.P, a.k, a.r, m0);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
  }
  return hipSuccess;
}

template <int K, int MAXE, int POL>
hipError_t run_decode_wave(const DecodeLaunch& a, hipStream_t s) {
  const uint32_t passes = (a.r + MAXE - 1) / MAXE;  // e <= r
  const uint32_t cap = occupancy_cap_lds(a.waves_per_cu ? a.waves_per_cu : knob(TestKnob::kDecodeWaves, kDecodeWavesPerCU), 4);
  for (uint32_t p = 0; p < passes; ++p) {
    const uint32_t m0 = p * MAXE;
    // kLdsTabs: per-wave slice of whole 1 KiB wave-loads covering this pass's rows
    const uint32_t rows = a.r - m0 < MAXE ? a.r - m0 : MAXE;
    const uint32_t slice = (POL & kLdsTabs) != 0 ? (rows * a.k * 2u + 63u) / 64u * 1024u : 0u;
    const uint32_t smem = cap > 4 * slice ? cap : 4 * slice;
    const uint64_t blocks = (a.groups + 3) / 4;
    const uint64_t max_blocks = max_wave_blocks();
    for (uint64_t b0 = 0; b0 < blocks; b0 += max_blocks) {
      const uint64_t bn = (blocks - b0 < max_blocks) ? blocks - b0 : max_blocks;
      const uint64_t g0 = b0 * 4;
      const uint64_t gn = (a.groups - g0 < bn * 4) ? a.groups - g0 : bn * 4;
      hipLaunchKernelGGL((decode_wave<K, MAXE, POL>), dim3(static_cast<uint32_t>(bn)), dim3(256), smem, s,
                         a.data + g0 * a.k * static_cast<uint64_t>(a.P),
                         a.parity + g0 * a.r * static_cast<uint64_t>(a.P), a.rec_off ? a.rec_off + g0 : nullptr, a.codebook, gn, a.P,
                         a.k, a.r, m0, (a.out ? a.out : a.data) + g0 * ((POL & kCompactOut) != 0 ? a.r : a.k) * static_cast<uint64_t>(a.P), 0u,
                         decode_swizzle(a, kDecodeWaveXcdSwizzle), slice);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
  }
  return hipSuccess;
}

template <int K, int MAXE, int POL, int NM, int NT, bool DIRECT = false, bool INLINE = DIRECT, int SCAN = 0>
hipError_t run_decode_fused(const DecodeLaunch& a, hipStream_t s) {
  constexpr uint64_t kGroupsPerBlock = SCAN > 64 ? SCAN : 4u * (SCAN > 0 ? SCAN : 1);
  const uint32_t passes = (a.r + MAXE - 1) / MAXE;
  const uint32_t smem = occupancy_cap_lds(a.waves_per_cu ? a.waves_per_cu : knob(TestKnob::kDecodeWaves, kDecodeWavesPerCU), 4);
  RankMeta rm{};
  for (int e = 1; e <= 3; ++e) {
    rm.base[e] = a.meta.base[e];
    rm.stride[e] = a.meta.stride[e];
    rm.count_r[e] = a.meta.count_r[e];
  }
  // Output of the chunk starting at group g0: packed rows are placed by their global row
  // start (rec_off), so every chunk gets the base; the other layouts are offset per chunk.
  auto out_at = [&](uint64_t g0) -> uint8_t* {
    if (a.packed_rows) return a.out;
    return (a.out ? a.out : a.data) + g0 * ((POL & kCompactOut) != 0 ? a.r : a.k) * static_cast<uint64_t>(a.P);
  };
  for (uint32_t p = 0; p < passes; ++p) {
    const uint32_t m0 = p * MAXE;
    const uint64_t blocks = (a.groups + kGroupsPerBlock - 1) / kGroupsPerBlock;
    const uint64_t max_blocks = max_wave_blocks();
    for (uint64_t b0 = 0; b0 < blocks; b0 += max_blocks) {
      const uint64_t bn = (blocks - b0 < max_blocks) ? blocks - b0 : max_blocks;
      const uint64_t g0 = b0 * kGroupsPerBlock;
      const uint64_t gn = (a.groups - g0 < bn * kGroupsPerBlock) ? a.groups - g0 : bn * kGroupsPerBlock;
      hipLaunchKernelGGL((decode_fused<K, MAXE, POL, NM, NT, DIRECT, INLINE, SCAN>), dim3(static_cast<uint32_t>(bn)), dim3(256), smem, s,
                         a.data + g0 * a.k * static_cast<uint64_t>(a.P),
                         a.parity + g0 * a.r * static_cast<uint64_t>(a.P), a.rec_off ? a.rec_off + g0 : nullptr, a.codebook, gn, a.P,
                         a.r, m0, out_at(g0), 0u, decode_swizzle(a, kDecodeFusedXcdSwizzle), DIRECT ? a.masks + g0 : nullptr, rm,
                         INLINE && a.status ? a.status + g0 : nullptr);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
  }
  return hipSuccess;
}

// The fused form for this (k, r, P), if instantiated; hipErrorNotSupported otherwise.
// Instantiated for every P in [16, 2048] of the compiled (k, r) shapes: NM 16-B and NT 4-B
// pieces per lane (P <= 256: one 4-B piece; the in-place decode of such packets takes the
// tiled form, the recover layout this one).  r <= 3 shapes only in the mask-addressed form (the one auto uses for
// them), r > 3 only in the record-addressed one; k=10 r=3 1200 B in both (probes).
// Measured at k=10 r=3, 2 erasures (tools/probe_decode.hip): 512 B 5.89 TB/s vs 3.12 for
// the looped wave kernel, 768 B 5.49 vs 3.24 (profiles/r01_probe_decode_small.txt).  The
// mask-addressed forms also load non-temporally (survivors are read once): +1.2..3.2% at
// 512 / 768 / 1200 / 1400 B in one process (profiles/r01_probe_decode_ntload.txt); loads
// alone without NT stores lose 14%.  The r > 3 record-addressed forms stage their tables
// through LDS (kLdsTabs): k=20 r=5, 5 erasures, 1200 B: 2.27 -> 4.73-4.92 TB/s
// (profiles/r01_probe_decode_ldstabs_k20.txt); at k=10 r=3, whose 286 records stay in the
// scalar cache, it gains nothing (profiles/r01_probe_decode_inline_k10.txt).
// dry: only report whether a form exists (hipSuccess) without launching it.
hipError_t try_decode_fused(const DecodeLaunch& a, hipStream_t s, bool direct, bool dry = false) {
  const uint32_t nm = a.P / 1024u, nt = (a.P % 1024u + 255u) / 256u;
#define QFEC_FUSED_D(KK, RR, NMM, NTT)                                                        \
  if (direct && a.k == KK && a.r == RR && nm == NMM && nt == NTT)                             \
    return dry ? hipSuccess                                                                   \
           : a.compact_out ? run_decode_fused<KK, RR, kNtStore | kNtLoad | kCompactOut, NMM, NTT, true>(a, s) \
                           : run_decode_fused<KK, RR, kNtStore | kNtLoad, NMM, NTT, true>(a, s);
  // k=10 r=3 (the BASELINE shape) also has the scan form, for sparse loss (DecodeLaunch::scan),
  // and the compact-output form (DecodeLaunch::compact_out)
#define QFEC_FUSED_DS(KK, RR, NMM, NTT)                                                       \
  if (direct && a.k == KK && a.r == RR && nm == NMM && nt == NTT) {                           \
    if (dry) return hipSuccess;                                                               \
    if (a.compact_out)                                                                        \
      return a.scan == kDecodeScanGroups                                                      \
                 ? run_decode_fused<KK, RR, kNtStore | kNtLoad | kCompactOut, NMM, NTT, true, true, kDecodeScanGroups>(a, s) \
                 : run_decode_fused<KK, RR, kNtStore | kNtLoad | kCompactOut, NMM, NTT, true>(a, s); \
    if (a.scan == kDecodeScanGroups)                                                          \
      return run_decode_fused<KK, RR, kNtStore | kNtLoad, NMM, NTT, true, true, kDecodeScanGroups>(a, s); \
    return run_decode_fused<KK, RR, kNtStore | kNtLoad, NMM, NTT, true>(a, s);                \
  }
#define QFEC_FUSED_R(KK, RR, NMM, NTT)                                                        \
  if (!direct && !a.compact_out && a.k == KK && a.r == RR && nm == NMM && nt == NTT)          \
    return dry ? hipSuccess : run_decode_fused<KK, RR, kNtStore, NMM, NTT, false>(a, s);
#define QFEC_FUSED_L(KK, RR, NMM, NTT)                                                        \
  if (!direct && a.k == KK && a.r == RR && nm == NMM && nt == NTT)                            \
    return dry ? hipSuccess                                                                   \
           : a.compact_out ? run_decode_fused<KK, RR, kNtStore | kNtLoad | kLdsTabs | kCoefBytes | kCompactOut, NMM, NTT, false>(a, s) \
                           : run_decode_fused<KK, RR, kNtStore | kNtLoad | kLdsTabs | kCoefBytes, NMM, NTT, false>(a, s);
#define QFEC_FUSED_P(M, KK, RR)                                                               \
  M(KK, RR, 0, 1) M(KK, RR, 0, 2) M(KK, RR, 0, 3) M(KK, RR, 0, 4) M(KK, RR, 1, 0) M(KK, RR, 1, 1) \
  M(KK, RR, 1, 2) M(KK, RR, 1, 3) M(KK, RR, 1, 4)
  QFEC_FUSED_P(QFEC_FUSED_DS, 10, 3)
  QFEC_FUSED_R(10, 3, 1, 1)
  QFEC_FUSED_P(QFEC_FUSED_L, 20, 5)
  QFEC_FUSED_P(QFEC_FUSED_D, 10, 1)
  QFEC_FUSED_P(QFEC_FUSED_D, 10, 2)
  QFEC_FUSED_P(QFEC_FUSED_D, 4, 2)
#undef QFEC_FUSED_P
#undef QFEC_FUSED_DS
#undef QFEC_FUSED_L
#undef QFEC_FUSED_R
#undef QFEC_FUSED_D
  return hipErrorNotSupported;
}

// Packets of at most this size decode in the tiled form (several groups per wave).
constexpr uint32_t kTiledMaxP = 256;

template <int K, int MAXE, int POL>
hipError_t run_decode_tiled(const DecodeLaunch& a, uint32_t tile, hipStream_t s) {
  const uint32_t cpp = (a.P + 15u) / 16u;
  const uint32_t bs = (tile * cpp + 63) / 64 * 64;
  const uint64_t blocks = (a.groups + tile - 1) / tile;
  const uint64_t max_blocks = kMaxThreadsPerLaunch / bs;  // blocks * bs stays a 32-bit grid
  for (uint64_t b0 = 0; b0 < blocks; b0 += max_blocks) {
    const uint64_t bn = (blocks - b0 < max_blocks) ? blocks - b0 : max_blocks;
    const uint64_t g0 = b0 * tile;
    const uint64_t gn = (a.groups - g0 < bn * tile) ? a.groups - g0 : bn * tile;
    hipLaunchKernelGGL((decode_tiled<K, MAXE, POL>), dim3(static_cast<uint32_t>(bn)), dim3(bs), 0, s,
                       a.data + g0 * a.k * static_cast<uint64_t>(a.P),
                       a.parity + g0 * a.r * static_cast<uint64_t>(a.P), a.rec_off ? a.rec_off + g0 : nullptr, a.codebook, gn, cpp,
                       a.P, a.r, tile,
                       (a.out ? a.out : a.data) + g0 * ((POL & kCompactOut) != 0 ? a.r : a.k) * static_cast<uint64_t>(a.P));
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// (k, r) shapes with a compiled tiled form (launch_decode's QFEC_TILED list)
bool has_tiled(uint32_t k, uint32_t r) {
  return (k == 10 && (r == 3 || r == 1)) || (k == 20 && r == 5) || (k == 4 && r == 2);
}

bool decode_tiled_form(const DecodeLaunch& a) {
  // the compact recover layout only where a tiled form is compiled; elsewhere the fused or
  // wave forms write it
  if (a.compact_out && !has_tiled(a.k, a.r)) return false;
  const uint32_t tile = a.P >= kVecMinP ? pick_tile((a.P + 15u) / 16u, a.k, a.P) : 0u;
  // auto leaves k=20 r=5 to the LDS-table fused form (P=200: 4.6 vs 2.8 TB/s, same box)
  const bool auto_tiled = a.variant == kDecodeAuto && a.P <= kTiledMaxP && !(a.k == 20 && a.r == 5);
  return tile > 0 && (auto_tiled || a.variant == kDecodeTiledPlain || a.variant == kDecodeTiledNt);
}

// Mask-addressed fused form (r <= 3): +1.2% at k=10 r=3 (tools/probe_decode.hip,
// r01_probe_decode_direct.txt); at k=20 r=5 its extra VGPRs cost a wave per SIMD (-30%), so
// auto takes it for r <= 3 only.  It classifies inline: one launch, no classify kernel.
bool decode_direct_form(const DecodeLaunch& a) {
  return a.P >= kVecMinP && !decode_tiled_form(a) && a.masks != nullptr && !a.rec_ready &&
         (a.variant == kDecodeFusedDirect || (a.variant == kDecodeAuto && a.r <= 3)) &&
         try_decode_fused(a, nullptr, true, /*dry=*/true) == hipSuccess;
}

}  // namespace

bool decode_needs_rec_off(const DecodeLaunch& a) { return a.groups > 0 && !decode_direct_form(a); }

// The record-addressed LDS-table forms (QFEC_FUSED_L: k=20 r=5, 256 < P < 2048) read compact
// codebooks; every other form reads CoefEntry records.
bool decode_compact_tables(const DecodeLaunch& a) {
  if (a.groups == 0 || a.P < kVecMinP || a.rec_ready || decode_tiled_form(a) || decode_direct_form(a)) return false;
  if (a.variant != kDecodeFused && a.variant != kDecodeAuto && a.variant != kDecodeFusedDirect) return false;
  const uint32_t nm = a.P / 1024u, nt = (a.P % 1024u + 255u) / 256u;
  return a.k == 20 && a.r == 5 && ((nm == 0 && nt >= 1) || nm == 1);  // QFEC_FUSED_P's (nm, nt)
}

uint64_t rows_prefix_workspace_bytes(uint64_t groups) {
  return ((groups + kRowsPerBlock - 1) / kRowsPerBlock) * sizeof(uint32_t);
}

hipError_t launch_rows_prefix(const uint64_t* masks, uint64_t groups, uint32_t k, uint32_t r, uint32_t* row_start,
                              uint32_t* block_sums, uint64_t* total, hipStream_t s) {
  if (groups == 0) return hipSuccess;
  const uint64_t nb = (groups + kRowsPerBlock - 1) / kRowsPerBlock;
  if (nb > 0xFFFFFFFFull) return hipErrorInvalidValue;
  // the two-launch form's block limit (the test library's TestKnob::kRowsDirectBlocks forces the other form)
  const uint64_t direct_max = static_cast<uint64_t>(knob(TestKnob::kRowsDirectBlocks, kRowsDirectBlocks));
  const dim3 grid(static_cast<uint32_t>(nb));
  hipLaunchKernelGGL(rows_block_sums, grid, dim3(256), 0, s, masks, groups, k, r, block_sums);
  if (nb <= direct_max) {
    hipLaunchKernelGGL(rows_write<true>, grid, dim3(256), 0, s, masks, groups, k, r, block_sums, row_start, total);
  } else {
    hipLaunchKernelGGL(rows_scan_blocks, dim3(1), dim3(256), 0, s, block_sums, static_cast<uint32_t>(nb), total);
    hipLaunchKernelGGL(rows_write<false>, grid, dim3(256), 0, s, masks, groups, k, r, block_sums, row_start,
                       nullptr);
  }
  return hipGetLastError();
}

namespace {

// The library's form: 8 waves per workgroup, 512 groups per tile, NT loads and stores (tools/
// probe_runs.hip over four boxes, C5: 0.229-0.251 ms vs 0.241-0.268 for the slot rows and
// 0.241-0.262 for the two-step packed rows; 4 waves x 256 groups 0.247-0.253; profiles/r04_probe_runs_*.txt).
constexpr int kRunWaves = 8;
constexpr uint32_t kRunGroups = 64u * kRunWaves;

uint64_t runs_blocks_per_launch(uint64_t groups) {
  const uint64_t nb = (groups + kRunGroups - 1) / kRunGroups;
  const uint64_t mb = max_wave_blocks();
  return nb < mb ? nb : mb;
}

// The tile recover's row stores are non-temporal.  Back-to-back recovers alone favour plain
// stores by 10-15% on round 5's boxes (profiles/r05c, r05e, r05i probe_runs_c5.txt), but there
// the 0.13 GB of rows stay in the Infinity Cache from one launch to the next (the form's time
// equals its no-store floor); in the bench's step, after the encode's 15.6 GB, the two policies
// recover in the same 0.254 ms and the plain rows' write-back lands in the next encode (+0.01 ms;
// profiles/r05j/ab_legs.jsonl).
template <int K, int R, int NM, int NT, int POL = kNtLoad | kNtStore>
hipError_t run_recover_runs(const RunsLaunch& a, uint32_t stage, hipStream_t s) {
  RankMeta rm{};
  for (int e = 1; e <= 3; ++e) {
    rm.base[e] = a.meta.base[e];
    rm.stride[e] = a.meta.stride[e];
    rm.count_r[e] = a.meta.count_r[e];
  }
  uint8_t* ws = static_cast<uint8_t*>(a.workspace);
  uint32_t* ticket = reinterpret_cast<uint32_t*>(ws);
  const uint64_t per = runs_blocks_per_launch(a.groups) * kRunGroups;
  const uint32_t launches = runs_launches(a.groups);
  uint64_t* totals = reinterpret_cast<uint64_t*>(ws + 64);
  uint64_t* lb = reinterpret_cast<uint64_t*>(ws + 64 + 8 * static_cast<uint64_t>(launches));
  for (uint32_t c = 0; c < launches; ++c) {
    const uint64_t g0 = c * per;
    const uint64_t gn = a.groups - g0 < per ? a.groups - g0 : per;
    const uint32_t nb = static_cast<uint32_t>((gn + kRunGroups - 1) / kRunGroups);
    hipLaunchKernelGGL((recover_runs<K, R, NM, NT, POL, kRunWaves>), dim3(nb), dim3(64 * kRunWaves), stage, s, a.data + g0 * K * static_cast<uint64_t>(a.P),
                       a.parity + g0 * R * static_cast<uint64_t>(a.P), a.masks + g0, gn, a.P, a.codebook, rm, a.out,
                       a.row_start + g0, a.status ? a.status + g0 : nullptr, lb, ticket, a.epoch + c, stage,
                       c > 0 ? totals + (c - 1) : nullptr, totals + c, c + 1 == launches ? a.total : nullptr, 0u);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

// (k, r, P) shapes with a compiled recover_runs: the mask-addressed decode's (try_decode_fused
// QFEC_FUSED_DS / _D lists), 256 < P <= 2048 or P <= 256 with one 4-B piece.
hipError_t try_recover_runs(const RunsLaunch& a, uint32_t stage, hipStream_t s, bool dry) {
  const uint32_t nm = a.P / 1024u, nt = (a.P % 1024u + 255u) / 256u;
#define QFEC_RUNS(KK, RR, NMM, NTT) \
  if (a.k == KK && a.r == RR && nm == NMM && nt == NTT) return dry ? hipSuccess : run_recover_runs<KK, RR, NMM, NTT>(a, stage, s);
#define QFEC_RUNS_P(KK, RR)                                                                                    \
  QFEC_RUNS(KK, RR, 0, 1) QFEC_RUNS(KK, RR, 0, 2) QFEC_RUNS(KK, RR, 0, 3) QFEC_RUNS(KK, RR, 0, 4)            \
  QFEC_RUNS(KK, RR, 1, 0) QFEC_RUNS(KK, RR, 1, 1) QFEC_RUNS(KK, RR, 1, 2) QFEC_RUNS(KK, RR, 1, 3) QFEC_RUNS(KK, RR, 1, 4)
  QFEC_RUNS_P(10, 3)
  QFEC_RUNS_P(10, 1)
  QFEC_RUNS_P(10, 2)
  QFEC_RUNS_P(4, 2)
#undef QFEC_RUNS_P
#undef QFEC_RUNS
  return hipErrorNotSupported;
}

}  // namespace

uint32_t runs_launches(uint64_t groups) {
  if (groups == 0) return 0;
  const uint64_t per = runs_blocks_per_launch(groups) * kRunGroups;
  return static_cast<uint32_t>((groups + per - 1) / per);
}

uint64_t runs_workspace_bytes(uint64_t groups) {
  return 64 + 8 * static_cast<uint64_t>(runs_launches(groups)) + 8 * runs_blocks_per_launch(groups);
}

bool runs_supported(uint32_t k, uint32_t r, uint32_t P) {
  RunsLaunch a{};
  a.k = k;
  a.r = r;
  a.P = P;
  return P >= kVecMinP && try_recover_runs(a, 0, nullptr, true) == hipSuccess;
}

uint32_t runs_stage_bytes(const RunsLaunch& a) {
  // the run image needs 16-B aligned row starts in LDS and in HBM
  if (a.P % 16u != 0 || reinterpret_cast<uintptr_t>(a.out) % 16u != 0) return 0;
  const int v = a.stage_bytes >= 0 ? a.stage_bytes : knob(TestKnob::kRunsStage, kRunsStageBytes);
  if (v <= 0) return 0;
  const uint32_t cap = 64u * 1024u;  // dynamic LDS per workgroup (160 KiB per CU)
  return static_cast<uint32_t>(v) < cap ? static_cast<uint32_t>(v) : cap;
}

hipError_t launch_recover_runs(const RunsLaunch& a, hipStream_t s) {
  if (a.groups == 0) return hipSuccess;
  if (a.workspace == nullptr || a.row_start == nullptr || a.out == nullptr || a.masks == nullptr) return hipErrorInvalidValue;
  return try_recover_runs(a, runs_stage_bytes(a), s, false);
}

hipError_t launch_decode(const DecodeLaunch& a, hipStream_t s) {
  if (a.groups == 0) return hipSuccess;
  // the codebook's format must be the one the chosen form reads
  if (a.compact_tables != decode_compact_tables(a)) return hipErrorInvalidValue;
  const uint32_t tile = a.P >= kVecMinP ? pick_tile((a.P + 15u) / 16u, a.k, a.P) : 0u;
  const bool tiled = decode_tiled_form(a);
  if (decode_direct_form(a)) return try_decode_fused(a, s, true);
  if (a.rec_off == nullptr) return hipErrorInvalidValue;  // every other form reads rec_off
  for (uint64_t g0 = 0; !a.rec_ready && g0 < a.groups; g0 += kMaxThreadsPerLaunch) {
    const uint64_t gn = (a.groups - g0 < kMaxThreadsPerLaunch) ? a.groups - g0 : kMaxThreadsPerLaunch;
    hipLaunchKernelGGL(classify, dim3(blocks_for(gn)), dim3(256), 0, s, a.masks + g0, gn, a.k, a.r,
                       a.binom, a.meta, a.rec_off ? a.rec_off + g0 : nullptr, a.status ? a.status + g0 : nullptr);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (a.P < kVecMinP) {
    const uint64_t gchunk = kMaxThreadsPerLaunch / a.P;
    for (uint64_t g0 = 0; g0 < a.groups; g0 += gchunk) {
      const uint64_t gn = (a.groups - g0 < gchunk) ? a.groups - g0 : gchunk;
      const uint32_t n = static_cast<uint32_t>(gn * a.P);
      hipLaunchKernelGGL(decode_bytes, dim3(blocks_for(n)), dim3(256), 0, s, a.data, a.parity,
                         a.rec_off, a.codebook, g0, n, a.P, a.k, a.r, a.out ? a.out : a.data,
                         a.compact_out ? 1u : 0u);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  if (a.compact_out) {
    // packets <= 256 B: the tiled form (several groups per wave), compact
    if (tiled) {
#define QFEC_TILED_C(KK, RR) \
  if (a.k == KK && a.r == RR) return run_decode_tiled<KK, RR, kNtStore | kCompactOut>(a, tile, s);
      QFEC_TILED_C(10, 3)
      QFEC_TILED_C(10, 1)
      QFEC_TILED_C(20, 5)
      QFEC_TILED_C(4, 2)
#undef QFEC_TILED_C
    }
    // fused forms were tried above; everything else: the runtime-k wave kernel, compact
    if (a.variant == kDecodeFused || a.variant == kDecodeAuto || a.variant == kDecodeFusedDirect) {
      const hipError_t e = try_decode_fused(a, s, false);
      if (e != hipErrorNotSupported) return e;
    }
    return run_decode_wave<0, 8, kNtStore | kNoCoefBranch | kCompactOut>(a, s);
  }
  if (tiled) {
#ifdef QUICFEC_PROBE_FORMS
    const bool nt = a.variant != kDecodeTiledPlain;
#else
    constexpr bool nt = true;  // the library never sets a variant (the plain forms are probe-only)
#endif
#define QFEC_TILED(KK, RR)                                                                   \
  if (a.k == KK && a.r == RR)                                                                \
    return nt ? run_decode_tiled<KK, RR, kNtStore>(a, tile, s) : QFEC_PROBE_ONLY(run_decode_tiled<KK, RR, 0>(a, tile, s));
    QFEC_TILED(10, 3)
    QFEC_TILED(10, 1)
    QFEC_TILED(20, 5)
    QFEC_TILED(4, 2)
#undef QFEC_TILED
  }
  // Fused passes win where many rows share each survivor (k=20 r=5, 5 losses: +21%); with
  // the XCD-aware order they also win at r = 3 (+2.6%; tools/probe_decode.hip), so auto
  // takes them wherever they are instantiated.
  // (the mask-addressed forms were tried above, before classify)
  if (a.variant == kDecodeFused || a.variant == kDecodeAuto || a.variant == kDecodeFusedDirect) {
    const hipError_t e = try_decode_fused(a, s, false);
    if (e != hipErrorNotSupported) return e;
  }
#ifdef QUICFEC_PROBE_FORMS
  // Probe-only forms (tools/probe_decode.hip sets DecodeLaunch::variant; the library never does):
  // no branch on coefficients 0 / 1, the plain-store wave kernel, 16-B lanes only (decode_v16).
  const bool separate_out = a.out != nullptr && a.out != a.data;  // decode_v16 lacks it
  if (a.variant == kDecodeWaveNoBranch && !separate_out) {
#define QFEC_WAVE_NB(KK, RR) \
  if (a.k == KK && a.r == RR) return run_decode_wave<KK, RR, kNtStore | kNoCoefBranch>(a, s);
    QFEC_WAVE_NB(10, 3)
    QFEC_WAVE_NB(20, 5)
#undef QFEC_WAVE_NB
  }
  if (a.variant == kDecodeWavePerGroup && !separate_out) {
    if (a.k == 10 && a.r == 3) return run_decode_v16<10, 3>(a, s);
    if (a.k == 10 && a.r == 1) return run_decode_v16<10, 1>(a, s);
    if (a.k == 20 && a.r == 5) return run_decode_v16<20, 5>(a, s);
    if (a.k == 4 && a.r == 2) return run_decode_v16<4, 2>(a, s);
    return run_decode_v16<0, 8>(a, s);
  }
  const bool nt = a.variant != kDecodeWavePlain;
#else
  constexpr bool nt = true;
#endif
  {
#define QFEC_WAVE(KK, RR)                                                                    \
  if (a.k == KK && a.r == RR)                                                                \
    return nt ? run_decode_wave<KK, RR, kNtStore>(a, s) : QFEC_PROBE_ONLY(run_decode_wave<KK, RR, 0>(a, s));
    QFEC_WAVE(10, 3)
    QFEC_WAVE(10, 1)
    QFEC_WAVE(20, 5)
    QFEC_WAVE(4, 2)
#undef QFEC_WAVE
    // Runtime k: multiplying by every coefficient (no branches on 0 / 1) wins at every shape
    // measured (tools/probe_decode.hip, profiles/r01_probe_decode_runtime_k.txt): k=10 r=2
    // 4.13 -> 4.79 TB/s, 12+6 2.62 -> 3.20, 16+4 2.67 -> 3.40.  Its tables staged through
    // LDS (kLdsTabs) lose here (2.2-2.8 TB/s): the records of these codebooks are hit often
    // enough in the scalar cache, and the wait for the tables precedes the survivor loads.
    return nt ? run_decode_wave<0, 8, kNtStore | kNoCoefBranch>(a, s) : QFEC_PROBE_ONLY(run_decode_wave<0, 8, 0>(a, s));
  }
}

hipError_t launch_fill_splitmix(uint8_t* dst, uint64_t nbytes, uint64_t seed, uint64_t byte_offset,
                                hipStream_t s) {
  if (nbytes == 0) return hipSuccess;
  const bool fast = (byte_offset % 8 == 0) && (reinterpret_cast<uintptr_t>(dst) % 16 == 0);
  uint64_t done = 0;
  if (fast) {
    const uint64_t n16 = nbytes / 16;
    for (uint64_t c0 = 0; c0 < n16; c0 += kMaxThreadsPerLaunch) {
      const uint64_t cn = (n16 - c0 < kMaxThreadsPerLaunch) ? n16 - c0 : kMaxThreadsPerLaunch;
      hipLaunchKernelGGL(fill_words, dim3(blocks_for(cn)), dim3(256), 0, s, dst + c0 * 16,
                         static_cast<uint32_t>(cn), seed, (byte_offset / 8) + 2 * c0);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
    done = n16 * 16;
  }
  for (uint64_t c0 = done; c0 < nbytes; c0 += kMaxThreadsPerLaunch) {
    const uint64_t cn = (nbytes - c0 < kMaxThreadsPerLaunch) ? nbytes - c0 : kMaxThreadsPerLaunch;
    hipLaunchKernelGGL(fill_bytes, dim3(blocks_for(cn)), dim3(256), 0, s, dst + c0,
                       static_cast<uint32_t>(cn), seed, byte_offset + c0);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_legacy_server(ServerSlot* ring, uint8_t* inl, uint64_t* done, ServerControl* ctl,
                                ServerCoord* coord, uint32_t classes, uint64_t gen, uint64_t idle_ticks,
                                uint64_t slow_ticks, uint64_t life_ticks, uint64_t* stamps, uint32_t epoch,
                                hipStream_t s) {
  if (epoch < 1u || epoch > kServerEpoch || (epoch & (epoch - 1u)) != 0) return hipErrorInvalidValue;
  // classes: a power of two (it divides kServerSlots), with the shared words when more than one;
  // gen fits the exit count's 56 bits
  if (classes < 1u || classes > kServerMaxClasses || (classes & (classes - 1u)) != 0 || (classes > 1u && !coord) ||
      gen == 0 || gen >= (1ull << 56))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(legacy_server, dim3(classes), dim3(kServerThreads), 0, s, ring, inl, done, ctl,
                     classes > 1u ? coord : nullptr, classes, gen, idle_ticks, slow_ticks, life_ticks, stamps, epoch);
  return hipGetLastError();
}

hipError_t launch_copy_words(const uint8_t* src, uint8_t* dst, uint64_t nbytes, hipStream_t s) {
  const uint64_t n16 = nbytes / 16;
  for (uint64_t c0 = 0; c0 < n16; c0 += kMaxThreadsPerLaunch) {
    const uint64_t cn = (n16 - c0 < kMaxThreadsPerLaunch) ? n16 - c0 : kMaxThreadsPerLaunch;
    hipLaunchKernelGGL(copy_words, dim3(blocks_for(cn)), dim3(256), 0, s,
                       reinterpret_cast<const uint4*>(src + c0 * 16), reinterpret_cast<uint4*>(dst + c0 * 16),
                       static_cast<uint32_t>(cn));
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

}  // namespace qfec
