// bitslice.hpp — bit-sliced GF(2^8) encode with the code's coefficients compiled in.
//
// Multiplying a byte by a constant c is a linear map over GF(2): bit u of c*x is the XOR
// of the bits b of x for which bit u of c*2^b is set (an 8x8 bit matrix per coefficient).
// With 32 bytes of one packet transposed into 8 bit planes (plane b = bit b of each of the
// 32 bytes, one dword), c*x for all 32 bytes is 8 plane XORs picked by that matrix, and a
// parity row is those XORs summed over the group's packets.  The parity matrix of the code
// (gf256.hpp's parity_matrix: Cauchy, normalised so row 0 and column 0 are all ones) is
// fixed by (k, r), so for a compile-time (K, R) every XOR is decided by the compiler: no
// table lookups, no selector preparation.  Per data dword at k=20 r=5 that is ~15 VALU
// operations (the 3-stage bit transpose 6, plane-subset XORs and row planes ~8, the row-0 XOR
// and the transposes back) against ~26 for the v_perm_b32 tables (fec_kernels.hip encode_v16,
// 97% VALU issue on MI355X, profiles/r03_sq/sq_c4.json) — the bytes produced are identical.
//
// Used by fec_kernels.hip (encode_bits) and checked on the CPU against the oracle
// (tests/csrc/kernel_emulation.cpp): the header is plain C++17 so the same code runs on both.
#pragma once

#include <cstdint>
#include <utility>

#include "coef_tables.hpp"  // QFEC_HD

#if defined(__clang__)
#define QFEC_UNROLL _Pragma("unroll")
#else
#define QFEC_UNROLL
#endif

namespace qfec {
namespace bs {

// ---- compile-time GF(2^8), polynomial 0x11D (the same field as gf256.hpp) ----
constexpr uint32_t cmul(uint32_t a, uint32_t b) {
  uint32_t p = 0, x = a & 0xFFu;
  for (int i = 0; i < 8; ++i) {
    if ((b >> i) & 1u) p ^= x;
    x <<= 1;
    if (x & 0x100u) x ^= 0x11Du;
  }
  return p;
}

constexpr uint32_t cinv(uint32_t a) {
  for (uint32_t x = 1; x < 256; ++x)
    if (cmul(a, x) == 1u) return x;
  return 0;
}

// gf256.hpp parity_matrix(K, R), evaluated by the compiler.
template <int K, int R>
struct CodeMatrix {
  static_assert(K > 0 && R > 0 && K + R <= 256, "code shape");
  uint8_t m[R][K];
  constexpr CodeMatrix() : m() {
    for (int i = 0; i < R; ++i)
      for (int j = 0; j < K; ++j) m[i][j] = static_cast<uint8_t>(cinv(uint32_t(i) ^ uint32_t(R + j)));
    for (int j = 0; j < K; ++j) {
      const uint32_t s = cinv(m[0][j]);
      for (int i = 0; i < R; ++i) m[i][j] = static_cast<uint8_t>(cmul(m[i][j], s));
    }
    for (int i = 1; i < R; ++i) {
      const uint32_t s = cinv(m[i][0]);
      for (int j = 0; j < K; ++j) m[i][j] = static_cast<uint8_t>(cmul(m[i][j], s));
    }
  }
};

// Row u of c's bit matrix: bit b set <=> bit u of c * 2^b.
constexpr uint32_t bitrow(uint32_t c, int u) {
  uint32_t r = 0;
  for (int b = 0; b < 8; ++b) r |= ((cmul(c, 1u << b) >> u) & 1u) << b;
  return r;
}

template <int K, int R>
struct Plan {
  uint8_t row[R][K][8];
  constexpr Plan() : row() {
    const CodeMatrix<K, R> M;
    for (int i = 0; i < R; ++i)
      for (int j = 0; j < K; ++j)
        for (int u = 0; u < 8; ++u) row[i][j][u] = static_cast<uint8_t>(bitrow(M.m[i][j], u));
  }
};

template <int K, int R>
struct PlanOf {
  static constexpr Plan<K, R> value{};
};

// ---- compile-time loops ----
template <class F, int... I>
QFEC_HD inline void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
QFEC_HD inline void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

// ---- 8 x 8 bit transpose per byte lane ----
// Rows d = the 8 dwords, columns b = bit b of each byte: afterwards x[b] bit (8q + d) is bit
// b of byte q of the old x[d].  A transpose, so it is its own inverse.  Stage S swaps the
// off-diagonal S x S blocks: row d's columns with bit S set <-> row d+S's columns with it
// clear; each pair costs two shifts and two bit selects (v_bfi_b32 / v_bitop3_b32).
template <int S>
QFEC_HD inline void swap_bits(uint32_t& a, uint32_t& b, uint32_t lo) {
  const uint32_t na = (a & lo) | ((b << S) & ~lo);
  const uint32_t nb = ((a >> S) & lo) | (b & ~lo);
  a = na;
  b = nb;
}

QFEC_HD inline void transpose8(uint32_t (&x)[8]) {
  swap_bits<4>(x[0], x[4], 0x0F0F0F0Fu);
  swap_bits<4>(x[1], x[5], 0x0F0F0F0Fu);
  swap_bits<4>(x[2], x[6], 0x0F0F0F0Fu);
  swap_bits<4>(x[3], x[7], 0x0F0F0F0Fu);
  swap_bits<2>(x[0], x[2], 0x33333333u);
  swap_bits<2>(x[1], x[3], 0x33333333u);
  swap_bits<2>(x[4], x[6], 0x33333333u);
  swap_bits<2>(x[5], x[7], 0x33333333u);
  swap_bits<1>(x[0], x[1], 0x55555555u);
  swap_bits<1>(x[2], x[3], 0x55555555u);
  swap_bits<1>(x[4], x[5], 0x55555555u);
  swap_bits<1>(x[6], x[7], 0x55555555u);
}

// a ^ b ^ c in one VALU operation (v_bitop3_b32 / v_xor3_b32 on the device)
QFEC_HD inline uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
#else
  return a ^ b ^ c;
#endif
}

// Hides v's expression from the optimiser.  Without it the compiler re-associates every
// row's XOR chain down to single planes (the chains share nothing any more, 2-3x the XORs)
// and keeps every packet's planes live to the end.
QFEC_HD inline uint32_t opaque(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  __asm__("" : "+v"(v));
#else
  __asm__("" : "+r"(v));
#endif
  return v;
}

// The XORs of the 4-plane half p[B0 .. B0+3] for every nonzero subset M (bit b = plane
// B0 + b): 11 operations for all 15; the compiler drops the ones no coefficient uses.
template <int B0>
struct Combos {
  uint32_t v[16];
  QFEC_HD explicit Combos(const uint32_t (&p)[8]) {
    v[0] = 0;
    v[1] = p[B0], v[2] = p[B0 + 1], v[4] = p[B0 + 2], v[8] = p[B0 + 3];
    v[3] = opaque(v[1] ^ v[2]), v[5] = opaque(v[1] ^ v[4]), v[6] = opaque(v[2] ^ v[4]);
    v[9] = opaque(v[1] ^ v[8]), v[10] = opaque(v[2] ^ v[8]), v[12] = opaque(v[4] ^ v[8]);
    v[7] = opaque(v[3] ^ v[4]), v[11] = opaque(v[3] ^ v[8]), v[13] = opaque(v[5] ^ v[8]);
    v[14] = opaque(v[6] ^ v[8]), v[15] = opaque(v[3] ^ v[12]);
  }
};

// Parity of one 32-byte chunk, streamed: load(j, dst) fetches 8 dwords of data packet j
// (any 8 dwords of the packet, the same positions for every j) into dst; out[i] receives the
// same bytes of parity row i.  At most W packets are held at once: packet j + W is fetched
// into packet j's registers as soon as j is folded in, so a wave keeps W packets of loads in
// flight while it computes and needs ~8W + 8R + 30 VGPRs instead of 8K + 8R + 30 (k=20 r=5
// with every packet held: 211 VGPRs, 2 waves per SIMD, and all of a CU's waves load and
// compute in lockstep; MI355X measured 43% VALU issue and slower than the tables).
template <int K, int R, int W, class Load>
QFEC_HD inline void encode_stream(Load&& load, uint32_t (&out)[R][8]) {
  static_assert(W >= 1 && W <= K, "window");
  uint32_t buf[W][8];
  static_for<W>([&](auto jj) { load(decltype(jj)::value, buf[decltype(jj)::value]); });
  uint32_t acc[R > 1 ? R - 1 : 1][8];
  static_for<K>([&](auto jj) {
    constexpr int j = decltype(jj)::value;
    uint32_t(&x)[8] = buf[j % W];
    // Row 0: the reference XOR (fec_xor_simd.cpp:411-427), in the byte domain.
    QFEC_UNROLL
    for (int d = 0; d < 8; ++d) out[0][d] = j == 0 ? x[d] : out[0][d] ^ x[d];
    if constexpr (R > 1) {
      transpose8(x);
      QFEC_UNROLL
      for (int b = 0; b < 8; ++b) x[b] = opaque(x[b]);
      if constexpr (j == 0) {
        // Column 0 of every row is 1: the planes of packet 0 as they are.
        QFEC_UNROLL
        for (int i = 0; i < R - 1; ++i)
          QFEC_UNROLL
          for (int u = 0; u < 8; ++u) acc[i][u] = x[u];
      } else {
        const Combos<0> lo(x);
        const Combos<4> hi(x);
        static_for<R - 1>([&](auto ii) {
          constexpr int i = decltype(ii)::value + 1;
          static_for<8>([&](auto uu) {
            constexpr int u = decltype(uu)::value;
            constexpr int br = PlanOf<K, R>::value.row[i][j][u];
            acc[i - 1][u] = xor3(acc[i - 1][u], lo.v[br & 15], hi.v[br >> 4]);
          });
        });
      }
    }
    if constexpr (j + W < K) load(j + W, x);
  });
  if constexpr (R > 1) {
    QFEC_UNROLL
    for (int i = 0; i < R - 1; ++i) {
      transpose8(acc[i]);
      QFEC_UNROLL
      for (int d = 0; d < 8; ++d) out[i + 1][d] = acc[i][d];
    }
  }
}

// The same with every packet already in registers (x is left transposed).
template <int K, int R>
QFEC_HD inline void encode_chunk(uint32_t (&x)[K][8], uint32_t (&out)[R][8]) {
  encode_stream<K, R, K>(
      [&](int j, uint32_t(&dst)[8]) {
        for (int d = 0; d < 8; ++d) dst[d] = x[j][d];
      },
      out);
}

}  // namespace bs
}  // namespace qfec
