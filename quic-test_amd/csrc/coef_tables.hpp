// coef_tables.hpp — the v_perm_b32 lookup tables of one GF(2^8) coefficient, computed from
// the coefficient alone.  Used by the kernels that receive bare coefficient bytes
// (fec_kernels.hip, kCoefBytes) and checked on the CPU against gf256.hpp's make_entry
// (tests/csrc/kernel_emulation.cpp).
//
// x -> c*x is linear over GF(2), so c*v for a 3-bit (or 2-bit) piece v of x is the XOR of
// c*2^b over the set bits b of the piece: eight products p_b = c*2^b (repeated doubling,
// x^8 = x^4 + x^3 + x^2 + 1) give every table byte with a few XORs.
#pragma once

#include <cstdint>

#if defined(__HIPCC__)
#define QFEC_HD __host__ __device__
#else
#define QFEC_HD
#endif

namespace qfec {

struct TabWords {
  uint32_t t0lo, t0hi;  // c * v        for v = 0..7  (bits 0..2 of x)
  uint32_t t1lo, t1hi;  // c * (v << 3) for v = 0..7  (bits 3..5)
  uint32_t t2;          // c * (v << 6) for v = 0..3  (bits 6..7)
};

QFEC_HD inline TabWords tab_words(uint32_t c) {
  uint32_t p[8];
  p[0] = c & 0xFFu;
  for (int b = 1; b < 8; ++b) p[b] = ((p[b - 1] << 1) ^ ((p[b - 1] & 0x80u) ? 0x1Du : 0u)) & 0xFFu;
  // bytes {0, a, b, a^b}: the products of the pieces 0..3 of a 2-bit piece basis (a, b)
  auto quad = [](uint32_t a, uint32_t b) { return (a << 8) | (b << 16) | ((a ^ b) << 24); };
  // bytes {d, a^d, b^d, a^b^d}: pieces 4..7 with the third basis product d
  auto quad_hi = [](uint32_t a, uint32_t b, uint32_t d) {
    return d | ((a ^ d) << 8) | ((b ^ d) << 16) | ((a ^ b ^ d) << 24);
  };
  TabWords t;
  t.t0lo = quad(p[0], p[1]);
  t.t0hi = quad_hi(p[0], p[1], p[2]);
  t.t1lo = quad(p[3], p[4]);
  t.t1hi = quad_hi(p[3], p[4], p[5]);
  t.t2 = quad(p[6], p[7]);
  return t;
}

}  // namespace qfec
