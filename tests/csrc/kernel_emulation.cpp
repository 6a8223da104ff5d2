// kernel_emulation.cpp — CPU check of the GPU library's table arithmetic (tests only).
//
// Re-executes, on the CPU, exactly the per-dword arithmetic of fec_kernels.hip
// (v_perm_b32 table lookups, the classify ranking, codebook-driven rebuild) using the
// product's own host code (quic-test_amd/csrc/gf256.hpp), and compares the bytes with the
// oracle restatement (oracle/liboracle.so).  Lets the CPU suite catch table / ranking /
// codebook-layout bugs before a GPU run.  Prints "OK <cases>" or the first mismatch.
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <random>
#include <vector>

#include "bitslice.hpp"
#include "coef_tables.hpp"
#include "gf256.hpp"

extern "C" {
int oracle_rs_encode(const uint8_t*, uint64_t, uint32_t, uint32_t, uint32_t, uint8_t*, int);
int64_t oracle_rs_decode(uint8_t*, const uint8_t*, const uint64_t*, uint64_t, uint32_t, uint32_t, uint32_t,
                         uint8_t*, int);
void oracle_fill_splitmix(uint8_t*, uint64_t, uint64_t, uint64_t);
}

using qfec::CoefEntry;

// v_perm_b32 (CDNA4 ISA): byte b of the result = byte sel_b of {S0:S1} for sel_b < 8.
static uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {
  const uint64_t d = (uint64_t(s0) << 32) | s1;
  uint32_t out = 0;
  for (int b = 0; b < 4; ++b) {
    const uint32_t s = (sel >> (8 * b)) & 0xFF;
    uint32_t v;
    if (s < 8) v = (d >> (8 * s)) & 0xFF;
    else if (s == 12) v = 0;
    else if (s >= 13) v = 0xFF;
    else v = ((d >> (16 * (s - 8) + 15)) & 1) ? 0xFF : 0;
    out |= v << (8 * b);
  }
  return out;
}

static uint32_t gmul(uint32_t w, const CoefEntry& t) {
  const uint32_t s0 = w & 0x07070707u, s1 = (w >> 3) & 0x07070707u, s2 = (w >> 6) & 0x03030303u;
  return perm(t.t0hi, t.t0lo, s0) ^ perm(t.t1hi, t.t1lo, s1) ^ perm(t.t2, t.t2, s2);
}

static uint32_t ld32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}
static void st32(uint8_t* p, uint32_t v) { std::memcpy(p, &v, 4); }

static int fail(const char* what, int a, int b, int c) {
  std::printf("MISMATCH %s (%d,%d,%d)\n", what, a, b, c);
  return 1;
}

// bitslice.hpp against gf256.hpp and the oracle: matrix, transpose, and groups of 1,208-byte
// packets encoded the way encode_bits maps lanes.
template <int K, int R>
static int bitslice_check(std::mt19937_64& rng) {
  std::vector<uint8_t> M;
  qfec::parity_matrix(K, R, M);
  constexpr qfec::bs::CodeMatrix<K, R> CM{};
  for (int i = 0; i < R; ++i)
    for (int j = 0; j < K; ++j)
      if (CM.m[i][j] != M[i * K + j]) return fail("bitslice matrix", K, R, i * K + j);
  uint32_t t[8], t0[8];
  for (auto& v : t) v = static_cast<uint32_t>(rng());
  std::memcpy(t0, t, sizeof t);
  qfec::bs::transpose8(t);
  for (int b = 0; b < 8; ++b)
    for (int q = 0; q < 4; ++q)
      for (int d = 0; d < 8; ++d)
        if (((t[b] >> (8 * q + d)) & 1u) != ((t0[d] >> (8 * q + b)) & 1u)) return fail("transpose8", b, q, d);
  qfec::bs::transpose8(t);
  if (std::memcmp(t, t0, sizeof t) != 0) return fail("transpose8 involution", K, R, 0);
  // encode_bits' lane mapping: one 16-byte column (the last shifted back to end at P) of
  // groups g and g + tile; a second group past the end repeats the first and is not stored.
  const uint32_t P = 1208, cpp = (P + 15) / 16, tile = 3;
  const uint64_t G = 5;
  std::vector<uint8_t> data(G * K * P), par(G * R * P), ref(G * R * P);
  oracle_fill_splitmix(data.data(), data.size(), rng(), 0);
  for (uint64_t g = 0; g < tile; ++g)
    for (uint32_t c = 0; c < cpp; ++c) {
      const uint32_t o = c * 16 + 16 <= P ? c * 16 : P - 16;
      const bool second = g + tile < G;
      const uint64_t gg[2] = {g, second ? g + tile : g};
      uint32_t x[K][8], out[R][8];
      for (int j = 0; j < K; ++j)
        for (int h = 0; h < 2; ++h)
          for (int w = 0; w < 4; ++w) x[j][4 * h + w] = ld32(&data[(gg[h] * K + j) * P + o + 4 * w]);
      qfec::bs::encode_chunk<K, R>(x, out);
      for (int i = 0; i < R; ++i)
        for (int h = 0; h < (second ? 2 : 1); ++h)
          for (int w = 0; w < 4; ++w) st32(&par[(gg[h] * R + i) * P + o + 4 * w], out[i][4 * h + w]);
    }
  oracle_rs_encode(data.data(), G, K, R, P, ref.data(), 1);
  if (par != ref) return fail("bitslice encode", K, R, int(P));
  return 0;
}

int main() {
  std::mt19937_64 rng(12345);
  int cases = 0;
  // The tables kernels build from a bare coefficient (kCoefBytes, coef_tables.hpp) are the
  // host's make_entry tables, for every coefficient.
  for (uint32_t c = 0; c < 256; ++c) {
    const CoefEntry e = qfec::make_entry(static_cast<uint8_t>(c));
    const qfec::TabWords w = qfec::tab_words(c);
    if (w.t0lo != e.t0lo || w.t0hi != e.t0hi || w.t1lo != e.t1lo || w.t1hi != e.t1hi || w.t2 != e.t2)
      return fail("tab_words", int(c), 0, 0);
    ++cases;
  }
  // A compact codebook holds exactly the coefficients of the full one, record for record.
  for (auto kr : {std::pair<uint32_t, uint32_t>{20, 5}, {10, 3}, {7, 4}}) {
    const uint32_t k = kr.first, r = kr.second;
    std::vector<uint8_t> M, full, comp;
    qfec::parity_matrix(k, r, M);
    qfec::CodebookLayout Lf, Lc;
    qfec::codebook_layout(k, r, 2ull << 30, Lf);
    qfec::codebook_layout(k, r, 2ull << 30, Lc, true);
    qfec::build_codebook(Lf, M, full);
    qfec::build_codebook(Lc, M, comp);
    for (uint32_t e = 1; e <= r; ++e) {
      if (Lc.level_count[e] != Lf.level_count[e] || Lc.level_stride[e] % 32 != 0) return fail("compact layout", int(k), int(r), int(e));
      for (uint64_t i = 0; i < Lf.level_count[e]; ++i) {
        const uint8_t* a = full.data() + Lf.level_base[e] + i * Lf.level_stride[e];
        const uint8_t* b = comp.data() + Lc.level_base[e] + i * Lc.level_stride[e];
        if (std::memcmp(a, b, qfec::kRecordHeader) != 0) return fail("compact header", int(k), int(e), int(i));
        const CoefEntry* ent = reinterpret_cast<const CoefEntry*>(a + qfec::kRecordHeader);
        for (uint32_t t = 0; t < e * k; ++t)
          if (b[qfec::kRecordHeader + t] != ent[t].coef) return fail("compact coef", int(k), int(e), int(t));
      }
    }
    ++cases;
  }
  // every product of the multiply tables against the field definition
  for (int c = 0; c < 256; ++c) {
    const CoefEntry e = qfec::make_entry(uint8_t(c));
    for (int x = 0; x < 256; ++x) {
      const uint32_t w = uint32_t(x) * 0x01010101u;
      if (gmul(w, e) != uint32_t(qfec::gf().mul(uint8_t(c), uint8_t(x))) * 0x01010101u) return fail("gmul", c, x, 0);
    }
  }
  // decode_fused<..., INLINE>: choose_small (fec_kernels.hip, the inline classify's C(n, t)
  // for t <= 3, same unsigned wrap-around for n < t) against the binomial table classify reads
  for (uint32_t n = 0; n < 64; ++n)
    for (uint32_t t = 1; t <= 3; ++t) {
      const uint64_t a = n, b = n - 1u, c = n - 2u;
      const uint64_t v = t == 1u ? a : t == 2u ? (a * b) >> 1 : (a * b * c) / 6u;
      if (v != qfec::binom().c[n][t]) return fail("choose_small", int(n), int(t), 0);
    }
  // encode_bits (bitslice.hpp): the compiled-in matrix is gf256.hpp's, the transpose is an
  // involution, and 32-byte chunks of the bit-sliced encode equal the oracle's parity.
  if (bitslice_check<20, 5>(rng) || bitslice_check<10, 3>(rng) || bitslice_check<10, 2>(rng) ||
      bitslice_check<4, 4>(rng) || bitslice_check<7, 4>(rng) || bitslice_check<9, 6>(rng))
    return 1;
  cases += 6;
  const uint32_t shapes[][3] = {{4, 2, 256}, {10, 3, 1200}, {10, 1, 64}, {20, 5, 96}, {7, 4, 32}, {3, 8, 16}, {1, 1, 8}, {16, 16, 16}, {32, 8, 8}};
  for (const auto& sh : shapes) {
    const uint32_t k = sh[0], r = sh[1], P = sh[2];
    const uint64_t G = 40;
    std::vector<uint8_t> data(G * k * P), par(G * r * P), ref_par(G * r * P);
    oracle_fill_splitmix(data.data(), data.size(), 0x1000 + k * 64 + r, 0);
    std::vector<uint8_t> M;
    qfec::parity_matrix(k, r, M);
    std::vector<CoefEntry> tabs;
    for (uint32_t i = 1; i < r; ++i)
      for (uint32_t j = 0; j < k; ++j) tabs.push_back(qfec::make_entry(M[i * k + j]));
    // encode_v16 arithmetic (row 0 and column 0 XOR, the rest table lookups)
    for (uint64_t g = 0; g < G; ++g)
      for (uint32_t b = 0; b < P; b += 4)
        for (uint32_t i = 0; i < r; ++i) {
          uint32_t acc = ld32(&data[(g * k + 0) * P + b]);
          for (uint32_t j = 1; j < k; ++j) {
            const uint32_t x = ld32(&data[(g * k + j) * P + b]);
            acc ^= (i == 0) ? x : gmul(x, tabs[(i - 1) * k + j]);
          }
          st32(&par[(g * r + i) * P + b], acc);
        }
    oracle_rs_encode(data.data(), G, k, r, P, ref_par.data(), 1);
    if (par != ref_par) return fail("encode", k, r, P);
    ++cases;
    if (k + r > 64) continue;
    // decode: classify ranking + codebook records
    qfec::CodebookLayout L;
    const bool dense = qfec::codebook_layout(k, r, 2ull << 30, L);
    if (!dense && k + r <= 25) return fail("layout", k, r, P);
    std::vector<uint8_t> book;
    if (dense && !qfec::build_codebook(L, M, book)) return fail("codebook", k, r, P);
    for (int trial = 0; trial < 6; ++trial) {
      std::vector<uint64_t> masks(G);
      for (uint64_t g = 0; g < G; ++g) {
        uint64_t m = 0;
        const uint32_t ne = uint32_t(rng() % (r + 2));
        for (uint32_t t = 0; t < ne; ++t) m |= 1ull << (rng() % (k + r));
        masks[g] = m;
      }
      std::vector<uint8_t> mine = data, ref = data;
      for (uint64_t g = 0; g < G; ++g)
        for (uint32_t j = 0; j < k; ++j)
          if ((masks[g] >> j) & 1) {
            std::memset(&mine[(g * k + j) * P], 0xEE, P);
            std::memset(&ref[(g * k + j) * P], 0xEE, P);
          }
      std::vector<uint8_t> st(G);
      const int64_t bad_ref = oracle_rs_decode(ref.data(), ref_par.data(), masks.data(), G, k, r, P, st.data(), 1);
      int64_t bad = 0;
      std::vector<uint32_t> sro;
      std::vector<uint8_t> sst;
      if (!dense && !qfec::build_sparse_plan(k, r, M, masks.data(), G, 0xFFFFFFFFu, 0xFFFFFFFEu, book, sro, sst))
        return fail("sparse", k, r, P);
      for (uint64_t g = 0; g < G; ++g) {
        // classify (fec_kernels.hip)
        const uint64_t kmask = (1ull << k) - 1, rmask = (r >= 64) ? ~0ull : ((1ull << r) - 1);
        uint64_t dm = masks[g] & kmask;
        const uint64_t pm = (masks[g] >> k) & rmask;
        const uint32_t e = __builtin_popcountll(dm);
        if (e == 0) continue;
        if (e > r - __builtin_popcountll(pm)) {
          ++bad;
          if (st[g] != 1) return fail("status", k, r, int(g));
          continue;
        }
        uint64_t rank_e = 0, rank_r = 0;
        for (uint32_t t = 0; dm; ++t) {
          rank_e += qfec::binom().c[__builtin_ctzll(dm)][t + 1];
          dm &= dm - 1;
        }
        uint64_t sp = ~pm & rmask;
        for (uint32_t t = 0; t < e; ++t) {
          rank_r += qfec::binom().c[__builtin_ctzll(sp)][t + 1];
          sp &= sp - 1;
        }
        const uint64_t off = dense ? L.level_base[e] + (rank_e * qfec::binom().c[r][e] + rank_r) * L.level_stride[e]
                                   : uint64_t(sro[g]) * 32;
        if (!dense && sst[g] != 0) return fail("sparse-status", k, r, int(g));
        if (off % 32) return fail("align", k, r, int(g));
        const uint8_t* rec = &book[off];
        if (rec[96] != e) return fail("record-e", k, r, int(g));
        // decode_fused<..., DIRECT>: survivor / erased ids from the mask must be the record's
        {
          const uint64_t lost = masks[g] & kmask;
          uint64_t alive = ~(masks[g] >> k) & rmask, rsel = 0;
          for (uint32_t t = 0; t < e; ++t) {
            rsel |= alive & (~alive + 1);
            alive &= alive - 1;
          }
          uint64_t surv = (~lost & kmask) | (rsel << k);
          for (uint32_t s = 0; s < k; ++s) {
            if (uint32_t(__builtin_ctzll(surv)) != rec[s]) return fail("direct-survivor", k, r, int(g));
            surv &= surv - 1;
          }
          uint64_t x = lost;
          for (uint32_t m = 0; m < e; ++m, x &= x - 1)
            if (uint32_t(__builtin_ctzll(x)) != rec[64 + m]) return fail("direct-erased", k, r, int(g));
          const bool xor_only = e == 1 && ((~(masks[g] >> k) & rmask) & 1u);
          if (xor_only != (rec[97] != 0)) return fail("direct-xor-only", k, r, int(g));
        }
        const CoefEntry* T = reinterpret_cast<const CoefEntry*>(rec + qfec::kRecordHeader);
        for (uint32_t b = 0; b < P; b += 4)
          for (uint32_t m = 0; m < e; ++m) {
            uint32_t acc = 0;
            for (uint32_t s = 0; s < k; ++s) {
              const uint32_t sid = rec[s];
              const uint32_t x = sid < k ? ld32(&data[(g * k + sid) * P + b]) : ld32(&ref_par[(g * r + sid - k) * P + b]);
              if ((sid < k) && ((masks[g] >> sid) & 1)) return fail("survivor-erased", k, r, int(g));
              const CoefEntry& t = T[m * k + s];
              acc ^= (t.coef == 1) ? x : (t.coef == 0 ? 0 : gmul(x, t));
            }
            st32(&mine[(g * k + rec[64 + m]) * P + b], acc);
          }
      }
      if (bad != bad_ref) return fail("bad-count", k, r, int(bad));
      if (mine != ref) return fail("decode", k, r, trial);
      ++cases;
    }
  }
  std::printf("OK %d\n", cases);
  return 0;
}
