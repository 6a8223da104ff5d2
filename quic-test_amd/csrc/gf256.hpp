// gf256.hpp — host-side GF(2^8) arithmetic and plan construction for libfec_hip.
//
// The reference FEC (internal/fec/fec_xor_simd.cpp) is XOR only.  This file defines the
// erasure code the GPU library computes (SURVEY.md §8(a) "code definition"):
//   GF(2^8) with polynomial x^8+x^4+x^3+x^2+1 (0x11D), generator 2;
//   parity matrix M (r x k): Cauchy 1/(x_i ^ y_j), x_i = i, y_j = r + j, then every
//   column divided by its row-0 entry (row 0 = all ones = the reference XOR row) and
//   every row i >= 1 divided by its column-0 entry (column 0 = all ones).
//
// GPU multiply tables ("coefficient entries"): multiplying a byte x by a constant c is
// linear over GF(2), so c*x = c*(x & 7) ^ c*(x & 0x38) ^ c*(x & 0xC0).  Each of the three
// pieces indexes a table of <= 8 bytes, which is exactly what one v_perm_b32 can look up
// for four bytes at once (selector bytes 0..7 pick bytes of a 64-bit {hi, lo} pair).
#pragma once

#include <cstdint>
#include <cstring>
#include <map>
#include <utility>
#include <vector>

namespace qfec {

struct GF256 {
  uint8_t exp[512];
  uint8_t log[256];
  GF256() {
    unsigned x = 1;
    for (int i = 0; i < 255; ++i) {
      exp[i] = static_cast<uint8_t>(x);
      log[x] = static_cast<uint8_t>(i);
      x <<= 1;
      if (x & 0x100) x ^= 0x11D;
    }
    for (int i = 255; i < 512; ++i) exp[i] = exp[i - 255];
    log[0] = 0;
  }
  uint8_t mul(uint8_t a, uint8_t b) const {
    return (a && b) ? exp[log[a] + log[b]] : 0;
  }
  uint8_t inv(uint8_t a) const { return a ? exp[255 - log[a]] : 0; }
};

inline const GF256& gf() {
  static const GF256 g;
  return g;
}

// One coefficient's GPU lookup tables, 32 bytes (one s_load_dwordx8).
struct CoefEntry {
  uint32_t t0lo, t0hi;  // c * v        for v = 0..7  (bits 0..2 of x)
  uint32_t t1lo, t1hi;  // c * (v << 3) for v = 0..7  (bits 3..5)
  uint32_t t2;          // c * (v << 6) for v = 0..3  (bits 6..7)
  uint32_t coef;        // c itself (0 / 1 take cheaper paths)
  uint32_t pad0, pad1;
};
static_assert(sizeof(CoefEntry) == 32, "CoefEntry must be 32 bytes");

inline CoefEntry make_entry(uint8_t c) {
  const GF256& g = gf();
  uint8_t t0[8], t1[8], t2[4];
  for (int v = 0; v < 8; ++v) {
    t0[v] = g.mul(c, static_cast<uint8_t>(v));
    t1[v] = g.mul(c, static_cast<uint8_t>(v << 3));
  }
  for (int v = 0; v < 4; ++v) t2[v] = g.mul(c, static_cast<uint8_t>(v << 6));
  auto pack = [](const uint8_t* b) {
    return uint32_t(b[0]) | uint32_t(b[1]) << 8 | uint32_t(b[2]) << 16 | uint32_t(b[3]) << 24;
  };
  CoefEntry e;
  e.t0lo = pack(t0);
  e.t0hi = pack(t0 + 4);
  e.t1lo = pack(t1);
  e.t1hi = pack(t1 + 4);
  e.t2 = pack(t2);
  e.coef = c;
  e.pad0 = e.pad1 = 0;
  return e;
}

// r x k parity matrix, row-major.  false if k == 0, r == 0 or k + r > 256.
inline bool parity_matrix(uint32_t k, uint32_t r, std::vector<uint8_t>& M) {
  if (k == 0 || r == 0 || k + r > 256) return false;
  const GF256& g = gf();
  M.assign(size_t(k) * r, 0);
  for (uint32_t i = 0; i < r; ++i)
    for (uint32_t j = 0; j < k; ++j) M[i * k + j] = g.inv(static_cast<uint8_t>(i ^ (r + j)));
  for (uint32_t j = 0; j < k; ++j) {
    const uint8_t s = g.inv(M[j]);
    for (uint32_t i = 0; i < r; ++i) M[i * k + j] = g.mul(M[i * k + j], s);
  }
  for (uint32_t i = 1; i < r; ++i) {
    const uint8_t s = g.inv(M[i * k]);
    for (uint32_t j = 0; j < k; ++j) M[i * k + j] = g.mul(M[i * k + j], s);
  }
  return true;
}

// Invert n x n (row-major) in place into `out`.  false if singular.
inline bool invert(std::vector<uint8_t> A, uint32_t n, std::vector<uint8_t>& out) {
  const GF256& g = gf();
  out.assign(size_t(n) * n, 0);
  for (uint32_t i = 0; i < n; ++i) out[i * n + i] = 1;
  for (uint32_t c = 0; c < n; ++c) {
    uint32_t p = c;
    while (p < n && A[p * n + c] == 0) ++p;
    if (p == n) return false;
    if (p != c)
      for (uint32_t j = 0; j < n; ++j) {
        std::swap(A[c * n + j], A[p * n + j]);
        std::swap(out[c * n + j], out[p * n + j]);
      }
    const uint8_t s = g.inv(A[c * n + c]);
    for (uint32_t j = 0; j < n; ++j) {
      A[c * n + j] = g.mul(A[c * n + j], s);
      out[c * n + j] = g.mul(out[c * n + j], s);
    }
    for (uint32_t i = 0; i < n; ++i) {
      const uint8_t f = A[i * n + c];
      if (i == c || f == 0) continue;
      for (uint32_t j = 0; j < n; ++j) {
        A[i * n + j] ^= g.mul(f, A[c * n + j]);
        out[i * n + j] ^= g.mul(f, out[c * n + j]);
      }
    }
  }
  return true;
}

// Binomial coefficients C(n, m), n <= 64, m <= 64 (saturating at UINT64_MAX).
struct Binom {
  uint64_t c[65][65];
  Binom() {
    std::memset(c, 0, sizeof(c));
    for (int n = 0; n <= 64; ++n) {
      c[n][0] = 1;
      for (int m = 1; m <= n; ++m) {
        const uint64_t a = c[n - 1][m - 1], b = (m <= n - 1) ? c[n - 1][m] : 0;
        c[n][m] = (a > UINT64_MAX - b) ? UINT64_MAX : a + b;
      }
    }
  }
};
inline const Binom& binom() {
  static const Binom b;
  return b;
}

// Colex rank of a sorted subset {c_0 < c_1 < ...}: sum_t C(c_t, t+1).
inline uint64_t colex_rank(const uint32_t* c, uint32_t n) {
  uint64_t r = 0;
  for (uint32_t t = 0; t < n; ++t) r += binom().c[c[t]][t + 1];
  return r;
}

// ---------------------------------------------------------------------------------
// Decode codebook.  One record per recoverable pattern (E, R): E = erased data shards
// (|E| = e, 1 <= e <= r), R = the e lowest surviving parity rows used to rebuild them.
// Pattern index inside level e = rank(E) * C(r, e) + rank(R).
//
// Record (all offsets in bytes, records 32-byte aligned):
//   [0, 64)    survivor shard ids, k bytes: surviving data shards ascending, then k+R_t
//   [64, 96)   erased data shard ids E_0 < ... < E_{e-1}
//   [96]       e
//   [97]       1 if every coefficient is 1 (single loss rebuilt from parity row 0: XOR)
//   [128, ...) e x k CoefEntry, row m (output E_m) major, survivor slot s minor
//              (compact books: e x k coefficient bytes instead, same order, padded to 32;
//              the kernels that read them compute the tables, coef_tables.hpp)
//
// Rebuild (syndrome form): with Inv = (M[R][E])^-1,
//   d_{E_m} = sum_t Inv[m][t] * p_{R_t}  ^  sum_{j in S} (sum_t Inv[m][t] * M[R_t][j]) * d_j
// which is the unique solution for the chosen survivors, i.e. the same linear map as
// inverting the full k x k survivor submatrix of [I ; M].
// ---------------------------------------------------------------------------------
constexpr uint32_t kRecordHeader = 128;
constexpr uint32_t kMaxDecodeShards = 64;  // k + r <= 64 (u64 erasure masks)

struct CodebookLayout {
  uint32_t k = 0, r = 0;
  bool compact = false;                                  // coefficient bytes, not CoefEntry
  uint64_t level_base[kMaxDecodeShards + 1] = {};   // byte offset of level e
  uint64_t level_stride[kMaxDecodeShards + 1] = {}; // record bytes at level e
  uint64_t level_count[kMaxDecodeShards + 1] = {};  // records at level e
  uint64_t total_bytes = 0;
};

inline uint64_t record_bytes(uint32_t k, uint32_t e, bool compact = false) {
  return kRecordHeader + (compact ? (uint64_t(e) * k + 31) / 32 * 32 : uint64_t(e) * k * sizeof(CoefEntry));
}

inline bool codebook_layout(uint32_t k, uint32_t r, uint64_t cap_bytes, CodebookLayout& L, bool compact = false) {
  if (k == 0 || r == 0 || k + r > kMaxDecodeShards) return false;
  L = CodebookLayout();
  L.k = k;
  L.r = r;
  L.compact = compact;
  uint64_t off = 0;
  for (uint32_t e = 1; e <= r && e <= k; ++e) {
    const uint64_t ce = binom().c[k][e], cr = binom().c[r][e];
    if (ce == UINT64_MAX || cr == UINT64_MAX) return false;
    const long double cnt = (long double)ce * (long double)cr;
    const uint64_t stride = record_bytes(k, e, compact);
    if (cnt * stride + off > (long double)cap_bytes) return false;
    L.level_base[e] = off;
    L.level_stride[e] = stride;
    L.level_count[e] = ce * cr;
    off += ce * cr * stride;
  }
  L.total_bytes = off;
  return true;
}

// Visit all e-subsets of [0, n) in lexicographic order.
template <class F>
inline void for_each_subset(uint32_t n, uint32_t e, F&& f) {
  if (e > n) return;
  uint32_t c[kMaxDecodeShards];
  for (uint32_t t = 0; t < e; ++t) c[t] = t;
  while (true) {
    f(static_cast<const uint32_t*>(c));
    int t = int(e) - 1;
    while (t >= 0 && c[t] == n - e + uint32_t(t)) --t;
    if (t < 0) return;
    ++c[t];
    for (uint32_t u = uint32_t(t) + 1; u < e; ++u) c[u] = c[u - 1] + 1;
  }
}

// Write the record of pattern (E, R) (sorted, |E| = |R| = e) at `rec` (record_bytes(k, e)
// bytes, zeroed by the caller).  false on a singular submatrix (cannot happen for this
// Cauchy construction; kept as a guard).
inline bool build_record(uint32_t k, const std::vector<uint8_t>& M, const uint32_t* E, const uint32_t* R,
                         uint32_t e, uint8_t* rec, bool compact = false) {
  const GF256& g = gf();
  // survivors: data not in E ascending, then parity rows R
  uint32_t ns = 0;
  uint32_t surv[kMaxDecodeShards];
  for (uint32_t j = 0, t = 0; j < k; ++j) {
    if (t < e && E[t] == j) {
      ++t;
      continue;
    }
    surv[ns++] = j;
  }
  for (uint32_t t = 0; t < e; ++t) surv[ns++] = k + R[t];
  for (uint32_t s = 0; s < k; ++s) rec[s] = static_cast<uint8_t>(surv[s]);
  for (uint32_t t = 0; t < e; ++t) rec[64 + t] = static_cast<uint8_t>(E[t]);
  rec[96] = static_cast<uint8_t>(e);
  std::vector<uint8_t> sub(size_t(e) * e, 0), inv;
  for (uint32_t a = 0; a < e; ++a)
    for (uint32_t b = 0; b < e; ++b) sub[a * e + b] = M[R[a] * k + E[b]];
  if (!invert(sub, e, inv)) return false;
  bool all_one = true;
  CoefEntry* ent = reinterpret_cast<CoefEntry*>(rec + kRecordHeader);
  for (uint32_t m = 0; m < e; ++m) {
    for (uint32_t s = 0; s < k; ++s) {
      uint8_t c = 0;
      if (surv[s] < k) {
        for (uint32_t t = 0; t < e; ++t) c ^= g.mul(inv[m * e + t], M[R[t] * k + surv[s]]);
      } else {
        c = inv[m * e + (s - (k - e))];
      }
      all_one &= (c == 1);
      if (compact) {
        rec[kRecordHeader + m * k + s] = c;
      } else {
        ent[m * k + s] = make_entry(c);
      }
    }
  }
  rec[97] = all_one ? 1 : 0;
  return true;
}

// Fill `out` (L.total_bytes) with every record.
inline bool build_codebook(const CodebookLayout& L, const std::vector<uint8_t>& M,
                           std::vector<uint8_t>& out) {
  const uint32_t k = L.k, r = L.r;
  out.assign(L.total_bytes, 0);
  bool ok = true;
  for (uint32_t e = 1; e <= r && e <= k; ++e) {
    const uint64_t cr = binom().c[r][e];
    for_each_subset(k, e, [&](const uint32_t* E) {
      const uint64_t rankE = colex_rank(E, e);
      for_each_subset(r, e, [&](const uint32_t* R) {
        const uint64_t idx = rankE * cr + colex_rank(R, e);
        ok &= build_record(k, M, E, R, e, out.data() + L.level_base[e] + idx * L.level_stride[e], L.compact);
      });
    });
  }
  return ok;
}

// Sparse plan: records only for the patterns present in one batch of masks (used when the
// dense codebook would exceed its cap).  rec_off[g] = record offset / 32, or the kRec*
// markers of fec_kernels.hpp (passed in as none / bad); status[g] = 1 if unrecoverable.
inline bool build_sparse_plan(uint32_t k, uint32_t r, const std::vector<uint8_t>& M, const uint64_t* masks,
                              uint64_t G, uint32_t rec_none, uint32_t rec_bad, std::vector<uint8_t>& book,
                              std::vector<uint32_t>& rec_off, std::vector<uint8_t>& status) {
  book.clear();
  rec_off.assign(G, rec_none);
  status.assign(G, 0);
  const uint64_t kmask = k >= 64 ? ~0ull : ((1ull << k) - 1);
  const uint64_t rmask = r >= 64 ? ~0ull : ((1ull << r) - 1);
  std::map<std::pair<uint64_t, uint64_t>, uint32_t> seen;
  for (uint64_t g = 0; g < G; ++g) {
    const uint64_t dm = masks[g] & kmask;
    if (!dm) continue;
    const uint64_t pm = k >= 64 ? 0 : (masks[g] >> k) & rmask;
    const uint32_t e = static_cast<uint32_t>(__builtin_popcountll(dm));
    if (e > r - static_cast<uint32_t>(__builtin_popcountll(pm))) {
      rec_off[g] = rec_bad;
      status[g] = 1;
      continue;
    }
    uint64_t rsel = 0, alive = ~pm & rmask;
    for (uint32_t t = 0; t < e; ++t) {
      rsel |= alive & (~alive + 1);  // lowest surviving parity row
      alive &= alive - 1;
    }
    auto key = std::make_pair(dm, rsel);
    auto it = seen.find(key);
    if (it == seen.end()) {
      uint32_t E[kMaxDecodeShards], R[kMaxDecodeShards];
      uint32_t ne = 0, nr = 0;
      for (uint64_t x = dm; x; x &= x - 1) E[ne++] = static_cast<uint32_t>(__builtin_ctzll(x));
      for (uint64_t x = rsel; x; x &= x - 1) R[nr++] = static_cast<uint32_t>(__builtin_ctzll(x));
      const uint64_t off = book.size();
      if ((off >> 5) >= rec_bad) return false;
      book.resize(off + record_bytes(k, e), 0);
      if (!build_record(k, M, E, R, e, book.data() + off)) return false;
      it = seen.emplace(key, static_cast<uint32_t>(off >> 5)).first;
    }
    rec_off[g] = it->second;
  }
  return true;
}

}  // namespace qfec
