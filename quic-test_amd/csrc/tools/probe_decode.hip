// probe_decode.hip — development probe: decode kernel variants A/B in one process, each
// verified to rebuild the poisoned shards exactly.  Not part of the library.
#include "../fec_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <random>
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
__global__ void poison(uint8_t* data, const uint64_t* masks, uint64_t groups, uint32_t k, uint32_t P) {
  const uint64_t t = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  const uint64_t g = t / (uint64_t(k) * P);
  if (g >= groups) return;
  const uint32_t j = uint32_t((t / P) % k);
  if ((masks[g] >> j) & 1) data[t] = 0xEE;
}
// Write-layout probe (k=10 r=3, 1200 B): one wave per group loads its 10 survivors (the mask's
// surviving data shards, then the lowest surviving parity rows, as the mask-addressed recover
// does), XORs them (the GF arithmetic is free at this size, r01/r02 probes) and stores the
// result as each of its e rebuilt rows, either at the recover API's slots (g*3 + m)*P
// (PACKED = 0) or back to back over all groups, row pre[g] + m (PACKED = 1: no gaps between
// groups' rows).  Timing only: the bytes are not the recovered packets.
template <int PACKED>
__global__ __launch_bounds__(256) void wr_layout(const uint8_t* __restrict__ data, const uint8_t* __restrict__ parity,
                                                 const uint64_t* __restrict__ masks, const uint32_t* __restrict__ pre,
                                                 uint8_t* __restrict__ out, uint64_t groups) {
  constexpr uint32_t K = 10, R = 3, P = 1200;
  const uint64_t g = uint64_t(blockIdx.x) * 4 + (threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63u;
  if (g >= groups) return;
  const uint64_t m = masks[g];
  const uint64_t lost = m & 0x3FFu;
  const uint32_t e = uint32_t(__popcll(lost));
  if (e == 0 || e > R - uint32_t(__popcll((m >> K) & 7u))) return;
  uint64_t alive = ~(m >> K) & 7u, rsel = 0;
  for (uint32_t t = 0; t < e; ++t) {
    rsel |= alive & (~alive + 1);
    alive &= alive - 1;
  }
  uint64_t surv = (~lost & 0x3FFu) | (rsel << K);
  const uint8_t* dg = data + g * K * P;
  const uint8_t* pg = parity + g * R * P;
  uint32_t toff = 1024u + lane * 4u;
  if (toff + 4u > P) toff = P - 4u;
  u32x4 a = {0u, 0u, 0u, 0u};
  uint32_t t4 = 0;
#pragma unroll
  for (int s = 0; s < int(K); ++s) {
    const uint32_t sid = uint32_t(__builtin_ctzll(surv));
    surv &= surv - 1;
    const uint8_t* src = sid < K ? dg + sid * P : pg + (sid - K) * P;
    a ^= __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(src + lane * 16u));
    t4 ^= __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(src + toff));
  }
  for (uint32_t i = 0; i < e; ++i) {
    uint8_t* dst = out + (PACKED ? uint64_t(pre[g]) + i : g * R + i) * P;
    __builtin_nontemporal_store(a, reinterpret_cast<u32x4*>(dst + lane * 16u));
    __builtin_nontemporal_store(t4, reinterpret_cast<uint32_t*>(dst + toff));
  }
}
}  // namespace
}  // namespace qfec

using namespace qfec;

int main(int argc, char** argv) {
  const uint32_t k = argc > 3 ? std::atoi(argv[3]) : 10, r = argc > 4 ? std::atoi(argv[4]) : 3;
  const uint32_t P = argc > 6 ? std::atoi(argv[6]) : 1200;
  const double loss = argc > 7 ? std::atof(argv[7]) : 0.0;  // > 0: iid loss per shard instead
  const uint32_t ners = argc > 5 ? std::atoi(argv[5]) : 2;
  const uint64_t G = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1000000;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 7;
  const uint64_t nd = G * k * P, np = G * r * P;
  uint8_t *data, *orig, *par;
  uint64_t* masks;
  uint32_t* rec;
  CK(hipMalloc(&data, nd));
  CK(hipMalloc(&orig, nd));
  CK(hipMalloc(&par, np));
  CK(hipMalloc(&masks, G * 8));
  CK(hipMalloc(&rec, G * 4));
  CK(launch_fill_splitmix(data, nd, 0x5EED0002, 0, nullptr));
  std::vector<uint8_t> M;
  parity_matrix(k, r, M);
  std::vector<CoefEntry> tab;
  for (uint32_t i = 1; i < r; ++i)
    for (uint32_t j = 0; j < k; ++j) tab.push_back(make_entry(M[i * k + j]));
  void* dtab = nullptr;
  if (!tab.empty()) {
    CK(hipMalloc(&dtab, tab.size() * 32));
    CK(hipMemcpy(dtab, tab.data(), tab.size() * 32, hipMemcpyHostToDevice));
  }
  EncodeLaunch el{data, nullptr, OffsetKind::kNone, par, G, k, r, P, dtab};
  CK(launch_encode(el, nullptr));
  CK(hipMemcpy(orig, data, nd, hipMemcpyDeviceToDevice));
  // exactly `ners` erasures per group, uniform over the k + r shards
  std::vector<uint64_t> hm(G);
  std::mt19937_64 rng(0x5EED0003);
  uint64_t alg = 0;
  for (uint64_t g = 0; g < G; ++g) {
    uint64_t m = 0;
    if (loss > 0) {  // resampled until recoverable, so every poisoned group is rebuilt
      do {
        m = 0;
        for (uint32_t j = 0; j < k + r; ++j)
          if (double(rng() >> 11) * 0x1.0p-53 < loss) m |= 1ull << j;
      } while (uint32_t(__builtin_popcountll(m & ((1ull << k) - 1))) > r - uint32_t(__builtin_popcountll((m >> k) & ((1ull << r) - 1))));
    } else {
      while (uint32_t(__builtin_popcountll(m)) < ners) m |= 1ull << (rng() % (k + r));
    }
    hm[g] = m;
    const uint32_t e = __builtin_popcountll(m & ((1ull << k) - 1));
    const uint32_t alive = r - __builtin_popcountll((m >> k) & ((1ull << r) - 1));
    if (e && e <= alive) alg += uint64_t(k + e) * P;
  }
  CK(hipMemcpy(masks, hm.data(), G * 8, hipMemcpyHostToDevice));
  CodebookLayout L;
  codebook_layout(k, r, 2ull << 30, L);
  std::vector<uint8_t> book;
  build_codebook(L, M, book);
  uint8_t* dbook;
  uint64_t* dbin;
  CK(hipMalloc(&dbook, book.size()));
  CK(hipMemcpy(dbook, book.data(), book.size(), hipMemcpyHostToDevice));
  CK(hipMalloc(&dbin, sizeof(binom().c)));
  CK(hipMemcpy(dbin, binom().c, sizeof(binom().c), hipMemcpyHostToDevice));
  DecodeLaunch dl;
  dl.data = data;
  dl.parity = par;
  dl.masks = masks;
  dl.rec_off = rec;
  dl.status = nullptr;
  dl.codebook = dbook;
  dl.binom = dbin;
  std::memset(&dl.meta, 0, sizeof(dl.meta));
  for (uint32_t e = 1; e <= 32; ++e) {
    dl.meta.base[e] = L.level_base[e];
    dl.meta.stride[e] = L.level_stride[e];
    dl.meta.count_r[e] = binom().c[r][e];
  }
  dl.groups = G;
  dl.k = k;
  dl.r = r;
  dl.P = P;
  // compact (coefficient-byte) book of the same patterns, for the forms that read one
  CodebookLayout Lc;
  codebook_layout(k, r, 2ull << 30, Lc, true);
  std::vector<uint8_t> cbook_h;
  build_codebook(Lc, M, cbook_h);
  uint8_t* cbook;
  CK(hipMalloc(&cbook, cbook_h.size()));
  CK(hipMemcpy(cbook, cbook_h.data(), cbook_h.size(), hipMemcpyHostToDevice));
  auto with_book = [&, cbook, Lc](DecodeLaunch a, bool compact) {  // the book a form reads
    a.compact_tables = compact;
    if (compact) {
      a.codebook = cbook;
      for (uint32_t e = 1; e <= 32; ++e) {
        a.meta.base[e] = Lc.level_base[e];
        a.meta.stride[e] = Lc.level_stride[e];
      }
    }
    return a;
  };
  struct Var {
    std::string name;
    int variant;
    int waves;
    int swz;
    std::vector<float> ms;
    std::function<hipError_t(const DecodeLaunch&)> fn = nullptr;  // custom launch (no check)
  };
  std::vector<Var> vars = {{"wave nt xcd", kDecodeWaveNt, -1, 1, {}},
                           {"auto (library default)", kDecodeAuto, 0, -1, {}},
                           {"fused nt xcd", kDecodeFused, -1, 1, {}},
                           {"direct xcd", kDecodeFusedDirect, -1, 1, {}},
                           {"direct xcd cap16", kDecodeFusedDirect, 16, 1, {}},
                           {"direct", kDecodeFusedDirect, -1, 0, {}}};
  if (loss > 0) {  // sparse-loss runs: the library forms only
    std::vector<Var> keep;
    for (auto& v : vars)
      if (v.name.rfind("auto", 0) == 0 || v.name.rfind("direct xcd", 0) == 0) keep.push_back(v);
    vars.swap(keep);
  }
  uint8_t* oop = nullptr;  // separate output buffer for the out-of-place probe
  CK(hipMalloc(&oop, nd));
  auto probe = [](const DecodeLaunch& a) -> hipError_t {
    hipLaunchKernelGGL(classify, dim3(blocks_for(a.groups)), dim3(256), 0, nullptr, a.masks, a.groups, a.k, a.r,
                       a.binom, a.meta, a.rec_off, a.status);
    return hipSuccess;
  };
  if (P < 1024) vars.push_back({"tiled nt", kDecodeTiledNt, -1, -1, {}});
#define PF(NAME, NT)                                                                             \
  {                                                                                              \
  vars.push_back({NAME, kDecodeFused, -1, 1, {}, [probe](const DecodeLaunch& a) {                \
                    probe(a);                                                                    \
                    return run_decode_fused<10, 3, kNtStore, 0, NT, true>(a, nullptr);           \
                  }});                                                                           \
  vars.push_back({NAME " nt-load", kDecodeFused, -1, 1, {}, [probe](const DecodeLaunch& a) {     \
                    probe(a);                                                                    \
                    return run_decode_fused<10, 3, kNtStore | kNtLoad, 0, NT, true>(a, nullptr); \
                  }});                                                                           \
  }
  if (k == 10 && r == 3 && P <= 256) PF("fused direct 4B x1", 1)
  if (k == 10 && r == 3 && P > 256 && P <= 512) PF("fused direct 4B x2", 2)
  if (k == 10 && r == 3 && P > 512 && P <= 768) PF("fused direct 4B x3", 3)
  if (k == 10 && r == 3 && P > 768 && P <= 1024) PF("fused direct 4B x4", 4)
#define PVD(NAME, CAP, POLF, NM, NT)                                                             \
  vars.push_back({NAME, kDecodeFused, CAP, 1, {}, [probe](const DecodeLaunch& a) {               \
                    probe(a);                                                                    \
                    return run_decode_fused<10, 3, (POLF), NM, NT, true>(a, nullptr);            \
                  }});
  if (k == 10 && r == 3 && P > 1280 && P <= 1536) {
    PVD("pol direct nt-store", -1, kNtStore, 1, 2)
    PVD("pol direct nt-load+store", -1, kNtStore | kNtLoad, 1, 2)
  }
  if (k == 10 && r == 3 && P == 1200) {
    PVD("pol direct nt-store", -1, kNtStore, 1, 1)
    PVD("pol direct nt-load+store", -1, kNtStore | kNtLoad, 1, 1)
    vars.push_back({"pol direct classify-launch", kDecodeFused, -1, 1, {}, [probe](const DecodeLaunch& a) {
                      probe(a);  // the previous form: classify kernel, then rec_off
                      return run_decode_fused<10, 3, kNtStore | kNtLoad, 1, 1, true, false>(a, nullptr);
                    }});
    vars.push_back({"pol direct inline-only", kDecodeFused, -1, 1, {}, [](const DecodeLaunch& a) {
                      return run_decode_fused<10, 3, kNtStore | kNtLoad, 1, 1, true, true>(a, nullptr);
                    }});
    PVD("pol direct nt-load", -1, kNtLoad, 1, 1)
    PVD("pol direct plain", -1, 0, 1, 1)
    PVD("pol direct nt-load+store cap12", 12, kNtStore | kNtLoad, 1, 1)
    vars.push_back({"pol encode (same buffers)", kDecodeFused, -1, 1, {}, [el](const DecodeLaunch&) {
                      return launch_encode(el, nullptr);  // rewrites identical parity
                    }});
    vars.push_back({"pol out-of-place", kDecodeFused, -1, 1, {}, [probe, oop](const DecodeLaunch& a) {
                      probe(a);
                      DecodeLaunch b = a;
                      b.out = oop;
                      return run_decode_fused<10, 3, kNtStore, 1, 1, true>(b, nullptr);
                    }});
  }
  // rebuilt packets written out of place, compact (group g's rows at (g*3+m)*P): the write
  // pattern of encode's parity instead of scattered in-place packets.  Unchecked (out of place).
  uint8_t* cout = nullptr;
  if (k == 10 && r == 3 && P == 1200) {
    CK(hipMalloc(&cout, G * 3 * P));
    vars.push_back({"compact-out", kDecodeFused, -1, 1, {}, [cout](const DecodeLaunch& a) {
                      DecodeLaunch b = a;
                      b.out = cout;
                      b.rec_off = nullptr;  // the inline forms read packed row starts from rec_off
                      return run_decode_fused<10, 3, kNtStore | kNtLoad | kCompactOut, 1, 1, true>(b, nullptr);
                    }});
    vars.push_back({"in-place same form", kDecodeFused, -1, 1, {}, [](const DecodeLaunch& a) {
                      return run_decode_fused<10, 3, kNtStore | kNtLoad, 1, 1, true>(a, nullptr);
                    }});
  }
  // write-layout probe: the recover API's slots vs rows packed back to back (prefix sums)
  if (k == 10 && r == 3 && P == 1200) {
    std::vector<uint32_t> hpre(G);
    uint32_t acc = 0;
    for (uint64_t g = 0; g < G; ++g) {
      hpre[g] = acc;
      acc += uint32_t(__builtin_popcountll(hm[g] & 0x3FFu));
    }
    uint32_t* dpre = nullptr;
    CK(hipMalloc(&dpre, G * 4));
    CK(hipMemcpy(dpre, hpre.data(), G * 4, hipMemcpyHostToDevice));
    uint8_t* wout = nullptr;
    CK(hipMalloc(&wout, G * 3 * P));
    const uint32_t wb = uint32_t((G + 3) / 4);
    vars.push_back({"wr slots", kDecodeFused, -1, 1, {}, [=](const DecodeLaunch& a) {
                      hipLaunchKernelGGL(wr_layout<0>, dim3(wb), dim3(256), 0, nullptr, a.data, a.parity, a.masks, dpre, wout, a.groups);
                      return hipGetLastError();
                    }});
    vars.push_back({"wr packed", kDecodeFused, -1, 1, {}, [=](const DecodeLaunch& a) {
                      hipLaunchKernelGGL(wr_layout<1>, dim3(wb), dim3(256), 0, nullptr, a.data, a.parity, a.masks, dpre, wout, a.groups);
                      return hipGetLastError();
                    }});
  }
  // SCAN groups per wave (mask-addressed inline form): sparse loss without a wave per group
#define PSCAN(T)                                                                                 \
  vars.push_back({"scan" #T, kDecodeFused, -1, 1, {}, [](const DecodeLaunch& a) {               \
                    return run_decode_fused<10, 3, kNtStore | kNtLoad, 1, 1, true, true, T>(a, nullptr); \
                  }});
  if (k == 10 && r == 3 && P == 1200) {
    PSCAN(2) PSCAN(4) PSCAN(8) PSCAN(16) PSCAN(32) PSCAN(64)
    PSCAN(256) PSCAN(512) PSCAN(1024)
    vars.push_back({"scan8 compact-out", kDecodeFused, -1, 1, {}, [cout](const DecodeLaunch& a) {
                      DecodeLaunch b = a;
                      b.out = cout;
                      b.rec_off = nullptr;  // the inline forms read packed row starts from rec_off
                      return run_decode_fused<10, 3, kNtStore | kNtLoad | kCompactOut, 1, 1, true, true, 8>(b, nullptr);
                    }});
  }
  // record-addressed fused form with the coefficient tables staged through LDS (kLdsTabs)
#define PLDS(KK, RR, NMM, NTT)                                                                    \
  if (k == KK && r == RR && P / 1024 == NMM && (P % 1024 + 255) / 256 == NTT) {                   \
    vars.push_back({"lds-tabs", kDecodeFused, -1, 1, {}, [probe](const DecodeLaunch& a) {         \
                      probe(a);                                                                   \
                      return run_decode_fused<KK, RR, kNtStore | kLdsTabs, NMM, NTT, false>(a, nullptr); \
                    }});                                                                          \
    vars.push_back({"lds-tabs nt-load", kDecodeFused, -1, 1, {}, [probe](const DecodeLaunch& a) { \
                      probe(a);                                                                   \
                      return run_decode_fused<KK, RR, kNtStore | kNtLoad | kLdsTabs, NMM, NTT, false>(a, nullptr); \
                    }});                                                                          \
    vars.push_back({"lds-tabs xcd0", kDecodeFused, -1, 0, {}, [probe](const DecodeLaunch& a) {    \
                      probe(a);                                                                   \
                      return run_decode_fused<KK, RR, kNtStore | kLdsTabs, NMM, NTT, false>(a, nullptr); \
                    }});                                                                          \
  }
  PLDS(20, 5, 1, 1)
  PLDS(10, 3, 1, 1)
  if (k == 20 && r == 5 && P == 1200) {
    vars.push_back({"coef-bytes", kDecodeFused, -1, 1, {}, [probe, with_book](const DecodeLaunch& a) {
                      const DecodeLaunch b = with_book(a, true);
                      probe(b);
                      return run_decode_fused<20, 5, kNtStore | kLdsTabs | kCoefBytes, 1, 1, false>(b, nullptr);
                    }});
    vars.push_back({"coef-bytes nt-load", kDecodeFused, -1, 1, {}, [probe, with_book](const DecodeLaunch& a) {
                      const DecodeLaunch b = with_book(a, true);
                      probe(b);
                      return run_decode_fused<20, 5, kNtStore | kNtLoad | kLdsTabs | kCoefBytes, 1, 1, false>(b, nullptr);
                    }});
  }
  if (k == 10 && r == 3 && P == 1200) {
    vars.push_back({"winbody direct w6 lds", kDecodeFused, -1, 1, {}, [](const DecodeLaunch& a) {
                      return run_decode_fused<10, 3, kNtStore | kNtLoad | kLdsTabs, 1, 1, true>(a, nullptr);
                    }});
  }
  // runtime-k wave kernel (any k, r): tables through the scalar cache vs through LDS
  vars.push_back({"wave0 scalar", kDecodeFused, -1, 1, {}, [probe](const DecodeLaunch& a) {
                    probe(a);
                    return run_decode_wave<0, 8, kNtStore>(a, nullptr);
                  }});
  vars.push_back({"wave0 nobranch", kDecodeFused, -1, 1, {}, [probe](const DecodeLaunch& a) {
                    probe(a);
                    return run_decode_wave<0, 8, kNtStore | kNoCoefBranch>(a, nullptr);
                  }});
  vars.push_back({"wave0 lds", kDecodeFused, -1, 1, {}, [probe](const DecodeLaunch& a) {
                    probe(a);
                    return run_decode_wave<0, 8, kNtStore | kNoCoefBranch | kLdsTabs>(a, nullptr);
                  }});
  if (std::getenv("PROBE_FILTER")) {  // keep variants whose name contains one of '|'-separated words
    const std::string f = std::getenv("PROBE_FILTER");
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
  for (auto& v : vars) {
    // custom launches are checked too (probe-only forms that skip stores or math mismatch by design)
    dl.variant = v.variant;
    dl.waves_per_cu = v.waves;
    dl.xcd_swizzle = v.swz;
    poison<<<uint32_t((nd + 255) / 256), 256>>>(data, masks, G, k, P);
    CK(v.fn ? v.fn(dl) : launch_decode(with_book(dl, decode_compact_tables(dl)), nullptr));
    CK(hipDeviceSynchronize());
    std::vector<uint8_t> a(nd), b(nd);
    CK(hipMemcpy(a.data(), data, nd, hipMemcpyDeviceToHost));
    CK(hipMemcpy(b.data(), orig, nd, hipMemcpyDeviceToHost));
    std::printf("check %-18s %s\n", v.name.c_str(), a == b ? "OK" : "MISMATCH (expected for out-of-place forms)");
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rd = 0; rd < rounds; ++rd)
    for (auto& v : vars) {
      dl.variant = v.variant;
      dl.waves_per_cu = v.waves;
      dl.xcd_swizzle = v.swz;
      CK(hipEventRecord(e0));
      CK(v.fn ? v.fn(dl) : launch_decode(with_book(dl, decode_compact_tables(dl)), nullptr));
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms);
    }
  std::printf("k=%u r=%u erasures=%u groups=%llu algorithmic bytes %.3f GB\n", k, r, ners, (unsigned long long)G, alg / 1e9);
  std::printf("%-20s %10s %10s %10s\n", "variant", "med_ms", "min_ms", "GB/s(med)");
  for (auto& v : vars) {
    std::sort(v.ms.begin(), v.ms.end());
    const float med = v.ms[v.ms.size() / 2];
    std::printf("%-20s %10.4f %10.4f %10.1f\n", v.name.c_str(), med, v.ms[0], alg / (med * 1e-3) / 1e9);
  }
  return 0;
}
