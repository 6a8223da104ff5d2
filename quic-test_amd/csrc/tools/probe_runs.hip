// probe_runs.hip — development probe: the one-launch packed recover (recover_runs) against the
// library's two-step packed recover (row prefix launches + decode_fused) and its slot-row
// recover, in one process, interleaved rounds.  Every recover_runs form is checked byte for
// byte (rows, row starts, total, status) against the two-step packed recover first.
// Not part of the library.
//
//   probe_runs [groups] [rounds] [loss]      loss > 0: iid per shard (C5: 0.01); 0: 2 erasures
//                                             per group uniform over the 13 shards (C3)
#include "../fec_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <random>
#include <string>
#include <vector>

#include "../gf256.hpp"

#define CK(x)                                                                                \
  do {                                                                                       \
    hipError_t e_ = (x);                                                                     \
    if (e_ != hipSuccess) {                                                                  \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                          \
    }                                                                                        \
  } while (0)

using namespace qfec;

// recover_runs in any probe form: one launch (no chunking), tile = 64 * WAVES groups
template <int POL, int WAVES, int TG = 64 * WAVES>
hipError_t runs_form(const RunsLaunch& a, uint32_t stage, uint32_t flags) {
  RankMeta rm{};
  for (int e = 1; e <= 3; ++e) {
    rm.base[e] = a.meta.base[e];
    rm.stride[e] = a.meta.stride[e];
    rm.count_r[e] = a.meta.count_r[e];
  }
  uint8_t* ws = static_cast<uint8_t*>(a.workspace);
  const uint32_t nb = uint32_t((a.groups + TG - 1) / TG);
  hipLaunchKernelGGL((recover_runs<10, 3, 1, 1, POL, WAVES, TG>), dim3(nb), dim3(64 * WAVES), stage, nullptr, a.data, a.parity,
                     a.masks, a.groups, a.P, a.codebook, rm, a.out, a.row_start, a.status,
                     reinterpret_cast<uint64_t*>(ws + 128), reinterpret_cast<uint32_t*>(ws), a.epoch, stage, nullptr,
                     reinterpret_cast<uint64_t*>(ws + 64), a.total, flags);
  return hipGetLastError();
}

int main(int argc, char** argv) {
  const uint64_t G = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1000000;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 9;
  const double loss = argc > 3 ? std::atof(argv[3]) : 0.01;
  const uint32_t k = 10, r = 3, P = 1200;
  const uint64_t nd = G * k * P, np = G * r * P;
  uint8_t *data, *par, *slots, *packA, *packB, *stA, *stB;
  uint64_t *masks, *totA, *totB;
  uint32_t *rsA, *rsB;
  CK(hipMalloc(&data, nd));
  CK(hipMalloc(&par, np));
  CK(hipMalloc(&slots, np));
  CK(hipMalloc(&packA, np));
  CK(hipMalloc(&packB, np));
  CK(hipMalloc(&stA, G));
  CK(hipMalloc(&stB, G));
  CK(hipMalloc(&masks, G * 8));
  CK(hipMalloc(&totA, 8));
  CK(hipMalloc(&totB, 8));
  CK(hipMalloc(&rsA, G * 4));
  CK(hipMalloc(&rsB, G * 4));
  CK(launch_fill_splitmix(data, nd, 0x5EED0002, 0, nullptr));
  std::vector<uint8_t> M;
  parity_matrix(k, r, M);
  std::vector<CoefEntry> tab;
  for (uint32_t i = 1; i < r; ++i)
    for (uint32_t j = 0; j < k; ++j) tab.push_back(make_entry(M[i * k + j]));
  void* dtab = nullptr;
  CK(hipMalloc(&dtab, tab.size() * 32));
  CK(hipMemcpy(dtab, tab.data(), tab.size() * 32, hipMemcpyHostToDevice));
  EncodeLaunch el{data, nullptr, OffsetKind::kNone, par, G, k, r, P, dtab};
  CK(launch_encode(el, nullptr));
  std::vector<uint64_t> hm(G);
  std::mt19937_64 rng(0x5EED0005);
  uint64_t alg = 0, rows_total = 0;
  for (uint64_t g = 0; g < G; ++g) {
    uint64_t m = 0;
    if (loss > 0) {
      for (uint32_t j = 0; j < k + r; ++j)
        if (double(rng() >> 11) * 0x1.0p-53 < loss) m |= 1ull << j;
    } else {
      while (__builtin_popcountll(m) < 2) m |= 1ull << (rng() % (k + r));
    }
    hm[g] = m;
    const uint32_t e = __builtin_popcountll(m & ((1ull << k) - 1));
    const uint32_t alive = r - __builtin_popcountll((m >> k) & ((1ull << r) - 1));
    if (e && e <= alive) {
      alg += uint64_t(k + e) * P;
      rows_total += e;
    }
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
  dl.rec_off = nullptr;
  dl.status = stA;
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
  dl.compact_out = true;
  const double share = double(rows_total) / double(G);
  dl.scan = share < 0.25 ? kDecodeScanGroups : 1;
  uint32_t* bsums;
  CK(hipMalloc(&bsums, rows_prefix_workspace_bytes(G) + 64));
  void* rws;
  const uint64_t rws_bytes = 128 + 8 * (G / 64 + 2);  // enough for the smallest probe tile
  CK(hipMalloc(&rws, rws_bytes));
  CK(hipMemset(rws, 0, rws_bytes));
  uint32_t epoch = 1;
  RunsLaunch ra{};
  ra.data = data;
  ra.parity = par;
  ra.masks = masks;
  ra.groups = G;
  ra.k = k;
  ra.r = r;
  ra.P = P;
  ra.codebook = dbook;
  ra.meta = dl.meta;
  ra.out = packB;
  ra.row_start = rsB;
  ra.total = totB;
  ra.status = stB;
  ra.workspace = rws;
  struct Var {
    std::string name;
    std::function<hipError_t()> fn;
    bool runs;
    std::vector<float> ms;
  };
  std::vector<Var> vars;
  vars.push_back({"lib slots", [&] {
                    DecodeLaunch a = dl;
                    a.out = slots;
                    return launch_decode(a, nullptr);
                  }, false, {}});
  vars.push_back({"lib packed (prefix+decode)", [&] {
                    DecodeLaunch a = dl;
                    a.out = packA;
                    a.rec_off = rsA;
                    a.packed_rows = true;
                    CK(launch_rows_prefix(masks, G, k, r, rsA, bsums, totA, nullptr));
                    return launch_decode(a, nullptr);
                  }, false, {}});
  for (int stage : {24576}) {
    vars.push_back({"runs stage " + std::to_string(stage), [&, stage] {
                      RunsLaunch a = ra;
                      a.stage_bytes = stage;
                      a.epoch = epoch;
                      epoch += runs_launches(G);
                      return launch_recover_runs(a, nullptr);
                    }, true, {}});
  }
#define RF(NAME, POL, W, TG, STAGE, FLAGS, CHECK, OUT)              \
  vars.push_back({NAME, [&, o = (OUT)] {                          \
                    RunsLaunch a = ra;                            \
                    a.out = o;                                    \
                    a.epoch = epoch++;                            \
                    return runs_form<POL, W, TG>(a, STAGE, FLAGS); \
                  }, CHECK, {}});
  constexpr int NL = kNtLoad, NS = kNtStore;
  // extra rebuilt-row buffers: the same forms on differently placed outputs (the
  // recover's rate moves with where its output lands)
  const int nbufs = std::getenv("PROBE_BUFS") ? std::atoi(std::getenv("PROBE_BUFS")) : 1;
  std::vector<uint8_t*> outs = {packB};
  for (int i = 1; i < nbufs; ++i) {
    uint8_t* o;
    CK(hipMalloc(&o, np));
    outs.push_back(o);
  }
  for (int i = 0; i < nbufs; ++i) {
    const std::string at = nbufs > 1 ? " @" + std::to_string(i) : "";
    const bool chk = i == 0;
    if (i > 0)
      vars.push_back({"lib packed" + at, [&, o = outs[i]] {
                        DecodeLaunch a = dl;
                        a.out = o;
                        a.rec_off = rsA;
                        a.packed_rows = true;
                        CK(launch_rows_prefix(masks, G, k, r, rsA, bsums, totA, nullptr));
                        return launch_decode(a, nullptr);
                      }, false, {}});
    RF("runs w8 nl st48K" + at, NL, 8, 512, 49152, 0, chk, outs[i])
    RF("runs w8 nl+ns st48K" + at, NL | NS, 8, 512, 49152, 0, chk, outs[i])
    if (loss == 0 && std::getenv("PROBE_SLOTS_POLICY")) {  // the slot-row recover's store policy by buffer
      vars.push_back({"slots nt-ld+nt-st (lib)" + at, [&, o = outs[i]] {
                        DecodeLaunch a = dl;
                        a.out = o;
                        return run_decode_fused<10, 3, kNtStore | kNtLoad | kCompactOut, 1, 1, true>(a, nullptr);
                      }, false, {}});
      vars.push_back({"slots nt-ld plain-st" + at, [&, o = outs[i]] {
                        DecodeLaunch a = dl;
                        a.out = o;
                        return run_decode_fused<10, 3, kNtLoad | kCompactOut, 1, 1, true>(a, nullptr);
                      }, false, {}});
      vars.push_back({"slots plain-ld nt-st" + at, [&, o = outs[i]] {
                        DecodeLaunch a = dl;
                        a.out = o;
                        return run_decode_fused<10, 3, kNtStore | kCompactOut, 1, 1, true>(a, nullptr);
                      }, false, {}});
      vars.push_back({"slots nostore-probe copy" + at, [&, o = outs[i]] {  // parity -> out copy of the rows' size
                        return launch_copy_words(par, o, uint64_t(G) * 3 * P / 2 / 16 * 16, nullptr);
                      }, false, {}});
      continue;
    }
    if (loss == 0) {  // dense: small tiles, every row in the image, look-back after the rebuild
      RF("runs w8 tg8 nl+ns st29K" + at, NL | NS, 8, 8, 28800, 0, chk, outs[i])
      RF("runs w8 tg8 nl st29K" + at, NL, 8, 8, 28800, 0, chk, outs[i])
      RF("runs w8 tg16 nl+ns st58K" + at, NL | NS, 8, 16, 57600, 0, chk, outs[i])
      RF("runs w4 tg8 nl+ns st29K" + at, NL | NS, 4, 8, 28800, 0, chk, outs[i])
      RF("runs w8 tg8 nostore" + at, NL, 8, 8, 28800, 1, false, outs[i])
      // several groups per wave, the next group's loads in flight during this one's rows (kRunPipe)
      RF("runs w4 tg16 nl+ns st58K" + at, NL | NS, 4, 16, 59392, 0, chk, outs[i])
      RF("runs w4 tg16 pipe nl+ns st58K" + at, NL | NS | kRunPipe, 4, 16, 59392, 0, chk, outs[i])
      RF("runs w8 tg32 pipe nl+ns st60K" + at, NL | NS | kRunPipe, 8, 32, 61440, 0, chk, outs[i])
    }
    if (loss > 0) {
      RF("runs w8 nl+ns st32K" + at, NL | NS, 8, 512, 32768, 0, chk, outs[i])
      RF("runs w4 nl+ns st24K" + at, NL | NS, 4, 256, 24576, 0, chk, outs[i])
      RF("runs w4 nl st24K" + at, NL, 4, 256, 24576, 0, chk, outs[i])
      RF("runs w8 nostore" + at, NL, 8, 512, 0, 1, false, outs[i])
      RF("runs w8 pipe nl+ns st48K" + at, NL | NS | kRunPipe, 8, 512, 49152, 0, chk, outs[i])
      // the store policy by path: the run image's copy-out plain, rows past it nt; a larger image
      RF("runs w8 nl+ns img-plain st48K" + at, NL | NS | kRunImgPlain, 8, 512, 49152, 0, chk, outs[i])
      RF("runs w8 nl+ns st64K" + at, NL | NS, 8, 512, 65536, 0, chk, outs[i])
      RF("runs w8 nl st64K" + at, NL, 8, 512, 65536, 0, chk, outs[i])
      RF("runs w8 nl+ns img-plain st64K" + at, NL | NS | kRunImgPlain, 8, 512, 65536, 0, chk, outs[i])
      RF("runs w4 tg256 pipe nl+ns st24K" + at, NL | NS | kRunPipe, 4, 256, 24576, 0, chk, outs[i])
    }
  }
  // reference output: the two-step packed recover
  CK(vars[1].fn());
  CK(hipDeviceSynchronize());
  std::vector<uint8_t> refp(rows_total * P), got(rows_total * P), refst(G), gotst(G);
  std::vector<uint32_t> refrs(G), gotrs(G);
  uint64_t reft = 0, gott = 0;
  CK(hipMemcpy(refp.data(), packA, rows_total * P, hipMemcpyDeviceToHost));
  CK(hipMemcpy(refrs.data(), rsA, G * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(refst.data(), stA, G, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&reft, totA, 8, hipMemcpyDeviceToHost));
  std::printf("groups %llu loss %.4f rows %llu (total from prefix %llu) algorithmic %.4f GB\n", (unsigned long long)G, loss,
              (unsigned long long)rows_total, (unsigned long long)reft, alg / 1e9);
  bool all_ok = reft == rows_total;
  for (auto& v : vars) {
    if (!v.runs) continue;
    for (int rep = 0; rep < 2; ++rep) {  // twice: the second launch runs on the first one's look-back words
      CK(hipMemset(packB, 0xA5, np));
      CK(hipMemset(rsB, 0xFF, G * 4));
      CK(hipMemset(totB, 0xFF, 8));
      CK(v.fn());
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(got.data(), packB, rows_total * P, hipMemcpyDeviceToHost));
      CK(hipMemcpy(gotrs.data(), rsB, G * 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(gotst.data(), stB, G, hipMemcpyDeviceToHost));
      CK(hipMemcpy(&gott, totB, 8, hipMemcpyDeviceToHost));
      const bool ok = got == refp && gotrs == refrs && gotst == refst && gott == reft;
      all_ok = all_ok && ok;
      std::printf("check %-28s rep %d %s (total %llu)\n", v.name.c_str(), rep, ok ? "OK" : "MISMATCH",
                  (unsigned long long)gott);
    }
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rd = 0; rd < rounds; ++rd)
    for (auto& v : vars) {
      CK(hipEventRecord(e0));
      CK(v.fn());
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms);
    }
  std::printf("%-30s %10s %10s %10s\n", "variant", "med_ms", "min_ms", "GB/s(med)");
  for (auto& v : vars) {
    std::sort(v.ms.begin(), v.ms.end());
    const float med = v.ms[v.ms.size() / 2];
    std::printf("%-30s %10.4f %10.4f %10.1f\n", v.name.c_str(), med, v.ms[0], alg / (med * 1e-3) / 1e9);
  }
  std::printf("all checks %s\n", all_ok ? "OK" : "FAILED");
  return all_ok ? 0 : 1;
}
