// call_site.cpp — the reference's unchanged FEC call site, timed for bench.py's `call_site`
// section.  Every stream owns a HybridFECEncoder (the C++ mirror of encoder_hybrid.go) and
// feeds it 1200-B packets back to back; the 10th packet of a group makes one fec_encode_batch
// call with that one group (encoder_hybrid.go:115 -> fec_cgo.go:138).  `raw` times
// fec_encode_batch alone with FECEncoderCXX's buffers (fec_cgo.go:64/76).  Every repair payload
// is checked against the XOR computed here -- no oracle, so bench.py may run it outside its
// cpu_baseline leg.  Links only libfec_hip.so and the mirror (libquicfec_host.so).
//
// `batcher` is the opt-in integration that changes the call site: every stream's
// BatchedFECEncoder shares one SharedFECBatcher (fec_batcher_*), submits its groups without
// waiting and collects the repair packets as batches finish; r rows per group, every row checked
// (row 0 the XOR, rows 1.. the code's GF(2^8) rows from fec_parity_matrix and a multiply here).
//
//   call_site raw CALLS
//   call_site streams S SECONDS
//   call_site batcher S SECONDS R
//   -> one JSON line: {"mode", "streams", "groups", "seconds", "groups_per_s", "delay_us": {p50, p99},
//                      "errors", "resident_calls", "resident_inline", "resident_vram"}
//      (batcher: "errors" = wrong or missing rows and failed calls; "expired" = groups whose
//       result the ring overwrote before their stream collected it, reported apart)
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "fec.hpp"
#include "fec_hip.h"

using namespace quicfec;
using Clock = std::chrono::steady_clock;

namespace {

constexpr uint32_t kK = 10, kP = 1200, kGroups = 16;

// kGroups groups of 10 packets and each group's XOR
struct Data {
  std::vector<uint8_t> pk, xr;
  Data() : pk(size_t(kGroups) * kK * kP), xr(size_t(kGroups) * kP, 0) {
    uint64_t x = 0x5EED0C5Eull;
    for (auto& b : pk) {
      x = x * 6364136223846793005ull + 1442695040888963407ull;
      b = static_cast<uint8_t>(x >> 56);
    }
    for (uint32_t g = 0; g < kGroups; ++g)
      for (uint32_t j = 0; j < kK; ++j)
        for (uint32_t i = 0; i < kP; ++i) xr[size_t(g) * kP + i] ^= pk[(size_t(g) * kK + j) * kP + i];
  }
};

// GF(2^8), polynomial 0x11D (include/fec_hip.h fec_parity_matrix's field)
uint8_t gf_mul(uint8_t a, uint8_t b) {
  uint8_t p = 0;
  for (; b; b >>= 1) {
    if (b & 1) p ^= a;
    a = static_cast<uint8_t>((a << 1) ^ ((a & 0x80) ? 0x1D : 0));
  }
  return p;
}

// Row i of every group of Data: sum over j of M[i][j] * packet j (row 0 = the XOR)
std::vector<uint8_t> expected_rows(const Data& d, uint32_t r) {
  std::vector<uint8_t> M(size_t(r) * kK);
  if (fec_parity_matrix(kK, r, M.data()) != 0) return {};
  std::vector<uint8_t> rows(size_t(kGroups) * r * kP, 0);
  for (uint32_t g = 0; g < kGroups; ++g)
    for (uint32_t i = 0; i < r; ++i)
      for (uint32_t j = 0; j < kK; ++j)
        for (uint32_t b = 0; b < kP; ++b)
          rows[(size_t(g) * r + i) * kP + b] ^= gf_mul(M[size_t(i) * kK + j], d.pk[(size_t(g) * kK + j) * kP + b]);
  return rows;
}

void report(const char* mode, int streams, std::vector<double>& us, double seconds, long errors) {
  std::sort(us.begin(), us.end());
  auto pct = [&](double p) { return us.empty() ? 0.0 : us[std::min(us.size() - 1, size_t(p * us.size()))]; };
  FECCoalesceStats cs{};
  fec_coalesce_stats_sized(&cs, sizeof(cs), 0);
  std::printf("{\"mode\": \"%s\", \"streams\": %d, \"groups\": %zu, \"seconds\": %.3f, \"groups_per_s\": %.1f, "
              "\"delay_us\": {\"p50\": %.2f, \"p99\": %.2f}, \"errors\": %ld, \"resident_calls\": %llu, "
              "\"resident_inline\": %llu, \"resident_vram\": %llu, \"resident_servers\": %llu}\n",
              mode, streams, us.size(), seconds, double(us.size()) / seconds, pct(0.5), pct(0.99), errors,
              (unsigned long long)cs.resident_calls, (unsigned long long)cs.resident_inline,
              (unsigned long long)cs.resident_vram, (unsigned long long)cs.resident_servers);
  std::fflush(stdout);
}

int raw(int calls) {
  const Data d;
  FECEncoderCtx* ctx = fec_encoder_new(0.1, 1024);
  if (!ctx) return 2;
  auto* slab = static_cast<uint8_t*>(fec_alloc_slab(size_t(kK) * kP));
  auto* rep = static_cast<uint8_t*>(fec_alloc_repair_buffer(kP));
  uint32_t offs[kK];
  for (uint32_t j = 0; j < kK; ++j) offs[j] = j * kP;
  FECCoalesceStats cs{};
  fec_coalesce_stats_sized(&cs, sizeof(cs), 1);
  std::vector<double> us;
  us.reserve(size_t(calls));
  long errors = 0;
  const auto t0 = Clock::now();
  for (int c = 0; c < calls; ++c) {
    const uint32_t g = uint32_t(c) % kGroups;
    std::memcpy(slab, d.pk.data() + size_t(g) * kK * kP, size_t(kK) * kP);  // the wrapper's copy into its slab
    const auto a = Clock::now();
    if (fec_encode_batch(ctx, slab, offs, 1, kP, rep) != 0) ++errors;
    us.push_back(std::chrono::duration<double, std::micro>(Clock::now() - a).count());
    if (std::memcmp(rep, d.xr.data() + size_t(g) * kP, kP) != 0) ++errors;
  }
  const double secs = std::chrono::duration<double>(Clock::now() - t0).count();
  report("raw", 1, us, secs, errors);
  fec_free_slab(slab);
  fec_free_repair_buffer(rep);
  fec_encoder_free(ctx);
  return errors ? 1 : 0;
}

int streams(int S, double seconds) {
  const Data d;
  FECCoalesceStats cs{};
  fec_coalesce_stats_sized(&cs, sizeof(cs), 1);
  std::mutex mu;
  std::vector<double> all;
  std::atomic<long> errors{0};
  const auto t0 = Clock::now();
  const auto t_end = t0 + std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(seconds));
  std::vector<std::thread> th;
  for (int s = 0; s < S; ++s)
    th.emplace_back([&, s] {
      HybridFECEncoder h(0.1);
      if (!h.UseCXX()) ++errors;  // the GPU library must serve it
      std::vector<double> lat;
      for (uint64_t i = 0;; ++i) {
        if (i % kK == 0 && Clock::now() >= t_end) break;
        const uint32_t g = uint32_t((uint64_t(s) * 7 + i / kK) % kGroups);
        const auto a = Clock::now();
        AddPacketResult res = h.AddPacket(d.pk.data() + (size_t(g) * kK + i % kK) * kP, kP, i);
        if (!res.err.ok()) ++errors;
        if (res.needsRedundancy) {
          lat.push_back(std::chrono::duration<double, std::micro>(Clock::now() - a).count());
          // the repair packet: an 11-byte header, then the group's XOR (encoder_hybrid.go)
          if (res.redundancy.size() != 11u + kP || std::memcmp(res.redundancy.data() + 11, d.xr.data() + size_t(g) * kP, kP))
            ++errors;
        }
      }
      h.Close();
      std::lock_guard<std::mutex> lk(mu);
      all.insert(all.end(), lat.begin(), lat.end());
    });
  for (auto& t : th) t.join();
  report("streams", S, all, std::chrono::duration<double>(Clock::now() - t0).count(), errors.load());
  return errors ? 1 : 0;
}

// The opt-in shared batcher: S streams, each a BatchedFECEncoder on one
// SharedFECBatcher (512-group batches, 1 ms deadline), submitting groups back to back without
// waiting and collecting repair packets as batches complete (at most 256 groups outstanding per
// stream).  delay = submit of a group's 10th packet until its rows were collected.
int batcher(int S, double seconds, int r) {
  const Data d;
  const std::vector<uint8_t> want = expected_rows(d, uint32_t(r));
  constexpr int kMaxGroups = 512;
  auto sb = SharedFECBatcher::New(kK, r, kP, kMaxGroups, 1000, -1, 8192 / kMaxGroups);
  if (!sb || want.empty()) {
    std::printf("{\"mode\": \"batcher\", \"error\": \"no batcher\"}\n");
    return 2;
  }
  std::mutex mu;
  std::vector<double> all;
  std::atomic<long> errors{0}, expired{0};
  const auto t0 = Clock::now();
  const auto t_end = t0 + std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(seconds));
  std::vector<std::thread> th;
  for (int s = 0; s < S; ++s)
    th.emplace_back([&, s] {
      BatchedFECEncoder be(sb);
      std::vector<Clock::time_point> sub;  // submit time of each outstanding group, in order
      std::vector<uint32_t> grp;           // its data group
      size_t head = 0;
      std::vector<double> lat;
      std::vector<Bytes> out;
      auto drain = [&](int64_t timeout) {
        out.clear();
        const Error e = be.Poll(&out, timeout);
        const auto now = Clock::now();
        if (out.size() % size_t(r) != 0) ++errors;
        for (size_t q = 0; q + size_t(r) <= out.size(); q += size_t(r), ++head) {
          lat.push_back(std::chrono::duration<double, std::micro>(now - sub[head]).count());
          for (int i = 0; i < r; ++i) {
            const Bytes& pkt = out[q + size_t(i)];
            const size_t hl = i == 0 ? 11u : 14u;  // FE C0 / FE C1 headers (host/fec.cpp MakeRepairPacket)
            if (pkt.size() != hl + kP ||
                std::memcmp(pkt.data() + hl, want.data() + (size_t(grp[head]) * r + i) * kP, kP) != 0)
              ++errors;
          }
        }
        // Poll stops at a ticket it could not collect and drops it: the rows before it are in
        // `out`, the dropped one is the next group.  A result the ring overwrote before this
        // stream came back for it (a thread descheduled while 2 * slabs * max_groups newer groups
        // were encoded) is counted as expired, any other failure as an error.
        if (!e.ok()) {
          if (e.code == FEC_ERR_RANGE) ++expired; else ++errors;
          if (head < sub.size()) ++head;
        }
      };
      for (uint64_t i = 0; Clock::now() < t_end; ++i) {
        const uint32_t g = uint32_t((uint64_t(s) * 7 + i) % kGroups);
        for (uint32_t j = 0; j < kK; ++j)
          if (!be.AddPacketAsync(d.pk.data() + (size_t(g) * kK + j) * kP, kP, i * kK + j).ok()) ++errors;
        sub.push_back(Clock::now());
        grp.push_back(g);
        drain(sub.size() - head >= 256 ? 100000 : 0);
      }
      if (!be.FlushAsync().ok()) ++errors;
      do drain(-1);  // a Poll that drops a ticket returns at it: go on with the rest
      while (be.outstanding() > 0);
      if (head != sub.size()) ++errors;
      std::lock_guard<std::mutex> lk(mu);
      all.insert(all.end(), lat.begin(), lat.end());
    });
  for (auto& t : th) t.join();
  const double wall = std::chrono::duration<double>(Clock::now() - t0).count();
  const std::vector<uint64_t> st = sb->Stats();  // groups, batches, full_flushes, deadline_flushes, max_batch
  std::sort(all.begin(), all.end());
  auto pct = [&](double p) { return all.empty() ? 0.0 : all[std::min(all.size() - 1, size_t(p * all.size()))]; };
  std::printf("{\"mode\": \"batcher\", \"streams\": %d, \"r\": %d, \"max_groups\": %d, \"deadline_us\": 1000, "
              "\"groups\": %zu, \"seconds\": %.3f, \"groups_per_s\": %.1f, \"delay_us\": {\"p50\": %.2f, \"p99\": %.2f}, "
              "\"errors\": %ld, \"expired\": %ld, \"batches\": %llu, \"max_batch\": %llu}\n",
              S, r, kMaxGroups, all.size(), wall, double(all.size()) / wall, pct(0.5), pct(0.99), errors.load(),
              expired.load(), (unsigned long long)(st.size() > 1 ? st[1] : 0),
              (unsigned long long)(st.size() > 4 ? st[4] : 0));
  std::fflush(stdout);
  return errors ? 1 : 0;
}

}  // namespace

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "raw";
  if (mode == "raw") return raw(argc > 2 ? std::atoi(argv[2]) : 20000);
  if (mode == "streams") return streams(argc > 2 ? std::atoi(argv[2]) : 16, argc > 3 ? std::atof(argv[3]) : 1.0);
  if (mode == "batcher")
    return batcher(argc > 2 ? std::atoi(argv[2]) : 16, argc > 3 ? std::atof(argv[3]) : 1.0, argc > 4 ? std::atoi(argv[4]) : 1);
  std::fprintf(stderr, "usage: call_site raw CALLS | call_site streams S SECONDS | call_site batcher S SECONDS R\n");
  return 2;
}
