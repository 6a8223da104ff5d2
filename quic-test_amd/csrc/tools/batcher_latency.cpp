// batcher_latency.cpp — repair delay and throughput of the shared batcher (fec_batcher_*,
// host mirror BatchedFECEncoder) under the reference's call pattern, next to the one-group
// GPU call and the CPU per-group cost.  Not part of the library; results in
// profiles/r02_batcher_latency.jsonl.
//
// The reference: every QUIC stream adds packets at --rate per second (default 100,
// main.go:32; client.go:1140-1143) and encodes one group per call on its 10th packet
// (encoder_hybrid.go:71-73, :115).
//
//   batcher_latency paced <streams> <rate_pps> <seconds> <r> <deadline_us>
//   batcher_latency saturate <streams> <seconds> <r> <deadline_us> <max_groups>
//   batcher_latency cpu                  (per-group CPU cost of the comparators, 1 core)
//   batcher_latency single <r> <calls>   (one group per synchronous call, no batcher)
//   batcher_latency raw <streams> <seconds> <r> <deadline_us> <max_groups> [depth]
//                                        (the C-ABI without the encoder API, and the copy cost)
//   batcher_latency decode <streams> <seconds> <r> <deadline_us> <max_groups> [depth]
//                                        (the decoder batcher at saturation, every packet checked)
//   batcher_latency legacy <streams> <rate_pps> <seconds>
//                                        (the reference's unchanged call site: every stream its own
//                                        HybridFECEncoder -> fec_encode_batch with one group; rate 0 =
//                                        back to back; QUICFEC_COALESCE=0/1 picks the library path)
#include <sys/resource.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "fec.hpp"
#include "fec_hip.h"

extern "C" {
void oracle_xor_avx2(const uint8_t* const*, size_t, size_t, uint8_t*);
int oracle_rs_encode_fast(const uint8_t*, uint64_t, uint32_t, uint32_t, uint32_t, uint8_t*, int);
int64_t oracle_rs_decode_fast(uint8_t*, const uint8_t*, const uint64_t*, uint64_t, uint32_t, uint32_t, uint32_t,
                              uint8_t*, int);
void oracle_fill_splitmix(uint8_t*, uint64_t, uint64_t, uint64_t);
}

using namespace quicfec;
using Clock = std::chrono::steady_clock;

namespace {

constexpr int kK = 10;
constexpr int kP = 1200;

double cpu_seconds() {
  rusage u{};
  getrusage(RUSAGE_SELF, &u);
  return u.ru_utime.tv_sec + u.ru_stime.tv_sec + (u.ru_utime.tv_usec + u.ru_stime.tv_usec) * 1e-6;
}

std::vector<Bytes> packets(int n, uint64_t seed) {
  std::vector<Bytes> v(n, Bytes(kP));
  for (int i = 0; i < n; ++i) oracle_fill_splitmix(v[i].data(), kP, seed, uint64_t(i) * kP);
  return v;
}

void print_lat(const char* mode, const std::string& cfg, std::vector<double>& us, double groups, double seconds,
               double cpu_s, SharedFECBatcher* sb) {
  std::sort(us.begin(), us.end());
  auto pct = [&](double p) { return us.empty() ? 0.0 : us[std::min(us.size() - 1, size_t(p * us.size()))]; };
  std::printf("{\"mode\": \"%s\", %s, \"groups\": %.0f, \"seconds\": %.3f, \"groups_per_s\": %.1f, "
              "\"payload_GiBps\": %.4f, \"delay_us\": {\"p50\": %.1f, \"p90\": %.1f, \"p99\": %.1f, \"max\": %.1f}, "
              "\"cpu_us_per_group\": %.3f",
              mode, cfg.c_str(), groups, seconds, groups / seconds, groups * kK * kP / seconds / (1u << 30), pct(0.5),
              pct(0.9), pct(0.99), us.empty() ? 0.0 : us.back(), cpu_s / groups * 1e6);
  if (sb) {
    auto st = sb->Stats();
    std::printf(", \"batches\": %llu, \"mean_batch\": %.2f, \"full_flushes\": %llu, \"deadline_flushes\": %llu, "
                "\"max_batch\": %llu",
                (unsigned long long)st[1], st[1] ? double(st[0]) / st[1] : 0.0, (unsigned long long)st[2],
                (unsigned long long)st[3], (unsigned long long)st[4]);
  }
  std::printf("}\n");
  std::fflush(stdout);
}

// Streams at a fixed packet rate, synchronous AddPacket (HybridFECEncoder's call shape):
// delay = the 10th packet's AddPacket call, which returns the repair packet(s).
int paced(int S, double rate, double seconds, int r, int deadline_us) {
  auto sb = SharedFECBatcher::New(kK, r, kP, 4096, deadline_us);
  if (!sb) return 2;
  const auto pk = packets(kK, 0x5EED0A);
  std::mutex mu;
  std::vector<double> all;
  std::atomic<long> groups{0}, errors{0};
  const auto t0 = Clock::now() + std::chrono::milliseconds(50);
  const double c0 = cpu_seconds();
  std::vector<std::thread> th;
  for (int s = 0; s < S; ++s)
    th.emplace_back([&, s] {
      BatchedFECEncoder be(sb);
      std::vector<double> lat;
      const double phase = double(s) / S / rate;  // streams spread over one packet interval
      for (long i = 0;; ++i) {
        const auto due = t0 + std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(phase + i / rate));
        if (due > t0 + std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(seconds))) break;
        std::this_thread::sleep_until(due);
        const auto a = Clock::now();
        AddPacketResult res = be.AddPacket(pk[i % kK], uint64_t(i));
        if (!res.err.ok()) ++errors;
        if (res.needsRedundancy) {
          lat.push_back(std::chrono::duration<double, std::micro>(Clock::now() - a).count());
          ++groups;
        }
      }
      std::lock_guard<std::mutex> lk(mu);
      all.insert(all.end(), lat.begin(), lat.end());
    });
  for (auto& t : th) t.join();
  const double cpu = cpu_seconds() - c0;
  char cfg[256];
  std::snprintf(cfg, sizeof(cfg), "\"streams\": %d, \"rate_pps\": %.0f, \"r\": %d, \"deadline_us\": %d, \"errors\": %ld", S,
                rate, r, deadline_us, errors.load());
  print_lat("paced", cfg, all, double(groups), seconds, cpu, sb.get());
  return errors ? 1 : 0;
}

// Every stream submits as fast as it can (async API, up to 256 groups outstanding each).
int saturate(int S, double seconds, int r, int deadline_us, int max_groups) {
  // Results stay collectable for 2 * slabs * max_groups newer groups: at ~3.5 M groups/s a
  // stream thread descheduled for a few ms (16 busy streams on 16 CPUs) must not lose its
  // results, so small batches get more slabs.
  auto sb = SharedFECBatcher::New(kK, r, kP, max_groups, deadline_us, -1, std::max(4, 8192 / max_groups));
  if (!sb) return 2;
  const auto pk = packets(kK, 0x5EED0B);
  std::mutex mu;
  std::vector<double> all;
  std::atomic<long> groups{0}, errors{0};
  const auto t_end = Clock::now() + std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(seconds));
  const auto t0 = Clock::now();
  const double c0 = cpu_seconds();
  std::vector<std::thread> th;
  for (int s = 0; s < S; ++s)
    th.emplace_back([&] {
      BatchedFECEncoder be(sb);
      std::vector<Clock::time_point> sub;  // submit time of each outstanding group, in order
      size_t head = 0;
      std::vector<double> lat;
      std::vector<Bytes> out;
      auto drain = [&](int64_t timeout) {
        out.clear();
        const bool ok = be.Poll(&out, timeout).ok();
        const auto now = Clock::now();
        for (size_t n = out.size() / size_t(r); n > 0; --n, ++head) {
          lat.push_back(std::chrono::duration<double, std::micro>(now - sub[head]).count());
          ++groups;
        }
        if (!ok) {  // Poll dropped the ticket after the rows it returned
          ++errors;
          if (head < sub.size()) ++head;
        }
      };
      while (Clock::now() < t_end) {
        for (int j = 0; j < kK; ++j)
          if (!be.AddPacketAsync(pk[j].data(), kP, 0).ok()) ++errors;
        sub.push_back(Clock::now());
        drain(sub.size() - head >= 256 ? 100000 : 0);
      }
      if (!be.FlushAsync().ok()) ++errors;
      do drain(-1);
      while (be.outstanding() > 0);
      std::lock_guard<std::mutex> lk(mu);
      all.insert(all.end(), lat.begin(), lat.end());
    });
  for (auto& t : th) t.join();
  const double wall = std::chrono::duration<double>(Clock::now() - t0).count();
  const double cpu = cpu_seconds() - c0;
  char cfg[256];
  std::snprintf(cfg, sizeof(cfg), "\"streams\": %d, \"r\": %d, \"deadline_us\": %d, \"max_groups\": %d, \"errors\": %ld", S,
                r, deadline_us, max_groups, errors.load());
  print_lat("saturate", cfg, all, double(groups), wall, cpu, sb.get());
  return errors ? 1 : 0;
}

// QUICFEC_BATCHER_DEVICES="0,1,..." (raw / decode modes): one batcher per listed device behind
// one handle (fec_batcher_new_multi); unset: fec_batcher_new on the current device.
std::vector<int> env_devices() {
  std::vector<int> d;
  const char* e = std::getenv("QUICFEC_BATCHER_DEVICES");
  for (const char* p = e; p && *p;) {
    d.push_back(std::atoi(p));
    p = std::strchr(p, ',');
    if (p) ++p;
  }
  return d;
}

FECBatcher* new_batcher(bool decoder, int r, int max_groups, int deadline_us) {
  const std::vector<int> d = env_devices();
  if (d.empty())
    return decoder ? fec_batcher_new_decoder(-1, kK, r, kP, max_groups, deadline_us, 4)
                   : fec_batcher_new(-1, kK, r, kP, max_groups, deadline_us, 4);
  return decoder ? fec_batcher_new_decoder_multi(d.data(), int(d.size()), kK, r, kP, max_groups, deadline_us, 4)
                 : fec_batcher_new_multi(d.data(), int(d.size()), kK, r, kP, max_groups, deadline_us, 4);
}

// The C-ABI alone (no BatchedFECEncoder): submit by packet pointers, keep up to 256 groups
// outstanding per stream, collect the oldest (payloads copied out).  And the cost of the
// submit's copy alone: 12 KB memcpy per group into page-locked or pageable memory.
int raw(int S, double seconds, int r, int deadline_us, int max_groups, int depth) {
  FECBatcher* b = new_batcher(false, r, max_groups, deadline_us);
  if (!b) return 2;
  // 64 different groups, so a batch that read stale slab bytes would show in row 0
  constexpr int NG = 64;
  Bytes data(size_t(NG) * kK * kP), xr(size_t(NG) * kP);
  oracle_fill_splitmix(data.data(), data.size(), 0x5EED0C, 0);
  for (int g = 0; g < NG; ++g) {
    const uint8_t* p[kK];
    for (int j = 0; j < kK; ++j) p[j] = data.data() + (size_t(g) * kK + j) * kP;
    oracle_xor_avx2(p, kK, kP, xr.data() + size_t(g) * kP);
  }
  std::atomic<long> groups{0}, errors{0};
  const auto t_end = Clock::now() + std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(seconds));
  const auto t0 = Clock::now();
  const double c0 = cpu_seconds();
  std::vector<std::thread> th;
  for (int s = 0; s < S; ++s)
    th.emplace_back([&, s] {
      std::mt19937_64 rng(5 + s);
      const uint8_t* ptrs[kK];
      uint32_t lens[kK];
      for (int j = 0; j < kK; ++j) lens[j] = kP;
      std::vector<uint8_t> rows(size_t(r) * kP);
      std::vector<std::pair<int64_t, int>> q;
      size_t head = 0;
      long n = 0;
      auto check = [&](int rc, int g) {
        if (rc != kP || std::memcmp(rows.data(), xr.data() + size_t(g) * kP, kP)) ++errors;
      };
      while (Clock::now() < t_end) {
        const int g = int(rng() % NG);
        for (int j = 0; j < kK; ++j) ptrs[j] = data.data() + (size_t(g) * kK + j) * kP;
        const int64_t t = fec_batcher_submit_packets(b, ptrs, lens, kK);
        if (t < 0) {
          ++errors;
          continue;
        }
        q.emplace_back(t, g);
        while (head < q.size()) {
          const int rc = fec_batcher_wait(b, q[head].first, rows.data(), kP, q.size() - head >= size_t(depth) ? -1 : 0);
          if (rc == FEC_ERR_AGAIN) break;
          check(rc, q[head].second);
          ++head;
          ++n;
        }
      }
      fec_batcher_flush(b);
      for (; head < q.size(); ++head, ++n) {
        const int rc = fec_batcher_wait(b, q[head].first, rows.data(), kP, -1);
        check(rc, q[head].second);
      }
      groups += n;
    });
  for (auto& t : th) t.join();
  const double wall = std::chrono::duration<double>(Clock::now() - t0).count();
  const double cpu = cpu_seconds() - c0;
  FECBatcherStats st{};
  fec_batcher_stats(b, &st);
  const int ndev = fec_batcher_devices(b);
  fec_batcher_free(b);
  std::printf("{\"mode\": \"raw\", \"devices\": %d, \"streams\": %d, \"r\": %d, \"deadline_us\": %d, \"max_groups\": %d, \"errors\": %ld, "
              "\"depth\": %d, \"groups_per_s\": %.1f, \"cpu_us_per_group\": %.3f, \"mean_batch\": %.1f}\n",
              ndev, S, r, deadline_us, max_groups, errors.load(), depth, groups / wall, cpu / groups * 1e6,
              st.batches ? double(st.groups) / st.batches : 0.0);
  std::fflush(stdout);
  if (std::getenv("QUICFEC_SKIP_COPY")) return errors ? 1 : 0;
  // the submit's copy alone
  for (int pinned = 0; pinned < 2; ++pinned) {
    const size_t region = size_t(4096) * kK * kP;
    std::vector<uint8_t*> dst(S);
    std::vector<std::vector<uint8_t>> pageable(S);
    for (int i = 0; i < S; ++i) {
      if (pinned) {
        dst[i] = static_cast<uint8_t*>(fec_alloc_slab(region));
      } else {
        pageable[i].assign(region, 0);
        dst[i] = pageable[i].data();
      }
    }
    std::atomic<long> copies{0};
    const auto e2 = Clock::now() + std::chrono::milliseconds(1000);
    const auto t2 = Clock::now();
    std::vector<std::thread> ct;
    for (int i = 0; i < S; ++i)
      ct.emplace_back([&, i] {
        long n = 0;
        while (Clock::now() < e2)
          for (int g = 0; g < 256; ++g, ++n)
            for (int j = 0; j < kK; ++j)
              std::memcpy(dst[i] + (size_t(n % 4096) * kK + j) * kP, data.data() + size_t(j) * kP, kP);
        copies += n;
      });
    for (auto& t : ct) t.join();
    const double w2 = std::chrono::duration<double>(Clock::now() - t2).count();
    std::printf("{\"mode\": \"copy\", \"streams\": %d, \"pinned\": %d, \"groups_per_s\": %.1f, \"GiBps\": %.2f}\n", S,
                pinned, copies / w2, copies * double(kK * kP) / w2 / (1u << 30));
    if (pinned)
      for (auto* d : dst) fec_free_slab(d);
  }
  return errors ? 1 : 0;
}

// The decoder batcher at saturation: every connection thread submits coded groups with
// losses (r = 1: one data shard; else two of the k + r shards, as C3), keeps `depth`
// outstanding, and checks every rebuilt packet against the original.
int draw(int S, double seconds, int r, int deadline_us, int max_groups, int depth) {
  FECBatcher* b = new_batcher(true, r, max_groups, deadline_us);
  if (!b) return 2;
  constexpr int NG = 64;
  Bytes data(size_t(NG) * kK * kP), par(size_t(NG) * r * kP);
  oracle_fill_splitmix(data.data(), data.size(), 0x5EED0E, 0);
  oracle_rs_encode_fast(data.data(), NG, kK, r, kP, par.data(), 1);
  std::atomic<long> groups{0}, errors{0};
  const auto t_end = Clock::now() + std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(seconds));
  const auto t0 = Clock::now();
  const double c0 = cpu_seconds();
  std::vector<std::thread> th;
  for (int s = 0; s < S; ++s)
    th.emplace_back([&, s] {
      std::mt19937_64 rng(99 + s);
      struct Out {
        int64_t t;
        int g;
        uint64_t mask;
      };
      std::vector<Out> q;
      size_t head = 0;
      std::vector<uint8_t> rows(size_t(r) * kP);
      long n = 0;
      auto check = [&](const Out& o, int rc, uint64_t got_mask) {
        int want = 0;
        bool ok = true;
        int first_bad = -1;
        for (int j = 0; j < kK; ++j) {
          if (!((o.mask >> j) & 1)) continue;
          if (rc > want) {
            const uint8_t* a = rows.data() + size_t(want) * kP;
            const uint8_t* e = data.data() + (size_t(o.g) * kK + j) * kP;
            for (int i = 0; i < kP && first_bad < 0; ++i)
              if (a[i] != e[i]) first_bad = want * 100000 + i;
          }
          if (rc <= want || first_bad >= 0) ok = false;
          ++want;
        }
        if (rc != want || got_mask != o.mask) ok = false;
        if (!ok && ++errors <= 6) {
          // what came back: zeros, another group's shard, or something else
          int zeros = 1, other = -1;
          for (int i = 0; i < kP; ++i) zeros &= rows[i] == 0;
          for (int gg = 0; gg < NG && other < 0; ++gg)
            for (int jj = 0; jj < kK; ++jj)
              if (!std::memcmp(rows.data(), data.data() + (size_t(gg) * kK + jj) * kP, kP)) other = gg * 100 + jj;
          std::fprintf(stderr, "decode error: stream %d ticket %lld group %d mask 0x%llx got rc %d mask 0x%llx, "
                               "first bad (row*1e5+byte) %d, row all zero %d, row = shard (g*100+j) %d, row[0..3] %02x%02x%02x%02x\n",
                       s, (long long)o.t, o.g, (unsigned long long)o.mask, rc, (unsigned long long)got_mask, first_bad, zeros,
                       other, rows[0], rows[1], rows[2], rows[3]);
        }
      };
      while (Clock::now() < t_end) {
        const int g = int(rng() % NG);
        uint64_t mask;
        if (r == 1) {
          mask = 1ull << (rng() % kK);
        } else {
          const int a = int(rng() % (kK + r));
          int c = int(rng() % (kK + r - 1));
          if (c >= a) ++c;
          mask = (1ull << a) | (1ull << c);
        }
        const uint8_t* shards[64];
        for (int j = 0; j < kK + r; ++j)
          shards[j] = (mask >> j) & 1 ? nullptr
                      : j < kK    ? data.data() + (size_t(g) * kK + j) * kP
                                  : par.data() + (size_t(g) * r + (j - kK)) * kP;
        const int64_t t = fec_batcher_submit_shards(b, shards, kP);
        if (t < 0) {
          ++errors;
          continue;
        }
        q.push_back(Out{t, g, mask});
        while (head < q.size()) {
          uint64_t m = 0;
          const int rc = fec_batcher_wait_rebuilt(b, q[head].t, rows.data(), kP, &m, q.size() - head >= size_t(depth) ? -1 : 0);
          if (rc == FEC_ERR_AGAIN) break;
          check(q[head], rc, m);
          ++head;
          ++n;
        }
      }
      fec_batcher_flush(b);
      for (; head < q.size(); ++head, ++n) {
        uint64_t m = 0;
        const int rc = fec_batcher_wait_rebuilt(b, q[head].t, rows.data(), kP, &m, -1);  // before m is read
        check(q[head], rc, m);
      }
      groups += n;
    });
  for (auto& t : th) t.join();
  const double wall = std::chrono::duration<double>(Clock::now() - t0).count();
  const double cpu = cpu_seconds() - c0;
  FECBatcherStats st{};
  fec_batcher_stats(b, &st);
  const int ndev = fec_batcher_devices(b);
  fec_batcher_free(b);
  std::printf("{\"mode\": \"decode_raw\", \"devices\": %d, \"streams\": %d, \"r\": %d, \"deadline_us\": %d, \"max_groups\": %d, "
              "\"depth\": %d, \"errors\": %ld, \"groups_per_s\": %.1f, \"cpu_us_per_group\": %.3f, \"mean_batch\": %.1f}\n",
              ndev, S, r, deadline_us, max_groups, depth, errors.load(), groups / wall, cpu / groups * 1e6,
              st.batches ? double(st.groups) / st.batches : 0.0);
  std::fflush(stdout);
  return errors ? 1 : 0;
}

// The one-group call of the reference's pattern without a batcher (HybridFECEncoder ->
// fec_encode_batch, one launch and synchronize per group), for comparison.
int single(int calls) {
  HybridFECEncoder h(0.1);
  if (!h.UseCXX()) return 2;
  const auto pk = packets(kK, 0x5EED0C);
  std::vector<double> us;
  const double c0 = cpu_seconds();
  const auto t0 = Clock::now();
  for (int c = 0; c < calls; ++c) {
    for (int j = 0; j < kK - 1; ++j) h.AddPacket(pk[j], 0);
    const auto a = Clock::now();
    AddPacketResult res = h.AddPacket(pk[kK - 1], 0);
    if (!res.needsRedundancy) return 1;
    us.push_back(std::chrono::duration<double, std::micro>(Clock::now() - a).count());
  }
  const double wall = std::chrono::duration<double>(Clock::now() - t0).count();
  print_lat("single_group_call", "\"streams\": 1, \"r\": 1, \"api\": \"HybridFECEncoder -> fec_encode_batch\"", us, calls,
            wall, cpu_seconds() - c0, nullptr);
  return 0;
}

// The unchanged HybridFECEncoder of every stream (its own FECEncoderCXX and context, one group
// per fec_encode_batch call, encoder_hybrid.go:115): paced at `rate` packets/s per stream, or
// back to back (rate 0).  Delay = the 10th packet's AddPacket; every repair payload is checked
// against the AVX2 XOR restatement.  Whether concurrent streams' calls share launches is the
// library's choice (QUICFEC_COALESCE, fec_coalesce.cpp); its stats are printed.
int legacy(int S, double rate, double seconds) {
  constexpr int NG = 16;
  Bytes data(size_t(NG) * kK * kP), xr(size_t(NG) * kP);
  oracle_fill_splitmix(data.data(), data.size(), 0x5EED0F, 0);
  for (int g = 0; g < NG; ++g) {
    const uint8_t* p[kK];
    for (int j = 0; j < kK; ++j) p[j] = data.data() + (size_t(g) * kK + j) * kP;
    oracle_xor_avx2(p, kK, kP, xr.data() + size_t(g) * kP);
  }
  FECCoalesceStats cs{};
  fec_coalesce_stats_sized(&cs, sizeof(cs), 1);
  std::mutex mu;
  std::vector<double> all;
  std::atomic<long> groups{0}, errors{0}, fallback{0};
  const auto t0 = Clock::now() + std::chrono::milliseconds(rate > 0 ? 200 : 0);
  const auto t_end = t0 + std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(seconds));
  const double c0 = cpu_seconds();
  std::vector<std::thread> th;
  for (int s = 0; s < S; ++s)
    th.emplace_back([&, s] {
      HybridFECEncoder h(0.1);
      if (!h.UseCXX()) ++fallback;
      std::vector<double> lat;
      const double phase = rate > 0 ? double(s) / S / rate : 0.0;
      for (long i = 0;; ++i) {
        if (rate > 0) {
          const auto due = t0 + std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(phase + i / rate));
          if (due > t_end) break;
          std::this_thread::sleep_until(due);
        } else if ((i % kK) == 0 && Clock::now() >= t_end) {
          break;
        }
        const int g = int((uint64_t(s) * 7 + uint64_t(i / kK)) % NG);
        const auto a = Clock::now();
        AddPacketResult res = h.AddPacket(data.data() + (size_t(g) * kK + i % kK) * kP, kP, uint64_t(i));
        if (!res.err.ok()) ++errors;
        if (res.needsRedundancy) {
          lat.push_back(std::chrono::duration<double, std::micro>(Clock::now() - a).count());
          ++groups;
          if (res.redundancy.size() != 11u + kP || std::memcmp(res.redundancy.data() + 11, xr.data() + size_t(g) * kP, kP))
            ++errors;
        }
      }
      h.Close();
      std::lock_guard<std::mutex> lk(mu);
      all.insert(all.end(), lat.begin(), lat.end());
    });
  for (auto& t : th) t.join();
  const double wall = rate > 0 ? seconds : std::chrono::duration<double>(Clock::now() - t0).count();
  const double cpu = cpu_seconds() - c0;
  fec_coalesce_stats_sized(&cs, sizeof(cs), 0);
  const char* co = std::getenv("QUICFEC_COALESCE");
  const char* res = std::getenv("QUICFEC_RESIDENT");
  char cfg[1024];
  std::snprintf(cfg, sizeof(cfg),
                "\"streams\": %d, \"rate_pps\": %.0f, \"r\": 1, \"coalesce\": %d, \"errors\": %ld, \"go_fallback\": %ld, "
                "\"coalesced_calls\": %llu, \"launches\": %llu, \"mean_batch\": %.2f, \"max_batch\": %llu, "
                "\"us_per_launch\": {\"close\": %.2f, \"launch\": %.2f, \"done\": %.2f}, \"resident\": %d, "
                "\"resident_calls\": %llu, \"resident_launches\": %llu, \"resident_inline\": %llu, \"resident_vram\": %llu, "
                "\"resident_servers\": %llu, \"resident_bad_slots\": %llu, \"resident_scrubs\": %llu, "
                "\"resident_us_per_call\": {\"pre\": %.2f, \"wait\": %.2f, \"post\": %.2f}",
                S, rate, co && co[0] == '0' ? 0 : 1, errors.load(), fallback.load(), (unsigned long long)cs.calls,
                (unsigned long long)cs.batches, cs.batches ? double(cs.groups) / cs.batches : 0.0,
                (unsigned long long)cs.max_batch, cs.batches ? cs.close_ns / 1e3 / cs.batches : 0.0,
                cs.batches ? cs.launch_ns / 1e3 / cs.batches : 0.0, cs.batches ? cs.done_ns / 1e3 / cs.batches : 0.0,
                res && res[0] == '0' ? 0 : 1, (unsigned long long)cs.resident_calls,
                (unsigned long long)cs.resident_launches, (unsigned long long)cs.resident_inline,
                (unsigned long long)cs.resident_vram, (unsigned long long)cs.resident_servers,
                (unsigned long long)cs.resident_bad_slots, (unsigned long long)cs.resident_scrubs,
                cs.resident_calls ? cs.resident_pre_ns / 1e3 / cs.resident_calls : 0.0,
                cs.resident_calls ? cs.resident_wait_ns / 1e3 / cs.resident_calls : 0.0,
                cs.resident_calls ? cs.resident_post_ns / 1e3 / cs.resident_calls : 0.0);
  print_lat("legacy", cfg, all, double(groups), wall, cpu, nullptr);
  return errors || fallback ? 1 : 0;
}

// fec_encode_batch alone, one group per call on page-locked buffers as FECEncoderCXX holds them
// (no Go-API mirror around it): the library's own per-call latency on whichever path it takes.
int legacy_raw(int calls) {
  FECEncoderCtx* ctx = fec_encoder_new(0.1, 1024);
  if (!ctx) return 2;
  auto* slab = static_cast<uint8_t*>(fec_alloc_slab(size_t(kK) * kP));
  auto* rep = static_cast<uint8_t*>(fec_alloc_repair_buffer(kP));
  oracle_fill_splitmix(slab, size_t(kK) * kP, 0x5EED10, 0);
  uint32_t offs[kK];
  for (int j = 0; j < kK; ++j) offs[j] = uint32_t(j * kP);
  Bytes xr(kP);
  const uint8_t* p[kK];
  for (int j = 0; j < kK; ++j) p[j] = slab + size_t(j) * kP;
  oracle_xor_avx2(p, kK, kP, xr.data());
  FECCoalesceStats cs{};
  fec_coalesce_stats_sized(&cs, sizeof(cs), 1);
  std::vector<double> us;
  long errors = 0;
  const auto t0 = Clock::now();
  for (int c = 0; c < calls; ++c) {
    const auto a = Clock::now();
    if (fec_encode_batch(ctx, slab, offs, 1, kP, rep) != 0) ++errors;
    us.push_back(std::chrono::duration<double, std::micro>(Clock::now() - a).count());
    if (std::memcmp(rep, xr.data(), kP)) ++errors;
  }
  const double wall = std::chrono::duration<double>(Clock::now() - t0).count();
  fec_coalesce_stats_sized(&cs, sizeof(cs), 0);
  // where the slowest calls are (the first call pays any lazily created state)
  const size_t imax = us.empty() ? 0 : size_t(std::max_element(us.begin(), us.end()) - us.begin());
  std::vector<double> rest(us.begin() + (us.empty() ? 0 : 1), us.end());
  const double first_us = us.empty() ? 0.0 : us[0], rest_max = rest.empty() ? 0.0 : *std::max_element(rest.begin(), rest.end());
  const char* co = std::getenv("QUICFEC_COALESCE");
  const char* res = std::getenv("QUICFEC_RESIDENT");
  char cfg[768];
  std::snprintf(cfg, sizeof(cfg),
                "\"streams\": 1, \"coalesce\": %d, \"resident\": %d, \"errors\": %ld, \"resident_calls\": %llu, "
                "\"resident_inline\": %llu, \"resident_vram\": %llu, "
                "\"resident_us_per_call\": {\"pre\": %.2f, \"wait\": %.2f, \"post\": %.2f}, "
                "\"max_at_call\": %zu, \"first_call_us\": %.1f, \"max_after_first_us\": %.1f, \"batches\": %llu",
                co && co[0] == '0' ? 0 : 1, res && res[0] == '0' ? 0 : 1, errors, (unsigned long long)cs.resident_calls,
                (unsigned long long)cs.resident_inline, (unsigned long long)cs.resident_vram,
                cs.resident_calls ? cs.resident_pre_ns / 1e3 / cs.resident_calls : 0.0,
                cs.resident_calls ? cs.resident_wait_ns / 1e3 / cs.resident_calls : 0.0,
                cs.resident_calls ? cs.resident_post_ns / 1e3 / cs.resident_calls : 0.0, imax, first_us, rest_max,
                (unsigned long long)cs.batches);
  print_lat("legacy_raw", cfg, us, calls, wall, 0.0, nullptr);
  fec_free_slab(slab);
  fec_free_repair_buffer(rep);
  fec_encoder_free(ctx);
  return errors ? 1 : 0;
}

// One core: the reference's computation per group (AVX2 XOR, xor_packets_avx2 restated) and
// the r = 3 code with GFNI (oracle fast form); 4096 groups of fresh data per pass.
int cpu() {
  const uint64_t G = 4096;
  Bytes data(G * kK * kP), rep(G * 3 * kP);
  oracle_fill_splitmix(data.data(), data.size(), 0x5EED0D, 0);
  auto time_it = [&](auto&& fn) {
    int reps = 0;
    const auto t0 = Clock::now();
    double s = 0;
    do {
      fn();
      ++reps;
      s = std::chrono::duration<double>(Clock::now() - t0).count();
    } while (s < 1.0);
    return s / (reps * double(G)) * 1e6;
  };
  const double xor_us = time_it([&] {
    const uint8_t* p[kK];
    for (uint64_t g = 0; g < G; ++g) {
      for (int j = 0; j < kK; ++j) p[j] = data.data() + (g * kK + j) * kP;
      oracle_xor_avx2(p, kK, kP, rep.data() + g * kP);
    }
  });
  const double rs3_us = time_it([&] { oracle_rs_encode_fast(data.data(), G, kK, 3, kP, rep.data(), 1); });
  // receiver side: 2 of the 13 shards lost per group (C3), rebuilt in place
  std::vector<uint64_t> masks(G);
  std::mt19937_64 rng(7);
  for (auto& m : masks) {
    const int a = int(rng() % 13);
    int b2 = int(rng() % 12);
    if (b2 >= a) ++b2;
    m = (1ull << a) | (1ull << b2);
  }
  const double dec3_us = time_it([&] { oracle_rs_decode_fast(data.data(), rep.data(), masks.data(), G, kK, 3, kP, nullptr, 1); });
  std::printf("{\"mode\": \"cpu_one_core\", \"us_per_group_avx2_xor_r1\": %.3f, \"us_per_group_gfni_r3\": %.3f, "
              "\"groups_per_s_avx2_xor_r1\": %.0f, \"groups_per_s_gfni_r3\": %.0f, \"us_per_group_gfni_decode_r3_2lost\": %.3f, "
              "\"groups_per_s_gfni_decode_r3_2lost\": %.0f}\n",
              xor_us, rs3_us, 1e6 / xor_us, 1e6 / rs3_us, dec3_us, 1e6 / dec3_us);
  return 0;
}

}  // namespace

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "cpu";
  auto arg = [&](int i, double d) { return argc > i ? std::atof(argv[i]) : d; };
  if (mode == "paced") return paced(int(arg(2, 10)), arg(3, 100), arg(4, 5), int(arg(5, 1)), int(arg(6, 1000)));
  if (mode == "saturate")
    return saturate(int(arg(2, 16)), arg(3, 3), int(arg(4, 1)), int(arg(5, 1000)), int(arg(6, 4096)));
  if (mode == "single") return single(int(arg(2, 2000)));
  if (mode == "legacy") return legacy(int(arg(2, 16)), arg(3, 0), arg(4, 3));
  if (mode == "legacy_raw") return legacy_raw(int(arg(2, 20000)));
  if (mode == "decode")
    return draw(int(arg(2, 16)), arg(3, 3), int(arg(4, 3)), int(arg(5, 1000)), int(arg(6, 4096)), int(arg(7, 1024)));
  if (mode == "raw")
    return raw(int(arg(2, 16)), arg(3, 3), int(arg(4, 1)), int(arg(5, 1000)), int(arg(6, 4096)), int(arg(7, 256)));
  return cpu();
}
