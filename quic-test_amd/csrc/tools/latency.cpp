// latency.cpp — per-call latency of the host-resident C-ABI at small batch sizes, called
// the way the reference's cgo wrapper calls it (fec_cgo.go:138: one fec_encode_batch per
// EncodeBatch, today with a single group per call, encoder_hybrid.go:115).  Links
// libfec_hip.so (and the HIP runtime for the device-resident floor).  Not part of the library.
//
//   latency [calls_per_point]   ->  one JSON object per line
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "fec_hip.h"

namespace {

using Clock = std::chrono::steady_clock;

template <typename F>
void run_point(const char* api, const char* mem, uint64_t G, uint32_t k, uint32_t P, int calls, F&& fn) {
  for (int i = 0; i < 10; ++i)
    if (fn() != 0) {
      std::printf("{\"api\": \"%s\", \"error\": \"%s\"}\n", api, fec_hip_last_error());
      std::exit(1);
    }
  std::vector<double> us(calls);
  for (int i = 0; i < calls; ++i) {
    const auto t0 = Clock::now();
    const int rc = fn();
    us[i] = std::chrono::duration<double, std::micro>(Clock::now() - t0).count();
    if (rc != 0) {
      std::printf("{\"api\": \"%s\", \"error\": \"%s\"}\n", api, fec_hip_last_error());
      std::exit(1);
    }
  }
  std::sort(us.begin(), us.end());
  const double med = us[us.size() / 2], p99 = us[us.size() * 99 / 100];
  std::printf("{\"api\": \"%s\", \"host_memory\": \"%s\", \"groups\": %llu, \"k\": %u, \"P\": %u, "
              "\"median_us\": %.2f, \"p99_us\": %.2f, \"min_us\": %.2f, \"payload_GiBps\": %.3f}\n",
              api, mem, (unsigned long long)G, k, P, med, p99, us[0], G * k * P / (med * 1e-6) / (1u << 30));
  std::fflush(stdout);
}

}  // namespace

int main(int argc, char** argv) {
  const int calls = argc > 1 ? std::atoi(argv[1]) : 200;
  // LATENCY_SCHED=spin|yield|blocking: the HIP runtime's wait mode, set before any context
  // exists (the library leaves the process default, auto)
  if (const char* m = std::getenv("LATENCY_SCHED")) {
    const unsigned f = !std::strcmp(m, "spin") ? hipDeviceScheduleSpin
                       : !std::strcmp(m, "yield") ? hipDeviceScheduleYield
                                                  : hipDeviceScheduleBlockingSync;
    if (hipSetDeviceFlags(f) != hipSuccess) std::fprintf(stderr, "hipSetDeviceFlags(%s) failed\n", m);
  }
  if (fec_hip_device_count() <= 0) {
    std::fprintf(stderr, "no GPU\n");
    return 2;
  }
  FECEncoderCtx* ctx = fec_encoder_new(0.10, 1024);
  if (!ctx) return 2;
  const uint32_t P = 1200, k = 10, r = 3;
  const uint64_t Gmax = 16384;
  uint8_t* slab = static_cast<uint8_t*>(fec_alloc_slab(Gmax * k * P));
  uint8_t* rep = static_cast<uint8_t*>(fec_alloc_repair_buffer(Gmax * r * P));
  std::vector<uint8_t> slab_pg(Gmax * k * P), rep_pg(Gmax * r * P);
  for (uint64_t i = 0; i < Gmax * k * P; ++i) slab[i] = slab_pg[i] = static_cast<uint8_t>(i * 2654435761u >> 13);
  std::vector<uint32_t> off(Gmax * k);
  for (uint64_t i = 0; i < off.size(); ++i) off[i] = static_cast<uint32_t>(i * P);
  std::vector<uint64_t> masks(Gmax);
  for (uint64_t g = 0; g < Gmax; ++g) masks[g] = 1ull << (g % k);  // one data loss per group
  // fec_encode_batch with nothing to do: the cost of crossing the C-ABI alone
  run_point("fec_encode_batch (0 groups)", "-", 0, k, P, calls,
            [&] { return fec_encode_batch(ctx, slab, off.data(), 0, P, rep); });
  // Floor: the same kernel on device-resident buffers (no PCIe), launch + synchronize.
  void *d_in = nullptr, *d_out = nullptr;
  if (hipMalloc(&d_in, k * P) == hipSuccess && hipMalloc(&d_out, r * P) == hipSuccess) {
    run_point("fec_encode_batch_rs_dev r=3 + fec_synchronize", "device", 1, k, P, calls, [&] {
      const int rc = fec_encode_batch_rs_dev(ctx, static_cast<uint8_t*>(d_in), 1, k, r, P, static_cast<uint8_t*>(d_out),
                                             nullptr);
      return rc != 0 ? rc : fec_synchronize(ctx);
    });
  }
  for (uint64_t G : {1ull, 4ull, 16ull, 64ull, 256ull, 1024ull, 4096ull, 16384ull}) {
    run_point("fec_encode_batch", "pinned", G, k, P, calls,
              [&] { return fec_encode_batch(ctx, slab, off.data(), static_cast<uint32_t>(G), P, rep); });
    run_point("fec_encode_batch", "pageable", G, k, P, calls,
              [&] { return fec_encode_batch(ctx, slab_pg.data(), off.data(), static_cast<uint32_t>(G), P, rep_pg.data()); });
    run_point("fec_encode_batch_rs r=3", "pinned", G, k, P, calls,
              [&] { return fec_encode_batch_rs(ctx, slab, nullptr, G, k, r, P, rep); });
    run_point("fec_decode_batch_rs r=3 (1 loss/group)", "pinned", G, k, P, calls, [&] {
      return fec_decode_batch_rs(ctx, slab, rep, masks.data(), G, k, r, P, nullptr, nullptr);
    });
  }
  (void)hipFree(d_in);
  (void)hipFree(d_out);
  fec_free_slab(slab);
  fec_free_repair_buffer(rep);
  fec_encoder_free(ctx);
  return 0;
}
