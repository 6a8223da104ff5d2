// ctx_isolation_test.cpp — many threads, one FECEncoderCtx each (one HybridFECEncoder per QUIC
// stream, client.go:783), each calling the reference's fec_encode_batch with one group per
// call (encoder_hybrid.go:115) on its own page-locked slab: random packet sizes, offsets
// shuffled inside the slab, every repair checked against the CPU XOR (fec_xor_simd.cpp:411-427).
// Contexts share nothing, so any cross-context aliasing of staging buffers shows up as a
// wrong repair.  Prints "PASS <calls>" or the first mismatches.
#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <algorithm>
#include <random>
#include <thread>
#include <vector>

#include "fec_hip.h"
#include "fec_xor_simd.h"

int main(int argc, char** argv) {
  const int threads = argc > 1 ? std::atoi(argv[1]) : 16;
  const int calls = argc > 2 ? std::atoi(argv[2]) : 2000;
  if (fec_hip_device_count() <= 0) {
    std::printf("no GPU\n");
    return 2;
  }
  std::atomic<long> bad{0}, done{0};
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t)
    th.emplace_back([&, t] {
      FECEncoderCtx* ctx = fec_encoder_new(0.10, 1024);
      const size_t slab_bytes = 10 * 1500 * 4;
      auto* slab = static_cast<uint8_t*>(fec_alloc_slab(slab_bytes));
      auto* rep = static_cast<uint8_t*>(fec_alloc_repair_buffer(1500));
      if (!ctx || !slab || !rep) {
        ++bad;
        return;
      }
      std::mt19937_64 rng(1000 + t);
      std::vector<uint32_t> off(10);
      std::vector<uint8_t> want(1500);
      for (int c = 0; c < calls; ++c) {
        const uint32_t P = 16 + uint32_t(rng() % 1485);
        // ten packet slots of P bytes at shuffled positions among 40 slots of the slab
        std::vector<uint32_t> slots(40);
        for (uint32_t i = 0; i < 40; ++i) slots[i] = i;
        std::shuffle(slots.begin(), slots.end(), rng);
        for (int j = 0; j < 10; ++j) off[j] = slots[j] * 1500;
        for (size_t i = 0; i < slab_bytes; i += 8) {
          const uint64_t v = rng();
          std::memcpy(slab + i, &v, 8);
        }
        std::memset(want.data(), 0, P);
        for (int j = 0; j < 10; ++j)
          for (uint32_t b = 0; b < P; ++b) want[b] ^= slab[off[j] + b];
        std::memset(rep, 0xA5, P);
        const int rc = fec_encode_batch(ctx, slab, off.data(), 1, P, rep);
        if (rc != 0 || std::memcmp(rep, want.data(), P) != 0) {
          if (bad.fetch_add(1) < 5) std::printf("thread %d call %d P=%u rc=%d: repair differs\n", t, c, P, rc);
        }
        ++done;
      }
      fec_free_repair_buffer(rep);
      fec_free_slab(slab);
      fec_encoder_free(ctx);
    });
  for (auto& x : th) x.join();
  if (bad) {
    std::printf("FAILED %ld of %ld calls\n", bad.load(), done.load());
    return 1;
  }
  std::printf("PASS %ld\n", done.load());
  return 0;
}
