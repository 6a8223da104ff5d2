// probe_placement.cpp — where does the C3 recover's placement penalty come from? (VERDICT r05
// "next round" item 1).  Not part of the library.
//
// One process: data (1M groups of k=10 x 1200 B) and parity are made once with the library
// (fec_fill_random_dev, fec_encode_batch_rs_dev); the slot-row recover (fec_recover_batch_rs_dev,
// 2 erasures per group, the bench's C3) is then timed into rebuilt buffers placed in different
// ways, 10 launches each on one stream (HIP events):
//   * plain hipMalloc buffers in allocation order (round 5: the first one is slow);
//   * hipExtMallocWithFlags(hipDeviceMallocContiguous) (round 3: slowest);
//   * buffers built with the virtual-memory API from `chunk`-byte physical handles, mapped in
//     allocation order, reversed, or in a seeded random order — the same physical pages with a
//     different virtual order, i.e. a different relation between the streams' physical addresses;
//   * data and rebuilt in ONE physically contiguous allocation, rebuilt at data_end + delta
//     (the data<->rebuilt relation, never swept before; parity<->rebuilt was, flat);
//   * the data itself copied into chunk-shuffled memory, with the first (slow) rebuilt buffer.
// One JSON object per line.
//
//   probe_placement [--chunk-mb 2] [--reps 10] [--groups 1000000] [--skip-delta] [--data-vmm] [--waves]
//
// --waves (built against libfec_hip_test.so, whose QUICFEC_DECODE_WAVES caps the recover's
// occupancy): the first plain buffer and a physically contiguous one at 8 .. 40 waves per CU and
// uncapped -- whether fewer requests in flight ease the slow placement's DRAM credit stalls.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <random>
#include <string>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "fec_hip.h"

namespace {

constexpr uint32_t K = 10, R = 3, P = 1200;

#define HIPCHK(x)                                                                          \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      std::printf("{\"error\": \"%s\", \"at\": %d}\n", hipGetErrorString(e_), __LINE__); \
      std::exit(1);                                                                        \
    }                                                                                      \
  } while (0)

uint64_t splitmix(uint64_t& s) {
  uint64_t z = (s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// A device buffer made of `chunk`-byte physical handles mapped into one virtual range in the
// given order (perm[i] = which handle backs virtual chunk i).
struct VmmBuffer {
  void* va = nullptr;
  size_t bytes = 0, chunk = 0, mapped = 0;
  std::vector<hipMemGenericAllocationHandle_t> handles;  // only the ones created
  const char* failed = nullptr;

  bool create(size_t want, size_t chunk_bytes, const std::vector<size_t>& perm_in, int dev) {
    chunk = chunk_bytes;
    const size_t n = (want + chunk - 1) / chunk;
    bytes = n * chunk;
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = dev;
    handles.reserve(n);
    for (size_t i = 0; i < n; ++i) {
      hipMemGenericAllocationHandle_t h{};
      if (hipMemCreate(&h, chunk, &prop, 0) != hipSuccess) return fail("hipMemCreate");
      handles.push_back(h);
    }
    if (hipMemAddressReserve(&va, bytes, chunk, nullptr, 0) != hipSuccess) {
      va = nullptr;
      return fail("hipMemAddressReserve");
    }
    std::vector<size_t> perm = perm_in;
    if (perm.size() != n) {
      perm.resize(n);
      std::iota(perm.begin(), perm.end(), 0);
    }
    for (size_t i = 0; i < n; ++i, ++mapped)
      if (hipMemMap(static_cast<char*>(va) + i * chunk, chunk, 0, handles[perm[i]], 0) != hipSuccess) return fail("hipMemMap");
    hipMemAccessDesc acc{};
    acc.location.type = hipMemLocationTypeDevice;
    acc.location.id = dev;
    acc.flags = hipMemAccessFlagsProtReadWrite;
    if (hipMemSetAccess(va, bytes, &acc, 1) != hipSuccess) return fail("hipMemSetAccess");
    return true;
  }
  bool fail(const char* what) {
    failed = what;
    (void)hipGetLastError();
    return false;
  }
  void destroy() {
    for (size_t i = 0; i < mapped; ++i) (void)hipMemUnmap(static_cast<char*>(va) + i * chunk, chunk);
    if (va) (void)hipMemAddressFree(va, bytes);
    for (auto h : handles) (void)hipMemRelease(h);
    handles.clear();
    va = nullptr;
    mapped = 0;
  }
};

}  // namespace

int main(int argc, char** argv) {
  size_t chunk_mb = 2;
  int reps = 10;
  uint64_t G = 1000000;
  bool skip_delta = false, data_vmm = false, waves_sweep = false;
  for (int i = 1; i < argc; ++i) {
    if (!std::strcmp(argv[i], "--chunk-mb") && i + 1 < argc) chunk_mb = std::strtoull(argv[++i], nullptr, 10);
    else if (!std::strcmp(argv[i], "--reps") && i + 1 < argc) reps = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "--groups") && i + 1 < argc) G = std::strtoull(argv[++i], nullptr, 10);
    else if (!std::strcmp(argv[i], "--skip-delta")) skip_delta = true;
    else if (!std::strcmp(argv[i], "--data-vmm")) data_vmm = true;
    else if (!std::strcmp(argv[i], "--waves")) waves_sweep = true;
  }
  if (fec_hip_device_count() <= 0) {
    std::printf("{\"error\": \"no GPU\"}\n");
    return 1;
  }
  const int dev = 0;
  HIPCHK(hipSetDevice(dev));
  FECEncoderCtx* ctx = fec_encoder_new_device(0.3, 1024, dev);
  if (!ctx) {
    std::printf("{\"error\": \"fec_encoder_new_device: %s\"}\n", fec_hip_last_error());
    return 1;
  }
  hipStream_t st;
  HIPCHK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const size_t data_bytes = G * K * P, par_bytes = G * R * P;

  hipMemAllocationProp prop{};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = dev;
  size_t gran = 0;
  HIPCHK(hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityMinimum));
  size_t chunk = std::max<size_t>(chunk_mb << 20, gran);
  chunk = (chunk + gran - 1) / gran * gran;
  std::printf("{\"kind\": \"setup\", \"groups\": %llu, \"granularity\": %zu, \"chunk\": %zu}\n",
              (unsigned long long)G, gran, chunk);

  uint8_t *data = nullptr, *parity = nullptr;
  uint64_t* masks = nullptr;
  HIPCHK(hipMalloc(&data, data_bytes));
  HIPCHK(hipMalloc(&parity, par_bytes));
  HIPCHK(hipMalloc(&masks, G * 8));
  if (fec_fill_random_dev(ctx, data, data_bytes, 0x5EED0002ull, 0, st) != 0 ||
      fec_encode_batch_rs_dev(ctx, data, G, K, R, P, parity, st) != 0) {
    std::printf("{\"error\": \"setup: %s\"}\n", fec_hip_last_error());
    return 1;
  }
  {  // 2 distinct erased shards of the 13 per group (the bench's C3 erasure model)
    std::vector<uint64_t> hm(G);
    uint64_t s = 0x5EED0003ull;
    for (uint64_t g = 0; g < G; ++g) {
      const uint32_t a = splitmix(s) % (K + R);
      uint32_t b = splitmix(s) % (K + R - 1);
      if (b >= a) ++b;
      hm[g] = (1ull << a) | (1ull << b);
    }
    HIPCHK(hipMemcpy(masks, hm.data(), G * 8, hipMemcpyHostToDevice));
  }
  uint64_t book = 0;
  if (fec_decode_prepare(ctx, K, R, &book) != 0) {
    std::printf("{\"error\": \"prepare: %s\"}\n", fec_hip_last_error());
    return 1;
  }
  HIPCHK(hipStreamSynchronize(st));

  hipEvent_t e0, e1;
  HIPCHK(hipEventCreate(&e0));
  HIPCHK(hipEventCreate(&e1));
  auto timed = [&](const uint8_t* d, uint8_t* rb) -> double {
    if (fec_recover_batch_rs_dev(ctx, d, parity, masks, G, K, R, P, rb, nullptr, st) != 0) {
      std::printf("{\"error\": \"recover: %s\"}\n", fec_hip_last_error());
      std::exit(1);
    }
    HIPCHK(hipEventRecord(e0, st));
    for (int i = 0; i < reps; ++i) (void)fec_recover_batch_rs_dev(ctx, d, parity, masks, G, K, R, P, rb, nullptr, st);
    HIPCHK(hipEventRecord(e1, st));
    HIPCHK(hipEventSynchronize(e1));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    return ms / reps;
  };
  auto out = [&](const char* kind, double ms, const void* rb, const char* extra = "") {
    std::printf("{\"kind\": \"%s\", \"ms\": %.4f, \"data\": \"%p\", \"parity\": \"%p\", \"rebuilt\": \"%p\"%s}\n",
                kind, ms, (const void*)data, (const void*)parity, rb, extra);
    std::fflush(stdout);
  };

  // 1. plain hipMalloc in allocation order
  std::vector<uint8_t*> plain;
  for (int i = 0; i < 3; ++i) {
    uint8_t* rb = nullptr;
    HIPCHK(hipMalloc(&rb, par_bytes));
    plain.push_back(rb);
    out("hipMalloc", timed(data, rb), rb, (",\"order\": " + std::to_string(i)).c_str());
  }
  // 2. physically contiguous
  {
    uint8_t* rb = nullptr;
    if (hipExtMallocWithFlags(reinterpret_cast<void**>(&rb), par_bytes, hipDeviceMallocContiguous) == hipSuccess) {
      out("contiguous", timed(data, rb), rb);
      HIPCHK(hipFree(rb));
    } else {
      std::printf("{\"kind\": \"contiguous\", \"error\": \"alloc\"}\n");
    }
  }
  if (waves_sweep) {
    uint8_t* rc = nullptr;
    const bool have_c =
        hipExtMallocWithFlags(reinterpret_cast<void**>(&rc), par_bytes, hipDeviceMallocContiguous) == hipSuccess;
    for (int pass = 0; pass < 2; ++pass)
      for (int w : {0, 8, 12, 16, 20, 24, 32, 40}) {
        if (w) setenv("QUICFEC_DECODE_WAVES", std::to_string(w).c_str(), 1);
        else unsetenv("QUICFEC_DECODE_WAVES");
        const std::string ex = ",\"waves\": " + std::to_string(w) + ", \"pass\": " + std::to_string(pass);
        out("waves_hipMalloc", timed(data, plain[0]), plain[0], ex.c_str());
        if (have_c) out("waves_contiguous", timed(data, rc), rc, ex.c_str());
      }
    unsetenv("QUICFEC_DECODE_WAVES");
    if (have_c) HIPCHK(hipFree(rc));
  }
  // 3. data and rebuilt in one physically contiguous allocation: rebuilt at data_end + delta
  if (!skip_delta) {
    const size_t MB = 1 << 20;
    const size_t deltas[] = {0, 4096, 65536, 256 * 1024, MB, 2 * MB, 3 * MB, 4 * MB, 6 * MB, 8 * MB,
                             12 * MB, 16 * MB, 24 * MB, 32 * MB, 64 * MB, 128 * MB, 256 * MB};
    const size_t span = (data_bytes + 2 * MB - 1) / (2 * MB) * (2 * MB);
    const size_t total = span + par_bytes + 256 * MB + 2 * MB;
    for (int alloc = 0; alloc < 2; ++alloc) {
      uint8_t* base = nullptr;
      const hipError_t rc = alloc == 0 ? hipExtMallocWithFlags(reinterpret_cast<void**>(&base), total,
                                                               hipDeviceMallocContiguous)
                                       : hipMalloc(&base, total);
      const char* an = alloc == 0 ? "contiguous" : "hipMalloc";
      if (rc != hipSuccess) {
        std::printf("{\"kind\": \"delta\", \"alloc\": \"%s\", \"error\": \"alloc\"}\n", an);
        continue;
      }
      if (fec_copy_dev(ctx, data, base, data_bytes, st) != 0) {
        std::printf("{\"error\": \"copy: %s\"}\n", fec_hip_last_error());
        return 1;
      }
      HIPCHK(hipStreamSynchronize(st));
      for (size_t d : deltas) {
        char extra[96];
        std::snprintf(extra, sizeof extra, ",\"alloc\": \"%s\", \"delta\": %zu", an, d);
        uint8_t* rb = base + span + d;
        const double ms = timed(base, rb);
        std::printf("{\"kind\": \"delta\", \"ms\": %.4f, \"data\": \"%p\", \"rebuilt\": \"%p\"%s}\n", ms,
                    (void*)base, (void*)rb, extra);
        std::fflush(stdout);
      }
      HIPCHK(hipFree(base));
    }
  }
  // 4. the first (slow?) plain buffer again, then the data copied into shuffled chunks
  out("hipMalloc_again", timed(data, plain[0]), plain[0], ",\"order\": 0");
  if (data_vmm) {  // (aborted inside the runtime on three boxes with 64-MB handles: opt-in)
    const size_t dchunk = std::max<size_t>(chunk, 64u << 20);  // fewer handles for 12 GB
    std::vector<size_t> dperm((data_bytes + dchunk - 1) / dchunk);
    std::iota(dperm.begin(), dperm.end(), 0);
    std::shuffle(dperm.begin(), dperm.end(), std::mt19937_64(0xDA7A));
    VmmBuffer d2;
    if (d2.create(data_bytes, dchunk, dperm, dev)) {
      // a kernel copy: the runtime's memcpy does not know virtual-memory ranges
      if (fec_copy_dev(ctx, data, static_cast<uint8_t*>(d2.va), data_bytes, st) != 0) {
        std::printf("{\"error\": \"copy: %s\"}\n", fec_hip_last_error());
        return 1;
      }
      HIPCHK(hipStreamSynchronize(st));
      for (int i = 0; i < 3; ++i)
        out("data_shuffled", timed(static_cast<uint8_t*>(d2.va), plain[i]), plain[i],
            (",\"order\": " + std::to_string(i)).c_str());
    } else {
      std::printf("{\"kind\": \"data_shuffled\", \"error\": \"%s\", \"handles\": %zu}\n", d2.failed, d2.handles.size());
    }
    d2.destroy();
  }
  // 5. virtual-memory buffers (last: after a virtual range is freed, the next large ordinary
  // allocation aborted inside the runtime on three boxes, "Memobj map does not have ptr"): the same physical handles in three virtual orders
  const size_t nchunks = (par_bytes + chunk - 1) / chunk;
  std::vector<size_t> ident(nchunks), rev(nchunks), shuf(nchunks);
  std::iota(ident.begin(), ident.end(), 0);
  std::reverse_copy(ident.begin(), ident.end(), rev.begin());
  shuf = ident;
  std::shuffle(shuf.begin(), shuf.end(), std::mt19937_64(0xC3C3));
  for (int pass = 0; pass < 2; ++pass) {
    const char* names[3] = {"vmm_in_order", "vmm_reversed", "vmm_shuffled"};
    const std::vector<size_t>* perms[3] = {&ident, &rev, &shuf};
    for (int v = 0; v < 3; ++v) {
      VmmBuffer b;
      if (!b.create(par_bytes, chunk, *perms[v], dev)) {
        std::printf("{\"kind\": \"%s\", \"error\": \"%s\"}\n", names[v], b.failed);
        b.destroy();
        continue;
      }
      out(names[v], timed(data, static_cast<uint8_t*>(b.va)), b.va, (",\"pass\": " + std::to_string(pass)).c_str());
      b.destroy();
    }
  }
  for (auto* p : plain) HIPCHK(hipFree(p));
  HIPCHK(hipFree(masks));
  HIPCHK(hipFree(parity));
  HIPCHK(hipFree(data));
  HIPCHK(hipStreamDestroy(st));
  fec_encoder_free(ctx);
  return 0;
}
