// probe_c4.hip — development probe: what bounds the C4 encode (k=20 r=5, 1200 B, 1M groups).
// The product's two forms (the v_perm tables, encode_v16; the bit-sliced two-groups-per-lane
// encode_bits) next to memory-only kernels with exactly their access patterns (the XOR of the
// packets instead of the GF rows, the same loads and stores): if encode_v16's pattern streams
// faster than encode_bits' without arithmetic, the bit-sliced form's memory pattern is what
// costs; if not, the k=20 r=5 read/write mix itself is the ceiling.  Not part of the library.
//
//   probe_c4 [groups] [rounds]
#include "../fec_kernels.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <functional>
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

namespace qfec {
namespace {
// encode_v16's tiled mapping (a workgroup owns `tile` whole groups, XCD-aware order), K loads
// of one 16-B column, their XOR stored as R rows (rotated so no store is folded away).
template <int K, int R>
__global__ __launch_bounds__(512) void v16_mem(const uint8_t* __restrict__ data, uint8_t* __restrict__ parity,
                                               uint32_t cpp, uint32_t P, uint32_t tile, uint64_t groups, uint32_t never) {
  extern __shared__ __attribute__((aligned(16))) uint8_t occupancy_lds[];
  if (never) occupancy_lds[threadIdx.x] = 0;
  const uint32_t lane = threadIdx.x;
  uint32_t gl = lane / cpp;
  const uint32_t col = lane - gl * cpp;
  if (gl >= tile) return;
  gl += xcd_tile(blockIdx.x, gridDim.x) * tile;
  if (gl >= groups) return;
  const uint64_t g = gl;
  const uint32_t o = col_off16(col, P);
  u32x4 d[K];
#pragma unroll
  for (int j = 0; j < K; ++j) d[j] = ld16<0>(data + (g * K + j) * static_cast<uint64_t>(P) + o);
  u32x4 a = d[0];
#pragma unroll
  for (int j = 1; j < K; ++j) a ^= d[j];
#pragma unroll
  for (int i = 0; i < R; ++i) {
    st16<kNtStore>(parity + (g * R + i) * static_cast<uint64_t>(P) + o, a);
    a = a.yzwx;
  }
}

// encode_bits' mapping (a lane owns one column of groups gl and gl + tile of its workgroup's
// 2 * tile groups; packets stream through a window of W), XOR only, 2R stores.
template <int K, int R, int W>
__global__ __launch_bounds__(512) void bits_mem(const uint8_t* __restrict__ data, uint8_t* __restrict__ parity,
                                                uint32_t cpp, uint32_t P, uint32_t tile, uint64_t groups, uint32_t never) {
  extern __shared__ __attribute__((aligned(16))) uint8_t occupancy_lds[];
  if (never) occupancy_lds[threadIdx.x] = 0;
  const uint32_t lane = threadIdx.x;
  uint32_t gl = lane / cpp;
  const uint32_t c = lane - gl * cpp;
  if (gl >= tile) return;
  gl += xcd_tile(blockIdx.x, gridDim.x) * (2 * tile);
  if (gl >= groups) return;
  const bool second = gl + tile < groups;
  const uint64_t g = gl, g2 = second ? g + tile : g;
  const uint32_t o = col_off16(c, P);
  const uint8_t* base = data + g * K * static_cast<uint64_t>(P) + o;
  const uint8_t* base2 = data + g2 * K * static_cast<uint64_t>(P) + o;
  u32x4 ba[W], bb[W];
#pragma unroll
  for (int j = 0; j < W; ++j) {
    ba[j] = ld16<0>(base + static_cast<uint64_t>(j) * P);
    bb[j] = ld16<0>(base2 + static_cast<uint64_t>(j) * P);
  }
  u32x4 a = {0u, 0u, 0u, 0u}, b = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int j = 0; j < K; ++j) {
    a ^= ba[j % W];
    b ^= bb[j % W];
    if (j + W < K) {
      ba[j % W] = ld16<0>(base + static_cast<uint64_t>(j + W) * P);
      bb[j % W] = ld16<0>(base2 + static_cast<uint64_t>(j + W) * P);
    }
  }
#pragma unroll
  for (int i = 0; i < R; ++i) {
    st16<kNtStore>(parity + (g * R + i) * static_cast<uint64_t>(P) + o, a);
    a = a.yzwx;
  }
  if (second) {
#pragma unroll
    for (int i = 0; i < R; ++i) {
      st16<kNtStore>(parity + (g2 * R + i) * static_cast<uint64_t>(P) + o, b);
      b = b.yzwx;
    }
  }
}
}  // namespace
}  // namespace qfec

using namespace qfec;

int main(int argc, char** argv) {
  constexpr uint32_t k = 20, r = 5, P = 1200;
  const uint64_t G = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1000000;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 7;
  const uint64_t nd = G * k * P, np = G * r * P, enc_bytes = nd + np;
  uint8_t *data, *par, *par2, *scratch;
  CK(hipMalloc(&data, nd));
  CK(hipMalloc(&par, np));
  CK(hipMalloc(&par2, np));
  CK(hipMalloc(&scratch, nd / 2));
  CK(launch_fill_splitmix(data, nd, 0x5EED0004, 0, nullptr));
  std::vector<uint8_t> M;
  parity_matrix(k, r, M);
  std::vector<CoefEntry> tab;
  for (uint32_t i = 1; i < r; ++i)
    for (uint32_t j = 0; j < k; ++j) tab.push_back(make_entry(M[i * k + j]));
  void* dtab = nullptr;
  CK(hipMalloc(&dtab, tab.size() * 32));
  CK(hipMemcpy(dtab, tab.data(), tab.size() * 32, hipMemcpyHostToDevice));
  EncodeLaunch el{data, nullptr, OffsetKind::kNone, par, G, k, r, P, dtab};
  const uint32_t cpp = (P + 15) / 16, tile = pick_tile(cpp, k, P), bs = (tile * cpp + 63) / 64 * 64;
  struct Var {
    std::string name;
    uint64_t bytes;
    std::function<void()> fn;
    std::vector<float> ms;
  };
  std::vector<Var> vars;
  vars.push_back({"copy16 (R=W)", nd, [&] { CK(launch_copy_words(data, scratch, nd / 2, nullptr)); }, {}});
  vars.push_back({"prod encode_bits (default)", enc_bytes, [&] {
                    unsetenv("QUICFEC_ENCODE_BITS");
                    CK(launch_encode(el, nullptr));
                  }, {}});
  vars.push_back({"prod encode_v16 tables", enc_bytes, [&] {
                    setenv("QUICFEC_ENCODE_BITS", "0", 1);
                    EncodeLaunch e2 = el;
                    e2.parity = par2;
                    CK(launch_encode(e2, nullptr));
                    unsetenv("QUICFEC_ENCODE_BITS");
                  }, {}});
  for (int per_cu : {2, 3, 4, 0}) {
    const uint32_t smem = occupancy_cap_lds(per_cu * int(bs / 64), bs / 64);
    vars.push_back({"v16_mem x" + std::to_string(per_cu), enc_bytes, [=] {
                      v16_mem<20, 5><<<uint32_t((G + tile - 1) / tile), bs, smem>>>(data, par2, cpp, P, tile, G, 0u);
                    }, {}});
  }
  const uint32_t b2 = uint32_t((G + 2 * tile - 1) / (2 * tile));
  vars.push_back({"bits_mem W4", enc_bytes, [=] { bits_mem<20, 5, 4><<<b2, bs, 0>>>(data, par2, cpp, P, tile, G, 0u); }, {}});
  vars.push_back({"bits_mem W8", enc_bytes, [=] { bits_mem<20, 5, 8><<<b2, bs, 0>>>(data, par2, cpp, P, tile, G, 0u); }, {}});
  vars.push_back({"bits_mem W20", enc_bytes, [=] { bits_mem<20, 5, 20><<<b2, bs, 0>>>(data, par2, cpp, P, tile, G, 0u); }, {}});
  // the two product forms give the same bytes
  vars[1].fn();
  vars[2].fn();
  CK(hipDeviceSynchronize());
  std::vector<uint8_t> a(np), b(np);
  CK(hipMemcpy(a.data(), par, np, hipMemcpyDeviceToHost));
  CK(hipMemcpy(b.data(), par2, np, hipMemcpyDeviceToHost));
  std::printf("check bits == tables: %s\n", a == b ? "OK" : "MISMATCH");
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rd = 0; rd < rounds; ++rd)
    for (auto& v : vars) {
      CK(hipEventRecord(e0));
      v.fn();
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      v.ms.push_back(ms);
    }
  std::printf("k=%u r=%u P=%u groups=%llu tile=%u bs=%u\n%-30s %10s %10s %10s\n", k, r, P, (unsigned long long)G, tile, bs,
              "variant", "med_ms", "min_ms", "GB/s(med)");
  for (auto& v : vars) {
    std::sort(v.ms.begin(), v.ms.end());
    const float med = v.ms[v.ms.size() / 2];
    std::printf("%-30s %10.4f %10.4f %10.1f\n", v.name.c_str(), med, v.ms[0], v.bytes / (med * 1e-3) / 1e9);
  }
  return a == b ? 0 : 1;
}
