// host_mirror_test.cpp — the reference's internal/fec/encoder_test.go, restated against the
// C++ mirror (quic-test_amd/host/fec.hpp) running on the GPU, with the byte-level
// assertions the reference tests never make checked against the oracle.
// Run by tests/test_host_mirror.py (GPU).  Prints "PASS <n>" or the failures.
#include <atomic>
#include <cstdio>
#include <cstring>
#include <random>
#include <thread>
#include <vector>

#include "fec.hpp"

extern "C" {
int64_t oracle_go_generate_redundancy(const uint8_t* const*, const size_t*, size_t, uint64_t, uint8_t*, size_t);
void oracle_xor_scalar(const uint8_t* const*, size_t, size_t, uint8_t*);
int oracle_rs_encode(const uint8_t*, uint64_t, uint32_t, uint32_t, uint32_t, uint8_t*, int);
void oracle_fill_splitmix(uint8_t*, uint64_t, uint64_t, uint64_t);
}

using namespace quicfec;

static int g_fail = 0, g_checks = 0;
#define CHECK(c)                                                          \
  do {                                                                    \
    ++g_checks;                                                           \
    if (!(c)) {                                                           \
      ++g_fail;                                                           \
      std::printf("FAIL %s:%d %s\n", __func__, __LINE__, #c);             \
    }                                                                     \
  } while (0)

static Bytes rep(uint8_t v, size_t n) { return Bytes(n, v); }
static Bytes rnd(size_t n, uint64_t seed) {
  Bytes b(n);
  oracle_fill_splitmix(b.data(), n, seed, 0);
  return b;
}

static Bytes go_redundancy(const std::vector<Bytes>& pk, uint64_t gid) {
  std::vector<const uint8_t*> p;
  std::vector<size_t> l;
  size_t mx = 0;
  for (auto& x : pk) {
    p.push_back(x.data());
    l.push_back(x.size());
    mx = std::max(mx, x.size());
  }
  Bytes out(11 + mx);
  const int64_t n = oracle_go_generate_redundancy(p.data(), l.data(), pk.size(), gid, out.data(), out.size());
  out.resize(n < 0 ? 0 : size_t(n));
  return out;
}

// encoder_test.go:9-36
static void TestNewFECEncoder() {
  for (double r : {0.10, 0.05, 0.20, -0.10, 0.0, 1.5}) {
    HybridFECEncoder e(r);
    CHECK(e.redundancy() > 0 && e.redundancy() <= 1);
    CHECK(e.UseCXX());
  }
}

// encoder_test.go:39-63
static void TestAddPacket() {
  HybridFECEncoder e(0.10);
  for (int i = 0; i < 5; ++i) {
    auto r = e.AddPacket(rep(uint8_t(i), 1200), i);
    CHECK(r.err.ok());
    CHECK(!r.needsRedundancy);
  }
  CHECK(e.GetMetrics().PacketsEncoded <= 5);
  CHECK(e.buffered() == 5);
}

// encoder_test.go:66-93, plus the known answer: FE C0 | 0 x8 | 0A | 1200 x 0x01
static void TestFECEncoderFullGroup() {
  HybridFECEncoder e(0.10);
  for (int i = 0; i < 10; ++i) {
    auto r = e.AddPacket(rep(uint8_t(i), 1200), i);
    CHECK(r.err.ok());
    if (i == 9) {
      CHECK(r.needsRedundancy);
      CHECK(r.redundancy.size() == 1211);
      const uint8_t hdr[11] = {0xFE, 0xC0, 0, 0, 0, 0, 0, 0, 0, 0, 10};
      CHECK(std::memcmp(r.redundancy.data(), hdr, 11) == 0);
      bool ones = true;
      for (size_t b = 11; b < r.redundancy.size(); ++b) ones &= r.redundancy[b] == 1;
      CHECK(ones);
    } else {
      CHECK(!r.needsRedundancy);
    }
  }
  CHECK(e.GetMetrics().GroupsProcessed >= 1);
}

// encoder_test.go:96-117
static void TestFECEncoderResetAfterGroup() {
  HybridFECEncoder e(0.10);
  for (int i = 0; i < 10; ++i) e.AddPacket(rep(uint8_t(i), 1200), i);
  auto r = e.AddPacket(rep(99, 1200), 10);
  CHECK(r.err.ok());
  CHECK(!r.needsRedundancy);
}

// encoder_test.go:120-151
static void TestDecoderBasics() {
  FECDecoder d;
  CHECK(d.groups() == 0);
  d.AddPacket(rep(0xAA, 1200), 1, 1);
  CHECK(d.GetMetrics().PacketsReceived == 1);
  CHECK(d.groups() == 1);
  CHECK(d.GetMetrics().PacketsReceived == 1);
}

// encoder_test.go:154-181, completed: the repair packet is fed to the decoder and the lost
// packet must come back byte for byte.
static void TestDecoderRecovery() {
  for (int order = 0; order < 2; ++order) {
    HybridFECEncoder e(0.10);
    FECDecoder d;
    std::vector<Bytes> pk;
    Bytes repair;
    for (int i = 0; i < 10; ++i) {
      pk.push_back(rnd(1200, 1000 + i));
      auto r = e.AddPacket(pk.back(), i);
      if (r.needsRedundancy) repair = r.redundancy;
    }
    CHECK(repair.size() == 1211);
    if (order == 0) {
      for (int i = 0; i < 10; ++i)
        if (i != 5) CHECK(!d.AddPacket(pk[i], i, 0));
      auto res = d.AddRedundancyPacket(repair);
      CHECK(res.first);
      CHECK(res.second.empty());  // reference quirk: rebuilt id already marked present
    } else {
      CHECK(!d.AddRedundancyPacket(repair).first);
      bool rec = false;
      for (int i = 0; i < 10; ++i)
        if (i != 5) rec = d.AddPacket(pk[i], i, 0);
      CHECK(rec);  // the 9th packet leaves one loss: recovered
      CHECK(d.GetMetrics().FailedRecoveries == 9);  // the repair and 8 arrivals saw > 1 missing
    }
    CHECK(d.GetPacket(0, 5) == pk[5]);
    CHECK(d.GetMetrics().PacketsRecovered == 1);
    CHECK(d.GetMetrics().RecoveryEvents == 1);
  }
}

// encoder_test.go:184-206
static void TestEncoderWithDifferentRedundancy() {
  for (double red : {0.05, 0.10, 0.15, 0.20}) {
    HybridFECEncoder e(red);
    for (int i = 0; i < 10; ++i) CHECK(e.AddPacket(rep(uint8_t(i), 1200), i).err.ok());
    CHECK(e.GetMetrics().PacketsEncoded != 0);
  }
}

// encoder_test.go:247-271
static void TestEncoderConcurrency() {
  HybridFECEncoder e(0.10);
  std::vector<std::thread> th;
  std::atomic<int> errors{0};
  for (int id = 0; id < 10; ++id)
    th.emplace_back([&, id] {
      for (int j = 0; j < 50; ++j)
        if (!e.AddPacket(rep(uint8_t(id), 1200), uint64_t(id * 100 + j)).err.ok()) errors++;
    });
  for (auto& t : th) t.join();
  CHECK(errors == 0);
  CHECK(e.GetMetrics().PacketsEncoded == 500);
  CHECK(e.GetMetrics().GroupsProcessed == 50);
}

// encoder_test.go:274-291, completed with an aged group
static void TestDecoderGroupsExpiration() {
  FECDecoder d;
  Bytes p(1200, 0);
  p[0] = 0xAA;
  d.AddPacket(p, 1, 1);
  d.CleanupGroups();
  CHECK(d.groups() == 1);
  d.AgeGroupsForTest(6);
  d.CleanupGroups();
  CHECK(d.groups() == 0);
  CHECK(d.GetMetrics().GroupsEvicted == 1);
}

// decoder.go:10, :98-103: more than 4096 live groups evicts the oldest
static void TestDecoderEviction() {
  FECDecoder d;
  Bytes p(100, 1);
  for (uint64_t g = 0; g < FECDecoder::kMaxActiveGroups + 3; ++g) d.AddPacket(p, 0, g);
  CHECK(d.groups() == FECDecoder::kMaxActiveGroups);
  CHECK(d.GetMetrics().GroupsEvicted == 3);
}

// Go semantics for uneven groups: zero padding to the longest packet; a Flush of a partial
// group XORs only the packets present (encoder.go:118-157)
static void TestVariableLengthAndFlushMatchGo() {
  HybridFECEncoder e(0.10);
  std::vector<Bytes> pk;
  std::mt19937 rng(7);
  Bytes repair;
  for (int i = 0; i < 10; ++i) {
    pk.push_back(rnd(200 + rng() % 1000, 2000 + i));
    auto r = e.AddPacket(pk.back(), i);
    if (r.needsRedundancy) repair = r.redundancy;
  }
  CHECK(repair == go_redundancy(pk, 0));
  std::vector<Bytes> part = {rnd(300, 1), rnd(77, 2), rnd(1500, 3)};
  for (size_t i = 0; i < part.size(); ++i) e.AddPacket(part[i], 100 + i);
  auto fl = e.Flush();
  CHECK(fl.second.ok());
  CHECK(fl.first == go_redundancy(part, 1));
  CHECK(e.Flush().first.empty());
}

// FECEncoderCXX.EncodeBatch over many groups, against the scalar XOR definition
static void TestEncodeBatchManyGroups() {
  auto enc = FECEncoderCXX::New(0.1, 16);
  CHECK(enc != nullptr);
  if (!enc) return;
  std::vector<FECBatchGroup> groups(300);
  for (size_t g = 0; g < groups.size(); ++g)
    for (int j = 0; j < 10; ++j) groups[g].Packets.push_back(rnd(1200, 50000 + g * 10 + j));
  std::vector<RepairPacket> out;
  CHECK(enc->EncodeBatch(groups, 1200, &out).ok());
  CHECK(out.size() == groups.size());
  bool all = true;
  for (size_t g = 0; g < groups.size(); ++g) {
    std::vector<const uint8_t*> p;
    for (auto& x : groups[g].Packets) p.push_back(x.data());
    Bytes exp(1200);
    oracle_xor_scalar(p.data(), p.size(), 1200, exp.data());
    all &= out[g] == exp;
  }
  CHECK(all);
  CHECK(enc->EncodeBatch({}, 1200, &out).ok() && out.empty());
  enc->Close();
  CHECK(!enc->EncodeBatch(groups, 1200, &out).ok());  // "encoder not initialized"
}

// batch extension: up to r losses per group
static void TestBatchRS() {
  const int k = 10, r = 3, P = 1200, G = 500;
  Bytes data = rnd(size_t(G) * k * P, 77), parity;
  CHECK(EncodeBatchRS(data, k, r, P, &parity).ok());
  Bytes ref(size_t(G) * r * P);
  oracle_rs_encode(data.data(), G, k, r, P, ref.data(), 4);
  CHECK(parity == ref);
  std::vector<uint64_t> er(G);
  std::mt19937_64 rng(3);
  Bytes broken = data;
  for (int g = 0; g < G; ++g) {
    uint64_t m = 0;
    while (__builtin_popcountll(m) < int(g % (r + 1))) m |= 1ull << (rng() % (k + r));
    er[g] = m;
    for (int j = 0; j < k; ++j)
      if ((m >> j) & 1) std::memset(&broken[(size_t(g) * k + j) * P], 0, P);
  }
  Error err;
  CHECK(RecoverBatchRS(broken, parity, er, k, r, P, &err) == 0);
  CHECK(err.ok());
  CHECK(broken == data);
}

int main() {
  TestNewFECEncoder();
  TestAddPacket();
  TestFECEncoderFullGroup();
  TestFECEncoderResetAfterGroup();
  TestDecoderBasics();
  TestDecoderRecovery();
  TestEncoderWithDifferentRedundancy();
  TestEncoderConcurrency();
  TestDecoderGroupsExpiration();
  TestDecoderEviction();
  TestVariableLengthAndFlushMatchGo();
  TestEncodeBatchManyGroups();
  TestBatchRS();
  if (g_fail) {
    std::printf("FAILED %d of %d checks\n", g_fail, g_checks);
    return 1;
  }
  std::printf("PASS %d\n", g_checks);
  return 0;
}
