// fec.cpp — C++ mirror of internal/fec (see fec.hpp) on top of libfec_hip.so's C-ABI.
#include "fec.hpp"

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstring>

#include "fec_hip.h"

namespace quicfec {

namespace {

Error errorf(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
Error errorf(const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  std::vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  return Error{buf};
}

double clamp_redundancy(double r) { return (r <= 0 || r > 1) ? 0.10 : r; }  // encoder.go:30-32

}  // namespace

// ===================================================================== FECEncoderCXX
std::unique_ptr<FECEncoderCXX> FECEncoderCXX::New(double redundancy, int maxGroups) {
  redundancy = clamp_redundancy(redundancy);  // fec_cgo.go:44-46
  if (maxGroups <= 0) maxGroups = 1024;       // fec_cgo.go:47-49
  std::unique_ptr<FECEncoderCXX> enc(new FECEncoderCXX());
  enc->maxGroups_ = maxGroups;
  enc->ctx_ = fec_encoder_new(redundancy, static_cast<uint32_t>(maxGroups));
  if (!enc->ctx_) return nullptr;
  // slab: maxGroups * 10 packets * 1200 B (+ one zero packet, see EncodeBatch)
  enc->slabSize_ = size_t(maxGroups) * 10 * 1200 + 1200;
  enc->slab_ = static_cast<uint8_t*>(fec_alloc_slab(enc->slabSize_));
  if (!enc->slab_) {
    fec_encoder_free(enc->ctx_);
    enc->ctx_ = nullptr;
    return nullptr;
  }
  enc->offsets_.reserve(size_t(maxGroups) * 10);
  enc->repairSize_ = size_t(maxGroups) * 1200;
  enc->repair_ = static_cast<uint8_t*>(fec_alloc_repair_buffer(enc->repairSize_));
  if (!enc->repair_) {
    fec_free_slab(enc->slab_);
    enc->slab_ = nullptr;
    fec_encoder_free(enc->ctx_);
    enc->ctx_ = nullptr;
    return nullptr;
  }
  enc->initialized_ = true;
  return enc;
}

FECEncoderCXX::~FECEncoderCXX() { Close(); }

Error FECEncoderCXX::resizeSlab(size_t newSize) {
  if (newSize <= slabSize_) return {};
  auto* p = static_cast<uint8_t*>(fec_alloc_slab(newSize));
  if (!p) return errorf("failed to allocate slab of size %zu", newSize);
  std::memcpy(p, slab_, slabSize_);
  fec_free_slab(slab_);
  slab_ = p;
  slabSize_ = newSize;
  return {};
}

Error FECEncoderCXX::resizeRepairBuffer(size_t newSize) {
  if (newSize <= repairSize_) return {};
  auto* p = static_cast<uint8_t*>(fec_alloc_repair_buffer(newSize));
  if (!p) return errorf("failed to allocate repair buffer of size %zu", newSize);
  fec_free_repair_buffer(repair_);
  repair_ = p;
  repairSize_ = newSize;
  return {};
}

Error FECEncoderCXX::EncodeBatch(const std::vector<FECBatchGroup>& groups, int packetSize,
                                 std::vector<RepairPacket>* out) {
  if (!initialized_) return errorf("encoder not initialized");  // fec_cgo.go:96-98
  if (out) out->clear();
  if (groups.empty()) return {};                                // :100-102
  if (packetSize <= 0) return errorf("invalid packet size %d", packetSize);
  std::lock_guard<std::mutex> lk(mu_);
  const size_t P = static_cast<size_t>(packetSize);
  // Slab layout: [zero packet][group 0 packet 0..9][group 1 ...], every packet padded to
  // packetSize.  Slots a group does not fill point at the zero packet, so a partial group
  // XORs exactly the packets it has (encoder.go:133-143).
  const size_t need = P + groups.size() * 10 * P;
  if (Error e = resizeSlab(need)) return errorf("failed to resize slab: %s", e.msg.c_str());
  if (need > 0xFFFFFFFFull) return errorf("batch exceeds the 4 GiB u32-offset slab (fec_xor_simd.h:71)");
  std::memset(slab_, 0, P);
  offsets_.clear();
  size_t off = P;
  for (const auto& g : groups) {
    if (g.Packets.size() > 10) return errorf("group of %zu packets: fec_encode_batch takes 10", g.Packets.size());
    for (size_t p = 0; p < 10; ++p) {
      if (p < g.Packets.size()) {
        const Bytes& pkt = g.Packets[p];
        const size_t n = std::min(pkt.size(), P);
        std::memcpy(slab_ + off, pkt.data(), n);
        if (n < P) std::memset(slab_ + off + n, 0, P - n);
        offsets_.push_back(static_cast<uint32_t>(off));
        off += P;
      } else {
        offsets_.push_back(0);
      }
    }
  }
  const size_t repairNeeded = groups.size() * P;
  if (Error e = resizeRepairBuffer(repairNeeded)) return errorf("failed to resize repair buffer: %s", e.msg.c_str());
  const int ret = fec_encode_batch(ctx_, slab_, offsets_.data(), static_cast<uint32_t>(groups.size()),
                                   static_cast<uint32_t>(P), repair_);
  if (ret != 0) return errorf("C++ encoding failed with code %d", ret);  // :147-149
  if (out) {
    out->resize(groups.size());
    for (size_t i = 0; i < groups.size(); ++i) (*out)[i].assign(repair_ + i * P, repair_ + (i + 1) * P);
  }
  return {};
}

Error FECEncoderCXX::Close() {
  std::lock_guard<std::mutex> lk(mu_);
  if (!initialized_) return {};
  if (ctx_) fec_encoder_free(ctx_);
  ctx_ = nullptr;
  if (slab_) fec_free_slab(slab_);
  slab_ = nullptr;
  if (repair_) fec_free_repair_buffer(repair_);
  repair_ = nullptr;
  initialized_ = false;
  return {};
}

// ===================================================================== HybridFECEncoder
HybridFECEncoder::HybridFECEncoder(double redundancy) : redundancy_(clamp_redundancy(redundancy)) {
  packets_.reserve(groupSize_);
  packetIDs_.reserve(groupSize_);
  cxx_ = FECEncoderCXX::New(redundancy_, 1024);  // encoder_hybrid.go:44
  useCXX_ = cxx_ && cxx_->initialized();
}

AddPacketResult HybridFECEncoder::AddPacket(const uint8_t* packet, size_t len, uint64_t packetID) {
  std::lock_guard<std::mutex> lk(mu_);
  packets_.emplace_back(packet, packet + len);  // the packet is copied (:64-65)
  packetIDs_.push_back(packetID);
  if (static_cast<int>(packets_.size()) >= groupSize_) return generateRedundancy();
  return {};
}

AddPacketResult HybridFECEncoder::generateRedundancy() {
  AddPacketResult res;
  if (!useCXX_) {
    res.err = errorf("GPU FEC engine unavailable: %s", fec_hip_last_error());
    return res;
  }
  if (packets_.empty()) {
    res.err = errorf("no packets in group");
    return res;
  }
  size_t maxSize = 0;
  for (const auto& p : packets_) maxSize = std::max(maxSize, p.size());
  if (maxSize == 0) {
    res.err = errorf("empty packets");
    return res;
  }
  FECBatchGroup group;
  group.Packets = packets_;
  for (const auto& p : packets_) group.Sizes.push_back(static_cast<uint32_t>(p.size()));
  std::vector<RepairPacket> repairs;
  if (Error e = cxx_->EncodeBatch({group}, static_cast<int>(maxSize), &repairs)) {
    res.err = errorf("C++ encoding failed: %s", e.msg.c_str());
    return res;
  }
  if (repairs.empty()) {
    res.err = errorf("no repair packet generated");
    return res;
  }
  res.redundancy = createFECPacket(repairs[0], static_cast<int>(packets_.size()));
  packets_.clear();
  packetIDs_.clear();
  ++groupID_;
  // metric updates exactly as encoder_hybrid.go:124-127 (PacketsEncoded counts groupSize)
  metrics_.GroupsProcessed++;
  metrics_.PacketsEncoded += groupSize_;
  metrics_.RedundancyPackets++;
  metrics_.RedundancyBytes += static_cast<int64_t>(res.redundancy.size());
  res.needsRedundancy = true;
  return res;
}

// encoder_hybrid.go:175-192: FE C0 | groupID u64 LE | count u8 | payload
Bytes HybridFECEncoder::createFECPacket(const Bytes& repair, int packetCount) {
  Bytes out(11 + repair.size());
  out[0] = 0xFE;
  out[1] = 0xC0;
  for (int b = 0; b < 8; ++b) out[2 + b] = static_cast<uint8_t>(groupID_ >> (8 * b));
  out[10] = static_cast<uint8_t>(packetCount);
  std::memcpy(out.data() + 11, repair.data(), repair.size());
  return out;
}

std::pair<Bytes, Error> HybridFECEncoder::Flush() {
  std::lock_guard<std::mutex> lk(mu_);
  if (packets_.empty()) return {{}, {}};
  AddPacketResult r = generateRedundancy();
  return {r.redundancy, r.err};
}

FECMetrics HybridFECEncoder::GetMetrics() {
  std::lock_guard<std::mutex> lk(mu_);
  return metrics_;
}

void HybridFECEncoder::ResetMetrics() {
  std::lock_guard<std::mutex> lk(mu_);
  metrics_ = FECMetrics();
}

Error HybridFECEncoder::Close() {
  std::lock_guard<std::mutex> lk(mu_);
  if (cxx_) return cxx_->Close();
  return {};
}

// ===================================================================== FECDecoder
namespace {

// decoder.go:62-69
Bytes padTo(const uint8_t* data, size_t len, size_t n) {
  Bytes out(n, 0);
  std::memcpy(out.data(), data, std::min(len, n));
  return out;
}

}  // namespace

FECDecoder::FECDecoder() = default;

bool FECDecoder::AddPacket(const uint8_t* packet, size_t len, uint64_t packetID, uint64_t groupID) {
  std::lock_guard<std::mutex> lk(mu_);
  if (groups_.find(groupID) == groups_.end() && groups_.size() >= kMaxActiveGroups) evictOldestGroup();
  auto it = groups_.find(groupID);
  if (it == groups_.end()) {
    Group g;
    g.groupID = groupID;
    g.createdAt = std::chrono::steady_clock::now();
    it = groups_.emplace(groupID, std::move(g)).first;
    metrics_.GroupsActive = static_cast<int64_t>(groups_.size());
  }
  Group& g = it->second;
  if (g.symbolLen == 0) g.symbolLen = static_cast<int>(std::min<size_t>(len, kMaxSymbolLen));
  g.packets[packetID] = padTo(packet, len, static_cast<size_t>(g.symbolLen));
  g.present[packetID] = true;
  g.received++;
  metrics_.PacketsReceived++;
  if ((g.hasRedundancy || !g.rows.empty()) && g.received < g.packetCount) return tryRecover(g, nullptr);
  return false;
}

std::pair<bool, std::vector<Recovered>> FECDecoder::AddRedundancyPacket(const uint8_t* b, size_t len) {
  std::lock_guard<std::mutex> lk(mu_);
  // parseRedundancyHeader, decoder.go:72-85, extended with the row 1..r-1 form
  RSRepairHeader h;
  const uint8_t* payload = nullptr;
  size_t plen = 0;
  if (!ParseRepairHeader(b, len, &h, &payload, &plen)) return {false, {}};
  const uint64_t groupID = h.groupID;
  const int packetCount = h.count;

  if (groups_.find(groupID) == groups_.end() && groups_.size() >= kMaxActiveGroups) evictOldestGroup();
  auto it = groups_.find(groupID);
  if (it == groups_.end()) {
    Group g;
    g.groupID = groupID;
    g.createdAt = std::chrono::steady_clock::now();
    g.packetCount = packetCount;
    it = groups_.emplace(groupID, std::move(g)).first;
    metrics_.GroupsActive = static_cast<int64_t>(groups_.size());
  }
  Group& g = it->second;
  const bool shapeConflict = h.row > 0 && g.k != 0 && (g.k != h.k || g.r != h.r);
  if ((g.packetCount != 0 && g.packetCount != packetCount) || shapeConflict) {  // conflicting: drop the group
    if (g.queued) pending_.erase(std::find(pending_.begin(), pending_.end(), groupID));
    groups_.erase(it);
    metrics_.GroupsActive = static_cast<int64_t>(groups_.size());
    return {false, {}};
  }
  g.packetCount = packetCount;
  if (g.symbolLen == 0) g.symbolLen = static_cast<int>(std::min<size_t>(plen, kMaxSymbolLen));
  if (h.row == 0) {
    g.redundancy = padTo(payload, plen, static_cast<size_t>(g.symbolLen));
    g.hasRedundancy = true;
  } else {
    g.k = h.k;
    g.r = h.r;
    g.rows[h.row] = padTo(payload, plen, static_cast<size_t>(g.symbolLen));
  }
  metrics_.RepairPacketsReceived++;
  if (g.received < g.packetCount) {
    std::vector<Recovered> list;
    if (tryRecover(g, &list)) {
      // Row 0 alone: decoder.go:170-178 lists ids still marked absent; the single-loss path
      // has just marked the rebuilt one present, so — as in the reference — the list comes
      // back empty.  The r > 1 path (new) returns what it rebuilt.
      return {true, list};
    }
  }
  return {false, {}};
}

bool FECDecoder::canRecoverRS(const Group& g) const {
  if (g.k <= 0 || g.r <= 0 || g.symbolLen <= 0 || g.packetCount > g.k) return false;
  int missing = 0;
  for (int id = 0; id < g.packetCount; ++id) {
    auto p = g.present.find(static_cast<uint64_t>(id));
    missing += (p == g.present.end() || !p->second) ? 1 : 0;
  }
  const int rows = (g.hasRedundancy ? 1 : 0) + static_cast<int>(g.rows.size());
  return missing >= 1 && missing <= rows;
}

bool FECDecoder::tryRecover(Group& g, std::vector<Recovered>* list) {  // decoder.go:216-248
  if (!g.hasRedundancy && g.rows.empty()) return false;
  if (g.received >= g.packetCount) return false;
  const int missing = g.packetCount - g.received;
  if (missing == 1 && g.hasRedundancy) {
    uint64_t id = 0;
    Bytes data;
    if (recoverSingle(g, &id, &data)) {
      g.packets[id] = std::move(data);
      g.present[id] = true;
      g.received++;
      metrics_.RecoveryEvents++;
      metrics_.PacketsRecovered++;
      return true;
    }
    metrics_.FailedRecoveries++;
    return false;
  }
  if (canRecoverRS(g)) {  // r > 1 (new): up to as many losses as rows received
    if (deferred_) {
      if (!g.queued) {
        g.queued = true;
        pending_.push_back(g.groupID);
      }
      return false;
    }
    std::vector<Group*> one{&g};
    std::vector<std::vector<Recovered>> lists;
    if (recoverRS(one, &lists)) {
      if (list) *list = std::move(lists[0]);
      return true;
    }
    return false;
  }
  metrics_.FailedRecoveries++;  // more losses than repair rows (row 0 alone: XOR recovers one)
  return false;
}

// decoder.go:255-287: out = parity ^ every other packet, on the GPU.
bool FECDecoder::recoverSingle(Group& g, uint64_t* id, Bytes* out) {
  if (!g.hasRedundancy || g.symbolLen == 0) return false;
  bool found = false;
  for (uint64_t i = 0; i < static_cast<uint64_t>(g.packetCount); ++i) {
    auto p = g.present.find(i);
    if (p == g.present.end() || !p->second) {
      *id = i;
      found = true;
      break;
    }
  }
  if (!found) return false;
  if (shared_ && shared_->r() == 1 && g.packetCount == shared_->k() && g.symbolLen <= shared_->slot()) {
    // the same XOR, in a batch shared with other connections
    std::vector<const uint8_t*> shards(static_cast<size_t>(g.packetCount) + 1, nullptr);
    for (auto& kv : g.packets)
      if (kv.first != *id && kv.first < static_cast<uint64_t>(g.packetCount)) shards[kv.first] = kv.second.data();
    shards.back() = g.redundancy.data();
    std::vector<std::pair<int, Bytes>> rebuilt;
    const Error e = shared_->Recover(shards, static_cast<uint32_t>(g.symbolLen), &rebuilt);
    if (!e.ok() || rebuilt.size() != 1 || rebuilt[0].first != static_cast<int>(*id)) return false;
    *out = std::move(rebuilt[0].second);
    return true;
  }
  std::vector<const uint8_t*> srcs;
  srcs.push_back(g.redundancy.data());
  for (auto& kv : g.packets)
    if (kv.first != *id) srcs.push_back(kv.second.data());  // every stored symbol is symbolLen long
  out->assign(static_cast<size_t>(g.symbolLen), 0);
  xor_impl_fn xor_gpu = fec_select_xor_impl();
  xor_gpu(srcs.data(), srcs.size(), static_cast<size_t>(g.symbolLen), out->data());
  // the xor entry points clear the thread's error text on entry and set it on failure
  const char* err = fec_hip_last_error();
  return !(err && err[0]);
}

void FECDecoder::evictOldestGroup() {  // decoder.go:306-325
  if (groups_.empty()) return;
  auto oldest = groups_.begin();
  for (auto it = groups_.begin(); it != groups_.end(); ++it)
    if (it->second.createdAt < oldest->second.createdAt) oldest = it;
  if (oldest->second.queued) pending_.erase(std::find(pending_.begin(), pending_.end(), oldest->first));
  groups_.erase(oldest);
  metrics_.GroupsEvicted++;
  metrics_.GroupsActive = static_cast<int64_t>(groups_.size());
}

void FECDecoder::CleanupGroups() {  // decoder.go:328-343
  std::lock_guard<std::mutex> lk(mu_);
  const auto now = std::chrono::steady_clock::now();
  for (auto it = groups_.begin(); it != groups_.end();) {
    if (now - it->second.createdAt > std::chrono::seconds(kGroupTTLSeconds)) {
      if (it->second.queued) pending_.erase(std::find(pending_.begin(), pending_.end(), it->first));
      it = groups_.erase(it);
      metrics_.GroupsEvicted++;
    } else {
      ++it;
    }
  }
  metrics_.GroupsActive = static_cast<int64_t>(groups_.size());
}

FECDecoderMetrics FECDecoder::GetMetrics() {
  std::lock_guard<std::mutex> lk(mu_);
  return metrics_;
}

void FECDecoder::ResetMetrics() {
  std::lock_guard<std::mutex> lk(mu_);
  metrics_ = FECDecoderMetrics();
}

Bytes FECDecoder::GetPacket(uint64_t groupID, uint64_t packetID) {
  std::lock_guard<std::mutex> lk(mu_);
  auto g = groups_.find(groupID);
  if (g == groups_.end()) return {};
  auto p = g->second.packets.find(packetID);
  return p == g->second.packets.end() ? Bytes{} : p->second;
}

void FECDecoder::AgeGroupsForTest(int seconds) {
  std::lock_guard<std::mutex> lk(mu_);
  for (auto& kv : groups_) kv.second.createdAt -= std::chrono::seconds(seconds);
}

// ===================================================================== batch extension
namespace {

FECEncoderCtx* shared_ctx() {
  static std::once_flag once;
  static FECEncoderCtx* ctx = nullptr;
  std::call_once(once, [] { ctx = fec_encoder_new(0.10, 1024); });
  return ctx;
}

}  // namespace

Error EncodeBatchRS(const Bytes& data, int k, int r, int packetSize, Bytes* parity) {
  FECEncoderCtx* ctx = shared_ctx();
  if (!ctx) return errorf("no usable GPU: %s", fec_hip_last_error());
  if (k <= 0 || r <= 0 || packetSize <= 0 || data.size() % (size_t(k) * packetSize) != 0)
    return errorf("data is not a whole number of %dx%d groups", k, packetSize);
  const uint64_t G = data.size() / (size_t(k) * packetSize);
  parity->assign(G * r * size_t(packetSize), 0);
  if (G == 0) return {};
  const int rc = fec_encode_batch_rs(ctx, data.data(), nullptr, G, k, r, packetSize, parity->data());
  if (rc != 0) return errorf("fec_encode_batch_rs failed with code %d: %s", rc, fec_hip_last_error());
  return {};
}

int64_t RecoverBatchRS(Bytes& data, const Bytes& parity, const std::vector<uint64_t>& erasures, int k, int r,
                       int packetSize, Error* err) {
  FECEncoderCtx* ctx = shared_ctx();
  if (!ctx) {
    if (err) *err = errorf("no usable GPU: %s", fec_hip_last_error());
    return -1;
  }
  const uint64_t G = erasures.size();
  if (data.size() < G * k * size_t(packetSize) || parity.size() < G * r * size_t(packetSize)) {
    if (err) *err = errorf("buffers too small for %llu groups", (unsigned long long)G);
    return -1;
  }
  if (G == 0) return 0;
  uint64_t bad = 0;
  const int rc = fec_decode_batch_rs(ctx, data.data(), parity.data(), erasures.data(), G, k, r, packetSize,
                                     nullptr, &bad);
  if (rc != 0) {
    if (err) *err = errorf("fec_decode_batch_rs failed with code %d: %s", rc, fec_hip_last_error());
    return -1;
  }
  return static_cast<int64_t>(bad);
}

// ===================================================================== batcher (new)
std::shared_ptr<SharedFECBatcher> SharedFECBatcher::New(int k, int r, int slotBytes, int maxGroups, int deadlineUs,
                                                         int device, int slabs) {
  if (k < 1 || r < 1 || k + r > 256 || k > FECDecoder::kMaxPacketCount || slotBytes < 1 || maxGroups < 1 ||
      deadlineUs < 0 || slabs < 0)
    return nullptr;
  std::shared_ptr<SharedFECBatcher> b(new SharedFECBatcher());
  b->b_ = fec_batcher_new(device, static_cast<uint32_t>(k), static_cast<uint32_t>(r), static_cast<uint32_t>(slotBytes),
                          static_cast<uint32_t>(maxGroups), static_cast<uint32_t>(deadlineUs),
                          static_cast<uint32_t>(slabs));
  if (!b->b_) return nullptr;
  b->k_ = k;
  b->r_ = r;
  b->slot_ = slotBytes;
  return b;
}

std::shared_ptr<SharedFECBatcher> SharedFECBatcher::NewMulti(const std::vector<int>& devices, int k, int r,
                                                              int slotBytes, int maxGroups, int deadlineUs, int slabs) {
  if (k < 1 || r < 1 || k + r > 256 || k > FECDecoder::kMaxPacketCount || slotBytes < 1 || maxGroups < 1 ||
      deadlineUs < 0 || slabs < 0)
    return nullptr;
  std::shared_ptr<SharedFECBatcher> b(new SharedFECBatcher());
  b->b_ = fec_batcher_new_multi(devices.empty() ? nullptr : devices.data(), static_cast<int>(devices.size()),
                                static_cast<uint32_t>(k), static_cast<uint32_t>(r), static_cast<uint32_t>(slotBytes),
                                static_cast<uint32_t>(maxGroups), static_cast<uint32_t>(deadlineUs),
                                static_cast<uint32_t>(slabs));
  if (!b->b_) return nullptr;
  b->k_ = k;
  b->r_ = r;
  b->slot_ = slotBytes;
  return b;
}

SharedFECBatcher::~SharedFECBatcher() {
  if (b_) fec_batcher_free(b_);
}

void SharedFECBatcher::Flush() { fec_batcher_flush(b_); }

std::vector<uint64_t> SharedFECBatcher::Stats() {
  FECBatcherStats st{};
  fec_batcher_stats(b_, &st);
  return {st.groups, st.batches, st.full_flushes, st.deadline_flushes, st.max_batch};
}

std::shared_ptr<SharedFECDecodeBatcher> SharedFECDecodeBatcher::New(int k, int r, int slotBytes, int maxGroups,
                                                                     int deadlineUs, int device, int slabs) {
  if (k < 1 || r < 1 || k + r > 64 || slotBytes < 1 || maxGroups < 1 || deadlineUs < 0 || slabs < 0) return nullptr;
  std::shared_ptr<SharedFECDecodeBatcher> b(new SharedFECDecodeBatcher());
  b->b_ = fec_batcher_new_decoder(device, static_cast<uint32_t>(k), static_cast<uint32_t>(r),
                                  static_cast<uint32_t>(slotBytes), static_cast<uint32_t>(maxGroups),
                                  static_cast<uint32_t>(deadlineUs), static_cast<uint32_t>(slabs));
  if (!b->b_) return nullptr;
  b->k_ = k;
  b->r_ = r;
  b->slot_ = slotBytes;
  return b;
}

std::shared_ptr<SharedFECDecodeBatcher> SharedFECDecodeBatcher::NewMulti(const std::vector<int>& devices, int k, int r,
                                                                          int slotBytes, int maxGroups, int deadlineUs,
                                                                          int slabs) {
  if (k < 1 || r < 1 || k + r > 64 || slotBytes < 1 || maxGroups < 1 || deadlineUs < 0 || slabs < 0) return nullptr;
  std::shared_ptr<SharedFECDecodeBatcher> b(new SharedFECDecodeBatcher());
  b->b_ = fec_batcher_new_decoder_multi(devices.empty() ? nullptr : devices.data(), static_cast<int>(devices.size()),
                                        static_cast<uint32_t>(k), static_cast<uint32_t>(r),
                                        static_cast<uint32_t>(slotBytes), static_cast<uint32_t>(maxGroups),
                                        static_cast<uint32_t>(deadlineUs), static_cast<uint32_t>(slabs));
  if (!b->b_) return nullptr;
  b->k_ = k;
  b->r_ = r;
  b->slot_ = slotBytes;
  return b;
}

SharedFECDecodeBatcher::~SharedFECDecodeBatcher() {
  if (b_) fec_batcher_free(b_);
}

Error SharedFECDecodeBatcher::Recover(const std::vector<const uint8_t*>& shards, uint32_t len,
                                      std::vector<std::pair<int, Bytes>>* out) {
  out->clear();
  if (shards.size() != static_cast<size_t>(k_ + r_)) return errorf("expected %d shards, got %zu", k_ + r_, shards.size());
  const int64_t t = fec_batcher_submit_shards(b_, shards.data(), len);
  if (t < 0) return errorf("fec_batcher_submit_shards failed with code %lld: %s", static_cast<long long>(t),
                           fec_batcher_last_error());
  std::vector<uint8_t> rows(static_cast<size_t>(r_) * slot_);
  uint64_t mask = 0;
  const int n = fec_batcher_wait_rebuilt(b_, t, rows.data(), static_cast<uint32_t>(slot_), &mask, -1);
  if (n < 0) return errorf("fec_batcher_wait_rebuilt failed with code %d: %s", n, fec_batcher_last_error());
  int row = 0;
  for (int j = 0; j < k_ && row < n; ++j)
    if ((mask >> j) & 1) {
      const uint8_t* src = rows.data() + static_cast<size_t>(row++) * slot_;
      out->emplace_back(j, Bytes(src, src + len));
    }
  return Error{};
}

void SharedFECDecodeBatcher::Flush() { fec_batcher_flush(b_); }

std::vector<uint64_t> SharedFECDecodeBatcher::Stats() {
  FECBatcherStats st{};
  fec_batcher_stats(b_, &st);
  return {st.groups, st.batches, st.full_flushes, st.deadline_flushes, st.max_batch};
}

BatchedFECEncoder::BatchedFECEncoder(std::shared_ptr<SharedFECBatcher> batcher) : b_(std::move(batcher)) {
  packets_.reserve(b_ ? b_->k() : 10);
}

void BatchedFECEncoder::addLocked(const uint8_t* packet, size_t len) {
  if (npk_ < packets_.size()) {
    packets_[npk_].assign(packet, packet + len);  // reuses the buffer of an earlier group
  } else {
    packets_.emplace_back(packet, packet + len);
  }
  ++npk_;
}

Error BatchedFECEncoder::submitLocked(Ticket* t) {
  if (!b_) return errorf("GPU FEC engine unavailable");
  if (npk_ == 0) return errorf("no packets in group");  // encoder_hybrid.go:84-86
  lens_.clear();
  ptrs_.clear();
  size_t maxSize = 0;
  for (size_t i = 0; i < npk_; ++i) {
    const Bytes& p = packets_[i];
    ptrs_.push_back(p.data());
    lens_.push_back(static_cast<uint32_t>(p.size()));
    maxSize = std::max(maxSize, p.size());
  }
  // encoder_hybrid.go:95-97.  The reference keeps the packets after this error (every later
  // AddPacket of the stream then fails the same way); the group is dropped here instead.
  if (maxSize == 0) {
    npk_ = 0;
    return errorf("empty packets");
  }
  const int64_t tk =
      fec_batcher_submit_packets(b_->raw(), ptrs_.data(), lens_.data(), static_cast<uint32_t>(lens_.size()));
  if (tk < 0) {  // refused (e.g. a packet wider than the slot): the group is dropped
    npk_ = 0;
    return errorf("fec_batcher_submit failed with code %lld: %s", static_cast<long long>(tk), fec_batcher_last_error());
  }
  t->ticket = tk;
  t->groupID = groupID_++;
  t->count = static_cast<int>(npk_);
  npk_ = 0;  // the buffers stay for the next group (their capacity is reused)
  return {};
}

Error BatchedFECEncoder::collect(const Ticket& t, int64_t timeoutUs, std::vector<Bytes>* rows, bool* ready) {
  const int r = b_->r();
  rowbuf_.resize(size_t(r) * b_->slot());
  const int rc = fec_batcher_wait(b_->raw(), t.ticket, rowbuf_.data(), static_cast<uint32_t>(b_->slot()), timeoutUs);
  *ready = rc != FEC_ERR_AGAIN;
  if (rc == FEC_ERR_AGAIN) return {};
  if (rc < 0) {
    Error e = errorf("C++ encoding failed: %s", fec_batcher_last_error());
    e.code = rc;  // FEC_ERR_RANGE: the result expired (a ticket of this encoder is always issued once)
    return e;
  }
  const size_t len = static_cast<size_t>(rc);
  for (int row = 0; row < r; ++row) {
    RSRepairHeader h;
    h.groupID = t.groupID;
    h.count = t.count;
    h.row = row;
    h.r = r;
    h.k = b_->k();
    // row 0: encoder_hybrid.go:175-192's packet (FE C0 | groupID | count | payload)
    rows->push_back(MakeRepairPacket(h, rowbuf_.data() + size_t(row) * b_->slot(), len));
    metrics_.RedundancyPackets++;
    metrics_.RedundancyBytes += static_cast<int64_t>(rows->back().size());
  }
  // encoder_hybrid.go:124-127 (PacketsEncoded counts the group size)
  metrics_.GroupsProcessed++;
  metrics_.PacketsEncoded += b_->k();
  return {};
}

AddPacketResult BatchedFECEncoder::AddPacket(const uint8_t* packet, size_t len, uint64_t packetID) {
  (void)packetID;
  std::lock_guard<std::mutex> lk(mu_);
  AddPacketResult res;
  addLocked(packet, len);  // copied, as encoder_hybrid.go:64-65
  if (static_cast<int>(npk_) < (b_ ? b_->k() : 10)) return res;
  Ticket t;
  if ((res.err = submitLocked(&t))) return res;
  std::vector<Bytes> rows;
  bool ready = false;
  if ((res.err = collect(t, -1, &rows, &ready))) return res;
  res.needsRedundancy = true;
  res.redundancy = std::move(rows[0]);
  res.extra.assign(std::make_move_iterator(rows.begin() + 1), std::make_move_iterator(rows.end()));
  return res;
}

Error BatchedFECEncoder::AddPacketAsync(const uint8_t* packet, size_t len, uint64_t packetID) {
  (void)packetID;
  std::lock_guard<std::mutex> lk(mu_);
  addLocked(packet, len);
  if (static_cast<int>(npk_) < (b_ ? b_->k() : 10)) return {};
  Ticket t;
  if (Error e = submitLocked(&t)) return e;
  outstanding_.push_back(t);
  return {};
}

Error BatchedFECEncoder::Poll(std::vector<Bytes>* out, int64_t timeoutUs) {
  std::lock_guard<std::mutex> lk(mu_);
  bool first = true;
  while (!outstanding_.empty()) {
    bool ready = false;
    const int64_t wait = timeoutUs < 0 ? -1 : (first ? timeoutUs : 0);
    if (Error e = collect(outstanding_.front(), wait, out, &ready)) {
      outstanding_.pop_front();
      return e;
    }
    if (!ready) break;
    outstanding_.pop_front();
    first = false;
  }
  return {};
}

AddPacketResult BatchedFECEncoder::Flush() {
  std::lock_guard<std::mutex> lk(mu_);
  AddPacketResult res;
  if (npk_ == 0) return res;
  Ticket t;
  if ((res.err = submitLocked(&t))) return res;
  b_->Flush();
  std::vector<Bytes> rows;
  bool ready = false;
  if ((res.err = collect(t, -1, &rows, &ready))) return res;
  res.needsRedundancy = true;
  res.redundancy = std::move(rows[0]);
  res.extra.assign(std::make_move_iterator(rows.begin() + 1), std::make_move_iterator(rows.end()));
  return res;
}

Error BatchedFECEncoder::FlushAsync() {
  std::lock_guard<std::mutex> lk(mu_);
  if (npk_ != 0) {
    Ticket t;
    if (Error e = submitLocked(&t)) return e;
    outstanding_.push_back(t);
  }
  if (b_) b_->Flush();
  return {};
}

FECMetrics BatchedFECEncoder::GetMetrics() {
  std::lock_guard<std::mutex> lk(mu_);
  return metrics_;
}

// ===================================================================== r > 1 (new)
bool ParseRepairHeader(const uint8_t* b, size_t len, RSRepairHeader* h, const uint8_t** payload, size_t* plen) {
  if (len < kRepairHeaderLen || b[0] != 0xFE || (b[1] != 0xC0 && b[1] != 0xC1)) return false;
  RSRepairHeader x;
  for (int i = 0; i < 8; ++i) x.groupID |= uint64_t(b[2 + i]) << (8 * i);
  x.count = b[10];
  if (x.count <= 0 || x.count > FECDecoder::kMaxPacketCount) return false;  // decoder.go:80-82
  size_t hl = kRepairHeaderLen;
  if (b[1] == 0xC1) {
    if (len < kRSRepairHeaderLen) return false;
    x.row = b[11];
    x.r = b[12];
    x.k = b[13];
    if (x.row < 1 || x.row >= x.r || x.k < 1 || x.count > x.k || x.k + x.r > 64) return false;
    hl = kRSRepairHeaderLen;
  }
  *h = x;
  *payload = b + hl;
  *plen = len - hl;
  return true;
}

Bytes MakeRepairPacket(const RSRepairHeader& h, const uint8_t* payload, size_t plen) {
  const size_t hl = h.row == 0 ? kRepairHeaderLen : kRSRepairHeaderLen;
  Bytes out(hl + plen);
  out[0] = 0xFE;
  out[1] = h.row == 0 ? 0xC0 : 0xC1;
  for (int b = 0; b < 8; ++b) out[2 + b] = static_cast<uint8_t>(h.groupID >> (8 * b));
  out[10] = static_cast<uint8_t>(h.count);
  if (h.row != 0) {
    out[11] = static_cast<uint8_t>(h.row);
    out[12] = static_cast<uint8_t>(h.r);
    out[13] = static_cast<uint8_t>(h.k);
  }
  if (plen) std::memcpy(out.data() + hl, payload, plen);
  return out;
}

// ---------------------------------------------------------------- FECDecoder, r > 1
bool FECDecoder::recoverRS(const std::vector<Group*>& gs, std::vector<std::vector<Recovered>>* lists) {
  lists->assign(gs.size(), {});
  if (gs.empty()) return true;
  FECEncoderCtx* ctx = shared_ctx();
  if (!ctx) return false;
  const int k = gs[0]->k, r = gs[0]->r;
  size_t L = 0;
  for (Group* g : gs) L = std::max(L, static_cast<size_t>(g->symbolLen));
  const size_t G = gs.size();
  // Symbols zero-padded to the widest group's length: bytewise coding keeps every group's
  // own prefix exact.  Slots count..k-1 are the encoder's zero packets (present).
  Bytes data(G * k * L, 0), parity(G * r * L, 0), status(G, 0);
  std::vector<uint64_t> masks(G, 0);
  for (size_t i = 0; i < G; ++i) {
    Group& g = *gs[i];
    for (int id = 0; id < g.packetCount; ++id) {
      auto p = g.present.find(static_cast<uint64_t>(id));
      if (p == g.present.end() || !p->second) {
        masks[i] |= 1ull << id;
      } else {
        const Bytes& pk = g.packets[static_cast<uint64_t>(id)];
        std::memcpy(&data[(i * k + id) * L], pk.data(), std::min(pk.size(), L));
      }
    }
    for (int row = 0; row < r; ++row) {
      const Bytes* src = nullptr;
      if (row == 0 && g.hasRedundancy) src = &g.redundancy;
      if (row > 0) {
        auto rw = g.rows.find(row);
        if (rw != g.rows.end()) src = &rw->second;
      }
      if (src) std::memcpy(&parity[(i * r + row) * L], src->data(), std::min(src->size(), L));
      else masks[i] |= 1ull << (k + row);
    }
  }
  uint64_t bad = 0;
  const int rc = fec_decode_batch_rs(ctx, data.data(), parity.data(), masks.data(), G, static_cast<uint32_t>(k),
                                     static_cast<uint32_t>(r), static_cast<uint32_t>(L), status.data(), &bad);
  if (rc != 0) {
    metrics_.FailedRecoveries += static_cast<int64_t>(G);
    return false;
  }
  for (size_t i = 0; i < G; ++i) {
    Group& g = *gs[i];
    g.queued = false;
    if (status[i] != 0) {
      metrics_.FailedRecoveries++;
      continue;
    }
    for (int id = 0; id < g.packetCount; ++id) {
      if (!((masks[i] >> id) & 1)) continue;
      const uint8_t* src = &data[(i * k + id) * L];
      Bytes sym(src, src + g.symbolLen);
      g.packets[static_cast<uint64_t>(id)] = sym;
      g.present[static_cast<uint64_t>(id)] = true;
      g.received++;
      metrics_.PacketsRecovered++;
      (*lists)[i].push_back({static_cast<uint64_t>(id), std::move(sym)});
    }
    metrics_.RecoveryEvents++;
  }
  return true;
}

void FECDecoder::SetSharedBatcher(std::shared_ptr<SharedFECDecodeBatcher> batcher) {
  std::lock_guard<std::mutex> lk(mu_);
  shared_ = std::move(batcher);
}

void FECDecoder::SetDeferredRecovery(bool deferred) {
  std::lock_guard<std::mutex> lk(mu_);
  deferred_ = deferred;
}

std::vector<std::pair<uint64_t, std::vector<Recovered>>> FECDecoder::RecoverPending(Error* err) {
  std::lock_guard<std::mutex> lk(mu_);
  std::vector<std::pair<uint64_t, std::vector<Recovered>>> out;
  // one library call per code shape
  std::map<std::pair<int, int>, std::vector<Group*>> byShape;
  for (uint64_t id : pending_) {
    auto it = groups_.find(id);
    if (it == groups_.end() || !it->second.queued) continue;
    it->second.queued = false;
    if (!canRecoverRS(it->second)) continue;  // completed by data packets meanwhile
    byShape[{it->second.k, it->second.r}].push_back(&it->second);
  }
  pending_.clear();
  for (auto& kv : byShape) {
    std::vector<std::vector<Recovered>> lists;
    if (!recoverRS(kv.second, &lists)) {
      if (err) *err = errorf("fec_decode_batch_rs failed: %s", fec_hip_last_error());
      continue;
    }
    for (size_t i = 0; i < kv.second.size(); ++i)
      if (!lists[i].empty()) out.emplace_back(kv.second[i]->groupID, std::move(lists[i]));
  }
  return out;
}

// ---------------------------------------------------------------- RSBatchEncoder
std::unique_ptr<RSBatchEncoder> RSBatchEncoder::New(int k, int r, int batchGroups, int slotSize) {
  if (k < 1 || r < 1 || k + r > 64 || k > FECDecoder::kMaxPacketCount || r > 255 || batchGroups < 1 ||
      slotSize < 1)
    return nullptr;
  std::unique_ptr<RSBatchEncoder> e(new RSBatchEncoder());
  e->k_ = k;
  e->r_ = r;
  e->batch_ = batchGroups;
  e->slot_ = (static_cast<size_t>(slotSize) + 15) / 16 * 16;  // 16-byte packets: the vector kernels
  e->ctx_ = fec_encoder_new(0.10, static_cast<uint32_t>(batchGroups));
  if (!e->ctx_) return nullptr;
  e->slab_ = static_cast<uint8_t*>(fec_alloc_slab(size_t(batchGroups) * k * e->slot_));
  e->parity_ = static_cast<uint8_t*>(fec_alloc_repair_buffer(size_t(batchGroups) * r * e->slot_));
  if (!e->slab_ || !e->parity_) return nullptr;  // the destructor frees what was allocated
  e->count_.assign(batchGroups, 0);
  e->maxLen_.assign(batchGroups, 0);
  return e;
}

RSBatchEncoder::~RSBatchEncoder() { Close(); }

Error RSBatchEncoder::Close() {
  std::lock_guard<std::mutex> lk(mu_);
  if (slab_) fec_free_slab(slab_);
  if (parity_) fec_free_repair_buffer(parity_);
  if (ctx_) fec_encoder_free(ctx_);
  slab_ = parity_ = nullptr;
  ctx_ = nullptr;
  open_ = 0;
  return {};
}

Error RSBatchEncoder::encodeLocked(int groups, std::vector<Bytes>* out) {
  if (groups <= 0) return {};
  // zero the slots a partial last group does not fill (the slab is reused across batches)
  const int last = groups - 1;
  for (uint32_t j = count_[last]; j < static_cast<uint32_t>(k_); ++j)
    std::memset(slab_ + (size_t(last) * k_ + j) * slot_, 0, slot_);
  const int rc = fec_encode_batch_rs(ctx_, slab_, nullptr, static_cast<uint64_t>(groups), static_cast<uint32_t>(k_),
                                     static_cast<uint32_t>(r_), static_cast<uint32_t>(slot_), parity_);
  if (rc != 0) return errorf("fec_encode_batch_rs failed with code %d: %s", rc, fec_hip_last_error());
  Error firstErr;
  for (int g = 0; g < groups; ++g) {
    const uint64_t gid = groupID_++;
    if (maxLen_[g] == 0) {  // encoder_hybrid.go:105-107 refuses a group of empty packets
      if (!firstErr) firstErr = errorf("empty packets in group %llu", static_cast<unsigned long long>(gid));
      continue;
    }
    for (int row = 0; row < r_; ++row) {
      RSRepairHeader h;
      h.groupID = gid;
      h.count = static_cast<int>(count_[g]);
      h.row = row;
      h.r = r_;
      h.k = k_;
      Bytes pkt = MakeRepairPacket(h, parity_ + (size_t(g) * r_ + row) * slot_, maxLen_[g]);
      metrics_.RedundancyPackets++;
      metrics_.RedundancyBytes += static_cast<int64_t>(pkt.size());
      if (out) out->push_back(std::move(pkt));
    }
    metrics_.GroupsProcessed++;
  }
  open_ = 0;
  return firstErr;
}

Error RSBatchEncoder::widenLocked(size_t newSlot, std::vector<Bytes>* out) {
  const bool partial = open_ > 0 && count_[open_ - 1] < static_cast<uint32_t>(k_);
  const int complete = open_ - (partial ? 1 : 0);
  Bytes keep;
  uint32_t keepCount = 0, keepMax = 0;
  if (partial) {
    keepCount = count_[open_ - 1];
    keepMax = maxLen_[open_ - 1];
    const uint8_t* src = slab_ + size_t(open_ - 1) * k_ * slot_;
    keep.assign(src, src + size_t(keepCount) * slot_);
  }
  if (complete > 0) {
    if (Error e = encodeLocked(complete, out)) return e;
  }
  open_ = 0;
  auto* slab = static_cast<uint8_t*>(fec_alloc_slab(size_t(batch_) * k_ * newSlot));
  auto* parity = static_cast<uint8_t*>(fec_alloc_repair_buffer(size_t(batch_) * r_ * newSlot));
  if (!slab || !parity) {
    if (slab) fec_free_slab(slab);
    if (parity) fec_free_repair_buffer(parity);
    return errorf("failed to widen the slab to %zu-byte slots", newSlot);
  }
  fec_free_slab(slab_);
  fec_free_repair_buffer(parity_);
  slab_ = slab;
  parity_ = parity;
  const size_t old = slot_;
  slot_ = newSlot;
  if (partial) {
    for (uint32_t j = 0; j < keepCount; ++j) {
      std::memcpy(slab_ + size_t(j) * slot_, keep.data() + size_t(j) * old, old);
      std::memset(slab_ + size_t(j) * slot_ + old, 0, slot_ - old);
    }
    count_[0] = keepCount;
    maxLen_[0] = keepMax;
    open_ = 1;
  }
  return {};
}

Error RSBatchEncoder::AddPacket(const uint8_t* packet, size_t len, std::vector<Bytes>* out) {
  std::lock_guard<std::mutex> lk(mu_);
  if (!ctx_) return errorf("encoder closed");
  if (len > 0xFFFFu) return errorf("packet of %zu bytes is too large", len);
  if (len > slot_) {
    if (Error e = widenLocked((len + 15) / 16 * 16, out)) return e;
  }
  if (open_ == 0 || count_[open_ - 1] == static_cast<uint32_t>(k_)) {
    count_[open_] = 0;
    maxLen_[open_] = 0;
    ++open_;
  }
  const int g = open_ - 1;
  uint8_t* dst = slab_ + (size_t(g) * k_ + count_[g]) * slot_;
  if (len) std::memcpy(dst, packet, len);
  std::memset(dst + len, 0, slot_ - len);
  count_[g]++;
  maxLen_[g] = std::max<uint32_t>(maxLen_[g], static_cast<uint32_t>(len));
  metrics_.PacketsEncoded++;
  if (open_ == batch_ && count_[g] == static_cast<uint32_t>(k_)) return encodeLocked(open_, out);
  return {};
}

Error RSBatchEncoder::Flush(std::vector<Bytes>* out) {
  std::lock_guard<std::mutex> lk(mu_);
  if (!ctx_) return errorf("encoder closed");
  return encodeLocked(open_, out);
}

FECMetrics RSBatchEncoder::GetMetrics() {
  std::lock_guard<std::mutex> lk(mu_);
  return metrics_;
}

}  // namespace quicfec
