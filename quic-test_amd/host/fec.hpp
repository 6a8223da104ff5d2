// fec.hpp — C++ mirror of the reference's Go FEC API (internal/fec), running on
// libfec_hip.so through its C-ABI.  Same type and method names, argument meaning and
// error behaviour as the Go code, so callers and tests read like the reference's own.
//
//   FECEncoderCXX     internal/fec/fec_cgo.go:25-247
//   HybridFECEncoder  internal/fec/encoder_hybrid.go:9-237
//   FECDecoder        internal/fec/decoder.go:24-343
//
// Deliberate differences:
//   * No CPU fallback lives here.  The reference's hybrid encoder falls back to its pure-Go
//     FECEncoder when the native library is unavailable (encoder_hybrid.go:44-52); in this
//     library a failed GPU init leaves UseCXX() false and AddPacket reports an error.
//   * Packets shorter than the group's largest are zero-padded and partial groups XOR only
//     the packets present (the Go semantics, encoder.go:133-143), where the reference's C++
//     path reads past short packets and reuses stale offsets.
//   * FECDecoder recovery runs on the GPU (xor_packets via fec_select_xor_impl) and, as a
//     batch extension, RecoverBatchRS rebuilds up to r losses per group.
#pragma once

#include <chrono>
#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

struct FECEncoderCtx;

namespace quicfec {

using Bytes = std::vector<uint8_t>;

// Go's `error`: empty = nil.
struct Error {
  std::string msg;
  bool ok() const { return msg.empty(); }
  explicit operator bool() const { return !msg.empty(); }
};

using RepairPacket = Bytes;

// fec_cgo.go:251-254
struct FECBatchGroup {
  std::vector<Bytes> Packets;
  std::vector<uint32_t> Sizes;
};

// fec_cgo.go:25-247
class FECEncoderCXX {
 public:
  // NewFECEncoderCXX: nullptr when the GPU library cannot be initialised (fec_cgo.go:56-82).
  static std::unique_ptr<FECEncoderCXX> New(double redundancy, int maxGroups);
  ~FECEncoderCXX();
  FECEncoderCXX(const FECEncoderCXX&) = delete;
  FECEncoderCXX& operator=(const FECEncoderCXX&) = delete;

  // One repair packet (packetSize bytes) per group, in one C call (fec_cgo.go:95-171).
  Error EncodeBatch(const std::vector<FECBatchGroup>& groups, int packetSize, std::vector<RepairPacket>* out);
  Error Close();
  bool initialized() const { return initialized_; }

 private:
  FECEncoderCXX() = default;
  Error resizeSlab(size_t newSize);
  Error resizeRepairBuffer(size_t newSize);

  FECEncoderCtx* ctx_ = nullptr;
  uint8_t* slab_ = nullptr;  // pinned (fec_alloc_slab)
  size_t slabSize_ = 0;
  std::vector<uint32_t> offsets_;
  uint8_t* repair_ = nullptr;
  size_t repairSize_ = 0;
  int maxGroups_ = 1024;
  std::mutex mu_;
  bool initialized_ = false;
};

// encoder.go:20-26
struct FECMetrics {
  int64_t PacketsEncoded = 0;
  int64_t RedundancyPackets = 0;
  int64_t RedundancyBytes = 0;
  int64_t GroupsProcessed = 0;
};

struct AddPacketResult {
  bool needsRedundancy = false;
  Bytes redundancy;
  Error err;
};

// encoder_hybrid.go:9-237
class HybridFECEncoder {
 public:
  explicit HybridFECEncoder(double redundancy);
  AddPacketResult AddPacket(const uint8_t* packet, size_t len, uint64_t packetID);
  AddPacketResult AddPacket(const Bytes& p, uint64_t id) { return AddPacket(p.data(), p.size(), id); }
  std::pair<Bytes, Error> Flush();
  FECMetrics GetMetrics();
  void ResetMetrics();
  bool UseCXX() const { return useCXX_; }
  Error Close();
  double redundancy() const { return redundancy_; }
  size_t buffered() {
    std::lock_guard<std::mutex> lk(mu_);
    return packets_.size();
  }

 private:
  AddPacketResult generateRedundancy();
  Bytes createFECPacket(const Bytes& repair, int packetCount);

  double redundancy_;
  int groupSize_ = 10;
  bool useCXX_ = false;
  std::unique_ptr<FECEncoderCXX> cxx_;
  std::vector<Bytes> packets_;
  std::vector<uint64_t> packetIDs_;
  uint64_t groupID_ = 0;
  std::mutex mu_;
  FECMetrics metrics_;
};

// decoder.go:29-34
struct Recovered {
  uint64_t PacketID = 0;
  Bytes Data;
};

// decoder.go:43-51
struct FECDecoderMetrics {
  int64_t PacketsReceived = 0;
  int64_t RepairPacketsReceived = 0;
  int64_t PacketsRecovered = 0;
  int64_t RecoveryEvents = 0;
  int64_t FailedRecoveries = 0;
  int64_t GroupsActive = 0;
  int64_t GroupsEvicted = 0;
};

// decoder.go:24-343
class FECDecoder {
 public:
  static constexpr size_t kMaxActiveGroups = 4096;       // decoder.go:10
  static constexpr int kGroupTTLSeconds = 5;             // decoder.go:11
  static constexpr int kMaxSymbolLen = 1500;             // decoder.go:12
  static constexpr int kMaxPacketCount = 255;            // decoder.go:13

  FECDecoder();
  bool AddPacket(const uint8_t* packet, size_t len, uint64_t packetID, uint64_t groupID);
  bool AddPacket(const Bytes& p, uint64_t id, uint64_t gid) { return AddPacket(p.data(), p.size(), id, gid); }
  std::pair<bool, std::vector<Recovered>> AddRedundancyPacket(const uint8_t* pkt, size_t len);
  std::pair<bool, std::vector<Recovered>> AddRedundancyPacket(const Bytes& p) {
    return AddRedundancyPacket(p.data(), p.size());
  }
  void CleanupGroups();
  FECDecoderMetrics GetMetrics();
  void ResetMetrics();
  size_t groups() {
    std::lock_guard<std::mutex> lk(mu_);
    return groups_.size();
  }
  // Test hook: age every group by `seconds` (the reference's TTL is wall-clock).
  void AgeGroupsForTest(int seconds);
  // Stored symbol of (groupID, packetID), empty if absent (recovered packets included).
  Bytes GetPacket(uint64_t groupID, uint64_t packetID);

 private:
  struct Group {
    uint64_t groupID = 0;
    std::chrono::steady_clock::time_point createdAt;
    int packetCount = 0;
    int symbolLen = 0;
    std::map<uint64_t, bool> present;
    std::map<uint64_t, Bytes> packets;
    Bytes redundancy;
    bool hasRedundancy = false;
    int received = 0;
  };
  bool tryRecover(Group& g);
  bool recoverSingle(Group& g, uint64_t* id, Bytes* out);
  void evictOldestGroup();

  std::map<uint64_t, Group> groups_;
  std::mutex mu_;
  FECDecoderMetrics metrics_;
};

// Batch extension (new): rebuild up to r lost packets per group on the GPU.
// data: groups*k*packetSize, parity: groups*r*packetSize, erasures: bit s = shard s lost.
// Returns the number of unrecoverable groups, or -1 with err set.
int64_t RecoverBatchRS(Bytes& data, const Bytes& parity, const std::vector<uint64_t>& erasures, int k, int r,
                       int packetSize, Error* err);
Error EncodeBatchRS(const Bytes& data, int k, int r, int packetSize, Bytes* parity);

}  // namespace quicfec
