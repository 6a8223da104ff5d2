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
//   * FECDecoder recovery runs on the GPU (xor_packets via fec_select_xor_impl).  New for
//     r > 1: RSBatchEncoder, the row 1..r-1 wire header, FECDecoder's multi-loss path and
//     RecoverBatchRS (see "r > 1" below).
#pragma once

#include <chrono>
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

struct FECEncoderCtx;
struct FECBatcher;

namespace quicfec {

using Bytes = std::vector<uint8_t>;

// Go's `error`: empty = nil.
struct Error {
  std::string msg;
  int code = 0;  // the library's FEC_ERR_* when a library call failed (e.g. a batcher result
                 // that expired: FEC_ERR_RANGE from fec_batcher_wait), else 0
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
  std::vector<Bytes> extra;  // BatchedFECEncoder with r > 1: rows 1..r-1 (FE C1 packets)
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
class SharedFECDecodeBatcher;

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

  // r > 1 (new).  Deferred mode: groups that become recoverable by rows >= 1 are queued
  // instead of decoded one by one; RecoverPending rebuilds every queued group in one library
  // call per (k, r) and returns the recovered packets keyed by group id.  Immediate mode
  // (the default) decodes such a group as soon as it is recoverable.
  void SetDeferredRecovery(bool deferred);
  // New: single-loss rebuilds of groups of the batcher's k (row 0 only, r = 1 batchers) go
  // through a batch shared with other connections' decoders; results are unchanged.
  void SetSharedBatcher(std::shared_ptr<SharedFECDecodeBatcher> batcher);
  std::vector<std::pair<uint64_t, std::vector<Recovered>>> RecoverPending(Error* err = nullptr);
  size_t pending() {
    std::lock_guard<std::mutex> lk(mu_);
    return pending_.size();
  }

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
    // r > 1 (new): rows 1..r-1 by index, and the code shape from their headers
    std::map<int, Bytes> rows;
    int k = 0, r = 0;
    bool queued = false;
  };
  bool tryRecover(Group& g, std::vector<Recovered>* list);
  bool canRecoverRS(const Group& g) const;
  // One library call over groups of one (k, r); fills lists[i] for gs[i].  True when the
  // call ran (per-group failures are counted in FailedRecoveries).
  bool recoverRS(const std::vector<Group*>& gs, std::vector<std::vector<Recovered>>* lists);
  bool recoverSingle(Group& g, uint64_t* id, Bytes* out);
  void evictOldestGroup();
  std::shared_ptr<SharedFECDecodeBatcher> shared_;

  std::map<uint64_t, Group> groups_;
  std::mutex mu_;
  FECDecoderMetrics metrics_;
  bool deferred_ = false;
  std::vector<uint64_t> pending_;
};

// ===================================================================== r > 1 (new)
// a batched encoder that emits r repair packets per group, the
// wire header for rows 1..r-1, and the decoder path that rebuilds up to r losses.
//
// Wire format.  Row 0 keeps the reference's 11-byte header and payload byte for byte
// (encoder_hybrid.go:175-192, encoder.go:146-160): FE C0 | groupID u64 LE | count u8.  A
// receiver that only knows the reference format recovers single losses from it as before.
// Rows i >= 1 carry a 14-byte header the reference parser rejects (decoder.go:73 checks
// b[1] == 0xC0), so old receivers ignore them:
//   FE C1 | groupID u64 LE | count u8 | row u8 (1..r-1) | r u8 | k u8 | payload
// count = data packets in the group (<= k; slots count..k-1 are zero), payload = the
// group's largest packet length.  Coding is bytewise, so any common truncation or zero
// padding of a group's symbols keeps the recovered prefix exact (what lets the decoder keep
// the reference's symbol-length rule, decoder.go:115-120).
constexpr size_t kRepairHeaderLen = 11;    // row 0, the reference's header
constexpr size_t kRSRepairHeaderLen = 14;  // rows 1..r-1

struct RSRepairHeader {
  uint64_t groupID = 0;
  int count = 0;  // data packets in the group
  int row = 0;    // parity row 0..r-1
  int r = 0;      // 0 when unknown (a row-0 packet)
  int k = 0;      // 0 when unknown (a row-0 packet)
};

// Parse either header form; false for anything else (the same bounds as decoder.go:72-85,
// plus row < r and k + r <= 64 for the new form).
bool ParseRepairHeader(const uint8_t* b, size_t len, RSRepairHeader* h, const uint8_t** payload, size_t* plen);
Bytes MakeRepairPacket(const RSRepairHeader& h, const uint8_t* payload, size_t plen);

// Groups of k packets, batchGroups groups per library call (one fec_encode_batch_rs over a
// pinned slab), r repair packets per group.  Row 0 of every group is byte-identical to
// HybridFECEncoder's repair packet for the same packets and group id.
class RSBatchEncoder {
 public:
  // nullptr when the GPU library cannot be initialised or the shape is invalid
  // (1 <= k, 1 <= r, k + r <= 64, batchGroups >= 1).  slotSize = the widest packet expected;
  // larger packets widen the slot on the fly.
  static std::unique_ptr<RSBatchEncoder> New(int k, int r, int batchGroups, int slotSize = 1200);
  ~RSBatchEncoder();
  RSBatchEncoder(const RSBatchEncoder&) = delete;
  RSBatchEncoder& operator=(const RSBatchEncoder&) = delete;

  // Copies the packet into the slab; when the batch is full, encodes it and appends every
  // group's r repair packets (group order, row order) to *out.
  Error AddPacket(const uint8_t* packet, size_t len, std::vector<Bytes>* out);
  Error AddPacket(const Bytes& p, std::vector<Bytes>* out) { return AddPacket(p.data(), p.size(), out); }
  // Encodes the complete groups and the partial one (count < k) now.
  Error Flush(std::vector<Bytes>* out);
  FECMetrics GetMetrics();
  Error Close();
  int k() const { return k_; }
  int r() const { return r_; }
  int slotSize() const { return slot_; }
  uint64_t nextGroupID() const { return groupID_; }

 private:
  RSBatchEncoder() = default;
  Error encodeLocked(int groups, std::vector<Bytes>* out);
  Error widenLocked(size_t newSlot, std::vector<Bytes>* out);

  FECEncoderCtx* ctx_ = nullptr;
  int k_ = 0, r_ = 0, batch_ = 0;
  size_t slot_ = 0;
  uint8_t* slab_ = nullptr;    // pinned, batch_ * k_ * slot_
  uint8_t* parity_ = nullptr;  // pinned, batch_ * r_ * slot_
  std::vector<uint32_t> count_, maxLen_;  // per group of the open batch
  int open_ = 0;                          // groups started in the open batch
  uint64_t groupID_ = 0;
  std::mutex mu_;
  FECMetrics metrics_;
};

// ===================================================================== batcher (new)
// SURVEY.md §8(f) item 1.  The reference runs one HybridFECEncoder per QUIC stream and
// encodes one group per call (encoder_hybrid.go:115).  Here every stream's encoder hands its
// finished groups to one process-wide SharedFECBatcher (fec_batcher_*, include/fec_hip.h),
// which encodes them together when maxGroups are pending or deadlineUs after the oldest
// pending group, whichever comes first: a repair is at most deadlineUs + one encode late.
class SharedFECBatcher {
 public:
  // nullptr when the GPU library cannot be initialised or the shape is invalid.
  static std::shared_ptr<SharedFECBatcher> New(int k, int r, int slotBytes = 1500, int maxGroups = 4096,
                                               int deadlineUs = 1000, int device = -1, int slabs = 3);
  // One batcher per listed GPU behind this handle (fec_batcher_new_multi; repeats allowed, empty
  // = every visible GPU): host-resident batches are bound by their GPU's PCIe link.
  static std::shared_ptr<SharedFECBatcher> NewMulti(const std::vector<int>& devices, int k, int r,
                                                    int slotBytes = 1500, int maxGroups = 4096, int deadlineUs = 1000,
                                                    int slabs = 3);
  ~SharedFECBatcher();
  SharedFECBatcher(const SharedFECBatcher&) = delete;
  SharedFECBatcher& operator=(const SharedFECBatcher&) = delete;
  FECBatcher* raw() const { return b_; }
  int k() const { return k_; }
  int r() const { return r_; }
  int slot() const { return slot_; }
  void Flush();
  // groups, batches, full_flushes, deadline_flushes, max_batch
  std::vector<uint64_t> Stats();

 private:
  SharedFECBatcher() = default;
  FECBatcher* b_ = nullptr;
  int k_ = 0, r_ = 0, slot_ = 0;
};

// One batch of recoveries for the receivers of every connection (fec_batcher_new_decoder):
// the reference's FECDecoder rebuilds one group per call (decoder.go:255-287), a GPU launch
// per group; FECDecoder::SetSharedBatcher routes those rebuilds through this instead.
class SharedFECDecodeBatcher {
 public:
  // nullptr when the GPU library cannot be initialised or the shape is invalid (k + r <= 64).
  static std::shared_ptr<SharedFECDecodeBatcher> New(int k, int r, int slotBytes = 1500, int maxGroups = 4096,
                                                     int deadlineUs = 200, int device = -1, int slabs = 3);
  // One decoder batcher per listed GPU behind this handle (fec_batcher_new_decoder_multi).
  static std::shared_ptr<SharedFECDecodeBatcher> NewMulti(const std::vector<int>& devices, int k, int r,
                                                          int slotBytes = 1500, int maxGroups = 4096,
                                                          int deadlineUs = 200, int slabs = 3);
  ~SharedFECDecodeBatcher();
  SharedFECDecodeBatcher(const SharedFECDecodeBatcher&) = delete;
  SharedFECDecodeBatcher& operator=(const SharedFECDecodeBatcher&) = delete;
  int k() const { return k_; }
  int r() const { return r_; }
  int slot() const { return slot_; }
  // Rebuilds a group's lost data shards and waits for its batch (at most the deadline plus
  // one launch).  shards: k data shards then r parity rows, nullptr = lost, each `len` bytes.
  // out: (shard id, rebuilt bytes) in ascending shard order.
  Error Recover(const std::vector<const uint8_t*>& shards, uint32_t len, std::vector<std::pair<int, Bytes>>* out);
  void Flush();
  // groups, batches, full_flushes, deadline_flushes, max_batch
  std::vector<uint64_t> Stats();

 private:
  SharedFECDecodeBatcher() = default;
  FECBatcher* b_ = nullptr;
  int k_ = 0, r_ = 0, slot_ = 0;
};

// One stream's encoder on a shared batcher: HybridFECEncoder's API, groups of k packets,
// and its wire bytes -- the row-0 repair packet (FE C0 | groupID | count | XOR payload) is
// byte-identical to HybridFECEncoder's for the same packets -- plus rows 1..r-1 as FE C1
// packets (AddPacketResult::extra) when the batcher's r > 1.
class BatchedFECEncoder {
 public:
  explicit BatchedFECEncoder(std::shared_ptr<SharedFECBatcher> batcher);
  // Synchronous, like HybridFECEncoder::AddPacket: the k-th packet submits the group and
  // waits for its batch (at most the deadline plus one encode).
  AddPacketResult AddPacket(const uint8_t* packet, size_t len, uint64_t packetID);
  AddPacketResult AddPacket(const Bytes& p, uint64_t id) { return AddPacket(p.data(), p.size(), id); }
  // Asynchronous: the k-th packet submits without waiting; Poll appends the repair packets
  // of finished groups (in group order, row order) and waits up to timeoutUs for the oldest
  // outstanding one (0: no wait, < 0: all of them).  A group it cannot collect (its result
  // expired in the batcher's ring, or its batch failed) is dropped from the outstanding list
  // and ends the call with that error; the rows appended before it stay in `out`.
  Error AddPacketAsync(const uint8_t* packet, size_t len, uint64_t packetID);
  Error Poll(std::vector<Bytes>* out, int64_t timeoutUs = 0);
  size_t outstanding() {
    std::lock_guard<std::mutex> lk(mu_);
    return outstanding_.size();
  }
  // The partial group (count < k) now, synchronously, as HybridFECEncoder::Flush (its rows
  // 1..r-1 in `extra`).  FlushAsync submits it without waiting and closes the batch now.
  AddPacketResult Flush();
  Error FlushAsync();
  FECMetrics GetMetrics();

 private:
  struct Ticket {
    int64_t ticket;
    uint64_t groupID;
    int count;
  };
  Error submitLocked(Ticket* t);
  Error collect(const Ticket& t, int64_t timeoutUs, std::vector<Bytes>* rows, bool* ready);

  std::shared_ptr<SharedFECBatcher> b_;
  void addLocked(const uint8_t* packet, size_t len);
  std::vector<Bytes> packets_;  // packet buffers, kept across groups; the first npk_ are this group's
  size_t npk_ = 0;
  uint64_t groupID_ = 0;
  std::deque<Ticket> outstanding_;
  Bytes rowbuf_;
  std::vector<const uint8_t*> ptrs_;
  std::vector<uint32_t> lens_;
  std::mutex mu_;
  FECMetrics metrics_;
};

// Batch extension (new): rebuild up to r lost packets per group on the GPU.
// data: groups*k*packetSize, parity: groups*r*packetSize, erasures: bit s = shard s lost.
// Returns the number of unrecoverable groups, or -1 with err set.
int64_t RecoverBatchRS(Bytes& data, const Bytes& parity, const std::vector<uint64_t>& erasures, int k, int r,
                       int packetSize, Error* err);
Error EncodeBatchRS(const Bytes& data, int k, int r, int packetSize, Bytes* parity);

}  // namespace quicfec
