// fec_kernels.hpp — launch interface between the C-ABI shim (fec_shim.cpp) and the
// gfx950 kernels (fec_kernels.hip).  Internal to libfec_hip.so.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace qfec {

// Byte offsets of packets, when the data shards are not contiguous.
// kAddr: `offsets` holds one absolute device address per packet (u64), `data` is unused --
// the legacy-call coalescer (fec_coalesce.cpp) gathers packets from many callers' buffers.
enum class OffsetKind : int { kNone = 0, kU32 = 1, kU64 = 2, kAddr = 3 };

// Packets of any size P >= 16 at any byte address run on the 16-byte-column kernels
// (fec_kernels.hip header); shorter ones on the byte kernels.
struct EncodeLaunch {
  const uint8_t* data;       // base of the data shards (device address)
  const void* offsets;       // device u32/u64 offsets (k per group) or nullptr
  OffsetKind off_kind;
  uint8_t* parity;           // parity row (g, i) at (g * r + i) * P
  uint64_t groups;
  uint32_t k, r, P;
  const void* tables;        // (r-1) x k CoefEntry (rows 1..r-1), device
  int waves_per_cu = 0;      // occupancy cap of the streaming kernel (0 = tuned default)
};

// Tuned occupancy caps (waves per CU) of the streaming kernels: fewer concurrent waves
// than the hardware allows keep the HBM request stream more local and measured faster
// (tools/probe_encode.hip, tools/probe_decode.hip).
// Encode: 2 workgroups per CU (k=10/1200 B: 2 x 5 waves, 5.70 vs 5.26 TB/s uncapped;
// 1024 B: 2 x 4 waves 6.12 vs 5.92 at 3; 1216 B: 2 x 6 waves 5.92 vs 5.25 at 1); one more
// for r >= 4 (k=20 r=5: 5.47 at 3 vs 4.99 at 2); none for the runtime-k kernel
// (k=10 r=2: 5.61 uncapped vs 3.66 at 2).  profiles/r01_encode_blocks_sweep.txt.
constexpr int kEncodeBlocksPerCU = 2;
constexpr int kEncodeXorWavesPerCU = 15;  // r = 1 (XOR row only), rounded to whole workgroups
constexpr int kDecodeWavesPerCU = 0;   // measured: any cap below ~20 waves/CU is slower

// Dynamic LDS bytes that cap a workgroup of `waves_per_block` waves at about
// `waves_per_cu` waves per CU (160 KiB LDS per CU); 0 = no cap.
inline uint32_t occupancy_cap_lds(int waves_per_cu, uint32_t waves_per_block) {
  if (waves_per_cu <= 0 || waves_per_block == 0) return 0;
  // nearest whole number of workgroups (a 6-wave workgroup under a 10-wave cap gets 2, not 1)
  uint32_t blocks = (static_cast<uint32_t>(waves_per_cu) + waves_per_block / 2) / waves_per_block;
  if (blocks == 0) blocks = 1;
  if (blocks * waves_per_block >= 32) return 0;
  return 160u * 1024u / (blocks + 1) + 16u;
}

struct LevelMeta {           // codebook levels e = 1..32 (see gf256.hpp)
  uint64_t base[33];
  uint64_t stride[33];
  uint64_t count_r[33];      // C(r, e)
};

// Decode kernel selection (tests / probes; the library uses kDecodeAuto).
constexpr int kDecodeAuto = 0;           // the measured best of the forms below
constexpr int kDecodeWavePerGroup = 1;   // one wave per group, 16-B lanes only
constexpr int kDecodeTiledPlain = 2;     // workgroup = whole groups, per-lane records
constexpr int kDecodeTiledNt = 3;        //   same, non-temporal stores
constexpr int kDecodeWavePlain = 4;      // one wave per group, 16-B passes + 4-B tail
constexpr int kDecodeWaveNt = 5;         //   same, non-temporal stores (the default)
constexpr int kDecodeWaveNoBranch = 6;   //   same, no branch on coefficient 0 / 1
constexpr int kDecodeFused = 7;          // one wave per group, 16-B and 4-B pieces fused
constexpr int kDecodeFusedDirect = 8;    //   same, survivor addresses from the erasure mask

struct DecodeLaunch {
  int variant = kDecodeAuto;
  // Where rebuilt shards are stored, same layout as `data`; nullptr = in place in `data`.
  // May be a device-visible pointer to page-locked host memory (zero-copy writes).
  uint8_t* out = nullptr;
  uint8_t* data;
  const uint8_t* parity;
  const uint64_t* masks;
  uint32_t* rec_off;         // workspace, one u32 per group
  uint8_t* status;           // nullable
  const uint8_t* codebook;   // device
  const uint64_t* binom;     // device, 65 x 65
  LevelMeta meta;
  uint64_t groups;
  uint32_t k, r, P;
  int waves_per_cu = 0;      // occupancy cap of the decode kernel (0 = tuned default)
  bool rec_ready = false;    // rec_off already filled by the host (sparse plan): no classify
  int xcd_swizzle = -1;      // XCD-aware group order: -1 tuned default, 0 off, 1 on
  // Groups per wave of the mask-addressed decode (kDecodeScanGroups or 1).  One wave per
  // group is best when most groups lost data (C3: 5.35 TB/s vs 4.92 at 8 per wave); when few
  // did (C5, iid 1% loss: ~10% of groups) 8 per wave saves the dispatch and mask-load latency
  // of the waves that find nothing to do (0.257 -> 0.243 ms per 1M groups,
  // profiles/r02_probe_decode_scan.txt).  The host paths that know the masks pick it.
  uint32_t scan = 1;
  // `codebook` holds coefficient bytes (compact layout, gf256.hpp) rather than CoefEntry
  // tables: set exactly when decode_compact_tables(*this) (launch_decode checks).
  bool compact_tables = false;
  // Rebuilt shards go to out + (g * r + m) * P (m-th lost data shard of group g, ascending),
  // `data` is only read (fec_recover_batch_rs_dev); else in place / at `out` like `data`.
  bool compact_out = false;
  // compact_out with rec_off = the packed rows' row_start (fec_recover_batch_rs_dev_packed):
  // rows are placed by global row index, so chunked launches must not offset `out`.
  bool packed_rows = false;
};

constexpr uint32_t kDecodeScanGroups = 8;
// Share of groups needing a rebuild below which the host paths use the scan form.
constexpr double kDecodeScanMaxShare = 0.25;

constexpr int kDecodeFusedXcdSwizzle = 1;  // tuned per kernel (fec_kernels.hip decode_swizzle)
constexpr int kDecodeWaveXcdSwizzle = 1;

hipError_t launch_encode(const EncodeLaunch& a, hipStream_t s);
hipError_t launch_decode(const DecodeLaunch& a, hipStream_t s);
// Packed recover rows: row_start[g] = exclusive prefix sum of the rows each group rebuilds
// (lost data shards when recoverable, else 0); *total (nullable) = all rows.  block_sums:
// rows_prefix_workspace_bytes(groups) of device workspace.
uint64_t rows_prefix_workspace_bytes(uint64_t groups);
hipError_t launch_rows_prefix(const uint64_t* masks, uint64_t groups, uint32_t k, uint32_t r, uint32_t* row_start,
                              uint32_t* block_sums, uint64_t* total, hipStream_t s);
// Packed recover in one launch (recover_runs, fec_kernels.hip): every workgroup owns 512
// consecutive groups, finds its run's first row by decoupled look-back (no prefix launches)
// and writes its rebuilt rows as one contiguous run, staged through an LDS image of up to
// stage bytes.  Mask-addressed shapes only (runs_supported).
struct RunsLaunch {
  const uint8_t* data;
  const uint8_t* parity;
  const uint64_t* masks;
  uint64_t groups;
  uint32_t k, r, P;
  const uint8_t* codebook;   // dense CoefEntry codebook (the mask-addressed decode's)
  LevelMeta meta;
  uint8_t* out;              // packed rows
  uint32_t* row_start;       // one u32 per group (written)
  uint64_t* total;           // nullable: all rows
  uint8_t* status;           // nullable
  // runs_workspace_bytes(groups) of device memory, zeroed when first allocated, kept by the
  // caller stream: ticket counter, chunk totals, look-back words
  void* workspace;
  // look-back epoch of the first launch; a call takes runs_launches(groups) epochs, never
  // reused while the workspace lives (the caller counts; < 2^30, then re-zero the workspace)
  uint32_t epoch;
  int stage_bytes = -1;      // LDS run image: -1 tuned default (test switch kRunsStage), 0 none
};
// LDS run image per workgroup of 512 groups (tools/probe_runs.hip; DESIGN_HISTORY.md §5 round 4): C5's
// ~59 rows per tile fit 48 KB (40 rows) mostly; two workgroups per CU.
// recover_runs' run image per workgroup.
constexpr int kRunsStageBytes = 48 * 1024;
bool runs_supported(uint32_t k, uint32_t r, uint32_t P);
uint32_t runs_launches(uint64_t groups);
uint64_t runs_workspace_bytes(uint64_t groups);
uint32_t runs_stage_bytes(const RunsLaunch& a);
hipError_t launch_recover_runs(const RunsLaunch& a, hipStream_t s);
// Whether launch_decode(a) uses the rec_off workspace (every form but the mask-addressed
// one, which classifies inline).  The caller then provides a workspace private to the call.
bool decode_needs_rec_off(const DecodeLaunch& a);
// Whether launch_decode(a) runs a form that reads a compact codebook (coefficient bytes).
bool decode_compact_tables(const DecodeLaunch& a);
// ---- resident legacy encoder (fec_coalesce.cpp "resident server") ----
// A ring of submission slots (page-locked coherent host memory, or VRAM written through the BAR).
// The host fills slot seq % kServerSlots with a legacy call's groups: every 8-B word of a slot
// carries the slot's tag, server_tag(seq), in its top 16 bits, so the device recognises a
// complete slot by the tags alone, whatever order its reads of the host's stores land in.  An
// aligned 8-B store is the unit the host's stores are assumed to arrive in (x86 quadword
// atomicity); nothing larger is assumed to arrive in one piece, so every 8-B word is
// self-validating.  Resident workgroups serve the slots in seq order (one per serving class,
// below) and store done[seq % kServerSlots] = seq + 1.  Calls are served without a kernel launch
// each.
//
// Tags and the epoch.  A slot's tag is (lap & (epoch - 1)) + 1 with lap = seq / kServerSlots and
// epoch a power of two (no division on the server's critical path), so the tags of one slot
// repeat every `epoch` laps (32768; shorter in the test library, fec_knobs.hpp kResidentEpoch).  A word left from the previous epoch could carry the current tag (a word written
// exactly `epoch` laps ago and not since, e.g. a later group's address word under inline-only
// calls), so the slot is scrubbed at every epoch boundary: the server zeroes the slot's words
// and its inline data area after serving the last lap of an epoch, before that slot's done word
// (its next occupant writes only after it has seen the done word, so the zeroes are in place
// first), and the host zeroes the slot's inline output staging before publishing the first lap
// of an epoch.  Within an epoch every tag of a slot is used once, so no stale word matches;
// tag 0 (the zeroed state) never matches.
constexpr uint32_t kServerSlots = 1024;
constexpr uint32_t kServerMaxGroups = 8;  // groups per slot (legacy calls of 1..8 groups)
constexpr uint32_t kServerPackets = 10;   // the legacy call's packets per group
constexpr uint64_t kServerTagShift = 48;  // addresses below 2^48 (x86-64 user virtual addresses)
constexpr uint64_t kServerAddrMask = (1ull << kServerTagShift) - 1;
constexpr uint32_t kServerEpoch = 32768;  // laps per tag epoch, a power of two (tags 1 .. epoch fit 16 bits)
__host__ __device__ inline uint32_t server_tag(uint64_t seq, uint32_t epoch) {
  return (static_cast<uint32_t>(seq / kServerSlots) & (epoch - 1u)) + 1u;
}
// Whether the server scrubs the slot of seq after serving it (the last lap of an epoch).
__host__ __device__ inline bool server_scrub_after(uint64_t seq, uint32_t epoch) {
  return (static_cast<uint32_t>(seq / kServerSlots) & (epoch - 1u)) == epoch - 1u;
}
struct alignas(64) ServerSlot {
  uint64_t out;             // tag | device address of the repair rows, row g at out + g * P
  uint64_t shape;           // tag | P (bits 0..15) | groups (bits 16..23; 0 = nothing to do) | kServerInline
  uint64_t addr[kServerMaxGroups * kServerPackets];  // tag | device address of packet (g, j) at [g * 10 + j]
};
// VRAM ring (large-BAR devices, fec_coalesce.cpp Resident): the slots and the packets of small
// calls live in uncached device memory that the host writes through the BAR, so the server's
// poll and packet loads stay on the device.  An inline slot (shape bit kServerInline) carries
// no addresses: its packets are copied by the host into the slot's data area, packet (g, j) as
// 16-B chunks at chunk (g * 10 + j) * nch + c, nch = ceil(P / 12).  A chunk is two 8-B halves,
// each 6 payload bytes and the slot's 16-bit tag in its top two bytes:
//   bytes 0..5 = payload [12c, 12c + 6), bytes 6..7 = tag, bytes 8..13 = payload [12c + 6,
//   12c + 12), bytes 14..15 = tag (payload zero past P),
// so each half validates itself (a 16-B write-combined store may reach the device as two 8-B
// pieces) and no ordering of the host's stores through the BAR is assumed.  The rows come back
// the same way: an inline slot's `out` is its output staging in page-locked host memory, repair
// chunk (g, c) in the same two-half form at out + (g * nch + c) * 16, and the host takes the rows
// once both halves of every chunk carry the tag (the done word then only says "consumed").
constexpr uint64_t kServerInline = 1ull << 24;
constexpr uint32_t kInlineMaxGroups = 4;
constexpr uint32_t kInlineMaxP = 1536;
constexpr uint32_t kInlinePayload = 12;  // payload bytes of a 16-B chunk (6 per 8-B half)
constexpr uint32_t kInlineSlotBytes = kInlineMaxGroups * kServerPackets * (kInlineMaxP / kInlinePayload) * 16;
// Serving classes.  An instance is `classes` workgroups (a power of two, 1 .. kServerMaxClasses,
// so it divides kServerSlots): workgroup c serves the seqs with seq % classes == c, in order, so
// concurrent callers are served by independent poll -> serve -> done cycles.
constexpr uint32_t kServerMaxClasses = 8;
constexpr uint32_t kServerPoll = 16;  // slots of its class a workgroup reads per poll (the longest run it serves)
struct alignas(64) ServerControl {
  uint64_t stop;            // host -> device: leave at the next poll
  uint64_t pad0[7];
  uint64_t exited;          // device -> host: generation of the last instance that left (its last workgroup)
  uint64_t pad1[7];
  uint64_t progress[kServerMaxClasses];   // device -> host: every seq of class c below progress[c] was served
  uint64_t bad_slots[kServerMaxClasses];  // device -> host: polls that found a slot with a word not yet landed (diagnostic)
  uint64_t scrubs[kServerMaxClasses];     // device -> host: slots scrubbed at an epoch boundary (diagnostic)
};
// Device memory the workgroups of one instance share (uncached: they run on different XCDs, each
// with its own L2).  Words are tagged with the instance's generation, so nothing is reset
// between instances.
struct alignas(64) ServerCoord {
  uint64_t leave;                      // gen: every workgroup of instance gen leaves at its next poll
  uint64_t exits;                      // (gen << 8) | workgroups of instance gen that have left
  uint64_t pad[6];
  uint64_t idle[kServerMaxClasses];    // gen while class c's workgroup has been idle for idle_ticks, else 0
};
// The coordination rules, shared by legacy_server and the CPU model (tests/csrc/ring_protocol_test.cpp).
// Whether every class of instance gen is idle: this one (idle, now) and the others by the flags
// it last read (idle_seen[c] == gen; a flag of an earlier instance never counts).
__host__ __device__ inline bool server_all_idle(bool idle, const uint64_t* idle_seen, uint32_t classes, uint32_t cls,
                                                uint64_t gen) {
  bool all = idle;
  for (uint32_t c = 0; c < classes; ++c) all = all && (c == cls || idle_seen[c] == gen);
  return all;
}
// The exit count: a workgroup leaving instance gen turns the word v into this (the word still
// holds the previous instance's count until the first of this one's); the workgroup whose new
// word counts all `classes` is the last out and stores ctl->exited = gen.
__host__ __device__ inline uint64_t server_exits_next(uint64_t v, uint64_t gen) {
  return (v >> 8) == gen ? v + 1 : (gen << 8) | 1u;
}
__host__ __device__ inline bool server_exits_last(uint64_t nv, uint32_t classes) { return (nv & 0xFFu) == classes; }
// One resident instance serving the ring, each class from its progress mark, until every class
// has found nothing to do for idle_ticks, or it lived life_ticks (wall-clock ticks,
// hipDeviceAttributeWallClockRate), or the host sets ctl->stop; on leaving a workgroup stores its
// class's progress, and the last one to leave stores exited = gen.
// coord: nullptr when classes == 1.  slow_ticks: a workgroup other than class 0's without work
// for that long polls slowly (~5 us apart instead of ~1.5) until it finds some.
// stamps: nullptr, or 256 x 8 words of host memory for the diagnostic phase stamps of class 0
// (test library, fec_knobs.hpp kResidentStamps).
// inl: the inline data areas (kInlineSlotBytes per slot) when the ring is in VRAM, else nullptr;
// then the host's stop word (host memory) is read by every 16th poll only, not every poll.
// epoch: laps per tag epoch (server_tag), a power of two, 1 .. kServerEpoch.
hipError_t launch_legacy_server(ServerSlot* ring, uint8_t* inl, uint64_t* done, ServerControl* ctl,
                                ServerCoord* coord, uint32_t classes, uint64_t gen, uint64_t idle_ticks,
                                uint64_t slow_ticks, uint64_t life_ticks, uint64_t* stamps, uint32_t epoch,
                                hipStream_t s);

hipError_t launch_fill_splitmix(uint8_t* dst, uint64_t nbytes, uint64_t seed, uint64_t byte_offset,
                                hipStream_t s);
// dst <- src, nbytes a multiple of 16, both 16-B aligned (box calibration).
hipError_t launch_copy_words(const uint8_t* src, uint8_t* dst, uint64_t nbytes, hipStream_t s);

// Records marking "nothing to do" / "unrecoverable" in rec_off.
constexpr uint32_t kRecNone = 0xFFFFFFFFu;
constexpr uint32_t kRecBad = 0xFFFFFFFEu;

}  // namespace qfec
