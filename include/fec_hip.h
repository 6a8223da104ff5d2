/*
 * fec_hip.h — batch GF(2^8) erasure-coding API of libfec_hip.so (new; the reference has
 * no equivalent).  These are the entry points SURVEY.md §8(b) "New entry points" asks
 * for: explicit k and r, 64-bit layout, device-pointer variants on a caller stream,
 * device selection.  Plain C types only.
 *
 * Code: byte-wise GF(2^8), polynomial 0x11D, systematic generator
 * [I_k ; M] with M an r x k Cauchy matrix normalised so that row 0 and column 0 are all
 * ones.  Parity row 0 is therefore the reference XOR repair packet
 * (fec_xor_simd.cpp:411-427) byte for byte.  MDS for k + r <= 256.
 *
 * Layout (contiguous form):
 *   data   : G*k*P bytes, data shard (g,j) at (g*k + j)*P
 *   parity : G*r*P bytes, parity row (g,i) at (g*r + i)*P
 * Erasure mask of a group: bit s set (s < k+r) => shard s lost; s < k is data shard s,
 * s >= k is parity row s-k.  Decode requires k + r <= 64.
 *
 * Decode rule: erased data shards are rebuilt in place in `data` from every surviving
 * data shard plus the lowest-indexed surviving parity rows (as many as there are erased
 * data shards).  A single lost data shard with parity row 0 alive is therefore the
 * reference XOR recovery (decoder.go:255-287).  Groups with more erased data shards than
 * surviving parity rows are left untouched and reported unrecoverable.
 */
#ifndef FEC_HIP_H
#define FEC_HIP_H

#include <stddef.h>
#include <stdint.h>

#include "fec_xor_simd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Return codes.  -1 keeps the reference's meaning (NULL argument, fec_xor_simd.cpp:564). */
#define FEC_OK 0
#define FEC_ERR_NULL (-1)      /* a required pointer is NULL                      */
#define FEC_ERR_HIP (-2)       /* the HIP runtime reported an error               */
#define FEC_ERR_RANGE (-3)     /* k, r, packet size or group count unsupported     */
#define FEC_ERR_NODEV (-4)     /* no usable GPU                                   */
#define FEC_ERR_NOMEM (-5)     /* device or pinned allocation failed              */
#define FEC_ERR_AGAIN (-6)     /* fec_batcher_wait: not ready within the timeout   */
#define FEC_ERR_UNRECOVERABLE (-7) /* fec_batcher_wait_rebuilt: too many shards lost */

/* Number of visible HIP devices (0 when none or the runtime is unusable). */
int fec_hip_device_count(void);

/* Message of the calling thread's last failing call ("" if none; entry points taking a
 * context clear it on entry). */
const char* fec_hip_last_error(void);

/* Message of the last failing call on `ctx`, whichever thread made it (Go: a goroutine may
 * move to another OS thread between the failing call and the read, so the thread-local
 * text above may be empty or another call's).  Copies at most buflen-1 bytes plus a NUL
 * into buf (when buf != NULL and buflen > 0) and returns the message's full length; 0 for
 * a NULL context or no failure yet.  Replaces the cgo wrapper's code-only message
 * (fec_cgo.go:147-149). */
size_t fec_ctx_last_error(FECEncoderCtx* ctx, char* buf, size_t buflen);

/* fec_encoder_new on an explicit device ordinal (shards of a multi-GPU job). */
FECEncoderCtx* fec_encoder_new_device(double redundancy, uint32_t max_groups, int device);

/* Device ordinal a context is bound to, or -1 for NULL. */
int fec_encoder_device(const FECEncoderCtx* ctx);

/* Library build identifier, for logs: "libfec_hip <version> gfx950 src=<sha256 of the sources it was
 * built from>" (quic-test_amd/csrc/src_hash.py defines the hash; tests/test_abi.py checks it). */
const char* fec_hip_version(void);

/* The r x k parity matrix M, row-major (r*k bytes).  0, or FEC_ERR_RANGE. */
int fec_parity_matrix(uint32_t k, uint32_t r, uint8_t* out);

/* ---- synchronous API: host or device pointers (auto-detected) ----
 * offsets: NULL for the contiguous layout, else k*num_groups u64 byte offsets into
 * `data` (data shard (g,j) at data + offsets[g*k + j]); parity is always contiguous. */
int fec_encode_batch_rs(FECEncoderCtx* ctx, const uint8_t* data, const uint64_t* offsets,
                        uint64_t num_groups, uint32_t k, uint32_t r, uint32_t packet_size,
                        uint8_t* parity_out);

/* status_out (nullable): one byte per group, 0 = recovered or nothing lost,
 * 1 = unrecoverable.  unrecoverable_out (nullable): count of status 1. */
int fec_decode_batch_rs(FECEncoderCtx* ctx, uint8_t* data, const uint8_t* parity,
                        const uint64_t* erasure_masks, uint64_t num_groups, uint32_t k,
                        uint32_t r, uint32_t packet_size, uint8_t* status_out,
                        uint64_t* unrecoverable_out);

/* ---- device-resident API: device pointers only, asynchronous on `stream`
 * (a hipStream_t; NULL = the context's own stream).  Contiguous layout only. ---- */
int fec_encode_batch_rs_dev(FECEncoderCtx* ctx, const uint8_t* d_data, uint64_t num_groups,
                            uint32_t k, uint32_t r, uint32_t packet_size, uint8_t* d_parity,
                            void* stream);

/* d_status (nullable) as status_out above, written on the device. */
int fec_decode_batch_rs_dev(FECEncoderCtx* ctx, uint8_t* d_data, const uint8_t* d_parity,
                            const uint64_t* d_erasure_masks, uint64_t num_groups, uint32_t k,
                            uint32_t r, uint32_t packet_size, uint8_t* d_status, void* stream);

/* Recover: decode without touching d_data.  The rebuilt data shards of group g go to
 * d_rebuilt + (g*r + m)*P, m = 0..e-1 over the group's lost data shards in ascending shard
 * order -- the reference decoder hands recovered packets back as separate buffers
 * (decoder.go:16-22 Recovered{PacketID, Data}, the list built at :195-207), and a device-resident receiver
 * consumes them the same way.  d_rebuilt holds num_groups*r*P bytes; slots m >= e of a
 * group, and all slots of an unrecoverable group, are left unwritten.  Writing the rebuilt
 * packets back to back (the write pattern of encode's parity rows) instead of scattered
 * among the data shards measured 2.32 vs 2.47 ms at k=10 r=3, 2 erasures, 1M groups. */
int fec_recover_batch_rs_dev(FECEncoderCtx* ctx, const uint8_t* d_data, const uint8_t* d_parity,
                             const uint64_t* d_erasure_masks, uint64_t num_groups, uint32_t k, uint32_t r,
                             uint32_t packet_size, uint8_t* d_rebuilt, uint8_t* d_status, void* stream);

/* Build (and upload) the decode codebook for (k, r) ahead of the first decode.  The
 * codebook holds the recovery tables of every recoverable erasure pattern; its size is
 * returned in *bytes_out (nullable).  When it would exceed the 2 GiB cap (e.g. k=16 r=16)
 * decode instead builds records for the patterns present in each call ("sparse plan":
 * masks are read back to the host and the call completes synchronously); *bytes_out is
 * then 0.  FEC_ERR_RANGE if k + r > 64. */
int fec_decode_prepare(FECEncoderCtx* ctx, uint32_t k, uint32_t r, uint64_t* bytes_out);

/* The same recovery with the rebuilt packets of all groups back to back ("packed"), the
 * shape of decoder.go's Recovered list (:29-34): group g's m-th lost data shard (ascending
 * shard id) at d_rebuilt + (d_row_start[g] + m) * packet_size, where d_row_start[g] (u32, one
 * per group, written by the call) is the number of rows rebuilt for groups 0..g-1;
 * unrecoverable groups and groups without lost data rebuild none.  *d_total (nullable, device)
 * = all rows.  d_rebuilt holds at most num_groups * r rows.  No gaps between groups' rows:
 * the stores stream like encode's parity (C5-style sparse loss: 15% faster than the slot
 * layout in the probe, profiles/r02_probe_recover_write_layout.txt).  Mask-addressed shapes
 * only (k + r with an inline-classify form, r <= 3, 256 < P <= 2048); others return
 * FEC_ERR_RANGE.  Asynchronous on `stream` like the call above. */
int fec_recover_batch_rs_dev_packed(FECEncoderCtx* ctx, const uint8_t* d_data, const uint8_t* d_parity,
                                    const uint64_t* d_masks, uint64_t num_groups, uint32_t k, uint32_t r,
                                    uint32_t packet_size, uint8_t* d_rebuilt, uint32_t* d_row_start,
                                    uint64_t* d_total, uint8_t* d_status, void* stream);

/* Expected share (0..1) of groups that lost data shards in this context's device-resident
 * decode calls, e.g. 1 - (1 - p)^k for iid loss p (the receiver knows its network profile;
 * satellite p = 0.01, k = 10: ~0.10).  Below 0.25 the decode checks several groups per
 * wave instead of dispatching one wave per group, which saves the waves that would find
 * nothing to do; results are identical either way.  share < 0 or > 1: unknown (default,
 * treated as dense loss).  The host-pointer calls measure the share from the masks. */
int fec_decode_loss_hint(FECEncoderCtx* ctx, double share);

/* ---- utilities for benchmarks and tests ---- */
/* Fill d_dst with the counter-based splitmix64 stream (byte i of the stream at
 * byte_offset + i), asynchronously on stream. */
int fec_fill_random_dev(FECEncoderCtx* ctx, uint8_t* d_dst, uint64_t nbytes, uint64_t seed,
                        uint64_t byte_offset, void* stream);

/* d_dst <- d_src with the engine's own 16-B-per-lane access pattern, asynchronously on
 * stream: the HBM copy rate a box achieves, which the benchmark reports the FEC kernels
 * against.  nbytes and both addresses must be multiples of 16 (else FEC_ERR_RANGE). */
int fec_copy_dev(FECEncoderCtx* ctx, const uint8_t* d_src, uint8_t* d_dst, uint64_t nbytes, void* stream);

/* Wait for the context's own stream. */
int fec_synchronize(FECEncoderCtx* ctx);

/* ---- device groups: one host batch sharded over several GPUs ----
 * Groups are independent: shard i of n takes groups [G*i/n, G*(i+1)/n) on its own
 * context (device, streams, staging buffers) from its own host thread; no data moves
 * between devices.  Host buffers only (page-locked ones from
 * fec_alloc_slab stream at DMA rate); a device buffer gives FEC_ERR_RANGE.  Return codes
 * as the single-context calls; on failure fec_hip_last_error() names the shard. */
typedef struct FECDeviceGroup FECDeviceGroup;

/* devices: ordinals to use (repeats allowed), or NULL / ndevices <= 0 for every visible
 * device.  NULL when no GPU is usable or an ordinal is out of range. */
FECDeviceGroup* fec_group_new(const int* devices, int ndevices);
void fec_group_free(FECDeviceGroup* group);
int fec_group_size(const FECDeviceGroup* group);
/* Context of shard i (for device-resident work on that GPU), NULL if out of range. */
FECEncoderCtx* fec_group_context(FECDeviceGroup* group, int i);

int fec_group_encode_batch_rs(FECDeviceGroup* group, const uint8_t* data, uint64_t num_groups,
                              uint32_t k, uint32_t r, uint32_t packet_size, uint8_t* parity_out);

int fec_group_decode_batch_rs(FECDeviceGroup* group, uint8_t* data, const uint8_t* parity,
                              const uint64_t* erasure_masks, uint64_t num_groups, uint32_t k,
                              uint32_t r, uint32_t packet_size, uint8_t* status_out,
                              uint64_t* unrecoverable_out);

/* ---- batcher: one process-wide batch for the groups of many streams ----
 * The reference encodes one group per call (encoder_hybrid.go:115, one HybridFECEncoder per
 * QUIC stream, client.go:783).  A batcher collects finished groups from every stream of the
 * process and encodes them in one launch when max_groups are pending OR deadline_us have
 * passed since the oldest pending group arrived (deadline_us = 0: as soon as the flusher is
 * free; groups arriving meanwhile share the next launch).  A repair therefore waits at most
 * deadline_us plus one encode.  Groups are k slots of slot_bytes (shorter packets
 * zero-padded, a group of count < k packets has zero slots count..k-1, as encoder.go:133-143
 * XORs only the packets present); each group's r repair payloads are as long as its longest
 * packet (the reference's repair length, encoder_hybrid.go:91-98).  Memory: `slabs` (>= 2)
 * page-locked slabs of max_groups groups; submitters wait while every slab is in use.
 * Thread-safe; one flusher thread per batcher.  NULL on failure (fec_batcher_last_error). */
typedef struct FECBatcher FECBatcher;

typedef struct {
  uint64_t groups;            /* groups encoded                                    */
  uint64_t batches;           /* launches                                          */
  uint64_t full_flushes;      /* batches closed because max_groups were pending    */
  uint64_t deadline_flushes;  /* batches closed by the deadline (or fec_batcher_flush) */
  uint64_t max_batch;         /* largest batch                                     */
  uint64_t expired;           /* results dropped uncollected (see fec_batcher_wait) */
} FECBatcherStats;

FECBatcher* fec_batcher_new(int device, uint32_t k, uint32_t r, uint32_t slot_bytes, uint32_t max_groups,
                            uint32_t deadline_us, uint32_t slabs);
/* Encodes what is pending, then frees.  No call may be in flight on the batcher. */
void fec_batcher_free(FECBatcher* b);

/* One group: `count` (1..k) packets back to back in `packed`, packet j `lens[j]` bytes
 * (<= slot_bytes; not all empty).  Returns the group's ticket (>= 0) or a negative code. */
int64_t fec_batcher_submit(FECBatcher* b, const uint8_t* packed, const uint32_t* lens, uint32_t count);

/* The same with the packets where they are (packet j at packets[j]): one copy fewer for
 * C / C++ callers (cgo may not pass Go memory that holds Go pointers, so Go packs). */
int64_t fec_batcher_submit_packets(FECBatcher* b, const uint8_t* const* packets, const uint32_t* lens,
                                   uint32_t count);

/* Waits for a ticket's batch (timeout_us < 0: no limit; 0: poll) and copies its r repair
 * payloads to out (row i at out + i*out_stride; NULL: discard).  Returns the payload length,
 * FEC_ERR_AGAIN on timeout (the ticket stays valid), or another negative code.  Each ticket
 * can be collected once; the payloads are copied straight from the batcher's page-locked
 * parity ring.  A result not collected before 2 * slabs * max_groups newer groups are encoded
 * may be dropped (FEC_ERR_RANGE).  Polling (timeout 0) a ticket never issued returns
 * FEC_ERR_AGAIN; a blocking wait on it returns FEC_ERR_RANGE. */
int fec_batcher_wait(FECBatcher* b, int64_t ticket, uint8_t* out, uint32_t out_stride, int64_t timeout_us);

/* ---- decoder batcher: the receiving side's FECDecoder rebuilds one group per call
 * (decoder.go:216-287); a decoder batcher shares launches across every connection the same
 * way.  k + r <= 64.  A connection submits a group's k + r shards (data shards, then parity
 * rows 0..r-1; NULL = lost), each `len` <= slot_bytes bytes (the group's symbol length,
 * shorter packets zero-padded as decoder.go:62-69 does), and gets a ticket.  The batch runs
 * fec_recover_batch_rs_dev.  fec_batcher_flush / _stats / _free / _last_error apply. */
FECBatcher* fec_batcher_new_decoder(int device, uint32_t k, uint32_t r, uint32_t slot_bytes, uint32_t max_groups,
                                    uint32_t deadline_us, uint32_t slabs);
int64_t fec_batcher_submit_shards(FECBatcher* b, const uint8_t* const* shards, uint32_t len);

/* Waits as fec_batcher_wait and copies the group's rebuilt data shards, in ascending shard
 * order, to out (row i at out + i*out_stride, `len` bytes each); *lost_mask (nullable) = the
 * submitted erasure mask.  Returns the number of rows (0: nothing was lost),
 * FEC_ERR_UNRECOVERABLE when more shards were lost than parity rows survive, FEC_ERR_AGAIN,
 * or another negative code. */
int fec_batcher_wait_rebuilt(FECBatcher* b, int64_t ticket, uint8_t* out, uint32_t out_stride, uint64_t* lost_mask,
                             int64_t timeout_us);

/* Several GPUs behind one handle (SURVEY.md §8(e) for the host-resident path): one batcher
 * per listed device (ordinals, repeats allowed; NULL / ndevices <= 0: every visible device),
 * each with its own context, slabs, output ring and flusher thread.  A host-resident batch is
 * bound by its GPU's PCIe link, so N devices give N links.  Groups are dealt round robin,
 * passing over a device whose slabs are all busy while another has room; tickets stay unique
 * (device i of n hands out its ticket t as t * n + i) and every fec_batcher_* call above takes
 * the handle.  Stats sum over the devices (max_batch: the largest).  With one device this is
 * fec_batcher_new / fec_batcher_new_decoder.  NULL on failure (fec_batcher_last_error names
 * the device). */
FECBatcher* fec_batcher_new_multi(const int* devices, int ndevices, uint32_t k, uint32_t r, uint32_t slot_bytes,
                                  uint32_t max_groups, uint32_t deadline_us, uint32_t slabs);
FECBatcher* fec_batcher_new_decoder_multi(const int* devices, int ndevices, uint32_t k, uint32_t r,
                                          uint32_t slot_bytes, uint32_t max_groups, uint32_t deadline_us,
                                          uint32_t slabs);
/* Devices behind a batcher handle (1 for fec_batcher_new / _new_decoder). */
int fec_batcher_devices(const FECBatcher* b);

/* Closes the pending batch now (e.g. at the end of a stream) instead of at its deadline. */
int fec_batcher_flush(FECBatcher* b);

int fec_batcher_stats(FECBatcher* b, FECBatcherStats* out);

/* Message of the calling thread's last failing fec_batcher_* call. */
const char* fec_batcher_last_error(void);

/* ---- legacy-call coalescing (fec_coalesce.cpp) ----
 * Calls from page-locked slabs (fec_alloc_slab, as the Go wrapper packs them) of 1..8 groups
 * go to a resident encoder instead: one workgroup per device that stays launched while calls
 * keep coming and serves a ring of submission slots, so a call costs no kernel launch
 * (QUICFEC_RESIDENT=0 turns it off).  On a large-BAR device the ring is in device memory the
 * host writes directly (QUICFEC_RESIDENT_VRAM=0: page-locked host memory), and calls of at most
 * 4 groups with packet_size <= 1536 and a multiple of 4 have their packets copied into their
 * slot -- from any host memory, pageable slabs included.  The rest:
 * The reference's unchanged call site encodes one group per fec_encode_batch call, each stream
 * on its own context (encoder_hybrid.go:115 via fec_cgo.go:138, client.go:783).  Host-resident
 * legacy calls of at most QUICFEC_COALESCE_MAX_GROUPS groups (default 64) are joined, across
 * every context of the process, into shared launches on their device: a caller records its
 * packets' addresses (page-locked slabs are read in place, pageable ones copied to page-locked
 * staging), the first caller to find no launch slot busy closes the batch and launches it
 * (group commit: no flusher thread, so a lone caller pays no hand-off), and every caller gets
 * its own repair rows back with the legacy return codes (fec_xor_simd.cpp:556-594).
 * QUICFEC_COALESCE=0 turns it off (one launch and synchronize per call on the caller's context). */
typedef struct {
  uint64_t calls;      /* legacy calls that went through the coalescer */
  uint64_t groups;     /* their groups */
  uint64_t batches;    /* launches */
  uint64_t max_batch;  /* groups in the largest launch */
  uint64_t max_calls;  /* calls in the largest launch */
  uint64_t close_ns;   /* sums over launches: leader waiting for the batch's address writes, */
  uint64_t launch_ns;  /*   the launch calls, */
  uint64_t done_ns;    /*   and launch until the leader saw the batch complete */
  uint64_t resident_calls;     /* legacy calls served by the resident encoder instead */
  uint64_t resident_launches;  /* instances of the resident encoder launched */
  uint64_t resident_pre_ns;    /* sums over resident calls: entry until the slot was published, */
  uint64_t resident_wait_ns;   /*   published until its done word was seen, */
  uint64_t resident_post_ns;   /*   and from there to the return */
  uint64_t resident_inline;    /* resident calls whose packets the host copied into the slot */
  uint64_t resident_vram;      /* devices whose resident ring is in device memory (not reset) */
  uint64_t resident_bad_slots; /* polls that found a published slot with a word not yet landed, retried (not reset) */
  uint64_t resident_scrubs;    /* slots the resident encoder zeroed at a tag-epoch boundary (not reset) */
  uint64_t resident_servers;   /* serving workgroups per resident instance (QUICFEC_RESIDENT_SERVERS), the
                                  largest over devices; 0 before any resident encoder exists (not reset) */
} FECCoalesceStats;

/* Process-wide totals over every device and packet size; reset = 1 zeroes them after the read.
 * Writes min(out_bytes, sizeof(FECCoalesceStats)) bytes: pass sizeof(*out) of the struct the
 * caller was built with, so fields a later library appends are never written past it.
 * FEC_ERR_RANGE when out_bytes is below the first published layout (15 words). */
int fec_coalesce_stats_sized(FECCoalesceStats* out, size_t out_bytes, int reset);

/* The first published form: writes the first 15 fields only (calls .. resident_vram). */
int fec_coalesce_stats(FECCoalesceStats* out, int reset);

#ifdef __cplusplus
}
#endif

#endif /* FEC_HIP_H */
