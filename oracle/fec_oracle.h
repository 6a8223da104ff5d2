/*
 * fec_oracle.h — CPU restatement of the reference FEC hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (quic-test_amd/, include/)
 * links, loads or calls this code.  It is used by tests/ (as the checker),
 * by __graft_entry__.smoke() (as the checker) and by bench.py's cpu_baseline
 * leg (as the timed CPU comparator).
 *
 * What it restates (reference = twogc/quic-test @ 2025-12-12):
 *   - xor_packets_scalar      internal/fec/fec_xor_simd.cpp:411-427
 *   - xor_packets_avx2        internal/fec/fec_xor_simd.cpp:74-204
 *   - fec_encode_batch        internal/fec/fec_xor_simd.cpp:556-594 (k fixed to 10 at :580)
 *   - FECEncoder.generateRedundancy  internal/fec/encoder.go:113-163 (zero-pad XOR + 11-B header)
 *   - FECDecoder.recoverSingle       internal/fec/decoder.go:255-287 (+ padTo :62-69)
 *   - GF(2^8) systematic Cauchy code for parity rows 1..r-1 and multi-erasure
 *     decode: NEW (the reference is XOR-only, SURVEY.md §0.1, §8(a) "code
 *     definition").  Row 0 of the code is the reference XOR by construction.
 *
 * Parity pinning:
 *   - XOR row 0 / single-erasure XOR decode: pinned against the reference C++
 *     compiled from /root/reference (oracle/_ref; the tests/golden npz fixtures, generated
 *     by tests/golden/make_golden.py).
 *   - GF rows 1..r-1 and 2..r erasure decode: the reference has no such code, so
 *     these are "parity unpinned by the reference"; they are pinned by the
 *     committed matrix fixture (tests/golden/parity_matrices.json), the
 *     committed GF fixtures made by this restatement, and the MDS round-trip
 *     property (encode -> erase <= r -> decode == original).
 */
#ifndef FEC_ORACLE_H
#define FEC_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- synthetic data (counter-based splitmix64; identical on the device) ---- */
/* byte i of the stream = little-endian byte (i % 8) of mix(seed + (i/8 + 1) * 0x9E3779B97F4A7C15) */
void oracle_fill_splitmix(uint8_t* dst, uint64_t nbytes, uint64_t seed, uint64_t byte_offset);

/* ---- XOR (parity row 0) ---- */
void oracle_xor_scalar(const uint8_t* const* pkts, size_t n, size_t packet_size, uint8_t* out);
void oracle_xor_avx2(const uint8_t* const* pkts, size_t n, size_t packet_size, uint8_t* out);

/* fec_encode_batch semantics: 10 packets per group gathered through u32 offsets.
 * Returns -1 when slab/offsets/repair is NULL, 0 otherwise (also for 0 groups / 0 size). */
int oracle_encode_batch_legacy(const uint8_t* slab, const uint32_t* offsets, uint32_t num_groups,
                               uint32_t packet_size, uint8_t* repair_out, int use_avx2);

/* Contiguous XOR encode of G groups of k packets (packet (g,j) at (g*k+j)*P), AVX2, threaded. */
void oracle_xor_encode_contig(const uint8_t* data, uint64_t G, uint32_t k, uint32_t P,
                              uint8_t* repair, int nthreads);

/* Calls xor_fn (an xor_packets_* of the reference's signature, fec_xor_simd.h:22-24) once per
 * group over the G groups of k contiguous packets -- the C1 leg's driver, so the reference's
 * own AVX2 function is timed without a foreign-call cost per group. */
typedef void (*oracle_xor_fn)(const uint8_t* const* pkts, size_t n, size_t packet_size, uint8_t* out);
void oracle_xor_groups(oracle_xor_fn xor_fn, const uint8_t* data, uint64_t G, uint32_t k, uint32_t P,
                       uint8_t* repair);

/* ---- GF(2^8), polynomial 0x11D, generator 2 ---- */
uint8_t oracle_gf_mul(uint8_t a, uint8_t b);
uint8_t oracle_gf_inv(uint8_t a);        /* a != 0 */

/* r x k parity matrix, row-major.  Returns 0, or -1 if k==0, r==0 or k+r > 256. */
int oracle_parity_matrix(uint32_t k, uint32_t r, uint8_t* M);

/* parity shard (g,i) at (g*r+i)*P.  Returns 0 / -1 (bad k,r). */
int oracle_rs_encode(const uint8_t* data, uint64_t G, uint32_t k, uint32_t r, uint32_t P,
                     uint8_t* parity, int nthreads);

/* Decode in place.  erasure_masks[g] bit s (s < k+r) set => shard s of group g lost
 * (s < k: data shard s, s >= k: parity row s-k).  Survivor rule: every surviving data
 * shard plus the lowest-indexed surviving parity rows, as many as there are erased data
 * shards.  Erased data shards are rewritten in `data`; nothing else is written.
 * status[g] = 0 recovered (or nothing to do), 1 unrecoverable (data untouched).
 * Returns number of unrecoverable groups, or -1 on bad arguments (k+r > 64). */
int64_t oracle_rs_decode(uint8_t* data, const uint8_t* parity, const uint64_t* erasure_masks,
                         uint64_t G, uint32_t k, uint32_t r, uint32_t P, uint8_t* status,
                         int nthreads);

/* ---- Fast CPU comparator (bench.py cpu_baseline leg) ----
 * Same results as oracle_rs_encode / oracle_rs_decode (tests check byte equality), computed
 * the way a tuned CPU library (ISA-L style) does: multiplication by a constant is an 8x8
 * GF(2) bit matrix applied with GFNI's affine instruction (VGF2P8AFFINEQB), 64 bytes per
 * instruction with AVX-512 (32 with AVX2+GFNI), recovery rows cached per erasure pattern.
 * Falls back to the table code above when the CPU lacks GFNI or the shape exceeds
 * k <= 32, e <= 8.  oracle_fast_isa(): 2 = AVX-512+GFNI, 1 = AVX2+GFNI, 0 = tables. */
int oracle_fast_isa(void);
uint64_t oracle_gf_affine(uint8_t c);  /* the affine matrix of x -> c*x */
int oracle_rs_encode_fast(const uint8_t* data, uint64_t G, uint32_t k, uint32_t r, uint32_t P,
                          uint8_t* parity, int nthreads);
int64_t oracle_rs_decode_fast(uint8_t* data, const uint8_t* parity, const uint64_t* erasure_masks,
                              uint64_t G, uint32_t k, uint32_t r, uint32_t P, uint8_t* status,
                              int nthreads);

/* ---- Go-path semantics ---- */
/* encoder.go:113-163.  Writes 11 + maxLen bytes into out (cap checked).  Returns the
 * length, -1 for "no packets in group", -2 for "empty packets", -3 if cap too small. */
int64_t oracle_go_generate_redundancy(const uint8_t* const* pkts, const size_t* lens, size_t n,
                                      uint64_t group_id, uint8_t* out, size_t out_cap);

/* decoder.go:255-287.  `present` has packet_count flags; `pkts[i]` (lens[i]) valid when
 * present[i].  Symbols are normalised with padTo(symbol_len) as the decoder does on
 * ingestion (:62-69, :132, :197).  Writes symbol_len bytes to out; returns the recovered
 * packet id, or -1 if nothing is missing. */
int64_t oracle_go_recover_single(const uint8_t* const* pkts, const size_t* lens,
                                 const uint8_t* present, size_t packet_count,
                                 const uint8_t* parity_payload, size_t parity_len,
                                 size_t symbol_len, uint8_t* out);

#ifdef __cplusplus
}
#endif
#endif /* FEC_ORACLE_H */
