/*
 * fec_xor_simd.h — drop-in C-ABI of libfec_hip.so for the quic-test internal/fec cgo
 * wrapper.  Same eleven declarations, same argument meaning and return codes as the
 * reference header internal/fec/fec_xor_simd.h; every function here executes its
 * arithmetic on an MI355X (gfx950) through HIP kernels.  There is no CPU compute path.
 *
 * Differences a maintainer must know (DESIGN.md §2 has the full list):
 *   - all symbols have default visibility (the reference's -fvisibility=hidden build,
 *     internal/fec/Makefile:30, exports none of them);
 *   - fec_encoder_new returns NULL when no usable GPU exists, so the Go hybrid encoder
 *     falls back to its pure-Go path (encoder_hybrid.go:44-52);
 *   - fec_encode_batch returns distinct negative codes for HIP failures (fec_hip.h);
 *   - repair offsets are computed in 64 bits (the reference multiplies two uint32_t,
 *     fec_xor_simd.cpp:589, which wraps above 4 GiB of repair output);
 *   - the ISA-suffixed xor_packets_* names are kept for ABI compatibility; in this
 *     library they all run the same GPU XOR kernel.
 */
#ifndef FEC_XOR_SIMD_H
#define FEC_XOR_SIMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Opaque context.  Reference: fec_xor_simd.h:14, struct at fec_xor_simd.cpp:532-536.
 * Here it also owns a HIP stream, device buffers and per-(k,r) plans. */
typedef struct FECEncoderCtx FECEncoderCtx;

/* Reference fec_xor_simd.h:22 / fec_xor_simd.cpp:538-544.  redundancy outside (0,1]
 * becomes 0.10, max_groups 0 becomes 1024.  Binds the calling thread's current HIP
 * device.  Returns NULL if no GPU is usable (HIP error text: fec_hip_last_error()). */
FECEncoderCtx* fec_encoder_new(double redundancy, uint32_t max_groups);

/* Reference fec_xor_simd.h:29 / .cpp:469-484: 64-byte aligned, size rounded up to 64.
 * Here: page-locked (pinned) host memory, so H2D/D2H copies run at DMA rate. */
void* fec_alloc_slab(size_t size);

/* Reference fec_xor_simd.h:37 / .cpp:486-510.  numa_node >= 0: page-aligned anonymous
 * memory bound to that node with mbind(MPOL_BIND, MPOL_MF_MOVE) -- best effort, as in the
 * reference -- then page-locked with hipHostRegister (so the pages fault in on the node);
 * without a usable GPU it stays pageable, which is what the reference returns.
 * numa_node < 0: fec_alloc_slab.  Free with fec_free_slab. */
void* fec_alloc_slab_numa(size_t size, int numa_node);

/* Reference fec_xor_simd.h:44 / .cpp:512-514: same allocator as fec_alloc_slab. */
void* fec_alloc_repair_buffer(size_t size);

/* Reference fec_xor_simd.h:50 / .cpp:516-518.  NULL is a no-op. */
void fec_free_repair_buffer(void* ptr);

/* Reference fec_xor_simd.h:68-75 / .cpp:556-594.
 * For g < num_groups: repair_out[g*packet_size + i] = XOR over p < 10 of
 * slab[offsets[g*10 + p] + i], i < packet_size.  Exactly ten packets per group
 * (fec_xor_simd.cpp:580).  Returns -1 if ctx, slab, offsets or repair_out is NULL,
 * 0 on success or when num_groups == 0 or packet_size == 0, and a negative FEC_ERR_*
 * code (fec_hip.h) if the GPU fails.  Host or device pointers are accepted. */
int fec_encode_batch(FECEncoderCtx* ctx, const uint8_t* slab, const uint32_t* offsets,
                     uint32_t num_groups, uint32_t packet_size, uint8_t* repair_out);

/* Reference fec_xor_simd.h:81 / .cpp:546-550.  NULL is a no-op. */
void fec_encoder_free(FECEncoderCtx* ctx);

/* Reference fec_xor_simd.h:87 / .cpp:520-526.  NULL is a no-op. */
void fec_free_slab(void* ptr);

/* Reference fec_xor_simd.h:94-99. */
typedef void (*xor_impl_fn)(const uint8_t* packets[], size_t num_packets, size_t packet_size,
                            uint8_t* repair);

/* Reference fec_xor_simd.h:104 / .cpp:435-463.  Returns the GPU XOR entry point. */
xor_impl_fn fec_select_xor_impl(void);

/* Reference fec_xor_simd.h:107-137 / .cpp:74-427.  repair[i] = XOR of packets[p][i] for
 * p < num_packets, i < packet_size; nothing is written when num_packets or packet_size
 * is 0.  Runs on the GPU of a process-wide default context; on GPU failure repair is
 * left unwritten and fec_hip_last_error() says why. */
void xor_packets_scalar(const uint8_t* packets[], size_t num_packets, size_t packet_size,
                        uint8_t* repair);
void xor_packets_avx2(const uint8_t* packets[], size_t num_packets, size_t packet_size,
                      uint8_t* repair);
void xor_packets_avx512(const uint8_t* packets[], size_t num_packets, size_t packet_size,
                        uint8_t* repair);
void xor_packets_neon(const uint8_t* packets[], size_t num_packets, size_t packet_size,
                      uint8_t* repair);

#ifdef __cplusplus
}
#endif

#endif /* FEC_XOR_SIMD_H */
