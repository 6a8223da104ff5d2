// fec_internal.hpp — what the C-ABI shim (fec_shim.cpp) lends the legacy-call coalescer
// (fec_coalesce.cpp).  Internal to libfec_hip.so (hidden visibility).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "fec_hip.h"

namespace qfec {

enum class HostMem { kPageable, kPinned, kDevice };

// Where `p` lives; for page-locked host memory *dev = the address kernels use for it.
HostMem classify_host_pointer(const void* p, void** dev);

// Row 0 .. r-1 of G groups of k packets at absolute device addresses d_addr[g * k + j] (row 0
// = XOR), parity row (g, i) at d_parity + (g * r + i) * P; queued on `s`, which belongs to
// the context's device.  Locks the context and binds its device.
int encode_addr_batch(FECEncoderCtx* ctx, const uint64_t* d_addr, uint64_t G, uint32_t k, uint32_t r, uint32_t P,
                      uint8_t* d_parity, hipStream_t s);

// The calling thread's fec_hip_last_error text.
void set_last_error(const char* msg);

// The legacy fec_encode_batch call (10 packets per group at slab + offsets[i], packet_size
// bytes each, repair row g at repair_out + g * packet_size) joined into a shared launch on
// `device`.  Returns false when the call is not one the coalescer takes (device-resident
// buffers, too large, switched off); else true with the call's return code in *rc.  stream: the
// caller's context stream (a shared launch led by this caller goes there).
bool coalesce_legacy_encode(int device, const uint8_t* slab, const uint32_t* offsets, uint32_t num_groups,
                            uint32_t packet_size, uint8_t* repair_out, int* rc, hipStream_t stream);

// Sets up the resident encoder's page-locked ring for `device` ahead of the first legacy call
// (no kernel launch; that happens on the first call).
void coalesce_prepare(int device);

}  // namespace qfec
