//go:build cgo && fec_hip

// Batch GF(2^8) erasure coding on the GPU (include/fec_hip.h).  New API next to the
// reference's FECEncoderCXX (fec_cgo.go:25-247), which keeps working unchanged on top of
// the same library (its fec_encode_batch call, fec_cgo.go:138, now runs on the GPU).
//
// Status: written against the C-ABI in include/; not compiled here (no Go toolchain in
// the build image).  The same calls are exercised from Python (quicfec) and C++
// (quic-test_amd/host) by the test suite.

package fec

/*
#include <stdint.h>
#include <stdlib.h>
#include "fec_hip.h"
*/
import "C"

import (
	"fmt"
	"runtime"
	"sync"
	"unsafe"
)

// RSCodec encodes k data packets into r parity packets per group and rebuilds up to r
// lost packets, for whole batches of groups per call.  Parity row 0 is the XOR repair
// packet of FECEncoder/FECEncoderCXX byte for byte.
type RSCodec struct {
	ctx *C.FECEncoderCtx
	k   int
	r   int
	mu  sync.Mutex
}

// ctxError reads the failing call's message from the context itself (fec_ctx_last_error):
// the goroutine may have moved to another OS thread since the call, so the thread-local
// fec_hip_last_error could be empty or another call's.  The reference wrapper reports the
// code alone (fec_cgo.go:147-149).
func ctxError(ctx *C.FECEncoderCtx, what string, code C.int) error {
	var buf [512]C.char
	C.fec_ctx_last_error(ctx, &buf[0], C.size_t(len(buf)))
	return fmt.Errorf("%s failed with code %d: %s", what, int(code), C.GoString(&buf[0]))
}

// lockedError runs a call whose failure text is thread-local (fec_group_*, fec_batcher_*,
// context creation) with the goroutine pinned to its OS thread, so the text read after it
// is this call's.
func lockedError(call func() C.int, what string, lastError func() *C.char) error {
	runtime.LockOSThread()
	defer runtime.UnlockOSThread()
	if rc := call(); rc != 0 {
		return fmt.Errorf("%s failed with code %d: %s", what, int(rc), C.GoString(lastError()))
	}
	return nil
}

func hipLastError() *C.char { return C.fec_hip_last_error() }

// NewRSCodec binds a codec to GPU `device` (use -1 for the current HIP device).
func NewRSCodec(k, r, device int) (*RSCodec, error) {
	if k <= 0 || r <= 0 || k+r > 256 {
		return nil, fmt.Errorf("unsupported k=%d r=%d", k, r)
	}
	runtime.LockOSThread() // the creation error is thread-local
	defer runtime.UnlockOSThread()
	var ctx *C.FECEncoderCtx
	if device < 0 {
		ctx = C.fec_encoder_new(C.double(float64(r)/float64(k)), 1024)
	} else {
		ctx = C.fec_encoder_new_device(C.double(float64(r)/float64(k)), 1024, C.int(device))
	}
	if ctx == nil {
		return nil, fmt.Errorf("no usable GPU: %s", C.GoString(C.fec_hip_last_error()))
	}
	c := &RSCodec{ctx: ctx, k: k, r: r}
	runtime.SetFinalizer(c, (*RSCodec).Close)
	return c, nil
}

// EncodeBatch: data holds groups*k packets of packetSize bytes (packet (g,j) at
// (g*k+j)*packetSize); parity receives groups*r packets (row (g,i) at (g*r+i)*packetSize).
func (c *RSCodec) EncodeBatch(data []byte, packetSize int, parity []byte) error {
	if packetSize <= 0 || len(data)%(c.k*packetSize) != 0 {
		return fmt.Errorf("data length %d is not a whole number of %dx%d groups", len(data), c.k, packetSize)
	}
	groups := len(data) / (c.k * packetSize)
	if len(parity) < groups*c.r*packetSize {
		return fmt.Errorf("parity buffer too small")
	}
	if groups == 0 {
		return nil
	}
	c.mu.Lock()
	defer c.mu.Unlock()
	rc := C.fec_encode_batch_rs(c.ctx, (*C.uint8_t)(unsafe.Pointer(&data[0])), nil, C.uint64_t(groups),
		C.uint32_t(c.k), C.uint32_t(c.r), C.uint32_t(packetSize), (*C.uint8_t)(unsafe.Pointer(&parity[0])))
	runtime.KeepAlive(data)
	runtime.KeepAlive(parity)
	if rc != 0 {
		return ctxError(c.ctx, "fec_encode_batch_rs", rc)
	}
	return nil
}

// DecodeBatch rebuilds lost data packets in place.  erasures[g] bit s set means shard s
// of group g was lost (s < k data packet s, s >= k parity row s-k).  status[g] (optional,
// len >= groups) is 0 when the group is complete afterwards, 1 when it had more losses
// than surviving parity rows.  Returns the number of unrecoverable groups.
func (c *RSCodec) DecodeBatch(data, parity []byte, erasures []uint64, packetSize int, status []byte) (int, error) {
	if c.k+c.r > 64 { // one erasure bit per shard (include/fec_hip.h)
		return 0, fmt.Errorf("decode needs k+r <= 64 (k=%d r=%d)", c.k, c.r)
	}
	groups := len(erasures)
	if packetSize <= 0 || len(data) < groups*c.k*packetSize || len(parity) < groups*c.r*packetSize {
		return 0, fmt.Errorf("buffers too small for %d groups", groups)
	}
	if status != nil && len(status) < groups {
		return 0, fmt.Errorf("status buffer too small")
	}
	if groups == 0 {
		return 0, nil
	}
	c.mu.Lock()
	defer c.mu.Unlock()
	var st *C.uint8_t
	if status != nil {
		st = (*C.uint8_t)(unsafe.Pointer(&status[0]))
	}
	var bad C.uint64_t
	rc := C.fec_decode_batch_rs(c.ctx, (*C.uint8_t)(unsafe.Pointer(&data[0])), (*C.uint8_t)(unsafe.Pointer(&parity[0])),
		(*C.uint64_t)(unsafe.Pointer(&erasures[0])), C.uint64_t(groups), C.uint32_t(c.k), C.uint32_t(c.r),
		C.uint32_t(packetSize), st, &bad)
	runtime.KeepAlive(data)
	runtime.KeepAlive(parity)
	runtime.KeepAlive(erasures)
	runtime.KeepAlive(status)
	if rc != 0 {
		return 0, ctxError(c.ctx, "fec_decode_batch_rs", rc)
	}
	return int(bad), nil
}

// Close releases the GPU context.
func (c *RSCodec) Close() error {
	c.mu.Lock()
	defer c.mu.Unlock()
	if c.ctx != nil {
		C.fec_encoder_free(c.ctx)
		c.ctx = nil
	}
	return nil
}

// RSDeviceGroup is an RSCodec over several GPUs of one node: each batch is split into
// contiguous group ranges, one per device, run concurrently by the library (one context
// and host thread per device; include/fec_hip.h fec_group_*).  Host buffers only.
type RSDeviceGroup struct {
	grp *C.FECDeviceGroup
	k   int
	r   int
	mu  sync.Mutex
}

// NewRSDeviceGroup binds a group to the given device ordinals (nil: every visible GPU).
func NewRSDeviceGroup(k, r int, devices []int) (*RSDeviceGroup, error) {
	if k <= 0 || r <= 0 || k+r > 256 {
		return nil, fmt.Errorf("unsupported k=%d r=%d", k, r)
	}
	runtime.LockOSThread() // the creation error is thread-local
	defer runtime.UnlockOSThread()
	var grp *C.FECDeviceGroup
	if len(devices) == 0 {
		grp = C.fec_group_new(nil, 0)
	} else {
		ids := make([]C.int, len(devices))
		for i, d := range devices {
			ids[i] = C.int(d)
		}
		grp = C.fec_group_new(&ids[0], C.int(len(ids)))
	}
	if grp == nil {
		return nil, fmt.Errorf("no usable GPU group: %s", C.GoString(C.fec_hip_last_error()))
	}
	g := &RSDeviceGroup{grp: grp, k: k, r: r}
	runtime.SetFinalizer(g, (*RSDeviceGroup).Close)
	return g, nil
}

// Devices is the number of shards (devices, repeats counted).
func (g *RSDeviceGroup) Devices() int { return int(C.fec_group_size(g.grp)) }

// EncodeBatch: as RSCodec.EncodeBatch, sharded over the group's devices.
func (g *RSDeviceGroup) EncodeBatch(data []byte, packetSize int, parity []byte) error {
	if packetSize <= 0 || len(data)%(g.k*packetSize) != 0 {
		return fmt.Errorf("data length %d is not a whole number of %dx%d groups", len(data), g.k, packetSize)
	}
	groups := len(data) / (g.k * packetSize)
	if len(parity) < groups*g.r*packetSize {
		return fmt.Errorf("parity buffer too small")
	}
	if groups == 0 {
		return nil
	}
	g.mu.Lock()
	defer g.mu.Unlock()
	err := lockedError(func() C.int {
		return C.fec_group_encode_batch_rs(g.grp, (*C.uint8_t)(unsafe.Pointer(&data[0])), C.uint64_t(groups),
			C.uint32_t(g.k), C.uint32_t(g.r), C.uint32_t(packetSize), (*C.uint8_t)(unsafe.Pointer(&parity[0])))
	}, "fec_group_encode_batch_rs", hipLastError)
	runtime.KeepAlive(data)
	runtime.KeepAlive(parity)
	return err
}

// DecodeBatch: as RSCodec.DecodeBatch, sharded over the group's devices.
func (g *RSDeviceGroup) DecodeBatch(data, parity []byte, erasures []uint64, packetSize int, status []byte) (int, error) {
	if g.k+g.r > 64 {
		return 0, fmt.Errorf("decode needs k+r <= 64 (k=%d r=%d)", g.k, g.r)
	}
	groups := len(erasures)
	if packetSize <= 0 || len(data) < groups*g.k*packetSize || len(parity) < groups*g.r*packetSize {
		return 0, fmt.Errorf("buffers too small for %d groups", groups)
	}
	if status != nil && len(status) < groups {
		return 0, fmt.Errorf("status buffer too small")
	}
	if groups == 0 {
		return 0, nil
	}
	g.mu.Lock()
	defer g.mu.Unlock()
	var st *C.uint8_t
	if status != nil {
		st = (*C.uint8_t)(unsafe.Pointer(&status[0]))
	}
	var bad C.uint64_t
	err := lockedError(func() C.int {
		return C.fec_group_decode_batch_rs(g.grp, (*C.uint8_t)(unsafe.Pointer(&data[0])), (*C.uint8_t)(unsafe.Pointer(&parity[0])),
			(*C.uint64_t)(unsafe.Pointer(&erasures[0])), C.uint64_t(groups), C.uint32_t(g.k), C.uint32_t(g.r),
			C.uint32_t(packetSize), st, &bad)
	}, "fec_group_decode_batch_rs", hipLastError)
	runtime.KeepAlive(data)
	runtime.KeepAlive(parity)
	runtime.KeepAlive(erasures)
	runtime.KeepAlive(status)
	if err != nil {
		return 0, err
	}
	return int(bad), nil
}

// Close releases every device context of the group.
func (g *RSDeviceGroup) Close() error {
	g.mu.Lock()
	defer g.mu.Unlock()
	if g.grp != nil {
		C.fec_group_free(g.grp)
		g.grp = nil
	}
	return nil
}
