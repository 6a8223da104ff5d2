//go:build cgo && fec_hip

// One process-wide batch for the FEC groups of every QUIC stream (SURVEY.md §8(f) item 1).
//
// The reference runs one HybridFECEncoder per stream (client.go:783) and encodes one group
// per cgo call (encoder_hybrid.go:115).  On the GPU a call costs one launch (~15 us) however
// few groups it carries, so every stream's encoder here hands its finished groups to one
// SharedBatcher (fec_batcher_*, include/fec_hip.h), which encodes them together when
// maxGroups are pending or `deadline` after the oldest pending group arrived, whichever is
// first: a repair is at most deadline + one encode late.  BatchedFECEncoder keeps
// HybridFECEncoder's API and wire bytes: its row-0 repair packet is byte-identical.
//
// Same design as the C++ mirror (quic-test_amd/host/fec.hpp SharedFECBatcher /
// BatchedFECEncoder), which tests/csrc/host_mirror_test.cpp checks on MI355X.  Status:
// written against the C-ABI; not compiled here (no Go toolchain in the build image).

package fec

/*
#include <stdint.h>
#include <stdlib.h>
#include "fec_hip.h"
*/
import "C"

import (
	"errors"
	"fmt"
	"runtime"
	"sync"
	"time"
	"unsafe"
)

// SharedBatcher is shared by every stream of the process (create one per GPU).
type SharedBatcher struct {
	b       *C.FECBatcher
	k, r    int
	slot    int
	closeMu sync.RWMutex // calls hold it shared; Close takes it exclusively
}

func batcherLastError() *C.char { return C.fec_batcher_last_error() }

// ErrResultExpired: an async group's repair rows were overwritten in the batcher's ring before
// its stream collected them (2 * slabs * maxGroups newer groups were encoded meanwhile).  Poll
// returns it wrapped (errors.Is) after dropping that group.
var ErrResultExpired = errors.New("fec: batcher result expired before it was collected")

// NewSharedBatcher: groups of k packets of at most slotBytes, r repair packets per group,
// up to maxGroups per launch, flushed `deadline` after the oldest pending group (0: as soon
// as the flusher is free; groups that arrive meanwhile share the next launch).  device -1 is
// the current HIP device.
func NewSharedBatcher(k, r, slotBytes, maxGroups int, deadline time.Duration, device int) (*SharedBatcher, error) {
	if k < 1 || r < 1 || k+r > 256 || k > maxPacketCount || slotBytes < 1 || maxGroups < 1 || deadline < 0 {
		return nil, fmt.Errorf("unsupported batcher k=%d r=%d slot=%d maxGroups=%d", k, r, slotBytes, maxGroups)
	}
	runtime.LockOSThread() // the creation error is thread-local
	defer runtime.UnlockOSThread()
	b := C.fec_batcher_new(C.int(device), C.uint32_t(k), C.uint32_t(r), C.uint32_t(slotBytes), C.uint32_t(maxGroups),
		C.uint32_t(deadline/time.Microsecond), 3)
	if b == nil {
		return nil, fmt.Errorf("no usable GPU batcher: %s", C.GoString(C.fec_batcher_last_error()))
	}
	s := &SharedBatcher{b: b, k: k, r: r, slot: slotBytes}
	runtime.SetFinalizer(s, (*SharedBatcher).Close)
	return s, nil
}

// devicesArg passes a device list to the *_multi constructors (nil or empty: every visible
// GPU).  The C side copies the list during the call.
func devicesArg(devices []int) (*C.int, C.int, func()) {
	if len(devices) == 0 {
		return nil, 0, func() {}
	}
	p := (*C.int)(C.malloc(C.size_t(len(devices)) * C.size_t(unsafe.Sizeof(C.int(0)))))
	arr := unsafe.Slice(p, len(devices))
	for i, d := range devices {
		arr[i] = C.int(d)
	}
	return p, C.int(len(devices)), func() { C.free(unsafe.Pointer(p)) }
}

// NewSharedBatcherMulti: one batcher per listed GPU behind one handle (fec_batcher_new_multi;
// repeats allowed, nil = every visible GPU).  Host-resident batches are bound by their GPU's
// PCIe link, so N GPUs give N links; groups are dealt round robin and tickets stay unique.
func NewSharedBatcherMulti(k, r, slotBytes, maxGroups int, deadline time.Duration, devices []int) (*SharedBatcher, error) {
	if k < 1 || r < 1 || k+r > 256 || k > maxPacketCount || slotBytes < 1 || maxGroups < 1 || deadline < 0 {
		return nil, fmt.Errorf("unsupported batcher k=%d r=%d slot=%d maxGroups=%d", k, r, slotBytes, maxGroups)
	}
	runtime.LockOSThread() // the creation error is thread-local
	defer runtime.UnlockOSThread()
	dp, dn, free := devicesArg(devices)
	defer free()
	b := C.fec_batcher_new_multi(dp, dn, C.uint32_t(k), C.uint32_t(r), C.uint32_t(slotBytes), C.uint32_t(maxGroups),
		C.uint32_t(deadline/time.Microsecond), 3)
	if b == nil {
		return nil, fmt.Errorf("no usable GPU batcher: %s", C.GoString(C.fec_batcher_last_error()))
	}
	s := &SharedBatcher{b: b, k: k, r: r, slot: slotBytes}
	runtime.SetFinalizer(s, (*SharedBatcher).Close)
	return s, nil
}

// Flush closes the pending batch now instead of at its deadline.
func (s *SharedBatcher) Flush() {
	s.closeMu.RLock()
	defer s.closeMu.RUnlock()
	if s.b != nil {
		C.fec_batcher_flush(s.b)
	}
}

// Stats: groups, batches, full flushes, deadline flushes, largest batch, expired results.
func (s *SharedBatcher) Stats() [6]uint64 {
	s.closeMu.RLock()
	defer s.closeMu.RUnlock()
	var st C.FECBatcherStats
	if s.b != nil {
		C.fec_batcher_stats(s.b, &st)
	}
	return [6]uint64{uint64(st.groups), uint64(st.batches), uint64(st.full_flushes), uint64(st.deadline_flushes),
		uint64(st.max_batch), uint64(st.expired)}
}

// Close encodes what is pending and frees the batcher; no encoder may use it afterwards.
func (s *SharedBatcher) Close() error {
	s.closeMu.Lock()
	defer s.closeMu.Unlock()
	if s.b != nil {
		C.fec_batcher_free(s.b)
		s.b = nil
	}
	return nil
}

// submit packs a group's packets back to back (Go memory without Go pointers inside, so it
// may be passed to C for the call) and returns its ticket.
func (s *SharedBatcher) submit(packets [][]byte, packed []byte, lens []C.uint32_t) (int64, []byte, []C.uint32_t, error) {
	packed, lens = packed[:0], lens[:0]
	for _, p := range packets {
		packed = append(packed, p...)
		lens = append(lens, C.uint32_t(len(p)))
	}
	if len(packed) == 0 { // encoder_hybrid.go:95-97
		return 0, packed, lens, fmt.Errorf("empty packets")
	}
	s.closeMu.RLock()
	defer s.closeMu.RUnlock()
	if s.b == nil {
		return 0, packed, lens, fmt.Errorf("batcher closed")
	}
	runtime.LockOSThread()
	defer runtime.UnlockOSThread()
	t := C.fec_batcher_submit(s.b, (*C.uint8_t)(unsafe.Pointer(&packed[0])), &lens[0], C.uint32_t(len(lens)))
	runtime.KeepAlive(packed)
	if t < 0 {
		return 0, packed, lens, fmt.Errorf("fec_batcher_submit failed with code %d: %s", int64(t),
			C.GoString(C.fec_batcher_last_error()))
	}
	return int64(t), packed, lens, nil
}

// wait collects a ticket's r payloads into rows (r*slot bytes); returns the payload length,
// or ready == false on timeout.
func (s *SharedBatcher) wait(ticket int64, rows []byte, timeout time.Duration) (n int, ready bool, err error) {
	s.closeMu.RLock()
	defer s.closeMu.RUnlock()
	if s.b == nil {
		return 0, false, fmt.Errorf("batcher closed")
	}
	us := C.int64_t(-1)
	if timeout >= 0 {
		us = C.int64_t(timeout / time.Microsecond)
	}
	runtime.LockOSThread()
	defer runtime.UnlockOSThread()
	rc := C.fec_batcher_wait(s.b, C.int64_t(ticket), (*C.uint8_t)(unsafe.Pointer(&rows[0])), C.uint32_t(s.slot), us)
	runtime.KeepAlive(rows)
	switch {
	case rc == C.FEC_ERR_AGAIN:
		return 0, false, nil
	case rc == C.FEC_ERR_RANGE:
		// every ticket of a BatchedFECEncoder is issued and collected once: out of range = expired
		return 0, true, fmt.Errorf("%w: %s", ErrResultExpired, C.GoString(C.fec_batcher_last_error()))
	case rc < 0:
		return 0, true, fmt.Errorf("C++ encoding failed: %s", C.GoString(C.fec_batcher_last_error()))
	}
	return int(rc), true, nil
}

// BatchedFECEncoder is one stream's encoder on a SharedBatcher, with HybridFECEncoder's API.
type BatchedFECEncoder struct {
	mu          sync.Mutex
	s           *SharedBatcher
	packets     [][]byte
	groupID     uint64
	packed      []byte
	lens        []C.uint32_t
	rows        []byte
	outstanding []batchTicket
	metrics     FECMetrics
}

type batchTicket struct {
	ticket  int64
	groupID uint64
	count   int
}

// NewEncoder returns a stream encoder (groups of the batcher's k).
func (s *SharedBatcher) NewEncoder() *BatchedFECEncoder {
	return &BatchedFECEncoder{s: s, rows: make([]byte, s.r*s.slot)}
}

func (e *BatchedFECEncoder) submitLocked() (batchTicket, error) {
	var err error
	var t int64
	t, e.packed, e.lens, err = e.s.submit(e.packets, e.packed, e.lens)
	count := len(e.packets)
	e.packets = e.packets[:0] // refused groups are dropped so the stream keeps working
	if err != nil {
		return batchTicket{}, err
	}
	bt := batchTicket{ticket: t, groupID: e.groupID, count: count}
	e.groupID++
	return bt, nil
}

// collect turns a finished ticket into its r repair packets (row 0 with the reference
// header, encoder_hybrid.go:175-192; rows >= 1 with the FE C1 header).
func (e *BatchedFECEncoder) collect(t batchTicket, timeout time.Duration) ([][]byte, bool, error) {
	n, ready, err := e.s.wait(t.ticket, e.rows, timeout)
	if err != nil || !ready {
		return nil, ready, err
	}
	out := make([][]byte, e.s.r)
	for row := 0; row < e.s.r; row++ {
		out[row] = MakeRepairPacket(RepairHeader{GroupID: t.groupID, Count: t.count, Row: row, R: e.s.r, K: e.s.k},
			e.rows[row*e.s.slot:row*e.s.slot+n])
		e.metrics.RedundancyPackets++
		e.metrics.RedundancyBytes += int64(len(out[row]))
	}
	e.metrics.GroupsProcessed++
	e.metrics.PacketsEncoded += int64(e.s.k) // encoder_hybrid.go:124-127 counts the group size
	return out, true, nil
}

// AddPacket: HybridFECEncoder.AddPacket's contract (encoder_hybrid.go:59-74).  On the k-th
// packet the group is submitted and the call waits for its batch; returns (true, row-0
// repair packet, nil).  With r > 1 use AddPacketRows to get every row.
func (e *BatchedFECEncoder) AddPacket(packet []byte, packetID uint64) (bool, []byte, error) {
	rows, err := e.AddPacketRows(packet, packetID)
	if err != nil || rows == nil {
		return false, nil, err
	}
	return true, rows[0], nil
}

// AddPacketRows is AddPacket returning all r repair packets of a finished group.
func (e *BatchedFECEncoder) AddPacketRows(packet []byte, packetID uint64) ([][]byte, error) {
	e.mu.Lock()
	defer e.mu.Unlock()
	e.packets = append(e.packets, append([]byte(nil), packet...)) // copied (encoder_hybrid.go:64-65)
	if len(e.packets) < e.s.k {
		return nil, nil
	}
	t, err := e.submitLocked()
	if err != nil {
		return nil, err
	}
	rows, _, err := e.collect(t, -1)
	return rows, err
}

// AddPacketAsync submits a finished group without waiting; Poll collects repairs.
func (e *BatchedFECEncoder) AddPacketAsync(packet []byte, packetID uint64) error {
	e.mu.Lock()
	defer e.mu.Unlock()
	e.packets = append(e.packets, append([]byte(nil), packet...))
	if len(e.packets) < e.s.k {
		return nil
	}
	t, err := e.submitLocked()
	if err == nil {
		e.outstanding = append(e.outstanding, t)
	}
	return err
}

// Poll returns the repair packets of finished groups in group order (row order within a
// group), waiting up to timeout for the oldest outstanding one (0: no wait, < 0: for all).
// A group it cannot collect (its result expired in the batcher's ring, or its batch failed)
// is dropped and ends the call with that error, returned beside the rows collected before it.
func (e *BatchedFECEncoder) Poll(timeout time.Duration) ([][]byte, error) {
	e.mu.Lock()
	defer e.mu.Unlock()
	var out [][]byte
	for i := 0; len(e.outstanding) > 0; i++ {
		w := timeout
		if timeout >= 0 && i > 0 {
			w = 0
		}
		rows, ready, err := e.collect(e.outstanding[0], w)
		if err != nil {
			e.outstanding = e.outstanding[1:]
			return out, err
		}
		if !ready {
			break
		}
		out = append(out, rows...)
		e.outstanding = e.outstanding[1:]
	}
	return out, nil
}

// Flush encodes the partial group now (HybridFECEncoder.Flush): its row-0 repair packet.
func (e *BatchedFECEncoder) Flush() ([]byte, error) {
	e.mu.Lock()
	defer e.mu.Unlock()
	if len(e.packets) == 0 {
		return nil, nil
	}
	t, err := e.submitLocked()
	if err != nil {
		return nil, err
	}
	e.s.Flush()
	rows, _, err := e.collect(t, -1)
	if err != nil {
		return nil, err
	}
	return rows[0], nil
}

// GetMetrics returns a copy of the counters (encoder.go:20-26 fields).
func (e *BatchedFECEncoder) GetMetrics() FECMetrics {
	e.mu.Lock()
	defer e.mu.Unlock()
	return e.metrics
}

// SharedDecodeBatcher batches the receivers' recoveries across connections
// (fec_batcher_new_decoder): FECDecoder.recoverSingle (decoder.go:255-287) rebuilds one
// group per call; with this, every connection's single-loss rebuild of a k-packet group
// shares a launch with the others', at most `deadline` plus one launch later.
type SharedDecodeBatcher struct {
	b       *C.FECBatcher
	k, r    int
	slot    int
	closeMu sync.RWMutex
}

// NewSharedDecodeBatcher: groups of k data packets and r repair rows (k + r <= 64), symbols
// of at most slotBytes.
func NewSharedDecodeBatcher(k, r, slotBytes, maxGroups int, deadline time.Duration, device int) (*SharedDecodeBatcher, error) {
	if k < 1 || r < 1 || k+r > 64 || slotBytes < 1 || maxGroups < 1 || deadline < 0 {
		return nil, fmt.Errorf("unsupported decode batcher k=%d r=%d slot=%d maxGroups=%d", k, r, slotBytes, maxGroups)
	}
	runtime.LockOSThread() // the creation error is thread-local
	defer runtime.UnlockOSThread()
	b := C.fec_batcher_new_decoder(C.int(device), C.uint32_t(k), C.uint32_t(r), C.uint32_t(slotBytes),
		C.uint32_t(maxGroups), C.uint32_t(deadline/time.Microsecond), 3)
	if b == nil {
		return nil, fmt.Errorf("no usable GPU decode batcher: %s", C.GoString(C.fec_batcher_last_error()))
	}
	s := &SharedDecodeBatcher{b: b, k: k, r: r, slot: slotBytes}
	runtime.SetFinalizer(s, (*SharedDecodeBatcher).Close)
	return s, nil
}

// NewSharedDecodeBatcherMulti: one decoder batcher per listed GPU behind one handle
// (fec_batcher_new_decoder_multi; nil = every visible GPU).
func NewSharedDecodeBatcherMulti(k, r, slotBytes, maxGroups int, deadline time.Duration, devices []int) (*SharedDecodeBatcher, error) {
	if k < 1 || r < 1 || k+r > 64 || slotBytes < 1 || maxGroups < 1 || deadline < 0 {
		return nil, fmt.Errorf("unsupported decode batcher k=%d r=%d slot=%d maxGroups=%d", k, r, slotBytes, maxGroups)
	}
	runtime.LockOSThread() // the creation error is thread-local
	defer runtime.UnlockOSThread()
	dp, dn, free := devicesArg(devices)
	defer free()
	b := C.fec_batcher_new_decoder_multi(dp, dn, C.uint32_t(k), C.uint32_t(r), C.uint32_t(slotBytes),
		C.uint32_t(maxGroups), C.uint32_t(deadline/time.Microsecond), 3)
	if b == nil {
		return nil, fmt.Errorf("no usable GPU decode batcher: %s", C.GoString(C.fec_batcher_last_error()))
	}
	s := &SharedDecodeBatcher{b: b, k: k, r: r, slot: slotBytes}
	runtime.SetFinalizer(s, (*SharedDecodeBatcher).Close)
	return s, nil
}

// Close frees the batcher; no decoder may use it afterwards.
func (s *SharedDecodeBatcher) Close() error {
	s.closeMu.Lock()
	defer s.closeMu.Unlock()
	if s.b != nil {
		C.fec_batcher_free(s.b)
		s.b = nil
	}
	return nil
}

// Recover rebuilds the lost data shards of one group and waits for its batch.  shards holds
// the k data symbols then the r repair rows, nil for the lost ones, each symbolLen bytes
// (zero-padded as decoder.go:62-69 does).  Returns the rebuilt symbols by packet index.
func (s *SharedDecodeBatcher) Recover(shards [][]byte, symbolLen int) (map[int][]byte, error) {
	if len(shards) != s.k+s.r {
		return nil, fmt.Errorf("expected %d shards, got %d", s.k+s.r, len(shards))
	}
	if symbolLen < 1 || symbolLen > s.slot {
		return nil, fmt.Errorf("symbol length %d outside 1..%d", symbolLen, s.slot)
	}
	// the shards are copied into C memory: cgo forbids passing Go pointers inside Go memory
	buf := unsafe.Slice((*byte)(C.malloc(C.size_t(len(shards)*symbolLen))), len(shards)*symbolLen)
	defer C.free(unsafe.Pointer(&buf[0]))
	ptrs := unsafe.Slice((**C.uint8_t)(C.malloc(C.size_t(len(shards))*C.size_t(unsafe.Sizeof(uintptr(0))))), len(shards))
	defer C.free(unsafe.Pointer(&ptrs[0]))
	for j, sh := range shards {
		ptrs[j] = nil
		if sh != nil {
			if len(sh) < symbolLen {
				return nil, fmt.Errorf("shard %d shorter than the symbol length", j)
			}
			copy(buf[j*symbolLen:(j+1)*symbolLen], sh[:symbolLen])
			ptrs[j] = (*C.uint8_t)(unsafe.Pointer(&buf[j*symbolLen]))
		}
	}
	s.closeMu.RLock()
	defer s.closeMu.RUnlock()
	if s.b == nil {
		return nil, fmt.Errorf("decode batcher closed")
	}
	runtime.LockOSThread()
	defer runtime.UnlockOSThread()
	t := C.fec_batcher_submit_shards(s.b, &ptrs[0], C.uint32_t(symbolLen))
	if t < 0 {
		return nil, fmt.Errorf("fec_batcher_submit_shards failed with code %d: %s", int64(t), C.GoString(C.fec_batcher_last_error()))
	}
	rows := make([]byte, s.r*s.slot)
	var mask C.uint64_t
	n := C.fec_batcher_wait_rebuilt(s.b, t, (*C.uint8_t)(unsafe.Pointer(&rows[0])), C.uint32_t(s.slot), &mask, -1)
	runtime.KeepAlive(rows)
	if n < 0 {
		return nil, fmt.Errorf("fec_batcher_wait_rebuilt failed with code %d: %s", int(n), C.GoString(C.fec_batcher_last_error()))
	}
	out := make(map[int][]byte, int(n))
	row := 0
	for j := 0; j < s.k && row < int(n); j++ {
		if uint64(mask)>>uint(j)&1 == 1 {
			out[j] = append([]byte(nil), rows[row*s.slot:row*s.slot+symbolLen]...)
			row++
		}
	}
	return out, nil
}
