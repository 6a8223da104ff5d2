//go:build cgo && fec_hip

// r > 1 on the wire (SURVEY.md §8(f) items 1-2): the repair header for parity rows
// 1..r-1, a batched encoder that emits r repair packets per group from one library call
// per batch, and a decoder that rebuilds up to r lost packets per group.
//
// Same design as the C++ mirror in quic-test_amd/host/fec.{hpp,cpp} (RSBatchEncoder,
// ParseRepairHeader, FECDecoder's r > 1 path), which tests/csrc/host_mirror_test.cpp checks
// on MI355X.  Status: written against the C-ABI and the reference package's types
// (Recovered, FECDecoderMetrics, padTo and the limits in decoder.go:9-14); not compiled
// here (no Go toolchain in the build image).

package fec

/*
#include <stdint.h>
#include <stdlib.h>
#include "fec_hip.h"
*/
import "C"

import (
	"encoding/binary"
	"fmt"
	"runtime"
	"sync"
	"time"
	"unsafe"
)

// Wire format.  Row 0 keeps the reference header (encoder.go:146-160):
//
//	FE C0 | groupID u64 LE | count u8 | payload
//
// Rows 1..r-1 use a header the reference parser rejects (decoder.go:73), so receivers
// that predate it ignore them and still recover single losses from row 0:
//
//	FE C1 | groupID u64 LE | count u8 | row u8 | r u8 | k u8 | payload
const (
	RepairHeaderLen   = 11
	RSRepairHeaderLen = 14
)

// RepairHeader describes either header form; R and K are 0 for a row-0 packet.
type RepairHeader struct {
	GroupID uint64
	Count   int
	Row     int
	R       int
	K       int
}

// ParseRepairHeader accepts both forms, with decoder.go:72-85's bounds plus row < r,
// count <= k and k + r <= 64 for the new one.
func ParseRepairHeader(b []byte) (h RepairHeader, payload []byte, ok bool) {
	if len(b) < RepairHeaderLen || b[0] != 0xFE || (b[1] != 0xC0 && b[1] != 0xC1) {
		return h, nil, false
	}
	h.GroupID = binary.LittleEndian.Uint64(b[2:10])
	h.Count = int(b[10])
	if h.Count <= 0 || h.Count > maxPacketCount {
		return h, nil, false
	}
	if b[1] == 0xC0 {
		return h, b[RepairHeaderLen:], true
	}
	if len(b) < RSRepairHeaderLen {
		return h, nil, false
	}
	h.Row, h.R, h.K = int(b[11]), int(b[12]), int(b[13])
	if h.Row < 1 || h.Row >= h.R || h.K < 1 || h.Count > h.K || h.K+h.R > 64 {
		return h, nil, false
	}
	return h, b[RSRepairHeaderLen:], true
}

// MakeRepairPacket builds a row-0 packet (reference header) or a row >= 1 packet.
func MakeRepairPacket(h RepairHeader, payload []byte) []byte {
	hl := RepairHeaderLen
	if h.Row != 0 {
		hl = RSRepairHeaderLen
	}
	out := make([]byte, hl+len(payload))
	out[0] = 0xFE
	out[1] = 0xC0
	binary.LittleEndian.PutUint64(out[2:10], h.GroupID)
	out[10] = byte(h.Count)
	if h.Row != 0 {
		out[1] = 0xC1
		out[11], out[12], out[13] = byte(h.Row), byte(h.R), byte(h.K)
	}
	copy(out[hl:], payload)
	return out
}

// RSBatchEncoder groups packets k at a time and encodes batch groups per library call
// (fec_encode_batch_rs over a page-locked slab), instead of one cgo call per group
// (encoder_hybrid.go:115).  Row 0 of each group equals HybridFECEncoder's repair packet.
type RSBatchEncoder struct {
	mu      sync.Mutex
	ctx     *C.FECEncoderCtx
	k, r    int
	batch   int
	slot    int
	slab    []byte // page-locked (fec_alloc_slab), batch*k*slot
	parity  []byte // page-locked, batch*r*slot
	count   []int
	maxLen  []int
	open    int
	groupID uint64
	metrics FECMetrics
}

func pinned(n int) []byte {
	p := C.fec_alloc_slab(C.size_t(n))
	if p == nil {
		return nil
	}
	return unsafe.Slice((*byte)(p), n)
}

func freePinned(b []byte) {
	if len(b) > 0 {
		C.fec_free_slab(unsafe.Pointer(&b[0]))
	}
}

// NewRSBatchEncoder: slot is the widest packet expected (wider ones widen it on the fly).
func NewRSBatchEncoder(k, r, batch, slot int) (*RSBatchEncoder, error) {
	if k < 1 || r < 1 || k+r > 64 || batch < 1 || slot < 1 {
		return nil, fmt.Errorf("unsupported k=%d r=%d batch=%d slot=%d", k, r, batch, slot)
	}
	runtime.LockOSThread() // the creation error is thread-local
	ctx := C.fec_encoder_new(C.double(float64(r)/float64(k)), C.uint32_t(batch))
	if ctx == nil {
		err := fmt.Errorf("no usable GPU: %s", C.GoString(C.fec_hip_last_error()))
		runtime.UnlockOSThread()
		return nil, err
	}
	runtime.UnlockOSThread()
	e := &RSBatchEncoder{ctx: ctx, k: k, r: r, batch: batch, slot: (slot + 15) &^ 15,
		count: make([]int, batch), maxLen: make([]int, batch)}
	e.slab, e.parity = pinned(batch*k*e.slot), pinned(batch*r*e.slot)
	if e.slab == nil || e.parity == nil {
		e.Close()
		return nil, fmt.Errorf("failed to allocate page-locked buffers")
	}
	runtime.SetFinalizer(e, (*RSBatchEncoder).Close)
	return e, nil
}

// AddPacket copies the packet into the slab; a full batch is encoded and its repair
// packets (group order, row order) are returned.
func (e *RSBatchEncoder) AddPacket(packet []byte) ([][]byte, error) {
	e.mu.Lock()
	defer e.mu.Unlock()
	if e.ctx == nil {
		return nil, fmt.Errorf("encoder closed")
	}
	var out [][]byte
	if len(packet) > e.slot {
		var err error
		if out, err = e.widen((len(packet) + 15) &^ 15); err != nil {
			return out, err
		}
	}
	if e.open == 0 || e.count[e.open-1] == e.k {
		e.count[e.open], e.maxLen[e.open] = 0, 0
		e.open++
	}
	g := e.open - 1
	off := (g*e.k + e.count[g]) * e.slot
	n := copy(e.slab[off:off+e.slot], packet)
	clear(e.slab[off+n : off+e.slot])
	e.count[g]++
	if len(packet) > e.maxLen[g] {
		e.maxLen[g] = len(packet)
	}
	e.metrics.PacketsEncoded++
	if e.open == e.batch && e.count[g] == e.k {
		more, err := e.encode(e.open)
		return append(out, more...), err
	}
	return out, nil
}

// Flush encodes the open groups now, the last one possibly partial (count < k).
func (e *RSBatchEncoder) Flush() ([][]byte, error) {
	e.mu.Lock()
	defer e.mu.Unlock()
	if e.ctx == nil {
		return nil, fmt.Errorf("encoder closed")
	}
	return e.encode(e.open)
}

func (e *RSBatchEncoder) encode(groups int) ([][]byte, error) {
	if groups == 0 {
		return nil, nil
	}
	last := groups - 1
	clear(e.slab[(last*e.k+e.count[last])*e.slot : (last+1)*e.k*e.slot]) // unfilled slots are zero
	rc := C.fec_encode_batch_rs(e.ctx, (*C.uint8_t)(unsafe.Pointer(&e.slab[0])), nil, C.uint64_t(groups),
		C.uint32_t(e.k), C.uint32_t(e.r), C.uint32_t(e.slot), (*C.uint8_t)(unsafe.Pointer(&e.parity[0])))
	if rc != 0 {
		return nil, ctxError(e.ctx, "fec_encode_batch_rs", rc)
	}
	out := make([][]byte, 0, groups*e.r)
	var firstErr error
	for g := 0; g < groups; g++ {
		gid := e.groupID
		e.groupID++
		if e.maxLen[g] == 0 {
			if firstErr == nil {
				firstErr = fmt.Errorf("empty packets in group %d", gid)
			}
			continue
		}
		for row := 0; row < e.r; row++ {
			off := (g*e.r + row) * e.slot
			pkt := MakeRepairPacket(RepairHeader{GroupID: gid, Count: e.count[g], Row: row, R: e.r, K: e.k},
				e.parity[off:off+e.maxLen[g]])
			e.metrics.RedundancyPackets++
			e.metrics.RedundancyBytes += int64(len(pkt))
			out = append(out, pkt)
		}
		e.metrics.GroupsProcessed++
	}
	e.open = 0
	return out, firstErr
}

func (e *RSBatchEncoder) widen(slot int) ([][]byte, error) {
	partial := e.open > 0 && e.count[e.open-1] < e.k
	complete := e.open
	var keep []byte
	var keepCount, keepMax int
	if partial {
		complete--
		keepCount, keepMax = e.count[e.open-1], e.maxLen[e.open-1]
		base := (e.open - 1) * e.k * e.slot
		keep = append([]byte(nil), e.slab[base:base+keepCount*e.slot]...)
	}
	out, err := e.encode(complete)
	if err != nil {
		return out, err
	}
	slab, parity := pinned(e.batch*e.k*slot), pinned(e.batch*e.r*slot)
	if slab == nil || parity == nil {
		freePinned(slab)
		freePinned(parity)
		return out, fmt.Errorf("failed to widen the slab to %d-byte slots", slot)
	}
	freePinned(e.slab)
	freePinned(e.parity)
	old := e.slot
	e.slab, e.parity, e.slot, e.open = slab, parity, slot, 0
	if partial {
		for j := 0; j < keepCount; j++ {
			copy(e.slab[j*slot:], keep[j*old:(j+1)*old])
			clear(e.slab[j*slot+old : (j+1)*slot])
		}
		e.count[0], e.maxLen[0], e.open = keepCount, keepMax, 1
	}
	return out, nil
}

// GetMetrics returns a copy of the counters (encoder.go:20-26 fields).
func (e *RSBatchEncoder) GetMetrics() FECMetrics {
	e.mu.Lock()
	defer e.mu.Unlock()
	return e.metrics
}

// Close frees the page-locked buffers and the GPU context.
func (e *RSBatchEncoder) Close() error {
	e.mu.Lock()
	defer e.mu.Unlock()
	freePinned(e.slab)
	freePinned(e.parity)
	e.slab, e.parity = nil, nil
	if e.ctx != nil {
		C.fec_encoder_free(e.ctx)
		e.ctx = nil
	}
	return nil
}

// RSDecoder rebuilds up to r lost packets per group from RSBatchEncoder's stream.  It
// keeps FECDecoder's group bookkeeping (decoder.go:9-14 limits, TTL and eviction, the
// symbol-length rule of decoder.go:115-120: bytewise coding makes any common truncation
// exact).  With deferred set, recoverable groups are queued and RecoverPending rebuilds
// them all in one library call per (k, r).
type RSDecoder struct {
	mu       sync.Mutex
	codec    map[[2]int]*RSCodec
	groups   map[uint64]*rsGroup
	pending  []uint64
	deferred bool
	metrics  FECDecoderMetrics
}

type rsGroup struct {
	createdAt   time.Time
	packetCount int
	symbolLen   int
	k, r        int
	packets     map[int][]byte // data id -> symbol
	rows        map[int][]byte // parity row -> symbol
	queued      bool
}

func NewRSDecoder(deferred bool) *RSDecoder {
	return &RSDecoder{codec: map[[2]int]*RSCodec{}, groups: map[uint64]*rsGroup{}, deferred: deferred}
}

func (d *RSDecoder) group(id uint64) *rsGroup {
	g, ok := d.groups[id]
	if !ok {
		if len(d.groups) >= maxActiveGroups {
			d.evictOldest()
		}
		g = &rsGroup{createdAt: time.Now(), packets: map[int][]byte{}, rows: map[int][]byte{}}
		d.groups[id] = g
		d.metrics.GroupsActive = int64(len(d.groups))
	}
	return g
}

func (d *RSDecoder) setSymbolLen(g *rsGroup, n int) {
	if g.symbolLen == 0 {
		g.symbolLen = min(n, maxSymbolLen)
	}
}

// AddPacket stores data packet packetID (< count) of a group; returns what it rebuilt.
func (d *RSDecoder) AddPacket(packet []byte, packetID, groupID uint64) []Recovered {
	d.mu.Lock()
	defer d.mu.Unlock()
	g := d.group(groupID)
	d.setSymbolLen(g, len(packet))
	g.packets[int(packetID)] = padTo(packet, g.symbolLen)
	d.metrics.PacketsReceived++
	return d.try(groupID, g)
}

// AddRedundancyPacket takes a packet of either header form.
func (d *RSDecoder) AddRedundancyPacket(b []byte) []Recovered {
	d.mu.Lock()
	defer d.mu.Unlock()
	h, payload, ok := ParseRepairHeader(b)
	if !ok {
		return nil
	}
	g := d.group(h.GroupID)
	if (g.packetCount != 0 && g.packetCount != h.Count) || (h.Row > 0 && g.k != 0 && (g.k != h.K || g.r != h.R)) {
		d.drop(h.GroupID)
		return nil
	}
	g.packetCount = h.Count
	if h.Row > 0 {
		g.k, g.r = h.K, h.R
	}
	d.setSymbolLen(g, len(payload))
	g.rows[h.Row] = padTo(payload, g.symbolLen)
	d.metrics.RepairPacketsReceived++
	return d.try(h.GroupID, g)
}

// shape is (k, r) from the row >= 1 headers; a group that has only seen row 0 decodes as
// (count, 1), whose single parity row is the XOR (row 0 of every (k, r) code).
func (g *rsGroup) shape() [2]int {
	if g.k == 0 {
		return [2]int{g.packetCount, 1}
	}
	return [2]int{g.k, g.r}
}

func (g *rsGroup) missing() int {
	m := 0
	for id := 0; id < g.packetCount; id++ {
		if _, ok := g.packets[id]; !ok {
			m++
		}
	}
	return m
}

func (d *RSDecoder) try(id uint64, g *rsGroup) []Recovered {
	if g.packetCount == 0 || len(g.rows) == 0 {
		return nil
	}
	m := g.missing()
	if m == 0 {
		return nil
	}
	if g.k == 0 && m != 1 { // row 0 only: the reference's single-loss XOR (decoder.go:233-248)
		d.metrics.FailedRecoveries++
		return nil
	}
	if m > len(g.rows) {
		d.metrics.FailedRecoveries++
		return nil
	}
	if g.k == 0 { // row 0 only, one loss: the reference's XOR recovery (decoder.go:255-287)
		return d.recoverSingle(g)
	}
	if d.deferred {
		if !g.queued {
			g.queued = true
			d.pending = append(d.pending, id)
		}
		return nil
	}
	lists, _ := d.recover([]uint64{id})
	return lists[0]
}

// recoverSingle rebuilds a row-0-only group's one lost packet as parity XOR every present
// packet (decoder.go:255-287), on the GPU through the XOR entry point the reference binds
// (xor_packets_*, fec_xor_simd.h:107-137), so groups of any count up to 255 work (the batch
// decode's erasure masks stop at 64 shards).  cgo may not keep Go pointers in C memory, so
// the symbols are gathered into one C buffer first.
func (d *RSDecoder) recoverSingle(g *rsGroup) []Recovered {
	lost := -1
	for id := 0; id < g.packetCount; id++ {
		if _, ok := g.packets[id]; !ok {
			lost = id
			break
		}
	}
	L := g.symbolLen
	if lost < 0 || L <= 0 {
		return nil
	}
	n := g.packetCount // parity row 0 + the count-1 present packets
	buf := (*byte)(C.malloc(C.size_t(n * L)))
	ptrs := (*unsafe.Pointer)(C.malloc(C.size_t(n) * C.size_t(unsafe.Sizeof(unsafe.Pointer(nil)))))
	defer C.free(unsafe.Pointer(buf))
	defer C.free(unsafe.Pointer(ptrs))
	src := unsafe.Slice(buf, n*L)
	ps := unsafe.Slice(ptrs, n)
	copy(src[0:L], g.rows[0])
	ps[0] = unsafe.Pointer(&src[0])
	i := 1
	for id := 0; id < g.packetCount; id++ {
		if p, ok := g.packets[id]; ok {
			copy(src[i*L:(i+1)*L], p)
			ps[i] = unsafe.Pointer(&src[i*L])
			i++
		}
	}
	out := make([]byte, L)
	runtime.LockOSThread() // xor_packets_* report failure through the thread-local error text
	C.xor_packets_avx2((**C.uint8_t)(unsafe.Pointer(ptrs)), C.size_t(n), C.size_t(L), (*C.uint8_t)(unsafe.Pointer(&out[0])))
	failed := C.GoString(C.fec_hip_last_error()) != ""
	runtime.UnlockOSThread()
	if failed {
		d.metrics.FailedRecoveries++
		return nil
	}
	g.packets[lost] = out
	d.metrics.PacketsRecovered++
	d.metrics.RecoveryEvents++
	return []Recovered{{PacketID: uint64(lost), Data: out}}
}

// RecoverPending rebuilds every queued group, one library call per (k, r).
func (d *RSDecoder) RecoverPending() (map[uint64][]Recovered, error) {
	d.mu.Lock()
	defer d.mu.Unlock()
	byShape := map[[2]int][]uint64{}
	for _, id := range d.pending {
		g, ok := d.groups[id]
		if !ok || !g.queued {
			continue
		}
		g.queued = false
		if m := g.missing(); m == 0 || m > len(g.rows) {
			continue
		}
		byShape[g.shape()] = append(byShape[g.shape()], id)
	}
	d.pending = d.pending[:0]
	out := map[uint64][]Recovered{}
	var firstErr error
	for _, ids := range byShape {
		lists, err := d.recover(ids)
		if err != nil && firstErr == nil {
			firstErr = err
		}
		for i, id := range ids {
			if len(lists[i]) > 0 {
				out[id] = lists[i]
			}
		}
	}
	return out, firstErr
}

// recover runs one fec_decode_batch_rs over groups of one (k, r), symbols zero-padded to
// the widest group's length; slots count..k-1 are the encoder's zero packets.
func (d *RSDecoder) recover(ids []uint64) ([][]Recovered, error) {
	lists := make([][]Recovered, len(ids))
	shape := d.groups[ids[0]].shape()
	k, r := shape[0], shape[1]
	codec, ok := d.codec[shape]
	if !ok {
		var err error
		if codec, err = NewRSCodec(k, r, -1); err != nil {
			d.metrics.FailedRecoveries += int64(len(ids))
			return lists, err
		}
		d.codec[shape] = codec
	}
	L := 0
	for _, id := range ids {
		L = max(L, d.groups[id].symbolLen)
	}
	G := len(ids)
	data, parity := make([]byte, G*k*L), make([]byte, G*r*L)
	masks, status := make([]uint64, G), make([]byte, G)
	for i, id := range ids {
		g := d.groups[id]
		for j := 0; j < g.packetCount; j++ {
			if p, ok := g.packets[j]; ok {
				copy(data[(i*k+j)*L:], p)
			} else {
				masks[i] |= 1 << uint(j)
			}
		}
		for row := 0; row < r; row++ {
			if p, ok := g.rows[row]; ok {
				copy(parity[(i*r+row)*L:], p)
			} else {
				masks[i] |= 1 << uint(k+row)
			}
		}
	}
	if _, err := codec.DecodeBatch(data, parity, masks, L, status); err != nil {
		d.metrics.FailedRecoveries += int64(G)
		return lists, err
	}
	for i, id := range ids {
		g := d.groups[id]
		if status[i] != 0 {
			d.metrics.FailedRecoveries++
			continue
		}
		for j := 0; j < g.packetCount; j++ {
			if masks[i]&(1<<uint(j)) == 0 {
				continue
			}
			sym := append([]byte(nil), data[(i*k+j)*L:(i*k+j)*L+g.symbolLen]...)
			g.packets[j] = sym
			lists[i] = append(lists[i], Recovered{PacketID: uint64(j), Data: sym})
			d.metrics.PacketsRecovered++
		}
		d.metrics.RecoveryEvents++
	}
	return lists, nil
}

func (d *RSDecoder) drop(id uint64) {
	delete(d.groups, id)
	d.metrics.GroupsActive = int64(len(d.groups))
}

func (d *RSDecoder) evictOldest() {
	var oldest uint64
	var t time.Time
	first := true
	for id, g := range d.groups {
		if first || g.createdAt.Before(t) {
			oldest, t, first = id, g.createdAt, false
		}
	}
	if !first {
		d.drop(oldest)
		d.metrics.GroupsEvicted++
	}
}

// CleanupGroups drops groups older than the reference's TTL (decoder.go:328-343).
func (d *RSDecoder) CleanupGroups() {
	d.mu.Lock()
	defer d.mu.Unlock()
	now := time.Now()
	for id, g := range d.groups {
		if now.Sub(g.createdAt) > groupTTL {
			d.drop(id)
			d.metrics.GroupsEvicted++
		}
	}
}

// GetMetrics returns a copy of the counters (decoder.go:43-51 fields).
func (d *RSDecoder) GetMetrics() FECDecoderMetrics {
	d.mu.Lock()
	defer d.mu.Unlock()
	return d.metrics
}

// Packet returns the stored symbol of (groupID, packetID), nil if absent.
func (d *RSDecoder) Packet(groupID, packetID uint64) []byte {
	d.mu.Lock()
	defer d.mu.Unlock()
	if g, ok := d.groups[groupID]; ok {
		return g.packets[int(packetID)]
	}
	return nil
}
