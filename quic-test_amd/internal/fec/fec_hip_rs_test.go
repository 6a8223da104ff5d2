//go:build cgo && fec_hip

// Go-side checks a maintainer runs with `go test -tags fec_hip ./internal/fec/` on an
// MI355X host.  Status: unverified here (no Go toolchain in the build image); the same
// properties are checked from Python and C++ by tests/ in this repo.

package fec

import (
	"bytes"
	"fmt"
	"math/rand"
	"sync"
	"testing"
	"time"
)

// Parity row 0 of RSCodec equals the reference XOR repair (FECEncoderCXX / FECEncoder).
func TestRSCodecRow0IsXORRepair(t *testing.T) {
	c, err := NewRSCodec(10, 3, -1)
	if err != nil {
		t.Skipf("no GPU: %v", err)
	}
	defer c.Close()
	const P, G = 1200, 64
	data := make([]byte, G*10*P)
	rand.New(rand.NewSource(1)).Read(data)
	parity := make([]byte, G*3*P)
	if err := c.EncodeBatch(data, P, parity); err != nil {
		t.Fatal(err)
	}
	cxx := NewFECEncoderCXX(0.1, 16)
	if cxx == nil {
		t.Skip("no GPU library")
	}
	defer cxx.Close()
	for g := 0; g < G; g++ {
		grp := FECBatchGroup{}
		for j := 0; j < 10; j++ {
			grp.Packets = append(grp.Packets, data[(g*10+j)*P:(g*10+j+1)*P])
		}
		rep, err := cxx.EncodeBatch([]FECBatchGroup{grp}, P)
		if err != nil {
			t.Fatal(err)
		}
		if !bytes.Equal(rep[0], parity[g*3*P:g*3*P+P]) {
			t.Fatalf("group %d: row 0 differs from the XOR repair", g)
		}
	}
}

// Encode -> erase up to r shards per group -> decode restores the data.
func TestRSCodecRoundTrip(t *testing.T) {
	c, err := NewRSCodec(10, 3, -1)
	if err != nil {
		t.Skipf("no GPU: %v", err)
	}
	defer c.Close()
	const P, G = 1200, 500
	rng := rand.New(rand.NewSource(2))
	data := make([]byte, G*10*P)
	rng.Read(data)
	parity := make([]byte, G*3*P)
	if err := c.EncodeBatch(data, P, parity); err != nil {
		t.Fatal(err)
	}
	broken := append([]byte(nil), data...)
	erasures := make([]uint64, G)
	for g := 0; g < G; g++ {
		for _, s := range rng.Perm(13)[:g%4] {
			erasures[g] |= 1 << uint(s)
			if s < 10 {
				copy(broken[(g*10+s)*P:(g*10+s+1)*P], make([]byte, P))
			}
		}
	}
	bad, err := c.DecodeBatch(broken, parity, erasures, P, nil)
	if err != nil || bad != 0 {
		t.Fatalf("decode: bad=%d err=%v", bad, err)
	}
	if !bytes.Equal(broken, data) {
		t.Fatal("round trip mismatch")
	}
}

// BatchedFECEncoder on a SharedBatcher returns HybridFECEncoder's repair packets, from many
// goroutines at once (one stream each), with groups of different streams sharing launches.
func TestBatchedEncoderMatchesHybrid(t *testing.T) {
	sb, err := NewSharedBatcher(10, 1, 1500, 64, time.Millisecond, -1)
	if err != nil {
		t.Skipf("no GPU: %v", err)
	}
	defer sb.Close()
	var wg sync.WaitGroup
	errs := make(chan error, 16)
	for s := 0; s < 16; s++ {
		wg.Add(1)
		go func(seed int64) {
			defer wg.Done()
			be := sb.NewEncoder()
			hy := NewHybridFECEncoder(0.1)
			rng := rand.New(rand.NewSource(seed))
			for i := 0; i < 10*20+3; i++ {
				pkt := make([]byte, 1+rng.Intn(1400))
				rng.Read(pkt)
				a1, r1, e1 := be.AddPacket(pkt, uint64(i))
				a2, r2, e2 := hy.AddPacket(pkt, uint64(i))
				if e1 != nil || e2 != nil || a1 != a2 || !bytes.Equal(r1, r2) {
					errs <- fmt.Errorf("stream %d packet %d: batched and hybrid repairs differ", seed, i)
					return
				}
			}
			f1, e1 := be.Flush()
			f2, e2 := hy.Flush()
			if e1 != nil || e2 != nil || !bytes.Equal(f1, f2) {
				errs <- fmt.Errorf("stream %d: flush differs", seed)
			}
		}(int64(s))
	}
	wg.Wait()
	close(errs)
	for err := range errs {
		t.Fatal(err)
	}
	if st := sb.Stats(); st[0] != 16*21 || st[1] >= st[0] {
		t.Fatalf("stats %v: expected %d groups in fewer launches", st, 16*21)
	}
}

// One batcher per listed device behind one handle (the same GPU listed twice also works):
// repairs equal HybridFECEncoder's and the stats sum over both batchers.
func TestBatchedEncoderOnMultiDeviceBatcher(t *testing.T) {
	sb, err := NewSharedBatcherMulti(10, 1, 1500, 64, time.Millisecond, []int{0, 0})
	if err != nil {
		t.Skipf("no GPU: %v", err)
	}
	defer sb.Close()
	be := sb.NewEncoder()
	hy := NewHybridFECEncoder(0.1)
	rng := rand.New(rand.NewSource(7))
	for i := 0; i < 10*30; i++ {
		pkt := make([]byte, 1+rng.Intn(1400))
		rng.Read(pkt)
		a1, r1, e1 := be.AddPacket(pkt, uint64(i))
		a2, r2, e2 := hy.AddPacket(pkt, uint64(i))
		if e1 != nil || e2 != nil || a1 != a2 || !bytes.Equal(r1, r2) {
			t.Fatalf("packet %d: multi-device batched and hybrid repairs differ", i)
		}
	}
	if st := sb.Stats(); st[0] != 30 {
		t.Fatalf("stats %v: expected 30 groups", st)
	}
}
