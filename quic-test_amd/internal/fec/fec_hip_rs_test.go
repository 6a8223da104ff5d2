//go:build cgo && fec_hip

// Go-side checks a maintainer runs with `go test -tags fec_hip ./internal/fec/` on an
// MI355X host.  Status: unverified here (no Go toolchain in the build image); the same
// properties are checked from Python and C++ by tests/ in this repo.

package fec

import (
	"bytes"
	"math/rand"
	"testing"
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
