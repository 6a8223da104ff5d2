//go:build cgo && fec_hip

// Link glue for the MI355X library, replacing cgo_amd64.go (reference
// internal/fec/cgo_amd64.go:1-8, `-lfec_avx2 -lnuma`).  Select it with
// `go build -tags fec_hip`; cgo_amd64.go's constraint becomes `amd64 && cgo && !fec_hip`
// (INTEGRATION.md step 3).  ${SRCDIR} replaces the reference's cwd-relative `-L.`
// (fec_cgo.go:7-8), which only works when the linker runs inside internal/fec.
//
// Status: written against the C-ABI in include/; not compiled here (no Go toolchain in
// the build image).

package fec

/*
#cgo CFLAGS: -I${SRCDIR}/include
#cgo LDFLAGS: -L${SRCDIR}/lib -lfec_hip -Wl,-rpath,${SRCDIR}/lib
*/
import "C"
