// fec_knobs.hpp — the switches the library takes from the environment.
//
// Operational settings (the coalescer, the resident encoder's timings, host threads, the
// host-resident paths' thresholds; INTEGRATION.md §6 lists each with its default) are read by
// the product library where they are used.
//
// Test and tuning switches -- forcing a kernel form the library would not choose, sizes that
// make rare paths common (chunked launches, overflowing run images), fault injection into the
// resident encoder -- exist only in libfec_hip_test.so.  test_knob() is compiled twice
// (fec_knobs.cpp): in libfec_hip_test.so (-DQUICFEC_TEST_HOOKS) it reads the switch's
// environment variable at every call (tests change it inside one process); in libfec_hip.so it
// returns the default and no name of any such switch is in the library.  Both libraries are
// linked from the same kernel and shim objects.
#pragma once

namespace qfec {

enum class TestKnob : int {
  kMaxWaveBlocks,     // workgroups per wave-per-group launch (forces the chunked launches)
  kEncodeTile,        // groups per workgroup of the tiled encodes
  kEncodeBlocks,      // workgroups per CU of the tiled encodes
  kEncodeWaves,       // occupancy cap of the encodes, waves per CU
  kEncodeBits,        // 1: bit-sliced encode for every compiled shape, 0: never
  kEncodeStage,       // 1: parity rows staged through LDS, 0: direct stores
  kDecodeWaves,       // occupancy cap of the decodes, waves per CU
  kRowsDirectBlocks,  // block limit of the two-launch row prefix (forces the three-launch form)
  kRunsStage,         // run-image bytes of recover_runs (rows past it go straight to HBM)
  kDecodeScan,        // groups per wave of the mask-addressed decode
  kPackedRuns,        // 1: packed recover in one launch (recover_runs) whatever the loss, 0: never
  kResidentNoLaunch,  // resident encoder: record launches without launching (never serves)
  kResidentEpoch,     // resident encoder: tag epoch (short: scrubs within a few thousand calls)
  kResidentTear,      // resident encoder: store one chunk / later address words ~100 us late
  kResidentFailAt,    // resident encoder: this call (0 = first) fails as if its deadline passed
  kResidentSpread,    // resident encoder: every call to the next serving class
  kResidentStamps,    // resident encoder: phase time stamps of served batches, to stderr at exit
  kResidentSlowUs,    // resident encoder: slow-poll interval once idle
  kCoalesceStamps,    // coalescer: creation and first batches' phase times, to stderr
  kCoalesceSpinPause, // coalescer: a waiting caller's pause rounds before it yields
  kCoalesceSpinYield, // coalescer: ... and its yield rounds before it sleeps
  kCount
};

// The switch from the environment, or `def` when unset; always `def` in libfec_hip.so.
long test_knob(TestKnob k, long def);

// Whether this library reads the test switches (libfec_hip_test.so).
bool test_knobs_enabled();

}  // namespace qfec
