// fec_knobs.cpp — test and tuning switches (fec_knobs.hpp).  Compiled twice: plain for
// libfec_hip.so (every switch at its default, no environment read, no switch name in the
// library) and with -DQUICFEC_TEST_HOOKS for libfec_hip_test.so.
#include "fec_knobs.hpp"

#include <cstdlib>

namespace qfec {

#ifdef QUICFEC_TEST_HOOKS

namespace {
const char* const kNames[] = {
    "QUICFEC_MAX_WAVE_BLOCKS",     "QUICFEC_ENCODE_TILE",          "QUICFEC_ENCODE_BLOCKS",
    "QUICFEC_ENCODE_WAVES",        "QUICFEC_ENCODE_BITS",          "QUICFEC_ENCODE_STAGE",
    "QUICFEC_DECODE_WAVES",        "QUICFEC_ROWS_DIRECT_BLOCKS",   "QUICFEC_RUNS_STAGE",
    "QUICFEC_DECODE_SCAN",         "QUICFEC_PACKED_RUNS",          "QUICFEC_RESIDENT_TEST_NOLAUNCH",
    "QUICFEC_RESIDENT_TEST_EPOCH", "QUICFEC_RESIDENT_TEST_TEAR",   "QUICFEC_RESIDENT_TEST_FAIL_AT",
    "QUICFEC_RESIDENT_SPREAD",     "QUICFEC_RESIDENT_STAMPS",      "QUICFEC_RESIDENT_SLOW_US",
    "QUICFEC_COALESCE_STAMPS",     "QUICFEC_COALESCE_SPIN_PAUSE",  "QUICFEC_COALESCE_SPIN_YIELD",
};
static_assert(sizeof(kNames) / sizeof(kNames[0]) == static_cast<size_t>(TestKnob::kCount), "one name per switch");
}  // namespace

long test_knob(TestKnob k, long def) {
  const char* v = std::getenv(kNames[static_cast<int>(k)]);
  return v && *v ? std::atol(v) : def;
}

bool test_knobs_enabled() { return true; }

#else

long test_knob(TestKnob, long def) { return def; }

bool test_knobs_enabled() { return false; }

#endif

}  // namespace qfec
