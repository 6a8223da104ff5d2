"""CPU-side checks of the product library (no GPU compute calls).

- libfec_hip.so loads and exports every function include/*.h declares;
- behaviour that needs no device (NULL handling, no-GPU context creation, the code's
  parity matrix) matches the reference contract (fec_xor_simd.cpp:538-594);
- the kernels' table arithmetic, classify ranking and decode codebook, re-executed on the
  CPU from the product's own host code, match the oracle byte for byte.
"""
import json
import re
import subprocess
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parent.parent


def _declared_functions():
    names = set()
    for h in (REPO / "include").glob("*.h"):
        text = h.read_text()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b(\w+)\s*\(", text, flags=re.M):
            name = m.group(1)
            if name not in ("typedef",) and not text[m.start():m.end()].startswith("typedef"):
                names.add(name)
    return names


def test_headers_declare_reference_surface():
    names = _declared_functions()
    # the eleven reference functions (internal/fec/fec_xor_simd.h:22-137, 4 ISA variants)
    ref = {"fec_encoder_new", "fec_alloc_slab", "fec_alloc_slab_numa", "fec_alloc_repair_buffer",
           "fec_free_repair_buffer", "fec_encode_batch", "fec_encoder_free", "fec_free_slab",
           "fec_select_xor_impl", "xor_packets_scalar", "xor_packets_avx2", "xor_packets_avx512",
           "xor_packets_neon"}
    assert ref <= names


def test_library_exports_every_declared_symbol(quicfec_mod):
    lib_path = quicfec_mod.LIB_PATH
    out = subprocess.run(["nm", "-D", "--defined-only", str(lib_path)], capture_output=True, text=True,
                         check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    missing = _declared_functions() - exported
    assert not missing, missing
    assert set(quicfec_mod.REFERENCE_SYMBOLS) | set(quicfec_mod.HIP_SYMBOLS) <= exported


# The product library's only environment switches (INTEGRATION.md §6 lists them with defaults);
# the test and tuning switches (csrc/fec_knobs.hpp) exist in libfec_hip_test.so alone.
PRODUCT_KNOBS = {
    "QUICFEC_BATCHER_BLOCKING_SYNC", "QUICFEC_COALESCE", "QUICFEC_COALESCE_INFLIGHT", "QUICFEC_COALESCE_MAX_GROUPS",
    "QUICFEC_HOST_THREADS", "QUICFEC_NO_WARMUP", "QUICFEC_PIPE_CHUNK_BYTES", "QUICFEC_RESIDENT",
    "QUICFEC_RESIDENT_DEADLINE_MS", "QUICFEC_RESIDENT_IDLE_US", "QUICFEC_RESIDENT_LIFE_US", "QUICFEC_RESIDENT_SERVERS",
    "QUICFEC_RESIDENT_VRAM", "QUICFEC_SMALL_CALL_BYTES",
}


def _knob_names(path):
    data = Path(path).read_bytes()
    return {m.decode() for m in re.findall(rb"QUICFEC_[A-Z0-9_]+", data)}


def test_product_library_has_no_test_switches(quicfec_mod):
    """no fault-injection hook and no tuning switch in libfec_hip.so -- its
    environment names are exactly the operational ones; the test library holds the rest (and
    exports the same C-ABI)."""
    prod = _knob_names(quicfec_mod.LIB_PATH)
    assert prod == PRODUCT_KNOBS, sorted(prod ^ PRODUCT_KNOBS)
    assert not any("TEST" in n for n in prod)
    test = _knob_names(quicfec_mod.TEST_LIB_PATH)
    assert PRODUCT_KNOBS < test
    assert {"QUICFEC_RESIDENT_TEST_FAIL_AT", "QUICFEC_RESIDENT_TEST_TEAR", "QUICFEC_MAX_WAVE_BLOCKS",
            "QUICFEC_ENCODE_BITS", "QUICFEC_PACKED_RUNS"} <= test
    syms = []
    for lib in (quicfec_mod.LIB_PATH, quicfec_mod.TEST_LIB_PATH):
        out = subprocess.run(["nm", "-D", "--defined-only", str(lib)], capture_output=True, text=True,
                             check=True).stdout
        syms.append({ln.split()[-1] for ln in out.splitlines() if " T " in ln})
    assert syms[0] == syms[1]


def test_coalesce_stats_write_only_the_callers_struct(quicfec_mod):
    """FECCoalesceStats grew in round 5.  fec_coalesce_stats writes the 15
    words it was published with; fec_coalesce_stats_sized writes min(caller's size, this build's)
    and refuses a size below the first layout.  Guard words past the caller's struct stay put."""
    lib = quicfec_mod.load_library()
    n = len(quicfec_mod.COALESCE_STATS)
    guard = np.uint64(0xA5A5A5A5A5A5A5A5)
    for words, fn in ((15, "old"), (16, "sized"), (n, "sized"), (n + 4, "sized")):
        buf = np.full(n + 8, guard, dtype=np.uint64)
        rc = lib.fec_coalesce_stats(buf.ctypes.data, 0) if fn == "old" else \
            lib.fec_coalesce_stats_sized(buf.ctypes.data, words * 8, 0)
        assert rc == 0
        written = min(words, n)
        assert (buf[written:] == guard).all(), (fn, words)
        assert not (buf[:written] == guard).any(), (fn, words)   # every field of the caller's struct set
    buf = np.full(16, guard, dtype=np.uint64)
    assert lib.fec_coalesce_stats_sized(buf.ctypes.data, 14 * 8, 0) == quicfec_mod.FEC_ERR_RANGE
    assert (buf == guard).all()
    assert lib.fec_coalesce_stats_sized(None, 200, 0) == quicfec_mod.FEC_ERR_NULL


def test_library_is_built_from_this_tree(quicfec_mod):
    """The loaded libfec_hip.so embeds the hash of the sources it was built from
    (quic-test_amd/csrc/src_hash.py, compiled in by the Makefile); it must equal the hash of the
    tree this test runs from -- on the GPU box too, so a stale prebuilt library is caught
    (VERDICT r04 item 5)."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("src_hash", REPO / "quic-test_amd" / "csrc" / "src_hash.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    version = quicfec_mod.load_library().fec_hip_version().decode()
    assert re.fullmatch(r"libfec_hip \S+ gfx950 src=[0-9a-f]{64}", version), version
    assert version.endswith("src=" + mod.source_hash()), (version, mod.source_hash())


def test_library_is_gfx950_code_object(quicfec_mod):
    blob = quicfec_mod.LIB_PATH.read_bytes()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_null_arguments_need_no_gpu(quicfec_mod):
    lib = quicfec_mod.load_library()
    buf = np.zeros(16, dtype=np.uint8)
    off = np.zeros(10, dtype=np.uint32)
    # fec_xor_simd.cpp:564-566: NULL ctx/slab/offsets/repair -> -1 (checked before anything else)
    assert lib.fec_encode_batch(None, buf.ctypes.data, off.ctypes.data, 1, 8, buf.ctypes.data) == -1
    assert lib.fec_encode_batch(None, None, None, 0, 0, None) == -1
    assert lib.fec_encode_batch_rs(None, None, None, 0, 1, 1, 1, None) == quicfec_mod.FEC_ERR_NULL
    assert lib.fec_decode_batch_rs(None, None, None, None, 0, 1, 1, 1, None, None) == quicfec_mod.FEC_ERR_NULL
    lib.fec_encoder_free(None)
    lib.fec_free_slab(None)
    lib.fec_free_repair_buffer(None)
    assert lib.fec_encoder_device(None) == -1
    assert lib.fec_group_encode_batch_rs(None, None, 0, 1, 1, 1, None) == quicfec_mod.FEC_ERR_NULL
    assert lib.fec_group_decode_batch_rs(None, None, None, None, 0, 1, 1, 1, None, None) == quicfec_mod.FEC_ERR_NULL
    assert lib.fec_group_size(None) == 0
    assert not lib.fec_group_context(None, 0)
    lib.fec_group_free(None)
    # batchers: NULL handles and arguments are refused before anything touches a device
    assert lib.fec_batcher_submit(None, None, None, 0) == quicfec_mod.FEC_ERR_NULL
    assert lib.fec_batcher_submit_shards(None, None, 16) == quicfec_mod.FEC_ERR_NULL
    assert lib.fec_batcher_wait(None, 0, None, 0, 0) == quicfec_mod.FEC_ERR_NULL
    assert lib.fec_batcher_wait_rebuilt(None, 0, None, 0, None, 0) == quicfec_mod.FEC_ERR_NULL
    assert lib.fec_batcher_flush(None) == quicfec_mod.FEC_ERR_NULL
    assert lib.fec_batcher_stats(None, None) == quicfec_mod.FEC_ERR_NULL
    lib.fec_batcher_free(None)
    # unsupported shapes fail in the constructor, with a message, GPU or not
    assert not lib.fec_batcher_new(-1, 200, 57, 1200, 16, 100, 2)
    assert "unsupported" in lib.fec_batcher_last_error().decode()
    assert not lib.fec_batcher_new_decoder(-1, 60, 5, 1200, 16, 100, 2)      # k + r > 64
    assert "fec_batcher_new_decoder: unsupported" in lib.fec_batcher_last_error().decode()
    # several devices behind one handle: the same checks, the failing device named
    assert lib.fec_batcher_devices(None) == quicfec_mod.FEC_ERR_NULL
    devs = np.array([0, 1], dtype=np.int32)
    assert not lib.fec_batcher_new_multi(devs.ctypes.data, 2, 200, 57, 1200, 16, 100, 2)
    msg = lib.fec_batcher_last_error().decode()
    assert "fec_batcher_new_multi: device 0" in msg and "unsupported" in msg, msg
    assert not lib.fec_batcher_new_decoder_multi(devs.ctypes.data, 2, 60, 5, 1200, 16, 100, 2)
    assert "unsupported" in lib.fec_batcher_last_error().decode()
    neg = np.array([-3, 0], dtype=np.int32)
    assert not lib.fec_batcher_new_multi(neg.ctypes.data, 2, 10, 3, 1200, 16, 100, 2)
    assert "negative device ordinal" in lib.fec_batcher_last_error().decode()


def test_no_gpu_context_is_null_not_abort(quicfec_mod):
    if quicfec_mod.device_count() > 0:
        pytest.skip("a GPU is visible")
    lib = quicfec_mod.load_library()
    assert not lib.fec_encoder_new(0.1, 1024)
    assert "no HIP device" in quicfec_mod.last_error()
    with pytest.raises(quicfec_mod.FecError):
        quicfec_mod.Context()
    assert not lib.fec_group_new(None, 0)
    with pytest.raises(quicfec_mod.FecError):
        quicfec_mod.DeviceGroup()
    # the batchers fail loudly too: no CPU fallback
    with pytest.raises(quicfec_mod.FecError):
        quicfec_mod.Batcher(10, 3)
    with pytest.raises(quicfec_mod.FecError):
        quicfec_mod.DecodeBatcher(10, 3)
    with pytest.raises(quicfec_mod.FecError, match="no GPU visible"):
        quicfec_mod.Batcher(10, 3, devices=[])                 # every visible device: none
    with pytest.raises(quicfec_mod.FecError, match="device 0"):
        quicfec_mod.DecodeBatcher(10, 3, devices=[0, 0])


def test_parity_matrix_matches_oracle_and_fixture(quicfec_mod, oracle_mod, golden_dir):
    mats = json.loads((golden_dir / "parity_matrices.json").read_text())
    for key, M in mats.items():
        k, r = map(int, key.split(","))
        assert np.array_equal(quicfec_mod.parity_matrix(k, r), np.array(M, dtype=np.uint8))
    for k, r in ((1, 255), (128, 128), (200, 56)):
        assert np.array_equal(quicfec_mod.parity_matrix(k, r), oracle_mod.parity_matrix(k, r))
    with pytest.raises(quicfec_mod.FecError):
        quicfec_mod.parity_matrix(200, 57)
    with pytest.raises(quicfec_mod.FecError):
        quicfec_mod.parity_matrix(0, 3)


def test_kernel_arithmetic_emulation(tmp_path, oracle_mod):
    exe = tmp_path / "kernel_emulation"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", str(REPO / "quic-test_amd" / "csrc"),
                    str(REPO / "tests" / "csrc" / "kernel_emulation.cpp"), str(oracle_mod.ORACLE_LIB),
                    f"-Wl,-rpath,{oracle_mod.ORACLE_DIR}", "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and out.stdout.startswith("OK"), out.stdout + out.stderr


def test_resident_ring_protocol_model(tmp_path):
    """The resident ring's acceptance rules checked on the CPU against the product's own
    definitions (fec_kernels.hpp server_tag / server_scrub_after, the slot, control and
    coordination layouts): tags unique within an epoch and never 0, no stale 8-B word accepted
    over 40 epochs of torn, partly rewritten laps with the epoch scrub (and a stale acceptance
    without it, the control), serving classes' seqs confined to their own slots with the
    previous occupant seq - 1024, and the classes' shared idle / leave / exit-count words over
    4,500 modelled instances with random interleavings and late-dispatched workgroups: all leave
    together, none on an earlier instance's words, exactly one stores exited (ADVICE r05;
    controls without the generation checks must fail) (tests/csrc/ring_protocol_test.cpp)."""
    exe = tmp_path / "ring_protocol_test"
    subprocess.run(["g++", "-O2", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include",
                    "-I", str(REPO / "quic-test_amd" / "csrc"), str(REPO / "tests" / "csrc" / "ring_protocol_test.cpp"),
                    "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0 and out.stdout.startswith("OK"), out.stdout + out.stderr


def test_ctx_last_error_null_context(quicfec_mod):
    lib = quicfec_mod.load_library()
    import ctypes
    buf = ctypes.create_string_buffer(16)
    assert lib.fec_ctx_last_error(None, buf, 16) == 0


def _vma_policy(addr: int):
    """(mode, nodemask word 0) of the mapping at addr: get_mempolicy(MPOL_F_ADDR)."""
    import ctypes
    libc = ctypes.CDLL(None, use_errno=True)
    mode = ctypes.c_int(-1)
    mask = (ctypes.c_ulong * 16)()
    SYS_get_mempolicy, MPOL_F_ADDR = 239, 1 << 1
    rc = libc.syscall(SYS_get_mempolicy, ctypes.byref(mode), mask, ctypes.c_ulong(1024 + 1),
                      ctypes.c_void_p(addr), ctypes.c_ulong(MPOL_F_ADDR))
    if rc != 0:
        pytest.skip(f"get_mempolicy unavailable (errno {ctypes.get_errno()})")
    return mode.value, mask[0]


def test_alloc_slab_numa_binds_node(quicfec_mod):
    """fec_alloc_slab_numa(size, node) binds the pages to the node (fec_xor_simd.cpp:486-510
    mbinds with MPOL_BIND); read the policy back with get_mempolicy."""
    import ctypes
    lib = quicfec_mod.load_library()
    size = 3 * 4096 + 100
    p = lib.fec_alloc_slab_numa(size, 0)
    assert p, quicfec_mod.last_error()
    try:
        assert p % 4096 == 0
        ctypes.memset(p, 0xA5, size)              # usable memory, every byte
        assert ctypes.string_at(p + size - 1, 1) == b"\xa5"
        mode, nodes = _vma_policy(p)
        MPOL_BIND = 2
        assert mode == MPOL_BIND and nodes & 1, (mode, nodes)
    finally:
        lib.fec_free_slab(p)
    # node < 0: the plain allocator (NULL without a GPU, as fec_alloc_slab)
    q = lib.fec_alloc_slab_numa(64, -1)
    if q:
        lib.fec_free_slab(q)


def test_product_and_bench_tools_link_no_oracle():
    """The oracle is test infrastructure: the product library, the C++ mirror and the tool bench.py
    runs outside its cpu_baseline leg (lib/call_site, the call_site section) link none of it."""
    import subprocess
    lib = REPO / "quic-test_amd" / "lib"
    for name in ("libfec_hip.so", "libquicfec_host.so", "call_site"):
        f = lib / name
        assert f.exists(), f"{f} not built (__graft_entry__.build())"
        dyn = subprocess.run(["readelf", "-d", str(f)], capture_output=True, text=True, check=True).stdout
        needed = [ln for ln in dyn.splitlines() if "(NEEDED)" in ln]
        assert needed and not any("oracle" in ln or "fec_ref" in ln for ln in needed), (name, needed)


def test_bench_call_site_without_tool_is_skipped(monkeypatch, tmp_path):
    """bench.py's call_site section reports a missing tool instead of failing the bench line."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", REPO / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    monkeypatch.setattr(bench, "CALL_SITE_TOOL", tmp_path / "missing")
    assert "skipped" in bench.call_site()


def test_bench_call_site_reads_the_tool_lines(monkeypatch, tmp_path):
    """bench.py's call_site section runs the tool once per leg (raw, 1 and 16 streams, the shared
    batcher at r = 1 and 3) and keeps
    each leg's rate, delay percentiles, error and expiry counts and ring kind from its last JSON line."""
    import importlib.util
    import stat
    spec = importlib.util.spec_from_file_location("bench_mod2", REPO / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    tool = tmp_path / "call_site"
    tool.write_text("#!/bin/sh\necho 'warming up'\n"
                    "echo '{\"mode\": \"'$1'\", \"streams\": '${2:-1}', \"groups_per_s\": 1000.0, "
                    "\"delay_us\": {\"p50\": 5.5, \"p99\": 9.0}, \"errors\": 0, \"expired\": 0, "
                    "\"resident_inline\": 7, \"resident_vram\": 1, \"extra\": 3}'\n")
    tool.chmod(tool.stat().st_mode | stat.S_IEXEC)
    monkeypatch.setattr(bench, "CALL_SITE_TOOL", tool)
    out = bench.call_site(seconds=0.1)
    assert set(out) >= {"raw", "streams_1", "streams_16", "batcher_16_r1", "batcher_16_r3", "reference_call"}
    for leg in ("raw", "streams_1", "streams_16", "batcher_16_r1", "batcher_16_r3"):
        assert out[leg] == {"groups_per_s": 1000.0, "delay_us": {"p50": 5.5, "p99": 9.0}, "errors": 0,
                            "expired": 0, "resident_inline": 7, "resident_vram": 1}
    # beside the reference library on one core (cpu_baseline's ref_encode_batch_1t_GiBps)
    gib = 1000.0 * 12000 / 2**30
    out = bench.call_site(ref_1t_GiBps=2 * gib, seconds=0.1)
    assert out["ref_encode_batch_1t_groups_per_s"] == 2000.0
    assert out["batcher_16_r3"]["vs_ref_1t"] == 0.5


def test_test_switch_names_match_their_enum():
    """csrc/fec_knobs.cpp maps each TestKnob (fec_knobs.hpp) to its environment name by position:
    the two lists must line up one for one (kMaxWaveBlocks <-> QUICFEC_MAX_WAVE_BLOCKS, the
    resident test hooks under QUICFEC_RESIDENT_TEST_*), or a test would set one switch and move
    another."""
    csrc = REPO / "quic-test_amd" / "csrc"
    hpp = (csrc / "fec_knobs.hpp").read_text()
    enum = re.search(r"enum class TestKnob : int \{(.*?)\};", hpp, re.S).group(1)
    keys = [m.group(1) for m in re.finditer(r"^\s*k(\w+),?", enum, re.M)]
    assert keys[-1] == "Count"
    keys = keys[:-1]
    cpp = (csrc / "fec_knobs.cpp").read_text()
    names = re.findall(r'"(QUICFEC_[A-Z0-9_]+)"', re.search(r"kNames\[\] = \{(.*?)\};", cpp, re.S).group(1))
    assert len(names) == len(keys)

    def env_of(key):
        snake = re.sub(r"(?<!^)(?=[A-Z])", "_", key).upper()
        for hook in ("NO_LAUNCH", "EPOCH", "TEAR", "FAIL_AT"):   # the fault-injection hooks
            if snake == "RESIDENT_" + hook:
                return "QUICFEC_RESIDENT_TEST_" + hook.replace("NO_LAUNCH", "NOLAUNCH")
        return "QUICFEC_" + snake

    assert [env_of(k) for k in keys] == names


def test_headers_are_plain_c_and_link_from_c(tmp_path, quicfec_mod):
    """cgo compiles the preamble's headers with a C compiler (fec_cgo.go:10-14 includes
    fec_xor_simd.h; cgo_hip.go adds fec_hip.h): both headers compile as ISO C99 with -pedantic and
    no warning, and a C program that takes the address of every function they declare links
    against libfec_hip.so and runs (the version string; no GPU call)."""
    names = sorted(_declared_functions())
    src = tmp_path / "abi_c.c"
    src.write_text(
        '#include "fec_xor_simd.h"\n#include "fec_hip.h"\n#include <stdio.h>\n'
        "typedef void (*any_fn)(void);\n"
        "static const any_fn fns[] = {\n" + "".join(f"  (any_fn){n},\n" for n in names) + "};\n"
        "int main(void) {\n"
        "  size_t i, n = 0;\n"
        "  for (i = 0; i < sizeof fns / sizeof fns[0]; ++i) n += fns[i] != NULL;\n"
        '  printf("%zu %s\\n", n, fec_hip_version());\n'
        "  return 0;\n}\n")
    exe = tmp_path / "abi_c"
    lib_dir = Path(quicfec_mod.LIB_PATH).parent
    for std in ("c99", "c11"):
        subprocess.run(["gcc", f"-std={std}", "-Wall", "-Wextra", "-pedantic", "-Werror", "-I", str(REPO / "include"),
                        "-c", str(src), "-o", str(tmp_path / f"abi_{std}.o")], check=True)
    subprocess.run(["gcc", "-std=c99", "-I", str(REPO / "include"), str(src), "-o", str(exe), "-L", str(lib_dir),
                    "-lfec_hip", f"-Wl,-rpath,{lib_dir}"], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60, check=True).stdout.split()
    assert int(out[0]) == len(names) and out[1] == "libfec_hip", out
