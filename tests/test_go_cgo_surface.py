"""The Go files a maintainer adds (quic-test_amd/internal/fec/*.go) against the C headers.

There is no Go toolchain in this image, so the Go side is never compiled here (INTEGRATION.md
§7).  What can be checked without one is the cgo surface: every `C.<name>(...)` call in each Go
file names a function its own preamble's headers declare (cgo resolves names per file) with the
prototype's number of arguments, each argument that states its C type (`C.T(x)`, `(*C.T)(p)`,
`unsafe.Pointer(p)`) states the prototype's, and every `C.<Type>` / `C.<CONSTANT>` it uses is a type or
constant of those headers or of the C library.  This is what `go build -tags fec_hip` would
reject first; the semantics stay "unverified" until the Go files run."""
import re
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parent.parent
GO_DIR = REPO / "quic-test_amd" / "internal" / "fec"
INCLUDE = REPO / "include"

# cgo's numeric conversions and helpers, and what <stdint.h> / <stdlib.h> / <stddef.h> give
C_SCALARS = {"char", "schar", "uchar", "short", "ushort", "int", "uint", "long", "ulong", "longlong",
             "ulonglong", "float", "double", "size_t", "int8_t", "int16_t", "int32_t", "int64_t",
             "uint8_t", "uint16_t", "uint32_t", "uint64_t", "uintptr_t"}
CGO_HELPERS = {"GoString": 1, "GoStringN": 2, "GoBytes": 2, "CString": 1, "CBytes": 1}
STDLIB_FUNCS = {"malloc": 1, "free": 1, "calloc": 2}


def _strip_comments(text: str) -> str:
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    return re.sub(r"//[^\n]*", " ", text)


def _split_top(args: str) -> list[str]:
    """Top-level comma split of an argument list (nested (), [], {} and string literals kept)."""
    out, depth, cur, quote = [], 0, [], None
    for ch in args:
        if quote:
            cur.append(ch)
            if ch == quote:
                quote = None
            continue
        if ch in "\"'`":
            quote = ch
        elif ch in "([{":
            depth += 1
        elif ch in ")]}":
            depth -= 1
        elif ch == "," and depth == 0:
            out.append("".join(cur))
            cur = []
            continue
        cur.append(ch)
    if "".join(cur).strip():
        out.append("".join(cur))
    return [a.strip() for a in out]


def _header_surface(name: str, seen=None) -> tuple[dict, set, set]:
    """(function -> parameter count, type names, constant names) of one header and what it
    includes from include/."""
    seen = set() if seen is None else seen
    funcs, types, consts = {}, set(), set()
    if name in seen or not (INCLUDE / name).exists():
        return funcs, types, consts
    seen.add(name)
    raw = (INCLUDE / name).read_text()
    for inc in re.findall(r'#include\s+"([^"]+)"', raw):
        f, t, c = _header_surface(inc, seen)
        funcs.update(f)
        types |= t
        consts |= c
    # as a C compiler sees it: no `extern "C" {` / `}` of the C++ guard
    text = re.sub(r"#ifdef\s+__cplusplus.*?#endif", " ", _strip_comments(raw), flags=re.S)
    consts |= set(re.findall(r"^\s*#define\s+([A-Z][A-Z0-9_]+)\b", text, flags=re.M))
    for body in re.findall(r"\benum\b[^{;]*\{([^}]*)\}", text):
        consts |= {m.group(1) for m in re.finditer(r"\b([A-Z][A-Z0-9_]+)\s*(?:=|,|$)", body)}
    types |= set(re.findall(r"\btypedef\b[^;]*?\b(\w+)\s*;", text, flags=re.S))
    types |= set(re.findall(r"\btypedef\s+struct\s+\w*\s*\{[^}]*\}\s*(\w+)\s*;", text, flags=re.S))
    types |= set(re.findall(r"\btypedef\b[^;]*\(\s*\*\s*(\w+)\s*\)", text))
    flat = re.sub(r"\{[^{}]*\}", ";", text)  # struct bodies out of the way
    for m in re.finditer(r"([A-Za-z_][\w\s\*]*?)\b(\w+)\s*\(([^()]*)\)\s*;", flat):
        if m.group(1).strip().startswith("typedef") or m.group(2) in ("if", "while", "return"):
            continue
        params = m.group(3).strip()
        funcs[m.group(2)] = [] if params in ("", "void") else [_c_param_type(x) for x in _split_top(params)]
    return funcs, types, consts


GO_C_NAMES = {"uint": "unsigned int", "ulong": "unsigned long", "longlong": "long long",
              "ulonglong": "unsigned long long", "uchar": "unsigned char", "schar": "signed char",
              "ushort": "unsigned short"}


def _c_param_type(param: str) -> tuple[str, int]:
    """(base type, pointer depth) of one C parameter declaration: `const uint8_t* packets[]` ->
    ("uint8_t", 2); `uint32_t n` -> ("uint32_t", 0); `void* p` -> ("void", 1)."""
    depth = param.count("*") + param.count("[")
    words = re.sub(r"\[[^\]]*\]", " ", param).replace("*", " ").split()
    words = [w for w in words if w not in ("const", "volatile", "restrict", "struct")]
    if len(words) > 1:
        words = words[:-1]  # the parameter's name
    return " ".join(words), depth


def _go_arg_type(arg: str):
    """(base C type, pointer depth) of a Go argument that states its C type -- `C.T(x)`,
    `(*C.T)(p)`, `unsafe.Pointer(p)` -- or None (a variable, constant, nil or address)."""
    def whole(prefix_len: int) -> bool:
        depth = 0
        for i, ch in enumerate(arg[prefix_len - 1:], prefix_len - 1):
            depth += ch == "("
            depth -= ch == ")"
            if depth == 0:
                return i == len(arg) - 1
        return False
    m = re.match(r"C\.(\w+)\(", arg)
    if m and whole(m.end()):
        return GO_C_NAMES.get(m.group(1), m.group(1)), 0
    m = re.match(r"\((\*+)C\.(\w+)\)\(", arg)
    if m and whole(m.end()):
        return GO_C_NAMES.get(m.group(2), m.group(2)), len(m.group(1))
    m = re.match(r"unsafe\.Pointer\(", arg)
    if m and whole(m.end()):
        return "void", 1
    return None


def _go_files():
    return sorted(p for p in GO_DIR.glob("*.go"))


def test_go_files_present():
    names = {p.name for p in _go_files()}
    assert {"cgo_hip.go", "fec_hip_rs.go", "rs_stream.go", "batcher.go"} <= names


def test_no_cgo_in_go_test_files():
    """`go test` refuses `import "C"` in a _test.go file: the tests reach C through the package."""
    for p in _go_files():
        if p.name.endswith("_test.go"):
            assert 'import "C"' not in p.read_text(), p.name


def test_headers_parse_to_the_declared_surface():
    funcs, types, consts = _header_surface("fec_hip.h")
    # the reference's eleven, with their arities (internal/fec/fec_xor_simd.h:22-137)
    assert funcs["fec_encoder_new"] == [("double", 0), ("uint32_t", 0)]
    assert funcs["fec_encode_batch"] == [("FECEncoderCtx", 1), ("uint8_t", 1), ("uint32_t", 1), ("uint32_t", 0),
                                         ("uint32_t", 0), ("uint8_t", 1)]
    assert funcs["xor_packets_avx2"] == [("uint8_t", 2), ("size_t", 0), ("size_t", 0), ("uint8_t", 1)]
    assert funcs["fec_select_xor_impl"] == []
    assert {"FECEncoderCtx", "FECBatcher", "FECBatcherStats"} <= types
    assert "FEC_ERR_AGAIN" in consts


def _cgo_problems(text: str, name: str) -> tuple[list[str], int]:
    """(problems, number of C function calls checked) of one Go file's cgo references."""
    m = re.search(r"/\*(.*?)\*/\s*import \"C\"", text, flags=re.S)
    if m is None:
        return ([] if "C." not in _strip_comments(text) else [f"{name}: C. without a preamble"]), 0
    preamble = m.group(1)
    funcs, types, consts = {}, set(), set()
    for inc in re.findall(r'#include\s+"([^"]+)"', preamble):
        f, t, c = _header_surface(inc)
        assert f, f"{name}: {inc} not under include/"
        funcs.update(f)
        types |= t
        consts |= c
    stdlib = "stdlib.h" in preamble
    body = _strip_comments(text[m.end():])
    problems, calls = [], 0
    for ref in re.finditer(r"\bC\.(\w+)", body):
        cname = ref.group(1)
        after = body[ref.end():]
        if cname in C_SCALARS or cname in types or cname in consts:
            continue
        if not after.startswith("("):
            problems.append(f"C.{cname}: not a type or constant of the preamble's headers")
            continue
        depth, i = 0, 0
        for i, ch in enumerate(after):
            depth += ch == "("
            depth -= ch == ")"
            if depth == 0:
                break
        args = _split_top(after[1:i])
        calls += 1
        if cname in funcs:
            params = funcs[cname]
            if len(args) != len(params):
                problems.append(f"C.{cname}(): {len(args)} arguments, the prototype has {len(params)}")
                continue
            for k, (arg, want_t) in enumerate(zip(args, params)):
                got = _go_arg_type(arg)
                if got is not None and got != want_t:
                    problems.append(f"C.{cname}() argument {k + 1}: {got}, the prototype has {want_t}")
            continue
        want = CGO_HELPERS.get(cname, STDLIB_FUNCS.get(cname) if stdlib else None)
        if want is None:
            problems.append(f"C.{cname}(): not declared by the preamble's headers")
        elif len(args) != want:
            problems.append(f"C.{cname}(): {len(args)} arguments, the prototype has {want}")
    return sorted(set(problems)), calls


@pytest.mark.parametrize("go", _go_files(), ids=lambda p: p.name)
def test_every_cgo_reference_resolves_against_the_files_own_preamble(go):
    problems, _ = _cgo_problems(go.read_text(), go.name)
    assert not problems, (go.name, problems)


def test_cgo_check_sees_the_calls_and_catches_mistakes():
    """Control: the check covers the files' C calls, and a wrong arity, an undeclared function,
    an unknown type and a wrongly typed argument in mutated copies are each reported."""
    total = sum(_cgo_problems(p.read_text(), p.name)[1] for p in _go_files())
    assert total >= 30, total
    text = (GO_DIR / "batcher.go").read_text()
    assert "C.fec_batcher_flush(" in text and "C.FECBatcherStats" in text
    bad = text.replace("C.fec_batcher_flush(", "C.fec_batcher_flush(nil, ", 1)
    bad = bad.replace("C.FECBatcherStats", "C.FECBatcherStatz", 1)
    bad += "\nfunc broken() { C.fec_batcher_frobnicate(nil) }\n"
    problems, _ = _cgo_problems(bad, "batcher.go (mutated)")
    assert any(p.startswith("C.fec_batcher_flush(): ") and "arguments" in p for p in problems), problems
    assert "C.FECBatcherStatz: not a type or constant of the preamble's headers" in problems, problems
    assert "C.fec_batcher_frobnicate(): not declared by the preamble's headers" in problems, problems
    # a C scalar of the wrong type (cgo's types are distinct Go types: `go build` rejects it)
    rs = (GO_DIR / "fec_hip_rs.go").read_text()
    assert "C.fec_encoder_new(C.double(" in rs
    problems, _ = _cgo_problems(rs.replace("C.fec_encoder_new(C.double(", "C.fec_encoder_new(C.float(", 1), "rs")
    assert "C.fec_encoder_new() argument 1: ('float', 0), the prototype has ('double', 0)" in problems, problems
