"""The Julia drop-in (julia/SnappyMI355X.jl) checked as text: no Julia exists
in this image or on the GPU box, so the shim cannot run. What can be checked is that the
documented binding is the shipped file, that every symbol it ccalls is exported by the
library with the argument count `include/snappy_mi355x.h` declares, and that the 0.7-only
spellings appear only behind the VERSION gate (the reference pins `julia 0.6`, REQUIRE:1)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHIM = os.path.join(ROOT, "julia", "SnappyMI355X.jl")
LIB = os.path.join(ROOT, "snappy.jl_amd", "libsnappy_mi355x.so")
HDR = os.path.join(ROOT, "include", "snappy_mi355x.h")


def _shim():
    with open(SHIM) as f:
        return f.read()


def test_integration_block_is_the_shim():
    with open(os.path.join(ROOT, "INTEGRATION.md")) as f:
        doc = f.read()
    m = re.search(r"```julia\n(module Snappy.*?)```", doc, re.S)
    assert m, "INTEGRATION.md §1 lost its Julia block"
    shim = _shim()
    assert m.group(1) == shim[shim.index("module Snappy"):]


def _ccalls(src):
    # (:symbol, LIB), RetType, (ArgTypes...)
    out = []
    for m in re.finditer(r"ccall\(\(:(\w+), LIB\),\s*(\w+(?:\{\w+\})?),\s*\(([^()]*(?:\([^()]*\))?[^()]*)\)", src):
        args = [a.strip() for a in m.group(3).split(",") if a.strip()]
        out.append((m.group(1), len(args)))
    return out


def _header_arity():
    with open(HDR) as f:
        hdr = re.sub(r"/\*.*?\*/", "", f.read(), flags=re.S)
    arity = {}
    for m in re.finditer(r"\b(sm_\w+)\s*\(([^;{]*?)\)\s*;", hdr, re.S):
        params = m.group(2).strip()
        arity[m.group(1)] = 0 if params in ("", "void") else params.count(",") + 1
    return arity


def test_shim_ccalls_match_header():
    calls = _ccalls(_shim())
    assert len(calls) >= 10
    arity = _header_arity()
    for name, n in calls:
        assert name in arity, f"{name} is not declared in include/snappy_mi355x.h"
        assert arity[name] == n, f"{name}: shim passes {n} args, header declares {arity[name]}"


def test_shim_symbols_exported():
    if not os.path.exists(LIB):
        pytest.skip("library not built")
    lib = ctypes.CDLL(LIB)
    for name, _ in _ccalls(_shim()):
        assert hasattr(lib, name), name


def test_shim_julia06_spellings_gated():
    src = _shim()
    gate = src.index("@static if VERSION")
    end = src.index("\nend\n", gate)
    rest = src[:gate] + src[end:]
    code = "\n".join(l.split("#")[0] for l in rest.splitlines())
    assert "undef" not in code and "Cvoid" not in code
    assert "Vector{UInt8}(n)" in src[gate:end] and "Cvoid" in src[gate:end]
