"""The ctx-less snappy-c.h-shaped entry points (sm_snappy_*): the exact ccall shape of the
reference's libsnappy helper, test/libsnappy.jl:5-30 --
    snappy_max_compressed_length  Csize_t <- (Csize_t,)
    snappy_compress               Cint    <- (Ptr{UInt8}, Csize_t, Ptr{UInt8}, Ref{Csize_t})
    snappy_uncompressed_length    Cint    <- (Ptr{UInt8}, Csize_t, Ref{Csize_t})
    snappy_uncompress             Cint    <- (Ptr{UInt8}, Csize_t, Ptr{UInt8}, Ref{Csize_t})
so that a binding switches from libsnappy to this library by library and symbol name alone.
The ctypes functions below are bound with exactly those types and called the way
ccall_compress / ccall_uncompress do."""
import ctypes
import os
import re

import pytest

from conftest import ROOT, read_testfile

HEADER = os.path.join(ROOT, "include", "snappy_mi355x.h")
SNAPPY_C = "/opt/conda/include/snappy-c.h"


def _decl(text, name):
    m = re.search(r"(\w+)\s+" + name + r"\s*\(([^)]*)\)\s*;", text, re.S)
    assert m, name
    params = [re.sub(r"\s+", " ", p.strip()) for p in m.group(2).split(",")]
    types = [re.sub(r"\s*\b\w+$", "", p).replace(" *", "*") for p in params]  # drop the parameter name
    return m.group(1), types


@pytest.mark.parametrize("fn", ["compress", "uncompress", "max_compressed_length", "uncompressed_length",
                                "validate_compressed_buffer"])
def test_signatures_equal_snappy_c(fn):
    if not os.path.exists(SNAPPY_C):
        pytest.skip("snappy-c.h not present")
    ours = _decl(open(HEADER).read(), "sm_snappy_" + fn)
    theirs = _decl(open(SNAPPY_C).read(), "snappy_" + fn)
    assert ours[1] == theirs[1]
    # return types: size_t, or a 32-bit status (snappy_status is a C enum = int)
    assert (ours[0], theirs[0]) in {("size_t", "size_t"), ("sm_status", "snappy_status")}


def _bind(L):
    """ctypes twins of test/libsnappy.jl:5-30's ccall signatures."""
    u8p, csz = ctypes.c_char_p, ctypes.c_size_t
    L.sm_snappy_max_compressed_length.restype = csz
    L.sm_snappy_max_compressed_length.argtypes = [csz]
    L.sm_snappy_compress.restype = ctypes.c_int
    L.sm_snappy_compress.argtypes = [u8p, csz, u8p, ctypes.POINTER(csz)]
    L.sm_snappy_uncompressed_length.restype = ctypes.c_int
    L.sm_snappy_uncompressed_length.argtypes = [u8p, csz, ctypes.POINTER(csz)]
    L.sm_snappy_uncompress.restype = ctypes.c_int
    L.sm_snappy_uncompress.argtypes = [u8p, csz, u8p, ctypes.POINTER(csz)]
    L.sm_snappy_set_mode.restype = ctypes.c_int
    L.sm_snappy_set_mode.argtypes = [ctypes.c_int]
    return L


def ccall_compress(L, data):
    # ccall_compress, test/libsnappy.jl:4-15
    size_in = len(data)
    output = ctypes.create_string_buffer(L.sm_snappy_max_compressed_length(size_in))
    outputindex = ctypes.c_size_t(len(output))
    st = L.sm_snappy_compress(data, size_in, output, ctypes.byref(outputindex))
    return st, output.raw[: outputindex.value]


def ccall_uncompress(L, data):
    # ccall_uncompress, test/libsnappy.jl:17-30
    size_in = len(data)
    n = ctypes.c_size_t(0)
    st = L.sm_snappy_uncompressed_length(data, size_in, ctypes.byref(n))
    if st:
        return st, None
    output = ctypes.create_string_buffer(max(n.value, 1))
    st = L.sm_snappy_uncompress(data, size_in, output, ctypes.byref(n))
    return st, output.raw[: n.value]


def test_host_only_entry_points(sm):
    L = _bind(ctypes.CDLL(sm.library_path()))
    assert L.sm_snappy_max_compressed_length(65536) == 76490
    n = ctypes.c_size_t(0)
    assert L.sm_snappy_uncompressed_length(b"\x80\x80\x04", 3, ctypes.byref(n)) == 0 and n.value == 65536
    # snappy-c.h statuses: every error is 1 (SNAPPY_INVALID_INPUT); the ctx API keeps the detail
    assert L.sm_snappy_uncompressed_length(b"\x80\x80", 2, ctypes.byref(n)) == 1
    assert L.sm_uncompressed_length(b"\x80\x80", 2, ctypes.byref(n)) == 18  # "Could not decode varint32."
    assert L.sm_snappy_set_mode(7) == 33


@pytest.mark.gpu
def test_ccall_shape_roundtrip(sm, oracle, gpu_available):
    L = _bind(ctypes.CDLL(sm.library_path()))
    # the default mode is dense: the same bytes as the ctx API's SM_MODE_FAST_DENSE
    raw = read_testfile("alice29.txt")
    st, comp = ccall_compress(L, raw)
    assert st == 0 and comp == sm.compress(raw, mode="dense") and oracle.uncompress(comp) == raw
    for fname in ("html", "alice29.txt", "fireworks.jpeg", "urls.10K"):
        raw = read_testfile(fname)
        assert L.sm_snappy_set_mode(1) == 0  # SM_MODE_FAST
        st, comp = ccall_compress(L, raw)
        assert st == 0 and oracle.uncompress(comp) == raw
        st, back = ccall_uncompress(L, comp)
        assert st == 0 and back == raw
        assert L.sm_snappy_set_mode(0) == 0  # SM_MODE_REFERENCE: Snappy.jl's exact bytes
        st, comp = ccall_compress(L, raw)
        assert st == 0 and comp == oracle.compress(raw)
    L.sm_snappy_set_mode(2)  # back to the default
    st, _ = ccall_uncompress(L, read_testfile("baddata1.snappy"))
    assert st != 0
