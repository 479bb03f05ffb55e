"""ctypes wrapper around the CPU oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
module, and only as the checker / CPU baseline.  It restates krm01/Snappy.jl
(src/Snappy.jl, src/internal.jl, src/varint.jl) -- see snappy_oracle.c for per-function
citations and DESIGN.md "Oracle" for what pins it.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle_snappy.so")

MESSAGES = {
    16: "Input too large.",
    17: "Invalid input.",
    18: "Could not decode varint32.",
    19: "Invalid input: corrupt copy offset",
    20: "Invalid input: corrupt copy length",
    21: "Invalid input: corrupt literal",
}

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        c_u8p = ctypes.c_void_p
        L.smo_max_compressed_length.restype = ctypes.c_size_t
        L.smo_max_compressed_length.argtypes = [ctypes.c_size_t]
        L.smo_compress.restype = ctypes.c_int
        L.smo_compress.argtypes = [c_u8p, ctypes.c_size_t, c_u8p, ctypes.POINTER(ctypes.c_size_t), ctypes.c_int]
        L.smo_uncompress.restype = ctypes.c_int
        L.smo_uncompress.argtypes = [c_u8p, ctypes.c_size_t, c_u8p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
        L.smo_uncompressed_length.restype = ctypes.c_int
        L.smo_uncompressed_length.argtypes = [c_u8p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_size_t)]
        L.smo_parse32.restype = ctypes.c_int
        L.smo_parse32.argtypes = [c_u8p, ctypes.c_size_t, ctypes.c_size_t, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_size_t)]
        L.smo_encode32.restype = ctypes.c_size_t
        L.smo_encode32.argtypes = [c_u8p, ctypes.c_uint32]
        L.smo_find_match_length.restype = ctypes.c_long
        L.smo_find_match_length.argtypes = [c_u8p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t]
        L.smo_hashtable_size.restype = ctypes.c_uint32
        L.smo_hashtable_size.argtypes = [ctypes.c_size_t]
        L.smo_char_table.restype = ctypes.c_uint16
        L.smo_char_table.argtypes = [ctypes.c_uint8]
        L.smo_compress_fragment.restype = ctypes.c_int
        L.smo_compress_fragment.argtypes = [c_u8p, ctypes.c_size_t, c_u8p, ctypes.POINTER(ctypes.c_size_t), ctypes.c_size_t, ctypes.c_int]
        L.smo_compress_batch.restype = ctypes.c_int
        L.smo_compress_batch.argtypes = [c_u8p, c_u8p, c_u8p, ctypes.c_uint32, c_u8p, c_u8p, c_u8p, ctypes.c_int, ctypes.c_int]
        L.smo_uncompress_batch.restype = ctypes.c_int
        L.smo_uncompress_batch.argtypes = [c_u8p, c_u8p, c_u8p, ctypes.c_uint32, c_u8p, c_u8p, c_u8p, c_u8p, c_u8p, ctypes.c_int]
        _lib = L
    return _lib


def _buf(b):
    a = np.frombuffer(bytes(b), dtype=np.uint8) if not isinstance(b, np.ndarray) else np.ascontiguousarray(b, dtype=np.uint8)
    return a


class OracleError(Exception):
    def __init__(self, code):
        self.code = code
        super().__init__(MESSAGES.get(code, "status %d" % code))


def max_compressed_length(n):
    return lib().smo_max_compressed_length(n)


def compress(data, compat=False):
    src = _buf(data)
    out = np.empty(max_compressed_length(src.size) + 8, dtype=np.uint8)
    ol = ctypes.c_size_t(0)
    st = lib().smo_compress(src.ctypes.data, src.size, out.ctypes.data, ctypes.byref(ol), int(compat))
    if st:
        raise OracleError(st)
    return out[: ol.value].tobytes()


def compress_fragment(data, total_len, compat=False):
    """One <= 64 KiB fragment of a total_len-byte stream, as Snappy.jl's block loop emits it."""
    src = _buf(data)
    out = np.empty(max_compressed_length(src.size) + 8, dtype=np.uint8)
    ol = ctypes.c_size_t(0)
    st = lib().smo_compress_fragment(src.ctypes.data if src.size else None, src.size, out.ctypes.data,
                                     ctypes.byref(ol), total_len, int(compat))
    if st:
        raise OracleError(st)
    return out[: ol.value].tobytes()


def uncompressed_length(data):
    src = _buf(data)
    r = ctypes.c_size_t(0)
    st = lib().smo_uncompressed_length(src.ctypes.data if src.size else None, src.size, ctypes.byref(r))
    if st:
        raise OracleError(st)
    return r.value


def uncompress_status(data):
    """Returns (status, bytes-or-None)."""
    src = _buf(data)
    try:
        n = uncompressed_length(src)
    except OracleError as e:
        return e.code, None
    out = np.empty(max(n, 1), dtype=np.uint8)
    ol = ctypes.c_size_t(0)
    st = lib().smo_uncompress(src.ctypes.data, src.size, out.ctypes.data, n, ctypes.byref(ol))
    if st:
        return st, None
    return 0, out[: ol.value].tobytes()


def uncompress(data):
    st, out = uncompress_status(data)
    if st:
        raise OracleError(st)
    return out


def parse32(data, off=0):
    src = _buf(data)
    v = ctypes.c_uint32(0)
    nx = ctypes.c_size_t(0)
    st = lib().smo_parse32(src.ctypes.data if src.size else None, src.size, off, ctypes.byref(v), ctypes.byref(nx))
    if st:
        raise OracleError(st)
    return v.value, nx.value


def encode32(v):
    out = np.zeros(8, dtype=np.uint8)
    n = lib().smo_encode32(out.ctypes.data, v)
    return out[:n].tobytes()


def find_match_length(a, i1, i2, limit):
    src = _buf(a)
    return lib().smo_find_match_length(src.ctypes.data, src.size, i1, i2, limit)


def hashtable_size(n):
    return lib().smo_hashtable_size(n)


def char_table(c):
    return lib().smo_char_table(c)


def compress_batch(inp, in_off, in_len, out, out_off, out_len, compat=False, nthreads=1):
    """All arguments are numpy arrays (u8 / u64 / u32)."""
    return lib().smo_compress_batch(inp.ctypes.data, in_off.ctypes.data, in_len.ctypes.data, in_len.size,
                                    out.ctypes.data, out_off.ctypes.data, out_len.ctypes.data, int(compat), nthreads)


def uncompress_batch(inp, in_off, in_len, out, out_off, out_cap, out_len, status, nthreads=1):
    return lib().smo_uncompress_batch(inp.ctypes.data, in_off.ctypes.data, in_len.ctypes.data, in_len.size,
                                      out.ctypes.data, out_off.ctypes.data, out_cap.ctypes.data,
                                      out_len.ctypes.data, status.ctypes.data, nthreads)


# ---- libsnappy (third-party comparison for the CPU baseline; not the oracle) ----------------

LIBSNAPPY_PATH = "/opt/conda/lib/libsnappy.so.1"
_lsb = None


def libsnappy_batch():
    """ctypes handle of liblibsnappy_batch.so with libsnappy dlopen'ed, or None when libsnappy
    is absent on this host."""
    global _lsb
    if _lsb is None:
        path = os.path.join(HERE, "liblibsnappy_batch.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.lsb_open.restype = ctypes.c_int
        L.lsb_open.argtypes = [ctypes.c_char_p]
        vp = ctypes.c_void_p
        for fn in (L.lsb_compress_batch, L.lsb_uncompress_batch):
            fn.restype = ctypes.c_int
            fn.argtypes = [vp, vp, vp, ctypes.c_uint32, vp, vp, vp, vp, ctypes.c_int]
        if not os.path.exists(LIBSNAPPY_PATH) or L.lsb_open(LIBSNAPPY_PATH.encode()) != 0:
            _lsb = False
        else:
            _lsb = L
    return _lsb or None


def libsnappy_compress_batch(inp, in_off, in_len, out, out_off, out_cap, out_len, nthreads=1):
    return libsnappy_batch().lsb_compress_batch(inp.ctypes.data, in_off.ctypes.data, in_len.ctypes.data, in_len.size,
                                                out.ctypes.data, out_off.ctypes.data, out_cap.ctypes.data,
                                                out_len.ctypes.data, nthreads)


def libsnappy_uncompress_batch(inp, in_off, in_len, out, out_off, out_cap, out_len, nthreads=1):
    return libsnappy_batch().lsb_uncompress_batch(inp.ctypes.data, in_off.ctypes.data, in_len.ctypes.data,
                                                  in_len.size, out.ctypes.data, out_off.ctypes.data,
                                                  out_cap.ctypes.data, out_len.ctypes.data, nthreads)
