"""snappy.jl_amd -- MI355X-native Snappy codec with Snappy.jl's API surface.

Host-side mirror of krm01/Snappy.jl (src/Snappy.jl:1-94) over the C ABI in
include/snappy_mi355x.h (libsnappy_mi355x.so, hand-written gfx950 HIP kernels).

    compress(x)            -> bytes     Snappy.jl compress(::Vector{UInt8}) / (::String)  :20,:38
    uncompress(x)          -> bytes     Snappy.jl uncompress(::Vector{UInt8})            :46
    maxlength_compressed(n)             Snappy.jl:80
    length_uncompressed(x) -> (n, next) Snappy.jl:90  (next is a 0-based index here)
    parse32(buf, off) / encode32(v)     src/varint.jl:12 / :46 (0-based offsets)

Errors raise SnappyError carrying the reference's exact ErrorException message.
`mode="fast"` (default) uses the wave-parallel parse (valid snappy that decodes bit-exactly
under Snappy.jl's uncompress, different bytes); `mode="reference"` produces Snappy.jl's exact
bytes; `mode="dense"` is the fast parse with two chain candidates (smaller, slower).

Batched GPU path (the north-star hot path): compress_batch / uncompress_batch on host
arrays, and compress_batch_device / uncompress_batch_device on torch tensors already
resident in HBM.

There is no CPU fallback: importing works without a GPU, but every codec call needs the
HIP library and a device, and raises if either is missing.
"""
import ctypes
import os
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# SNAPPY_MI355X_LIB: alternate build of the same library (diagnostic/ablation builds only)
LIB_PATH = os.environ.get("SNAPPY_MI355X_LIB") or os.path.join(HERE, "libsnappy_mi355x.so")
BLOCK_SIZE = 65536

SM_OK = 0
SM_BUFFER_TOO_SMALL = 2
SM_ERR_DEVICE = 32
SM_OUT_LEN_ERROR = 0xFFF00000  # d_out_len[b] >= this: block b failed (include/snappy_mi355x.h)
MODES = {"reference": 0, "fast": 1, "dense": 2}

# exported symbols of include/snappy_mi355x.h (checked by tests/test_abi.py)
ABI_SYMBOLS = (
    "sm_status_message", "sm_max_compressed_length", "sm_uncompressed_length", "sm_parse32",
    "sm_encode32", "sm_ctx_create", "sm_ctx_destroy", "sm_ctx_stream", "sm_compress", "sm_uncompress",
    "sm_compress_batch_device", "sm_uncompress_batch_device", "sm_compress_batch",
    "sm_uncompress_batch", "sm_version", "sm_compress_fragments_device", "sm_ctx_last_path", "sm_ctx_set_small_decode",
    "sm_ctx_set_split_compress", "sm_ctx_last_compress_split",
    "sm_find_match_length", "sm_validate_batch_device", "sm_uncompressed_length_batch_device",
    "sm_validate_compressed_buffer", "sm_compress_batch_sharded", "sm_uncompress_batch_sharded",
    "sm_uncompress_fragments_device", "sm_place_fragments_device", "sm_snappy_compress", "sm_snappy_uncompress",
    "sm_snappy_max_compressed_length", "sm_snappy_uncompressed_length", "sm_snappy_validate_compressed_buffer",
    "sm_snappy_set_mode",
)


class SnappyError(Exception):
    """Mirrors the ErrorException the reference throws; .code is the sm_status."""

    def __init__(self, code, message=None):
        self.code = int(code)
        super().__init__(message if message is not None else status_message(code))


_lib = None
_ctx = {}
_ctx_lock = threading.Lock()


def library_path():
    return LIB_PATH


def lib():
    """Load libsnappy_mi355x.so (raises OSError if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OSError("libsnappy_mi355x.so not built (run __graft_entry__.build())")
        _lib = load_library(LIB_PATH)
    return _lib


def load_library(path):
    """A build of the C ABI at `path` with its prototypes set (lib() uses the shipped one; the
    GPU tests also load diagnostic variants built by the Makefile, e.g. the error-mark build)."""
    L = ctypes.CDLL(path)
    vp, sz, i32, u32 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int32, ctypes.c_uint32
    L.sm_status_message.restype = ctypes.c_char_p
    L.sm_status_message.argtypes = [i32]
    L.sm_max_compressed_length.restype = sz
    L.sm_max_compressed_length.argtypes = [sz]
    L.sm_uncompressed_length.restype = i32
    L.sm_uncompressed_length.argtypes = [vp, sz, ctypes.POINTER(sz)]
    L.sm_parse32.restype = i32
    L.sm_parse32.argtypes = [vp, sz, sz, ctypes.POINTER(u32), ctypes.POINTER(sz)]
    L.sm_encode32.restype = sz
    L.sm_encode32.argtypes = [vp, u32]
    L.sm_ctx_create.restype = vp
    L.sm_ctx_create.argtypes = [ctypes.c_int]
    L.sm_ctx_destroy.restype = None
    L.sm_ctx_destroy.argtypes = [vp]
    L.sm_ctx_stream.restype = vp
    L.sm_ctx_stream.argtypes = [vp]
    L.sm_compress.restype = i32
    L.sm_compress.argtypes = [vp, vp, sz, vp, ctypes.POINTER(sz), ctypes.c_int]
    L.sm_uncompress.restype = i32
    L.sm_uncompress.argtypes = [vp, vp, sz, vp, ctypes.POINTER(sz)]
    L.sm_compress_batch_device.restype = i32
    L.sm_compress_batch_device.argtypes = [vp, vp, vp, vp, u32, vp, vp, vp, ctypes.c_int, vp]
    L.sm_uncompress_batch_device.restype = i32
    L.sm_uncompress_batch_device.argtypes = [vp, vp, vp, vp, u32, vp, vp, vp, vp, vp, vp]
    L.sm_compress_batch.restype = i32
    L.sm_compress_batch.argtypes = [vp, vp, vp, vp, u32, vp, vp, vp, ctypes.c_int]
    L.sm_uncompress_batch.restype = i32
    L.sm_uncompress_batch.argtypes = [vp, vp, vp, vp, u32, vp, vp, vp, vp, vp]
    L.sm_compress_batch_sharded.restype = i32
    L.sm_compress_batch_sharded.argtypes = [vp, ctypes.c_int, vp, vp, vp, u32, vp, vp, vp, ctypes.c_int]
    L.sm_uncompress_batch_sharded.restype = i32
    L.sm_uncompress_batch_sharded.argtypes = [vp, ctypes.c_int, vp, vp, vp, u32, vp, vp, vp, vp, vp]
    L.sm_find_match_length.restype = i32
    L.sm_find_match_length.argtypes = [vp, sz, sz, sz, sz, ctypes.POINTER(sz)]
    L.sm_ctx_last_path.restype = ctypes.c_int
    L.sm_ctx_last_path.argtypes = [vp]
    L.sm_ctx_set_small_decode.restype = ctypes.c_int
    L.sm_ctx_set_small_decode.argtypes = [vp, ctypes.c_int]
    L.sm_ctx_set_split_compress.restype = ctypes.c_int
    L.sm_ctx_set_split_compress.argtypes = [vp, ctypes.c_int]
    L.sm_ctx_last_compress_split.restype = ctypes.c_int
    L.sm_ctx_last_compress_split.argtypes = [vp]
    L.sm_version.restype = ctypes.c_char_p
    L.sm_version.argtypes = []
    L.sm_compress_fragments_device.restype = i32
    L.sm_compress_fragments_device.argtypes = [vp, vp, vp, vp, u32, vp, vp, vp, ctypes.c_uint64, ctypes.c_int, vp]
    L.sm_validate_batch_device.restype = i32
    L.sm_validate_batch_device.argtypes = [vp, vp, vp, vp, u32, vp, vp]
    L.sm_uncompressed_length_batch_device.restype = i32
    L.sm_uncompressed_length_batch_device.argtypes = [vp, vp, vp, vp, u32, vp, vp, vp]
    L.sm_validate_compressed_buffer.restype = i32
    L.sm_validate_compressed_buffer.argtypes = [vp, vp, sz]
    L.sm_place_fragments_device.restype = i32
    L.sm_place_fragments_device.argtypes = [vp, vp, vp, vp, u32, vp, ctypes.c_uint64, ctypes.c_int, vp,
                                            ctypes.c_uint64, vp, vp, vp]
    L.sm_uncompress_fragments_device.restype = i32
    L.sm_uncompress_fragments_device.argtypes = [vp, vp, vp, vp, u32, vp, vp, vp, vp, vp, vp]
    # snappy-c.h shape (test/libsnappy.jl:5-30): (char*, size_t, char*, size_t*) -> int
    L.sm_snappy_compress.restype = i32
    L.sm_snappy_compress.argtypes = [vp, sz, vp, ctypes.POINTER(sz)]
    L.sm_snappy_uncompress.restype = i32
    L.sm_snappy_uncompress.argtypes = [vp, sz, vp, ctypes.POINTER(sz)]
    L.sm_snappy_max_compressed_length.restype = sz
    L.sm_snappy_max_compressed_length.argtypes = [sz]
    L.sm_snappy_uncompressed_length.restype = i32
    L.sm_snappy_uncompressed_length.argtypes = [vp, sz, ctypes.POINTER(sz)]
    L.sm_snappy_validate_compressed_buffer.restype = i32
    L.sm_snappy_validate_compressed_buffer.argtypes = [vp, sz]
    L.sm_snappy_set_mode.restype = i32
    L.sm_snappy_set_mode.argtypes = [ctypes.c_int]
    return L


def status_message(code):
    return lib().sm_status_message(int(code)).decode()


def _bytes(x):
    """Accept bytes / bytearray / memoryview / str / uint8 ndarray (String method, Snappy.jl:38)."""
    if isinstance(x, str):
        x = x.encode("utf-8")
    if isinstance(x, np.ndarray):
        return np.ascontiguousarray(x, dtype=np.uint8)
    return np.frombuffer(bytes(x), dtype=np.uint8)


def context(device=0):
    """Per-device sm_ctx (one HIP stream + scratch; the library serialises host-buffer calls on
    it).  Raises if no device is usable."""
    with _ctx_lock:
        c = _ctx.get(device)
        if c is None:
            c = lib().sm_ctx_create(device)
            if not c:
                raise SnappyError(32, "no usable HIP device %d for snappy_mi355x" % device)
            _ctx[device] = c
    return c


def contexts(devices):
    """One sm_ctx per entry of `devices` for the sharded calls; a device listed twice gets a
    second context (its own stream), so the sharding also runs on one GPU.  These contexts are
    separate from the single-call context(d) (the sharded call rejects a ctx listed twice)."""
    seen, out = {}, []
    for d in devices:
        k = seen.get(d, 0)
        seen[d] = k + 1
        key = ("shard", d, k)
        c = _ctx.get(key)
        if c is None:
            c = lib().sm_ctx_create(d)
            if not c:
                raise SnappyError(32, "no usable HIP device %d for snappy_mi355x" % d)
            _ctx[key] = c
        out.append(c)
    return (ctypes.c_void_p * len(out))(*out)


def _mode(mode):
    if mode not in MODES:
        raise ValueError("mode must be 'reference', 'fast' or 'dense'")
    return MODES[mode]


def maxlength_compressed(n):
    """Snappy.jl:80-82."""
    return lib().sm_max_compressed_length(int(n))


def parse32(buf, offset=0):
    """src/varint.jl:12-37 with a 0-based offset; returns (value, next_offset)."""
    a = _bytes(buf)
    v = ctypes.c_uint32(0)
    nx = ctypes.c_size_t(0)
    st = lib().sm_parse32(a.ctypes.data if a.size else None, a.size, int(offset), ctypes.byref(v), ctypes.byref(nx))
    if st:
        raise SnappyError(st)
    return v.value, nx.value


def encode32(value):
    """src/varint.jl:46-69; returns the varint bytes."""
    out = np.zeros(8, dtype=np.uint8)
    n = lib().sm_encode32(out.ctypes.data, int(value))
    return out[:n].tobytes()


def length_uncompressed(data):
    """Snappy.jl:90-92."""
    return parse32(data, 0)


_tls = threading.local()
_SCRATCH_MAX = 64 << 20  # single-call outputs up to this size land in a reused per-thread buffer


def _out_buffer(n):
    """(address, owner) of n writable bytes: the calling thread's reused scratch for outputs up
    to _SCRATCH_MAX (a single call's fixed cost is a few microseconds, so no allocation and no
    numpy address lookup per call), else a fresh array."""
    if n > _SCRATCH_MAX:
        a = np.empty(max(n, 1), dtype=np.uint8)
        return a.__array_interface__["data"][0], a
    buf = getattr(_tls, "buf", None)
    if buf is None or buf.size < n:
        buf = np.empty(max(n, 1 << 20), dtype=np.uint8)
        _tls.buf, _tls.ptr = buf, buf.__array_interface__["data"][0]
    return _tls.ptr, buf


def _in_arg(data):
    """(pointer argument, length, owner) of an input: bytes go to ctypes as they are (no copy)."""
    if isinstance(data, bytes):
        return (data if data else None), len(data), data
    a = _bytes(data)
    return (a.__array_interface__["data"][0] if a.size else None), a.size, a


def compress(data, mode="fast", device=0):
    """Snappy.jl:20-36 (and the String method :38), computed on the GPU."""
    src, n, keep = _in_arg(data)
    if n > 0xFFFFFFFF:
        raise SnappyError(16)
    cap = 32 + n + n // 6  # maxlength_compressed, Snappy.jl:80-82
    ptr, buf = _out_buffer(cap)
    ol = ctypes.c_size_t(cap)
    st = lib().sm_compress(context(device), src, n, ptr, ctypes.byref(ol), _mode(mode))
    if st:
        raise SnappyError(st)
    return ctypes.string_at(ptr, ol.value)


def find_match_length(buf, i1, i2, limit):
    """internal.jl:343-387 (0-based i1 < i2, inclusive limit); SnappyError where the
    reference would read past buf."""
    src = _bytes(buf)
    res = ctypes.c_size_t(0)
    st = lib().sm_find_match_length(src.ctypes.data if src.size else None, src.size, i1, i2, limit,
                                    ctypes.byref(res))
    if st:
        raise SnappyError(st)
    return res.value


def last_uncompress_path(device=0):
    """How the last uncompress() on this device decoded: 0 in order, 1 parallel fragments
    (block-structured stream), 2 parallel by origin pointers (copies cross 64 KiB blocks), 3 a
    large stream's first error found in parallel (its status returned, no output), 4 a small
    stream decoded by origin pointers entirely on the device."""
    return int(lib().sm_ctx_last_path(context(device)))


def set_small_decode(enable, device=0):
    """Diagnostic: path 4 (small streams on the device) on or off for uncompress() on this device."""
    st = lib().sm_ctx_set_small_decode(context(device), 1 if enable else 0)
    if st:
        raise SnappyError(st)


def set_split_compress(enable, device=0):
    """Diagnostic: compress() of small fast-mode inputs parses each 64 KiB fragment in parts on
    their own workgroups (on by default; the same bytes either way)."""
    st = lib().sm_ctx_set_split_compress(context(device), 1 if enable else 0)
    if st:
        raise SnappyError(st)


def last_compress_split(device=0):
    """Whether the last compress() on this device parsed its fragments in parts."""
    return int(lib().sm_ctx_last_compress_split(context(device))) == 1


def _declared_length(b):
    """The varint header's value (src/varint.jl:12-37), only to size the output: 0 when it does
    not parse (sm_uncompress then returns the reference's header error itself)."""
    v = 0
    for i in range(min(5, len(b))):
        c = b[i]
        v |= (c & 0x7F) << (7 * i)
        if c < 0x80:
            return v if v <= 0xFFFFFFFF else 0
    return 0


def uncompress(data, device=0):
    """Snappy.jl:46-52, computed on the GPU; raises SnappyError with the reference message."""
    src, n, keep = _in_arg(data)
    size = _declared_length(keep if isinstance(keep, bytes) else memoryview(keep))
    ptr, buf = _out_buffer(size)
    ol = ctypes.c_size_t(size)
    st = lib().sm_uncompress(context(device), src, n, ptr, ctypes.byref(ol))
    if st:
        raise SnappyError(st)
    return ctypes.string_at(ptr, ol.value)


# ---- batched host API ---------------------------------------------------------------

def pack_blocks(blocks):
    """list of byte strings -> (packed u8 array, u64 offsets, u32 lengths)."""
    lens = np.array([len(b) for b in blocks], dtype=np.uint32)
    offs = np.zeros(len(blocks), dtype=np.uint64)
    if len(blocks) > 1:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    buf = np.frombuffer(b"".join(bytes(b) for b in blocks), dtype=np.uint8) if blocks else np.zeros(0, np.uint8)
    return np.ascontiguousarray(buf), offs, lens


def slot_offsets(in_len):
    """Fixed output slots of max_compressed_length(len) bytes (16-B aligned)."""
    caps = (32 + in_len.astype(np.uint64) + in_len.astype(np.uint64) // 6 + 15) // 16 * 16
    offs = np.zeros(in_len.size, dtype=np.uint64)
    if in_len.size > 1:
        offs[1:] = np.cumsum(caps[:-1], dtype=np.uint64)
    return offs, caps


def compress_batch(blocks, mode="fast", device=0, devices=None):
    """Compress independent <=64 KiB blocks; returns a list of snappy streams (bytes).
    devices: a list of GPUs to shard the blocks over from this one process."""
    buf, in_off, in_len = pack_blocks(blocks)
    if np.any(in_len > BLOCK_SIZE):
        raise ValueError("batch blocks must be <= 65536 bytes")
    out_off, caps = slot_offsets(in_len)
    out = np.empty(int(out_off[-1] + caps[-1]) if len(blocks) else 1, dtype=np.uint8)
    out_len = np.zeros(len(blocks), dtype=np.uint32)
    if not blocks:
        return []
    args = (buf.ctypes.data, in_off.ctypes.data, in_len.ctypes.data, len(blocks), out.ctypes.data,
            out_off.ctypes.data, out_len.ctypes.data, _mode(mode))
    if devices is None:
        st = lib().sm_compress_batch(context(device), *args)
    else:  # one shard of the blocks per device, concurrently (sm_compress_batch_sharded)
        st = lib().sm_compress_batch_sharded(contexts(devices), len(devices), *args)
    if st:
        raise SnappyError(st)
    return [out[int(o): int(o) + int(l)].tobytes() for o, l in zip(out_off, out_len)]


def uncompress_batch(streams, capacities=None, device=0, devices=None):
    """Decode independent snappy streams; returns (list of bytes-or-None, status array).
    devices: as in compress_batch."""
    if not streams:
        return [], np.zeros(0, np.int32)
    buf, in_off, in_len = pack_blocks(streams)
    if capacities is None:
        caps = []
        for s in streams:
            try:
                caps.append(parse32(s)[0])
            except SnappyError:
                caps.append(0)
        capacities = caps
    cap = np.array(capacities, dtype=np.uint32)
    out_off = np.zeros(len(streams), dtype=np.uint64)
    if len(streams) > 1:
        out_off[1:] = np.cumsum(cap[:-1].astype(np.uint64), dtype=np.uint64)
    out = np.empty(max(int(cap.astype(np.uint64).sum()), 1), dtype=np.uint8)
    out_len = np.zeros(len(streams), dtype=np.uint32)
    status = np.zeros(len(streams), dtype=np.int32)
    args = (buf.ctypes.data, in_off.ctypes.data, in_len.ctypes.data, len(streams), out.ctypes.data,
            out_off.ctypes.data, cap.ctypes.data, out_len.ctypes.data, status.ctypes.data)
    if devices is None:
        st = lib().sm_uncompress_batch(context(device), *args)
    else:
        st = lib().sm_uncompress_batch_sharded(contexts(devices), len(devices), *args)
    if st:
        raise SnappyError(st)
    res = [out[int(o): int(o) + int(l)].tobytes() if s == 0 else None for o, l, s in zip(out_off, out_len, status)]
    return res, status


# ---- batched device API (torch tensors resident in HBM) -----------------------------

def _ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def _stream(stream, dev):
    import torch
    if stream is None:
        return torch.cuda.current_stream(dev).cuda_stream
    return stream.cuda_stream if hasattr(stream, "cuda_stream") else stream


def compress_batch_device(d_in, d_in_off, d_in_len, d_out, d_out_off, d_out_len, mode="fast", stream=None,
                          device=None):
    """All arguments are torch CUDA tensors (uint8 / int64 / int32).  Asynchronous on `stream`
    (a torch.cuda.Stream or raw hipStream_t int; default: torch's current stream)."""
    import torch
    dev = d_in.device.index if device is None else device
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    elif hasattr(stream, "cuda_stream"):
        stream = stream.cuda_stream
    st = lib().sm_compress_batch_device(context(dev), _ptr(d_in), _ptr(d_in_off), _ptr(d_in_len), d_in_len.numel(),
                                        _ptr(d_out), _ptr(d_out_off), _ptr(d_out_len), _mode(mode),
                                        ctypes.c_void_p(stream))
    if st:
        raise SnappyError(st)


def compress_fragments_device(d_in, d_in_off, d_in_len, d_out, d_out_off, d_out_len, total_len, mode="fast",
                              stream=None, device=None):
    """Fragments of ONE stream of total_len bytes (no per-fragment header; Q2 table size)."""
    import torch
    dev = d_in.device.index if device is None else device
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    elif hasattr(stream, "cuda_stream"):
        stream = stream.cuda_stream
    st = lib().sm_compress_fragments_device(context(dev), _ptr(d_in), _ptr(d_in_off), _ptr(d_in_len),
                                            d_in_len.numel(), _ptr(d_out), _ptr(d_out_off), _ptr(d_out_len),
                                            int(total_len), _mode(mode), ctypes.c_void_p(stream))
    if st:
        raise SnappyError(st)


def uncompress_batch_device(d_in, d_in_off, d_in_len, d_out, d_out_off, d_out_cap, d_out_len, d_status,
                            stream=None, device=None):
    import torch
    dev = d_in.device.index if device is None else device
    if stream is None:
        stream = torch.cuda.current_stream(dev).cuda_stream
    elif hasattr(stream, "cuda_stream"):
        stream = stream.cuda_stream
    st = lib().sm_uncompress_batch_device(context(dev), _ptr(d_in), _ptr(d_in_off), _ptr(d_in_len),
                                          d_in_len.numel(), _ptr(d_out), _ptr(d_out_off), _ptr(d_out_cap),
                                          _ptr(d_out_len), _ptr(d_status), ctypes.c_void_p(stream))
    if st:
        raise SnappyError(st)


def place_fragments_device(d_src, d_src_off, d_len, d_dst_off, d_dst, total_len, write_header, d_local_off=None,
                           d_status=None, stream=None, device=None):
    """Fragments of ONE stream at their offsets in it (sm_place_fragments_device): fragment b
    (d_len[b] bytes at d_src + d_src_off[b]) to d_dst + d_dst_off[b] - base, base = 0 with
    write_header (d_dst is the stream from byte 0; varint(total_len) is written there) or
    d_dst_off[0] (d_dst is this shard's byte range).  d_local_off (int64, optional) receives the
    fragments' offsets in d_dst; d_status (int32[1], optional, zeroed by the caller) turns
    SM_ERR_DEVICE on an error-mark length or a fragment past d_dst's end."""
    dev = d_dst.device.index if device is None else device
    nfrag = d_len.numel()
    nul = ctypes.c_void_p(0)
    st = lib().sm_place_fragments_device(context(dev), _ptr(d_src) if nfrag else nul, _ptr(d_src_off) if nfrag else nul,
                                         _ptr(d_len) if nfrag else nul, nfrag, _ptr(d_dst_off) if nfrag else nul,
                                         int(total_len), 1 if write_header else 0, _ptr(d_dst), d_dst.numel(),
                                         _ptr(d_local_off) if d_local_off is not None else nul,
                                         _ptr(d_status) if d_status is not None else nul,
                                         ctypes.c_void_p(_stream(stream, dev)))
    if st:
        raise SnappyError(st)


def uncompress_fragments_device(d_in, d_in_off, d_in_len, d_out, d_out_off, d_frag_len, d_out_len, d_status,
                                stream=None, device=None):
    """Fragments of ONE stream (no varint headers; sm_compress_fragments_device's output):
    fragment b must decode to exactly d_frag_len[b] bytes at d_out + d_out_off[b]."""
    dev = d_in.device.index if device is None else device
    st = lib().sm_uncompress_fragments_device(context(dev), _ptr(d_in), _ptr(d_in_off), _ptr(d_in_len),
                                              d_in_len.numel(), _ptr(d_out), _ptr(d_out_off), _ptr(d_frag_len),
                                              _ptr(d_out_len), _ptr(d_status), ctypes.c_void_p(_stream(stream, dev)))
    if st:
        raise SnappyError(st)


def validate_batch_device(d_in, d_in_off, d_in_len, d_status, stream=None, device=None):
    """d_status[b] = the status uncompress(block b) would return (no output written):
    batched snappy_validate_compressed_buffer."""
    dev = d_in.device.index if device is None else device
    st = lib().sm_validate_batch_device(context(dev), _ptr(d_in), _ptr(d_in_off), _ptr(d_in_len), d_in_len.numel(),
                                        _ptr(d_status), ctypes.c_void_p(_stream(stream, dev)))
    if st:
        raise SnappyError(st)


def uncompressed_length_batch_device(d_in, d_in_off, d_in_len, d_len, d_status, stream=None, device=None):
    """Batched length_uncompressed (Snappy.jl:90-92): the varint header of every block."""
    dev = d_in.device.index if device is None else device
    st = lib().sm_uncompressed_length_batch_device(context(dev), _ptr(d_in), _ptr(d_in_off), _ptr(d_in_len),
                                                   d_in_len.numel(), _ptr(d_len), _ptr(d_status),
                                                   ctypes.c_void_p(_stream(stream, dev)))
    if st:
        raise SnappyError(st)


def validate(data, device=0):
    """snappy_validate_compressed_buffer on the GPU: SM_OK (0) or the status uncompress(data)
    would raise with."""
    src = _bytes(data)
    return int(lib().sm_validate_compressed_buffer(context(device), src.ctypes.data if src.size else None, src.size))


def version():
    return lib().sm_version().decode()
