"""Hand-built snappy streams for decoder edge cases (test helper).

`build(ops)` encodes a list of ('lit', bytes) / ('copy', offset, length) operations with the
format's tags (src/internal.jl:16-19, 252-329: literal tags with 0..4 length bytes; copy-1
for len 4..11 and offset < 2048, copy-2 otherwise, copy-4 for offsets >= 65536) and returns
(stream, expected_output).  The expected output is the plain LZ77 meaning of the ops, the
semantics of decompress_all_tags! (src/internal.jl:411-466) on a valid stream.
"""
import numpy as np


def varint(n):
    out = bytearray()
    while n >= 0x80:
        out.append((n & 0x7F) | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def lit_tag(n):
    m = n - 1
    if m < 60:
        return bytes([m << 2])
    k = (m.bit_length() + 7) // 8
    return bytes([(59 + k) << 2]) + m.to_bytes(k, "little")


def copy_tag(offset, length):
    assert 1 <= length <= 64 and offset >= 1
    if 4 <= length < 12 and offset < 2048:
        return bytes([1 | ((length - 4) << 2) | ((offset >> 8) << 5), offset & 0xFF])
    if offset < 65536:
        return bytes([2 | ((length - 1) << 2)]) + offset.to_bytes(2, "little")
    return bytes([3 | ((length - 1) << 2)]) + offset.to_bytes(4, "little")


def build(ops):
    body = bytearray()
    out = bytearray()
    for op in ops:
        if op[0] == "lit":
            data = bytes(op[1])
            body += lit_tag(len(data)) + data
            out += data
        else:
            _, offset, length = op
            assert offset <= len(out)
            body += copy_tag(offset, length)
            for _ in range(length):
                out.append(out[-offset])
    return varint(len(out)) + bytes(body), bytes(out)


def random_ops(rng, target, max_lit=300, max_off=65535, long_lit_p=0.02, near=4096):
    """Seeded mix of literals (some long) and copies (any legal offset, len 1..64); half of
    the copies reach at most `near` bytes back."""
    ops, size = [], 0
    while size < target:
        if size == 0 or rng.random() < 0.3:
            n = int(rng.integers(201, 3000)) if rng.random() < long_lit_p else int(rng.integers(1, max_lit + 1))
            data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
            ops.append(("lit", data))
            size += n
        else:
            r = rng.random()
            if r < 0.3:
                off = int(rng.integers(1, min(size, 16) + 1))
            elif r < 0.8:
                off = int(rng.integers(1, min(size, near) + 1))
            else:
                off = int(rng.integers(1, min(size, max_off) + 1))
            ln = int(rng.integers(1, 65))
            ops.append(("copy", off, ln))
            size += ln
    return ops
