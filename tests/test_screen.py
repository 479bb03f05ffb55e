"""The incompressible screen (k_literal_screen, sm_compress_fast.hip): blocks whose content-defined
anchors (4-byte words hashing into the top 1/64) show (almost) no repeats are emitted as ONE literal -- header, emit_literal! tag
(src/internal.jl:271-284), the bytes -- by an aligned 16-B byte-shifting copy.  These tests put
that copy through every source/destination misalignment and ragged length, with and without the
varint header (fragments), check the exact literal-only size, that nothing outside a block's
output bytes is written, that the oracle (the restated Snappy.jl decoder) decodes every stream,
and that compressible and mixed blocks still take the parse.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _varint_len(n):
    k = 1
    while n >= 128:
        n >>= 7
        k += 1
    return k


def _lit_tag_len(n):
    return 1 if n - 1 < 60 else 2 if n - 1 < 256 else 3 if n - 1 < 65536 else 4


def _run(sm, blocks, in_shift, out_shift, header, mode="fast"):
    """Pack blocks at byte offsets shifted by in_shift[b] / out_shift[b] (any alignment) and
    compress them on the GPU; return host output buffer, offsets, sizes."""
    import torch
    dev = torch.device("cuda", 0)
    n = len(blocks)
    in_off, pos = [], 0
    for b, blk in enumerate(blocks):
        pos += in_shift[b]
        in_off.append(pos)
        pos += len(blk)
    inp = np.zeros(pos + 64, dtype=np.uint8)
    for b, blk in enumerate(blocks):
        inp[in_off[b]:in_off[b] + len(blk)] = np.frombuffer(blk, dtype=np.uint8)
    out_off, pos = [], 0
    for b, blk in enumerate(blocks):
        pos += 32 + out_shift[b]
        out_off.append(pos)
        pos += sm.maxlength_compressed(len(blk))
    outsz = pos + 64
    d_in = torch.from_numpy(inp).to(dev)
    d_in_off = torch.tensor(in_off, dtype=torch.int64, device=dev)
    d_in_len = torch.tensor([len(b) for b in blocks], dtype=torch.int32, device=dev)
    d_out = torch.full((outsz,), 0xA5, dtype=torch.uint8, device=dev)
    d_out_off = torch.tensor(out_off, dtype=torch.int64, device=dev)
    d_out_len = torch.zeros(n, dtype=torch.int32, device=dev)
    if header:
        sm.compress_batch_device(d_in, d_in_off, d_in_len, d_out, d_out_off, d_out_len, mode=mode)
    else:
        total = sum(len(b) for b in blocks)
        sm.compress_fragments_device(d_in, d_in_off, d_in_len, d_out, d_out_off, d_out_len, total, mode=mode)
    torch.cuda.synchronize()
    return d_out.cpu().numpy(), out_off, d_out_len.cpu().numpy().astype(np.int64)


def _check_untouched(out, out_off, lens):
    """Every byte outside [out_off[b], out_off[b] + lens[b]) still holds the 0xA5 canary."""
    mask = np.ones(out.size, dtype=bool)
    for o, l in zip(out_off, lens):
        mask[o:o + l] = False
    bad = np.nonzero(out[mask] != 0xA5)[0]
    assert bad.size == 0, "bytes written outside the streams: %d" % bad.size


@pytest.mark.parametrize("header", [True, False])
def test_literal_copy_every_alignment(sm, oracle, gpu_available, header):
    rng = np.random.default_rng(1234 + header)
    sizes = [65536, 65535, 65521, 8192, 8193, 40000, 16384 + 7, 65536 - 16, 12345, 65536]
    blocks, ish, osh = [], [], []
    for a in range(16):          # source misalignment
        for d in range(16):      # destination misalignment
            k = (16 * a + d) % len(sizes)
            blocks.append(rng.integers(0, 256, sizes[k], dtype=np.uint8).tobytes())
            ish.append(a)
            osh.append(d)
    out, out_off, lens = _run(sm, blocks, ish, osh, header)
    _check_untouched(out, out_off, lens)
    for b, blk in enumerate(blocks):
        n = len(blk)
        hv = _varint_len(n) if header else 0
        assert lens[b] == hv + _lit_tag_len(n) + n, (b, n, lens[b])
        s = out[out_off[b]:out_off[b] + lens[b]].tobytes()
        assert s[hv + _lit_tag_len(n):] == blk
        if header:
            assert oracle.uncompress(s) == blk
        else:  # a fragment: prefix the varint header and decode as a stream
            assert oracle.uncompress(bytes(sm.encode32(n)) + s) == blk


def test_screen_keeps_compressible_blocks(sm, oracle, gpu_available):
    """Text, structured data, half-random/half-text and runs take the parse (smaller than the input);
    so do constant blocks and short periods whose few distinct words all miss the anchor range
    (round 6: a block of 0x14 bytes was emitted as one literal -- too few anchors for random data)."""
    from conftest import read_testfile
    rng = np.random.default_rng(7)
    text = read_testfile("alice29.txt")[:65536]
    geo = read_testfile("geo.protodata")[:65536]
    rnd = rng.integers(0, 256, 65536, dtype=np.uint8).tobytes()
    mixed = rnd[:32768] + text[:32768]
    zeros_tail = rnd[:49152] + bytes(16384)
    blocks = [text, geo, mixed, zeros_tail, bytes(65536)]
    blocks += [bytes([c]) * 65536 for c in (0x14, 0x20, 0x41, 0x7f, 0xff)]
    blocks += [(bytes(rng.integers(0, 256, per, dtype=np.uint8)) * (65536 // per + 1))[:65536] for per in (2, 3, 5, 12)]
    out, out_off, lens = _run(sm, blocks, [0] * len(blocks), [0] * len(blocks), True)
    for b, blk in enumerate(blocks):
        s = out[out_off[b]:out_off[b] + lens[b]].tobytes()
        assert oracle.uncompress(s) == blk
        assert lens[b] < len(blk) * 0.95, (b, lens[b])


@pytest.mark.parametrize("fname", ["fireworks.jpeg", "paper-100k.pdf", "alice29.snappy"])
def test_screen_on_incompressible_corpus(sm, oracle, gpu_available, fname):
    """Real incompressible data: whatever the screen decides, the stream decodes and is no larger
    than the reference's own output + 0.1 %."""
    from conftest import read_testfile
    data = read_testfile(fname)
    blocks = [data[i:i + 65536] for i in range(0, len(data), 65536)]
    for mode in ("fast", "dense"):
        out, out_off, lens = _run(sm, blocks, [0] * len(blocks), [0] * len(blocks), True, mode)
        for b, blk in enumerate(blocks):
            s = out[out_off[b]:out_off[b] + lens[b]].tobytes()
            assert oracle.uncompress(s) == blk
            assert lens[b] <= len(oracle.compress(blk)) + len(blk) // 1000 + 8


def test_screen_long_range_repeats(sm, oracle, gpu_available):
    """repeats far apart (random content of period 4-48 KiB, a block made of
    two copies of one random 32 KiB half, a record file with a 64-B header every 1 KiB) are
    compressed, not screened as literal: each fast-mode stream is at most 1.1x the reference's
    (oracle) size + 64 B and decodes under the oracle."""
    rng = np.random.default_rng(2024)
    blocks, names = [], []
    for period in (4096, 8192, 16384, 32768, 49152):
        seg = rng.integers(0, 256, period, dtype=np.uint8).tobytes()
        blocks.append((seg * (65536 // period + 1))[:65536])
        names.append("period %d" % period)
    half = rng.integers(0, 256, 32768, dtype=np.uint8).tobytes()
    blocks.append(half + half)
    names.append("two halves")
    header = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
    rec = b"".join(header + rng.integers(0, 256, 960, dtype=np.uint8).tobytes() for _ in range(64))
    blocks.append(rec)
    names.append("64-B header every 1 KiB")
    out, out_off, lens = _run(sm, blocks, [0] * len(blocks), [0] * len(blocks), True)
    for b, blk in enumerate(blocks):
        s = out[out_off[b]:out_off[b] + lens[b]].tobytes()
        assert oracle.uncompress(s) == blk, names[b]
        ref = len(oracle.compress(blk))
        print("%-26s fast %6d  reference %6d" % (names[b], lens[b], ref))
        assert lens[b] <= 1.1 * ref + 64, (names[b], lens[b], ref)
