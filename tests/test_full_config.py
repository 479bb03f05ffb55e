"""Parity at the bench's full sizes (BASELINE.json configs 2-5), through the C ABI on the GPU.

* configs 2/3: the exact 10,000 text windows bench.py times (default_rng(0x5EED)), compressed in
  fast and dense mode on the GPU; EVERY stream is decoded by the oracle (the restated Snappy.jl
  decoder, OpenMP over blocks) and by the GPU decoder, and both must equal the input bytes.
* config 4: the 10,000 uniform random blocks (default_rng(0x5EED + 1)), same checks, plus the
  literal-only size (65,542 B per block at most 3 B over the input + header).
* reference mode: byte-identical to the oracle on all 10,000 blocks of config 2.
* the reference's max-blowup input (test/runtests.jl:147-154, seeded) and hand-built streams
  with valid copy-4 tags / offsets >= 65,536 through sm_uncompress (src/internal.jl:19,26-28:
  the decoder must not rely on the absence of long back-references).
* config 5 as fragments: sm_compress_fragments_device + sm_uncompress_fragments_device over the
  644 MiB stream; the stream placed on the device decodes under the oracle.
"""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT
from streams import build

pytestmark = pytest.mark.gpu
SLOT = 76496
BLOCK = 65536


def _bench():
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    import bench
    return bench


def _threads():
    return max(1, min(16, len(os.sched_getaffinity(0))))


def _gpu_batch(sm, blocks, mode):
    """Compress [nblk, 65536] blocks on the GPU (device API), decode on the GPU; return host
    copies of the slots, sizes, GPU-decoded bytes and statuses."""
    import torch
    nblk = blocks.shape[0]
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(blocks.reshape(-1)).to(dev)
    off = torch.arange(nblk, dtype=torch.int64, device=dev) * BLOCK
    ln = torch.full((nblk,), BLOCK, dtype=torch.int32, device=dev)
    d_c = torch.zeros(nblk * SLOT, dtype=torch.uint8, device=dev)
    c_off = torch.arange(nblk, dtype=torch.int64, device=dev) * SLOT
    c_len = torch.zeros(nblk, dtype=torch.int32, device=dev)
    sm.compress_batch_device(d_in, off, ln, d_c, c_off, c_len, mode=mode)
    d_d = torch.zeros(nblk * BLOCK, dtype=torch.uint8, device=dev)
    d_len = torch.zeros(nblk, dtype=torch.int32, device=dev)
    st = torch.full((nblk,), -1, dtype=torch.int32, device=dev)
    sm.uncompress_batch_device(d_c, c_off, c_len, d_d, off, ln, d_len, st)
    torch.cuda.synchronize()
    return d_c.cpu().numpy(), c_len.cpu().numpy().astype(np.uint32), d_d.cpu().numpy(), st.cpu().numpy(), \
        d_len.cpu().numpy()


def _oracle_decode(oracle, comp, comp_len, nblk):
    c_off = np.arange(nblk, dtype=np.uint64) * SLOT
    out = np.zeros(nblk * BLOCK, dtype=np.uint8)
    o_off = np.arange(nblk, dtype=np.uint64) * BLOCK
    cap = np.full(nblk, BLOCK, dtype=np.uint32)
    olen = np.zeros(nblk, dtype=np.uint32)
    st = np.zeros(nblk, dtype=np.int32)
    oracle.uncompress_batch(comp, c_off, comp_len, out, o_off, cap, olen, st, nthreads=_threads())
    return out, st, olen


@pytest.fixture(scope="module")
def text10k():
    return _bench().text_blocks(10000, 0x5EED)


@pytest.fixture(scope="module")
def random10k():
    return _bench().random_blocks(10000, 0x5EED + 1)


@pytest.mark.parametrize("mode", ["fast", "dense"])
def test_config2_text_full_batch(sm, oracle, gpu_available, text10k, mode):
    comp, clen, gdec, gst, glen = _gpu_batch(sm, text10k, mode)
    flat = text10k.reshape(-1)
    assert not gst.any() and (glen == BLOCK).all()
    assert np.array_equal(gdec, flat), "GPU decode of GPU streams"
    odec, ost, olen = _oracle_decode(oracle, comp, clen, text10k.shape[0])
    assert not ost.any() and (olen == BLOCK).all()
    bad = np.nonzero((odec.reshape(-1, BLOCK) != text10k).any(axis=1))[0]
    assert bad.size == 0, "oracle decode differs on blocks %s" % bad[:10]
    ratio = clen.astype(np.int64).sum() / flat.size
    assert ratio < 0.61, ratio  # the reference's own parse gives 0.606 on these blocks


@pytest.mark.parametrize("mode", ["fast", "dense"])
def test_config4_random_full_batch(sm, oracle, gpu_available, random10k, mode):
    comp, clen, gdec, gst, glen = _gpu_batch(sm, random10k, mode)
    assert not gst.any() and np.array_equal(gdec, random10k.reshape(-1))
    odec, ost, _ = _oracle_decode(oracle, comp, clen, random10k.shape[0])
    assert not ost.any() and np.array_equal(odec, random10k.reshape(-1))
    # (nearly) literal-only: header + a few literal tags (and the odd chance match); the
    # reference emits 65,542 B per block.  Bound: 0.1 % over the input.
    assert clen.max() <= 65536 + 65, clen.max()


def test_reference_mode_full_batch_byte_identical(sm, oracle, gpu_available, text10k):
    sub = np.ascontiguousarray(text10k)
    comp, clen, gdec, gst, _ = _gpu_batch(sm, sub, "reference")
    n = sub.shape[0]
    inp = sub.reshape(-1)
    o_comp = np.zeros(n * SLOT, dtype=np.uint8)
    o_len = np.zeros(n, dtype=np.uint32)
    oracle.compress_batch(inp, np.arange(n, dtype=np.uint64) * BLOCK, np.full(n, BLOCK, np.uint32), o_comp,
                          np.arange(n, dtype=np.uint64) * SLOT, o_len, compat=False, nthreads=_threads())
    assert np.array_equal(o_len, clen)
    for b in range(n):
        s = b * SLOT
        assert np.array_equal(comp[s:s + clen[b]], o_comp[s:s + o_len[b]]), b
    assert not gst.any() and np.array_equal(gdec, inp)


def test_max_blowup_on_gpu(sm, oracle, gpu_available):
    # test/runtests.jl:147-154: 20,000 random u32 then the same bytes reversed (seeded here)
    rng = np.random.default_rng(3)
    raw = rng.integers(0, 2**32, 20000, dtype=np.uint32).tobytes()
    raw = raw + raw[::-1]
    for mode in ("reference", "fast", "dense"):
        a = sm.compress(raw, mode=mode)
        if mode == "reference":
            assert a == oracle.compress(raw)
        assert a != raw
        assert oracle.uncompress(a) == raw
        assert sm.uncompress(a) == raw


def _copy4_streams(seed, n_streams=6):
    """Valid streams whose copies reach >= 65,536 bytes back (copy-4 tags, src/internal.jl:19)."""
    rng = np.random.default_rng(seed)
    out = []
    for k in range(n_streams):
        base = rng.integers(0, 256, 70000 + 4000 * k, dtype=np.uint8).tobytes()
        ops = [("lit", base)]
        size = len(base)
        n4 = 0
        while size < 300000:
            r = rng.random()
            if r < 0.4:
                off = int(rng.integers(65536, size + 1))          # copy-4
                n4 += 1
            elif r < 0.6:
                off = int(rng.integers(1, 65536))
            else:
                n = int(rng.integers(1, 200))
                ops.append(("lit", rng.integers(0, 256, n, dtype=np.uint8).tobytes()))
                size += n
                continue
            ln = int(rng.integers(1, 65))
            ops.append(("copy", off, ln))
            size += ln
        out.append(build(ops) + (n4,))
    return out


def test_copy4_long_offsets_uncompress(sm, oracle, gpu_available):
    for stream, expect, n4 in _copy4_streams(17):
        assert n4 > 100
        assert oracle.uncompress(stream) == expect
        assert sm.uncompress(stream) == expect
        assert sm.validate(stream) == 0


def test_config5_fragments_device_roundtrip(sm, oracle, gpu_available):
    """Config 5 through the fragment entry points the sharded bench uses (all fragments on one
    GPU here): the stream placed on the device by sm_place_fragments_device equals the checker's
    concatenation of the fragment slots behind the header and decodes under the oracle; the
    fragment decoder restores every fragment from the placed stream."""
    import torch
    bench = _bench()
    big = bench.large_corpus()
    sh = bench.StreamShard(big, 0, (big.size + BLOCK - 1) // BLOCK, torch.device("cuda", 0))
    sh.compress(sm)
    from importlib import import_module
    D = import_module("snappy_jl_amd.dist")
    sh.index(D, 0, 1)
    sh.place(sm)
    torch.cuda.synchronize()
    assert int(sh.place_status.item()) == 0
    placed = sh.d_stream[: sh.range_bytes()].cpu().numpy().tobytes()
    assert len(placed) == int(sh.stream_len.item())
    hl = D.varint32(big.size)
    lens = sh.comp_len.cpu().numpy().astype(np.int64)
    comp = sh.d_comp.cpu().numpy()
    stream = bytearray(hl)
    for f, n in enumerate(lens):
        stream += comp[f * SLOT: f * SLOT + n].tobytes()
    assert placed == bytes(stream)
    assert oracle.uncompress(placed) == big.tobytes()
    sh.d_dec.fill_(0)
    sh.uncompress(sm)
    torch.cuda.synchronize()
    assert int(sh.status.abs().sum()) == 0
    assert torch.equal(sh.d_dec, sh.d_in)
