"""Randomised round trips of the fast compressor on the GPU: structured blocks of ragged sizes
(periodic patterns, runs, small alphabets, mutated text, random tails, planted copies at
random distances, long repeats whose copies run to the 255-byte token cap across many rows) through fast and dense mode, decoded on the GPU and compared byte-for-byte,
and every stream decoded by the CPU oracle (the reference's decoder restated) as well.  Fast mode
has no byte-parity target: validity under the reference's decoder is the bar."""
import os

import numpy as np
import pytest

from conftest import TESTDATA

pytestmark = pytest.mark.gpu

SLOT = 76490 + 8  # sm_max_compressed_length(65536) + slack


def gen_block(rng, text):
    n = int(rng.choice([rng.integers(1, 300), rng.integers(300, 65537), 65536]))
    kind = int(rng.integers(0, 8))
    if kind == 0:  # periodic pattern, random period
        b = np.resize(rng.integers(0, 256, int(rng.integers(1, 300)), dtype=np.uint8), n)
    elif kind == 1:  # runs of random bytes and lengths
        out, tot = [], 0
        while tot < n:
            L = int(rng.integers(1, 200))
            out.append(np.full(L, rng.integers(0, 256), np.uint8))
            tot += L
        b = np.concatenate(out)[:n]
    elif kind == 2:  # small alphabet
        b = rng.integers(0, int(rng.integers(2, 5)), n, dtype=np.uint8)
    elif kind == 3:  # mutated text
        s = int(rng.integers(0, text.size - n)) if text.size > n else 0
        b = text[s:s + n].copy()
        m = rng.random(b.size) < rng.choice([0.0, 0.001, 0.05])
        b[m] = rng.integers(0, 256, int(m.sum()), dtype=np.uint8)
    elif kind == 4:  # text, then a random tail
        s = int(rng.integers(0, max(1, text.size - n)))
        b = text[s:s + n].copy()
        cut = int(rng.integers(0, b.size + 1))
        b[cut:] = rng.integers(0, 256, b.size - cut, dtype=np.uint8)
    elif kind == 6:  # a random segment repeated, sparsely mutated: long extended copies
        seg = rng.integers(0, 256, int(rng.integers(17, 5000)), dtype=np.uint8)
        b = np.resize(seg, n).copy()
        m = rng.random(b.size) < rng.choice([0.0, 0.0005, 0.005])
        b[m] = rng.integers(0, 256, int(m.sum()), dtype=np.uint8)
    elif kind == 7:  # a text segment repeated 2-4 times (html_x_4-like)
        k = int(rng.integers(2, 5))
        L = max(1, n // k)
        s = int(rng.integers(0, max(1, text.size - L)))
        b = np.resize(text[s:s + L], n).copy()
    else:  # random bytes with planted copies (long and overlapping matches)
        b = rng.integers(0, 256, n, dtype=np.uint8)
        for _ in range(int(rng.integers(1, 40))):
            L, d = int(rng.integers(4, 300)), int(rng.integers(1, 2000))
            p = int(rng.integers(0, max(1, n - L)))
            for k in range(min(L, n - p)):
                if p + k - d >= 0:
                    b[p + k] = b[p + k - d]
    return np.ascontiguousarray(b[:n], dtype=np.uint8)


# more seeds for a longer run: SM_FUZZ_SEEDS=40
@pytest.mark.parametrize("seed", range(1, 1 + int(os.environ.get("SM_FUZZ_SEEDS", "3"))))
def test_fast_modes_random_structured_blocks(sm, oracle, gpu_available, seed):
    import torch
    rng = np.random.default_rng(seed)
    text = np.frombuffer(open(os.path.join(TESTDATA, "lcet10.txt"), "rb").read(), np.uint8)
    blocks = [gen_block(rng, text) for _ in range(1500)]
    lens = np.array([b.size for b in blocks], np.int64)
    off = np.zeros(len(blocks), np.int64)
    off[1:] = np.cumsum(lens[:-1])
    dev = torch.device("cuda", 0)
    d_in = torch.from_numpy(np.concatenate(blocks)).to(dev)
    in_off = torch.from_numpy(off).to(dev)
    in_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
    comp_off = torch.arange(len(blocks), dtype=torch.int64, device=dev) * SLOT
    for mode in ("fast", "dense"):
        d_comp = torch.zeros(len(blocks) * SLOT, dtype=torch.uint8, device=dev)
        comp_len = torch.zeros(len(blocks), dtype=torch.int32, device=dev)
        sm.compress_batch_device(d_in, in_off, in_len, d_comp, comp_off, comp_len, mode=mode)
        d_dec = torch.zeros_like(d_in)
        dec_len = torch.zeros_like(in_len)
        status = torch.zeros_like(in_len)
        sm.uncompress_batch_device(d_comp, comp_off, comp_len, d_dec, in_off, in_len, dec_len, status)
        torch.cuda.synchronize()
        assert int(status.abs().sum()) == 0
        assert torch.equal(dec_len, in_len)
        assert torch.equal(d_dec, d_in)
        cl = comp_len.cpu().numpy()
        assert (cl.astype(np.int64) <= 32 + lens + lens // 6 + 5).all()  # within maxlength + header
        # EVERY stream through the oracle (the restated Snappy.jl decoder), OpenMP over blocks
        host = d_comp.cpu().numpy()
        odec = np.zeros(int(lens.sum()), np.uint8)
        olen = np.zeros(len(blocks), np.uint32)
        ost = np.zeros(len(blocks), np.int32)
        oracle.uncompress_batch(host, comp_off.cpu().numpy().astype(np.uint64), cl.astype(np.uint32), odec,
                                off.astype(np.uint64), lens.astype(np.uint32), olen, ost,
                                nthreads=max(1, min(16, len(os.sched_getaffinity(0)))))
        assert not ost.any(), (mode, np.nonzero(ost)[0][:5])
        assert np.array_equal(olen, lens.astype(np.uint32))
        assert np.array_equal(odec, np.concatenate(blocks)), mode


@pytest.mark.parametrize("seed", range(1, 1 + int(os.environ.get("SM_FUZZ_SEEDS", "3"))))
def test_single_calls_random_structured_inputs(sm, oracle, gpu_available, seed):
    """The single-buffer calls on multi-fragment inputs built from the same structured blocks
    (1 B .. ~1 MiB): compress in parts (k_compress_sc_span, parts gather) equals the
    whole-fragment parse byte for byte in both fast modes, every stream decodes under the oracle,
    and uncompress (path 4, path 0, pinned-staging results) returns the input."""
    rng = np.random.default_rng(1000 + seed)
    text = np.frombuffer(open(os.path.join(TESTDATA, "lcet10.txt"), "rb").read(), np.uint8)
    try:
        for _ in range(12):
            parts = [gen_block(rng, text) for _ in range(int(rng.integers(1, 17)))]
            raw = np.concatenate(parts).tobytes()
            for mode in ("fast", "dense"):
                sm.set_split_compress(False)
                whole = sm.compress(raw, mode=mode)
                sm.set_split_compress(True)
                split = sm.compress(raw, mode=mode)
                assert split == whole, (mode, len(raw))
                assert oracle.uncompress(split) == raw
                assert sm.uncompress(split) == raw
    finally:
        sm.set_split_compress(True)


@pytest.mark.parametrize("seed", range(1, 1 + int(os.environ.get("SM_FUZZ_SEEDS", "3"))))
def test_small_path_foreign_streams(sm, oracle, gpu_available, seed):
    """Path 4 (sm_api.hip small_uncompress: index, parallel-run chain, fill, resolve) on seeded
    foreign streams -- literal/copy mixes with no 64 KiB block structure, from copy-heavy (512-byte
    index chunks) to literal-heavy (1 KiB chunks, deep entries), copy-4 offsets, 1-byte copies --
    and on single-byte mutations of them: output and status equal the oracle's."""
    from streams import build, random_ops
    rng = np.random.default_rng(4000 + seed)
    for _ in range(8):
        target = int(rng.integers(5_000, 1_200_000))
        ops = random_ops(rng, target, max_lit=int(rng.choice([8, 60, 300, 2000])),
                         max_off=int(rng.choice([4096, 65535, 300_000])),
                         long_lit_p=float(rng.choice([0.0, 0.02, 0.2])), near=int(rng.choice([64, 4096])))
        s, e = build(ops)
        assert oracle.uncompress(s) == e
        assert sm.uncompress(s) == e, len(e)
        for _ in range(3):
            bad = bytearray(s)
            bad[int(rng.integers(2, len(bad)))] = int(rng.integers(0, 256))
            bad = bytes(bad)
            st_o, out_o = oracle.uncompress_status(bad)
            try:
                st_g, out_g = 0, sm.uncompress(bad)
            except sm.SnappyError as exc:
                st_g, out_g = exc.code, None
            assert st_g == st_o
            if st_o == 0:
                assert out_g == out_o
