"""GPU parity tests: the HIP path (through the C ABI) against the oracle on the same inputs.

* reference mode: compressed bytes identical to the oracle (= Snappy.jl) -- whole-buffer API
  (multi-fragment streams, quirk Q2) and batched 64 KiB blocks;
* fast mode: every stream decodes bit-exactly under the oracle decoder and libsnappy;
* decompress: output and status code identical to the oracle, incl. corrupted streams and
  a seeded mutation fuzz (first error in stream order, F6 leniencies).
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import ROOT, ROUNDTRIP_FILES, read_testfile

pytestmark = pytest.mark.gpu

GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))


def blocks_of(data, size=65536):
    return [data[i:i + size] for i in range(0, len(data), size)] or [b""]


@pytest.fixture(scope="module")
def corpus():
    return {f: read_testfile(f) for f in sorted(GOLDEN["corpus"])}


# ---- reference mode -------------------------------------------------------------------

@pytest.mark.parametrize("fname", sorted(GOLDEN["corpus"]))
def test_reference_mode_whole_file_matches_golden(sm, gpu_available, fname):
    raw = read_testfile(fname)
    out = sm.compress(raw, mode="reference")  # Snappy.jl compress(), multi-fragment, Q2 table
    g = GOLDEN["corpus"][fname]
    assert len(out) == g["c_reference"]
    assert hashlib.sha256(out).hexdigest() == g["sha256_reference"]


def test_reference_mode_batched_blocks(sm, oracle, gpu_available, corpus):
    blocks = []
    for raw in corpus.values():
        blocks.extend(blocks_of(raw))
    outs = sm.compress_batch(blocks, mode="reference")
    for blk, out in zip(blocks, outs):
        assert out == oracle.compress(blk)


def test_reference_mode_edge_strings(sm, oracle, gpu_available):
    from golden.make_golden import EDGE_STRINGS
    for s, g in zip(EDGE_STRINGS, GOLDEN["edge_strings"]):
        out = sm.compress(s, mode="reference")
        assert hashlib.sha256(out).hexdigest() == g["sha256_reference"]
        assert sm.uncompress(out) == s
    assert sm.compress("abc", mode="reference") == bytes.fromhex("0308616263")      # String method, Snappy.jl:38


def test_reference_mode_small_sizes(sm, oracle, gpu_available):
    rng = np.random.default_rng(11)
    blocks = []
    for n in list(range(0, 80)) + [255, 256, 257, 4095, 4096, 16383, 16384, 16385, 65535, 65536]:
        kind = n % 3
        if kind == 0:
            blk = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        elif kind == 1:
            blk = (b"abcab" * (n // 5 + 1))[:n]
        else:
            blk = rng.integers(0, 4, n, dtype=np.uint8).tobytes()
        blocks.append(blk)
    outs = sm.compress_batch(blocks, mode="reference")
    for blk, out in zip(blocks, outs):
        assert out == oracle.compress(blk), len(blk)


def test_reference_mode_dictionary_streams(sm, oracle, gpu_available):
    from test_oracle import dictionary_stream
    rng = np.random.default_rng(0x5EED)
    for _ in range(6):
        raw = dictionary_stream(rng, 1 << 14)
        assert sm.compress(raw, mode="reference") == oracle.compress(raw)


def test_reference_mode_fragments_device(sm, oracle, gpu_available):
    """Fragments of one stream (sharded-stream building block, dist.py): device output equals
    Snappy.jl's block loop (no headers, Q2 table size from the total length)."""
    import torch
    raw = read_testfile("html_x_4") + read_testfile("urls.10K")[:70000]
    total = len(raw)
    offs = list(range(0, total, 65536))
    lens = [min(65536, total - o) for o in offs]
    dev = torch.device("cuda", 0)
    d_in = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(dev)
    d_off = torch.tensor(offs, dtype=torch.int64, device=dev)
    d_len = torch.tensor(lens, dtype=torch.int32, device=dev)
    slot = 76496
    d_out = torch.empty(slot * len(offs), dtype=torch.uint8, device=dev)
    d_ooff = torch.arange(len(offs), dtype=torch.int64, device=dev) * slot
    d_olen = torch.zeros(len(offs), dtype=torch.int32, device=dev)
    sm.compress_fragments_device(d_in, d_off, d_len, d_out, d_ooff, d_olen, total, mode="reference")
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    ol = d_olen.cpu().numpy()
    frags = [out[i * slot: i * slot + int(ol[i])].tobytes() for i in range(len(offs))]
    for i, (o, l) in enumerate(zip(offs, lens)):
        assert frags[i] == oracle.compress_fragment(raw[o:o + l], total)
    assert oracle.encode32(total) + b"".join(frags) == oracle.compress(raw)


def test_reference_mode_block_end_exact(sm, oracle, gpu_available):
    """k_compress_exact reads the block in place through a buffer resource bounded at exactly
    n bytes: matches that run to the block's last byte, blocks of every length mod 4, at every
    address mod 4, with the block ending at the end of the device tensor."""
    import torch
    dev = torch.device("cuda", 0)
    rng = np.random.default_rng(17)
    for n in (65536, 65535, 65534, 65533, 4099, 1029, 31):
        for lead in (0, 1, 2, 3):
            pat = rng.integers(0, 256, 7, dtype=np.uint8).tobytes()
            head = rng.integers(0, 256, n // 3, dtype=np.uint8).tobytes()
            blk = (head + pat * (n // 7 + 1))[:n]  # a run of copies to the very end
            buf = bytes(lead) + blk
            d_in = torch.frombuffer(bytearray(buf), dtype=torch.uint8).to(dev)
            d_off = torch.tensor([lead], dtype=torch.int64, device=dev)
            d_len = torch.tensor([n], dtype=torch.int32, device=dev)
            d_out = torch.empty(76496, dtype=torch.uint8, device=dev)
            d_ooff = torch.zeros(1, dtype=torch.int64, device=dev)
            d_olen = torch.zeros(1, dtype=torch.int32, device=dev)
            sm.compress_batch_device(d_in, d_off, d_len, d_out, d_ooff, d_olen, mode="reference")
            torch.cuda.synchronize()
            out = d_out[:int(d_olen.item())].cpu().numpy().tobytes()
            assert out == oracle.compress(blk), (n, lead)


def _colliding_words(tbits, count, seed):
    """`count` distinct 4-byte words (little-endian u32) whose reference hash
    (w * 0x1e35a7bd) >> (32 - tbits) (src/internal.jl:94) is one and the same bucket."""
    rng = np.random.default_rng(seed)
    w = rng.integers(0, 2**32, 1 << 22, dtype=np.uint64)
    h = ((w * 0x1E35A7BD) & 0xFFFFFFFF) >> (32 - tbits)
    target = h[0]
    sel = np.unique(w[h == target])[:count]
    assert sel.size == count
    return sel.astype(np.uint32)


def test_reference_mode_same_bucket_blocks(sm, oracle, gpu_available):
    """Every probe of a batched step lands in one hash bucket (so the 64 lanes of one
    ds_mskor_rtn_b32 share an address): the byte-identical parse takes each lane's sequential
    candidate from the ascending-lane service order (sm_compress.hip), now guarded by cand < ip.
    Byte parity with the oracle on constant blocks, blocks of one word repeated at every
    alignment, and blocks of random sequences of words that share one bucket
    (src/internal.jl:190-193)."""
    rng = np.random.default_rng(0xB0C)
    words = _colliding_words(14, 8, 5)
    blocks = [bytes(65536), b"\x61" * 65536, b"\x61" * 40000 + bytes(25536)]
    for k in (2, 4, 8):  # sequences over k colliding words: every aligned position is one bucket
        seq = rng.integers(0, k, 16384)
        blocks.append(words[seq].astype("<u4").tobytes())
    for n in (65536, 65535, 20001, 4097):
        seq = rng.integers(0, 3, (n + 3) // 4)
        body = words[seq].astype("<u4").tobytes()
        lead = rng.integers(0, 256, 3, dtype=np.uint8).tobytes()
        blocks.append((lead + body)[:n])  # the same words at a shifted alignment
    # long runs of one colliding word between random bytes (deep copies after dense probes)
    parts = []
    while sum(map(len, parts)) < 65536:
        parts.append(rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8).tobytes())
        parts.append(words[int(rng.integers(0, 8))].astype("<u4").tobytes() * int(rng.integers(1, 200)))
    blocks.append(b"".join(parts)[:65536])
    outs = sm.compress_batch(blocks, mode="reference")
    for i, (blk, out) in enumerate(zip(blocks, outs)):
        assert out == oracle.compress(blk), i
        assert oracle.uncompress(out) == blk


# ---- fast mode --------------------------------------------------------------------------

FAST_MODES = ["fast", "dense"]


@pytest.mark.parametrize("mode", FAST_MODES)
@pytest.mark.parametrize("fname", ROUNDTRIP_FILES)
def test_fast_mode_roundtrip_whole_file(sm, oracle, libsnappy, gpu_available, fname, mode):
    raw = read_testfile(fname)
    out = sm.compress(raw, mode=mode)
    assert oracle.uncompress(out) == raw
    assert libsnappy.uncompress(out) == raw
    assert sm.uncompress(out) == raw


# per-file size bounds against the reference's own stream (the oracle = Snappy.jl's parse):
# dense mode compares both candidates of every copy over 16 bytes, as the reference's extension
# does for its one candidate (internal.jl:211-239); fast mode takes one by the SC_FAR rule
SIZE_BOUND = {"dense": 1.01, "fast": 1.04}


@pytest.mark.parametrize("mode", FAST_MODES)
def test_fast_mode_sizes_per_corpus_file(sm, oracle, gpu_available, mode):
    """every corpus file (test/runtests.jl:8-24 and the benchmark files) is at
    most SIZE_BOUND[mode] x the reference's stream + 64 B (profiles/r04_fast_sizes.txt)."""
    files = sorted(set(ROUNDTRIP_FILES + ["sample-tweet.json", "html_x_4"]))
    worst = 0.0
    for f in files:
        raw = read_testfile(f)
        got, ref = len(sm.compress(raw, mode=mode)), len(oracle.compress(raw))
        worst = max(worst, got / ref)
        print("%-18s %s %8d  reference %8d  (%.4f)" % (f, mode, got, ref, got / ref))
        assert got <= SIZE_BOUND[mode] * ref + 64, (f, got, ref)
    print("worst %.4f" % worst)


@pytest.mark.parametrize("mode", FAST_MODES)
def test_fast_mode_deterministic(sm, gpu_available, corpus, mode):
    """The parse has no order-dependent state: repeated launches give identical bytes."""
    blocks = []
    for raw in corpus.values():
        blocks.extend(blocks_of(raw))
    assert sm.compress_batch(blocks, mode=mode) == sm.compress_batch(blocks, mode=mode)


@pytest.mark.parametrize("mode", FAST_MODES)
def test_fast_mode_batched_roundtrip(sm, oracle, libsnappy, gpu_available, corpus, mode):
    rng = np.random.default_rng(5)
    blocks = []
    for raw in corpus.values():
        blocks.extend(blocks_of(raw))
    # sizes at the parse's chunk (256 B) and round (30 x 256 B fast, 15 x 256 B dense) boundaries;
    # k = 2, 3 rounds: the prologue hashes rounds 0 and 1, the parse waves the later ones
    edges = [k * m + d for m in (256, 3840, 7680) for k in (1, 2, 3, 17) for d in (-1, 0, 1) if 0 < k * m + d <= 65536]
    for n in list(range(0, 70)) + edges + [65535, 65536]:
        blocks.append(rng.integers(0, 3, n, dtype=np.uint8).tobytes())
    for n in edges[:6]:
        blocks.append(rng.integers(0, 256, n, dtype=np.uint8).tobytes())
    blocks.append(b"\x00" * 65536)
    blocks.append(rng.integers(0, 256, 65536, dtype=np.uint8).tobytes())
    outs = sm.compress_batch(blocks, mode=mode)
    for blk, out in zip(blocks, outs):
        assert oracle.uncompress(out) == blk
        assert libsnappy.uncompress(out) == blk
    ratio = sum(map(len, outs)) / sum(map(len, blocks))
    ref = sum(len(oracle.compress(b)) for b in blocks) / sum(map(len, blocks))
    assert ratio < ref * 1.10, (ratio, ref)   # fast parse stays within 10% of the reference size


@pytest.mark.parametrize("mode", FAST_MODES)
def test_fast_mode_largest_superchunk_outputs(sm, oracle, gpu_available, mode):
    """Blocks whose 1 KiB super-chunks come out as large as they can (k_compress_sc's staging
    slot holds 1,088 bytes; the bound is 1,040): literal runs of 61-64 bytes, each with a 2-byte
    tag, between short copies from more than 2 KiB back (3-byte tags), at every phase of the
    super-chunk grid, and runs that straddle lanes and super-chunks.  Every stream decodes under
    the oracle and is at most one literal of its block."""
    rng = np.random.default_rng(0x5107)
    base = rng.integers(0, 256, 4096, dtype=np.uint8).tobytes()
    blocks = []
    for run in (61, 62, 64, 60, 59):
        for phase in (0, 1, 7, 333):
            parts = [base, rng.integers(0, 256, phase, dtype=np.uint8).tobytes()]
            n = sum(map(len, parts))
            while n < 65536:
                lit = rng.integers(0, 256, run, dtype=np.uint8).tobytes()
                src = int(rng.integers(0, 4096 - 8))
                parts += [lit, base[src:src + 4]]
                n += run + 4
            blocks.append(b"".join(parts)[:65536])
    outs = sm.compress_batch(blocks, mode=mode)
    for blk, out in zip(blocks, outs):
        assert oracle.uncompress(out) == blk
        assert len(out) <= 3 + 3 + len(blk)


def superchunk_sizes(stream, sc=1024):
    """Output bytes per 1 KiB input super-chunk of a fast-mode stream: every tag (with its literal
    bytes) counted in the super-chunk where its input starts.  In k_compress_sc's streams no tag
    crosses a super-chunk end (copies stop there, literal runs are not merged across it), so these
    are the sizes the super-chunks had in their staging slots."""
    pos, ip = 0, 0
    while stream[ip] & 0x80:
        ip += 1
    ip += 1
    sizes = {}
    while ip < len(stream):
        c, start, tip = stream[ip], pos, ip
        kind = c & 3
        if kind == 0:
            n = c >> 2
            if n < 60:
                ip += 1
                n += 1
            else:
                k = n - 59
                n = int.from_bytes(stream[ip + 1: ip + 1 + k], "little") + 1
                ip += 1 + k
            ip += n
            pos += n
        else:
            ip += {1: 2, 2: 3, 3: 5}[kind]
            pos += 4 + ((c >> 2) & 7) if kind == 1 else (c >> 2) + 1
        s = start // sc
        assert (pos - 1) // sc == s, "a tag crosses a super-chunk end"
        sizes[s] = sizes.get(s, 0) + ip - tip
    return sizes


@pytest.mark.parametrize("mode", FAST_MODES)
def test_fast_mode_superchunk_bound_reached(sm, oracle, gpu_available, mode):
    """The staging slot's bound, reached: one super-chunk of each block is 61-64-byte
    literal runs (2-byte tags) between 4-byte copies from more than 2 KiB back (3-byte tags), the
    rest of the block a repeat, so the block keeps its parse (no whole-block literal fallback)
    and its stream shows every super-chunk's staged size.  The largest reaches the analytic bound
    of 1,040 bytes to within a few bytes and stays within kScSlot - 24 = 1,064."""
    rng = np.random.default_rng(0x5108)
    base = rng.integers(0, 256, 4096, dtype=np.uint8).tobytes()
    blocks = []
    for run in (61, 62, 63, 64):
        for phase in (0, 5, 31, 60):
            worst = [rng.integers(0, 256, phase, dtype=np.uint8).tobytes()]
            n = phase
            while n < 2048 + 128:
                src = int(rng.integers(0, 2048 - 8))
                worst += [rng.integers(0, 256, run, dtype=np.uint8).tobytes(), base[src:src + 4]]
                n += run + 4
            head = base + b"".join(worst)[:2048]  # the worst pattern over super-chunks 4 and 5
            blocks.append(head + base[:4096] * ((65536 - len(head)) // 4096 + 1))
    blocks = [b[:65536] for b in blocks]
    outs = sm.compress_batch(blocks, mode=mode)
    best = 0
    for blk, out in zip(blocks, outs):
        assert oracle.uncompress(out) == blk
        assert len(out) < len(blk) // 2  # the parse was kept
        sz = superchunk_sizes(out)
        assert max(sz.values()) <= 1040
        best = max(best, sz.get(4, 0), sz.get(5, 0))
    assert best >= 1030, best


# ---- decompress -------------------------------------------------------------------------

def test_decompress_corpus_and_golden(sm, oracle, libsnappy, gpu_available, corpus):
    streams = [oracle.compress(raw) for raw in corpus.values()]
    streams.append(read_testfile("alice29.snappy"))
    for s in streams:
        assert sm.uncompress(s) == oracle.uncompress(s)


def test_decompress_batched_blocks(sm, oracle, gpu_available, corpus):
    streams = []
    for raw in corpus.values():
        streams.extend(oracle.compress(b) for b in blocks_of(raw))
    outs, status = sm.uncompress_batch(streams)
    assert not status.any()
    for s, o in zip(streams, outs):
        assert o == oracle.uncompress(s)


@pytest.mark.parametrize("ndev", [2, 3])
def test_sharded_host_batches(sm, oracle, gpu_available, corpus, ndev):
    # sm_{,un}compress_batch_sharded: one context per shard (all on device 0 here), shards
    # rebased and run from concurrent host threads; results equal the single-context calls
    blocks = []
    for raw in corpus.values():
        blocks.extend(blocks_of(raw))
    blocks += [b"", b"a", bytes(range(256)) * 7]
    devs = [0] * ndev
    for mode in ("reference", "fast"):
        outs = sm.compress_batch(blocks, mode=mode, devices=devs)
        assert outs == sm.compress_batch(blocks, mode=mode)
        if mode == "reference":
            assert outs == [oracle.compress(b) for b in blocks]
    streams = [oracle.compress(b) for b in blocks]
    streams[5] = streams[5][:-3]  # a truncated stream: its own status, the rest decode
    dec, status = sm.uncompress_batch(streams, devices=devs)
    ref_dec, ref_status = sm.uncompress_batch(streams)
    assert list(status) == list(ref_status) and status[5] != 0 and not np.delete(status, 5).any()
    assert dec == ref_dec
    for i, (b, d) in enumerate(zip(blocks, dec)):
        assert d == (None if i == 5 else b)


def _status(sm, data):
    try:
        return 0, sm.uncompress(data)
    except sm.SnappyError as e:
        return e.code, None


def test_decompress_corrupted_matches_oracle(sm, oracle, gpu_available):
    from test_oracle import corrupted_cases
    for c in corrupted_cases(oracle):
        st_o, out_o = oracle.uncompress_status(c)
        st_g, out_g = _status(sm, c)
        assert st_o != 0
        assert (st_g, out_g) == (st_o, out_o)


def test_decompress_leniencies(sm, gpu_available, oracle):
    good = oracle.compress(b"hello hello hello hello")
    assert sm.uncompress(good + b"\x07") == b"hello hello hello hello"
    assert sm.uncompress(b"\x00\x00") == b""
    assert sm.uncompress(b"\x00") == b""
    assert _status(sm, b"\x00\x00\x00")[0] == 21
    assert _status(sm, bytes([0x40, 0x12, 0x00, 0x00]))[0] == 19


def _fuzz_cases(oracle, count, seed):
    """Seeded byte flips / truncations / extensions of valid streams."""
    rng = np.random.default_rng(seed)
    base = [oracle.compress(read_testfile(f)[:4096]) for f in ("html", "alice29.txt", "kppkn.gtb", "urls.10K")]
    base += [oracle.compress(b"ab" * 700), oracle.compress(bytes(range(256)) * 3)]
    cases = []
    for i in range(count):
        s = bytearray(base[i % len(base)])
        kind = rng.integers(0, 4)
        if kind == 0:
            for _ in range(int(rng.integers(1, 4))):
                s[int(rng.integers(0, len(s)))] = int(rng.integers(0, 256))
        elif kind == 1:
            s = s[: int(rng.integers(0, len(s)))]
        elif kind == 2:
            s += rng.integers(0, 256, int(rng.integers(1, 6)), dtype=np.uint8).tobytes()
        else:
            p = int(rng.integers(1, len(s)))
            s[p] = int(rng.integers(0, 256))
            s = s[: max(1, len(s) - int(rng.integers(0, 8)))]
        cases.append(bytes(s))
    return cases


def test_decompress_mutation_fuzz_batched(sm, oracle, gpu_available):
    """Seeded byte flips / truncations / extensions of valid streams: identical status codes
    (first error in stream order) and outputs vs the oracle, decoded as one GPU batch."""
    cases = _fuzz_cases(oracle, 3000, 1234)
    caps = []
    for c in cases:
        try:
            caps.append(min(oracle.uncompressed_length(c), 1 << 20))
        except oracle.OracleError:
            caps.append(0)
    outs, status = sm.uncompress_batch(cases, capacities=caps)
    for c, cap, o, st in zip(cases, caps, outs, status):
        try:
            n = oracle.uncompressed_length(c)
        except oracle.OracleError as e:
            assert st == e.code
            continue
        if n > cap:
            assert st == 2
            continue
        st_o, out_o = oracle.uncompress_status(c)
        assert int(st) == st_o
        assert o == out_o


def test_decompress_large_stream_global_path(sm, oracle, gpu_available):
    # > 64 KiB declared length: decoded straight into HBM (single stream)
    raw = read_testfile("html_x_4") + read_testfile("urls.10K")[:100000]
    comp = oracle.compress(raw)
    assert sm.uncompress(comp) == raw


# ---- decoder edge cases on hand-built streams (tests/streams.py) -------------------------

def _decode_all(sm, streams):
    outs, status = sm.uncompress_batch(streams)
    assert not np.asarray(status).any()
    return outs


def test_decompress_window_boundaries(sm, oracle, gpu_available):
    """Copies into long literals and across the LDS output window's reach (a linear window of
    kWin = 2,560 bytes that keeps the last kKeep = 480+ bytes when it shifts: sources inside it
    are read from LDS, older ones from HBM; round 4's ring reached 448), overlapping copies
    (offset < 16 runs in the in-order tail) after a long literal, and batches whose output
    exceeds the batch cap."""
    from streams import build
    rng = np.random.default_rng(3)
    big = rng.integers(0, 256, 5000, dtype=np.uint8).tobytes()
    cases = []
    for off in (1, 2, 7, 8, 15, 16, 17, 64, 100, 446, 447, 448, 449, 450, 479, 480, 481, 496, 511, 512, 513, 959,
                960, 961, 999, 1023, 1024, 1025, 2047, 2048, 2558, 2559, 2560, 2561, 3006, 3007, 3008, 3009, 3010,
                4000, 4095, 4096, 4097, 4999, 5000):
        for ln in (1, 4, 11, 12, 16, 33, 64):
            cases.append([("lit", big), ("copy", off, ln), ("copy", 3, 20), ("lit", b"xyz"), ("copy", off, ln)])
    mid = rng.integers(0, 256, 150, dtype=np.uint8).tobytes()  # a 65..200-byte literal
    for off in (1, 5, 8, 64, 149, 150):
        cases.append([("lit", mid), ("copy", off, 64), ("copy", off, 64)])
    cases.append([("lit", b"ab")] + [("copy", 2, 64)] * 100)            # > 1 KiB in one batch
    cases.append([("lit", b"a")] + [("copy", 1, 64)] * 1000)            # RLE, 64 KB
    cases.append([("lit", big), ("lit", big[:300])] + [("copy", 4500, 64)] * 50)
    built = [build(c) for c in cases]
    outs = _decode_all(sm, [s for s, _ in built])
    for (s, expect), o in zip(built, outs):
        assert o == expect
        assert oracle.uncompress(s) == expect


def test_decompress_random_op_streams(sm, gpu_available):
    """Seeded random literal/copy streams (any legal offset and length, some long
    literals), decoded as one GPU batch against the plain LZ77 meaning of the ops."""
    from streams import build, random_ops
    rng = np.random.default_rng(2024)
    built = [build(random_ops(rng, int(rng.integers(1, 65536)))) for _ in range(400)]
    # offsets around the decoder's LDS-window reach and batch cap (a source ending in the
    # unflushed tail before a batch; a batch-dependent copy after a long literal)
    built += [build(random_ops(rng, int(rng.integers(1, 65536)), long_lit_p=0.1, near=1200)) for _ in range(300)]
    outs = _decode_all(sm, [s for s, _ in built])
    for (s, expect), o in zip(built, outs):
        assert o == expect


def _nonminimal_streams(seed, count):
    """Streams whose literal tags carry 1..4 length bytes whatever the length (hi = 59 + k), a
    wrapped 4-byte length (1 + 0xffffffff = 0 in UInt32, internal.jl:456), and copies reaching
    back across them (LDS window and HBM sources)."""
    from streams import copy_tag, lit_tag, varint
    rng = np.random.default_rng(seed)
    streams = []
    for _ in range(count):
        body, out = bytearray(), bytearray()
        target = int(rng.integers(1, 20000))
        while len(out) < target:
            r = rng.random()
            if not out or r < 0.35:
                n = int(rng.choice([1, 2, 15, 16, 17, 60, 61, 64, 65, 100, 199, 200, 201, 300, 700]))
                data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
                k = int(rng.integers(1, 5))
                if n - 1 >= 1 << (8 * k):
                    body += lit_tag(n)
                else:
                    body += bytes([(59 + k) << 2]) + (n - 1).to_bytes(k, "little")
                body += data
                out += data
            elif r < 0.38:
                body += bytes([63 << 2]) + b"\xff\xff\xff\xff"  # a wrapped length: 0 bytes
            else:
                off = int(rng.integers(1, min(len(out), 3000) + 1))
                ln = int(rng.integers(1, 65))
                body += copy_tag(off, ln)
                for _ in range(ln):
                    out.append(out[-off])
        streams.append((varint(len(out)) + bytes(body), bytes(out)))
    return streams


def test_decompress_nonminimal_literals(sm, oracle, gpu_available):
    """Literal tags with more length bytes than needed (the batch walk leaves every hi >= 61
    literal to the general path and sizes hi = 60 ones in SWAR: sm_decompress.hip pack_sizes,
    tools/check_tag_sizes.c) and wrapped lengths, between copies: outputs equal the LZ77
    meaning and the oracle's, in one batch and through validate."""
    built = _nonminimal_streams(77, 300)
    outs = _decode_all(sm, [s for s, _ in built])
    for (s, expect), o in zip(built, outs):
        assert o == expect
        assert oracle.uncompress(s) == expect
    for s, expect in built[:40]:
        assert sm.validate(s) == 0
        assert sm.uncompress(s) == expect


def test_decompress_consecutive_nonminimal_literals(sm, oracle, gpu_available):
    """Long runs of consecutive short literals with 2-4 length bytes (each one a tag the batch walk
    stops at, decoded into the LDS window without a batch between them: many window shifts
    with no batch flush in between), then copies from anywhere before (window and HBM sources,
    offsets up to 65,535)."""
    from streams import copy_tag, varint
    rng = np.random.default_rng(0x6161)
    streams = []
    for _ in range(40):
        body, out = bytearray(), bytearray()
        target = int(rng.integers(3000, 65536))
        while len(out) < target:
            for _ in range(int(rng.integers(1, 80))):
                n = int(rng.integers(1, 201))
                k = int(rng.integers(2, 5))
                data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
                body += bytes([(59 + k) << 2]) + (n - 1).to_bytes(k, "little") + data
                out += data
            for _ in range(int(rng.integers(1, 4))):
                off = int(rng.integers(1, min(len(out), 65535) + 1))
                ln = int(rng.integers(4, 65))
                body += copy_tag(off, ln)
                for _ in range(ln):
                    out.append(out[-off])
        streams.append((varint(len(out)) + bytes(body), bytes(out)))
    outs = _decode_all(sm, [s for s, _ in streams])
    for (s, expect), o in zip(streams, outs):
        assert o == expect
        assert oracle.uncompress(s) == expect
    for s, expect in streams[:8]:
        assert sm.uncompress(s) == expect


# ---- one large stream: parallel fragment decode (sm_uncompress) ---------------------------

def _big_corpus(n):
    raw = b"".join(read_testfile(f) for f in sorted(GOLDEN["corpus"]))
    return (raw * (n // len(raw) + 1))[:n]


def small_path(sm, comp):
    """Whether sm_uncompress takes path 4 (small stream on the device, sm_api.hip
    small_uncompress) for this stream: 4 KiB..64 MiB of output from a body of <= 1024 index
    chunks of 1 KiB (1 MiB) and at most as long as the output (else all literals: path 0)."""
    size, hdr = sm.parse32(comp, 0)
    body = len(comp) - hdr
    return (4096 <= size <= (64 << 20) and body > 0 and (body + 1023) // 1024 <= 1024
            and body <= size)


def literal_path(sm, comp, limit=16):
    """Whether sm_uncompress takes path 5 (sm_api.hip literal_only): at most `limit` literal tags
    with at most 3 length bytes, covering the body and the declared length exactly."""
    size, p = sm.parse32(comp, 0)
    o = n = 0
    while p < len(comp):
        t = comp[p]
        if t & 3 or n == limit:
            return False
        ln, q = (t >> 2) + 1, p + 1
        if (t >> 2) >= 60:
            nb = (t >> 2) - 59
            if nb > 3 or q + nb > len(comp):
                return False
            ln, q = int.from_bytes(comp[q:q + nb], "little") + 1, q + nb
        if q + ln > len(comp) or o + ln > size:
            return False
        o, p, n = o + ln, q + ln, n + 1
    return n > 0 and o == size


def expected_small(sm, comp):
    """The single-call path of a stream with paths 4-5 on: 5, 4 or None (another path)."""
    if literal_path(sm, comp) and sm.parse32(comp, 0)[0] <= (16 << 20):
        return 5
    return 4 if small_path(sm, comp) else None


def _lit_stream(size, pieces, nb=None):
    """A stream of literal tags over `pieces` (bytes each), declared length `size`; nb forces the
    number of length bytes (a non-minimal encoding when the length would fit fewer)."""
    out = bytearray(bytes(encode32_py(size)))
    for b in pieces:
        v = len(b) - 1
        k = nb if nb is not None else (0 if v < 60 else 1 if v < 256 else 2 if v < 65536 else 3)
        out.append(v << 2 if k == 0 else (59 + k) << 2)
        out += v.to_bytes(k, "little") if k else b""
        out += b
    return bytes(out)


def encode32_py(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7f) | 0x80)
        v >>= 7
    out.append(v)
    return out


def test_uncompress_literal_only_streams(sm, oracle, libsnappy, gpu_available):
    """Path 5 (sm_api.hip literal_only + k_literal_spans): streams of at most 16 literal tags --
    incompressible inputs from every compressor, and hand-built ones with non-minimal length
    encodings -- decode bit-exactly in one copy kernel; everything that is not exactly such a
    stream (17 tags, a 4-byte length, a declared length the literals miss, a truncated or
    over-long body, a copy tag) takes the other paths with the oracle's status."""
    rng = np.random.default_rng(0x11)
    for n in (1, 15, 16, 17, 100, 4096, 65535, 65536, 65537, 123093, 1_000_000):
        data = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for comp in (sm.compress(data, mode="fast"), oracle.compress(data), libsnappy.compress(data)):
            assert literal_path(sm, comp), n
            assert sm.uncompress(comp) == data
            assert sm.last_uncompress_path() == 5
    data = rng.integers(0, 256, 70_000, dtype=np.uint8).tobytes()
    cuts = [0, 1, 61, 300, 4000, 20_000, 65_000, 70_000]
    pieces = [data[a:b] for a, b in zip(cuts, cuts[1:])]
    for nb in (None, 3):  # (nb 3: every literal with three length bytes)
        comp = _lit_stream(len(data), pieces, nb)
        assert oracle.uncompress(comp) == data
        assert sm.uncompress(comp) == data and sm.last_uncompress_path() == 5
    many = [data[i * 100:(i + 1) * 100] for i in range(17)]
    for k, want5 in ((16, True), (17, False)):
        comp = _lit_stream(100 * k, many[:k])
        assert sm.uncompress(comp) == data[:100 * k]
        assert (sm.last_uncompress_path() == 5) == want5
    # not literal-only, or not exactly covering: the reference's verdict through the other paths
    four = bytes(encode32_py(300)) + bytes([63 << 2]) + (299).to_bytes(4, "little") + data[:300]  # four length bytes
    bad = [four,
           _lit_stream(5000, [data[:4000]]),                # declared length longer than the literals
           _lit_stream(4000, [data[:4000]])[:-1],           # truncated body
           _lit_stream(4000, [data[:4000]]) + b"\x00",     # a byte after the last literal
           _lit_stream(4000, [data[:4000]]) + b"\x01\x02",  # a copy tag after it
           _lit_stream(3000, [data[:4000]])]                # literals longer than declared
    for comp in bad:
        st_o, out_o = oracle.uncompress_status(comp)
        try:
            st_g, out_g = 0, sm.uncompress(comp)
        except sm.SnappyError as exc:
            st_g, out_g = exc.code, None
        assert st_g == st_o, (st_g, st_o)
        if st_o == 0:
            assert out_g == out_o
        assert sm.last_uncompress_path() != 5


def test_uncompress_large_stream_parallel(sm, oracle, libsnappy, gpu_available):
    """Block-structured streams (Snappy.jl = oracle, libsnappy, this library's fast mode) of
    more than 4 fragments decode through the parallel fragment path, bit-exactly -- or, with a
    body of at most 1 MiB, through path 4; with path 4 off, all through the fragment path."""
    raw = _big_corpus(1_500_000)
    rng = np.random.default_rng(9)
    noise = rng.integers(0, 256, 1_000_000, dtype=np.uint8).tobytes()
    mixed = b"".join(raw[i:i + 50_000] + noise[i:i + 30_000] for i in range(0, 900_000, 80_000))
    # every 64 KiB block starting with a long literal (> 200 B: the batch path's big literals)
    blocky = b"".join(noise[i * 1000:i * 1000 + 700] + raw[i * 65536:i * 65536 + 64836] for i in range(8))
    seen = set()
    try:
        for small in (True, False):
            sm.set_small_decode(small)
            for data in (raw, noise, mixed, blocky):
                for comp in (oracle.compress(data), libsnappy.compress(data), sm.compress(data, mode="fast")):
                    assert sm.uncompress(comp) == data
                    want = (expected_small(sm, comp) or 1) if small else 1
                    assert sm.last_uncompress_path() == want
                    seen.add(want)
    finally:
        sm.set_small_decode(True)
    assert seen == {1, 4, 5}


def test_uncompress_large_stream_fallbacks(sm, oracle, gpu_available):
    """Valid streams that are not block-structured (copies into earlier 64 KiB blocks, a
    literal across a fragment start) decode in parallel by origin pointers (path 2) with the
    oracle's output; corrupted large streams report the oracle's status, their first error
    found in parallel over the tag path (path 3)."""
    from streams import build, random_ops
    rng = np.random.default_rng(31)
    s1, e1 = build(random_ops(rng, 400_000))                        # offsets up to 65535
    s2, e2 = build([("lit", rng.integers(0, 256, 70_000, dtype=np.uint8).tobytes())] +
                   [("copy", 1000, 64)] * 5000)                      # literal across 65536
    try:
        for small in (True, False):
            sm.set_small_decode(small)
            for s, e in ((s1, e1), (s2, e2)):
                assert oracle.uncompress(s) == e
                assert sm.uncompress(s) == e
                assert sm.last_uncompress_path() == (4 if small and small_path(sm, s) else 2)
    finally:
        sm.set_small_decode(True)
    good = oracle.compress(_big_corpus(600_000))
    paths = []
    for i in range(40):
        bad = bytearray(good)
        for _ in range(int(rng.integers(1, 4))):
            bad[int(rng.integers(5, len(bad)))] = int(rng.integers(0, 256))
        st_o, out_o = oracle.uncompress_status(bytes(bad))
        try:
            st_g, out_g = 0, sm.uncompress(bytes(bad))
        except sm.SnappyError as exc:
            st_g, out_g = exc.code, None
        assert st_g == st_o
        if st_o == 0:
            assert out_g == out_o
        elif st_o != 18:  # (a broken header never reaches the tag path)
            paths.append(sm.last_uncompress_path())
    assert paths and paths.count(3) >= len(paths) // 2, paths  # most errors are found in parallel


def _device_batch(streams):
    import torch
    dev = torch.device("cuda", 0)
    buf, in_off, in_len = _pack(streams)
    return (torch.from_numpy(buf).to(dev), torch.from_numpy(in_off.astype(np.int64)).to(dev),
            torch.from_numpy(in_len.astype(np.int32)).to(dev))


def _pack(streams):
    lens = np.array([len(x) for x in streams], dtype=np.uint32)
    offs = np.zeros(len(streams), dtype=np.uint64)
    if len(streams) > 1:
        offs[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    buf = np.frombuffer(b"".join(streams) + b"\0" * 16, dtype=np.uint8).copy()
    return buf, offs, lens


def _validate_statuses(sm, streams):
    import torch
    d_in, d_off, d_len = _device_batch(streams)
    d_st = torch.full((len(streams),), -1, dtype=torch.int32, device=d_in.device)
    sm.validate_batch_device(d_in, d_off, d_len, d_st)
    torch.cuda.synchronize()
    return d_st.cpu().numpy()


def test_validate_batch_matches_oracle(sm, oracle, gpu_available):
    """sm_validate_batch_device: the status uncompress() would return,
    without output -- corrupted, fuzzed, leniency and valid streams vs the oracle's decoder."""
    from test_oracle import corrupted_cases
    import streams as S
    rng = np.random.default_rng(77)
    cases = list(corrupted_cases(oracle)) + _fuzz_cases(oracle, 2000, 4321)
    cases += [oracle.compress(read_testfile(f)) for f in ("html", "alice29.txt", "fireworks.jpeg", "urls.10K")]
    cases += [S.build(S.random_ops(rng, 20000, long_lit_p=0.2))[0] for _ in range(20)]
    good = oracle.compress(b"hello hello hello hello")
    cases += [good + b"\x07", b"\x00\x00", b"\x00", b"\x00\x00\x00", bytes([0x40, 0x12, 0x00, 0x00]), b"",
              b"\xff\xff\xff\xff\x7f", b"\x80"]
    got = _validate_statuses(sm, cases)
    want = [oracle.uncompress_status(c)[0] for c in cases]
    bad = [(i, int(g), w) for i, (g, w) in enumerate(zip(got, want)) if int(g) != w]
    assert not bad, bad[:10]
    assert sum(1 for w in want if w == 0) >= 30 and sum(1 for w in want if w != 0) >= 500
    # the single-buffer entry point
    for c in cases[-40:]:
        assert sm.validate(c) == oracle.uncompress_status(c)[0]


def test_uncompressed_length_batch_device(sm, oracle, gpu_available):
    import torch
    cases = [b"", b"\x00", b"\x80", b"\x7f", b"\x80\x80\x04", b"\xff\xff\xff\xff\x0f", b"\xff\xff\xff\xff\x10",
             b"\xff\xff\xff\xff\xff\x01", oracle.compress(read_testfile("html"))]
    cases += [oracle.encode32(1 << i) for i in range(31)]
    d_in, d_off, d_len = _device_batch(cases)
    d_n = torch.zeros(len(cases), dtype=torch.int32, device=d_in.device)
    d_st = torch.full((len(cases),), -1, dtype=torch.int32, device=d_in.device)
    sm.uncompressed_length_batch_device(d_in, d_off, d_len, d_n, d_st)
    torch.cuda.synchronize()
    for c, n, st in zip(cases, d_n.cpu().numpy().view(np.uint32), d_st.cpu().numpy()):
        try:
            want = oracle.uncompressed_length(c)
            assert (int(st), int(n)) == (0, want), c
        except oracle.OracleError as e:
            assert (int(st), int(n)) == (e.code, 0), c


def test_config5_large_stream(sm, oracle, gpu_available):
    """SURVEY §8(d) config 5 (644 MiB = 10,304 fragments, the round-trip corpus tiled with
    seeded rotations) as ONE stream: reference-mode bytes equal the oracle's, the parallel
    single-stream decode restores it, and the fast-mode stream round-trips."""
    import hashlib
    sys_path_root()
    import bench
    raw = bench.large_corpus().tobytes()
    comp = sm.compress(raw, mode="reference")
    assert hashlib.sha256(comp).digest() == hashlib.sha256(oracle.compress(raw)).digest()
    assert sm.uncompress(comp) == raw
    assert sm.last_uncompress_path() == 1
    fast = sm.compress(raw, mode="fast")
    assert sm.uncompress(fast) == raw
    assert sm.last_uncompress_path() == 1


def test_config5_corrupted_stream_first_error(sm, oracle, gpu_available):
    """a corrupted config-5 stream (644 MiB, bytes flipped at 10 seeded
    positions) returns the oracle's status -- the first error in stream order, found by per-tag
    checks over the tag path in parallel (path 3; 18-33 ms of GPU work, the call well under a
    second with its upload) instead of the in-order decode's minute."""
    import time
    sys_path_root()
    import bench
    raw = bench.large_corpus().tobytes()
    comp = sm.compress(raw, mode="fast")
    rng = np.random.default_rng(0xBAD5)
    hdr = len(sm.encode32(len(raw)))
    for trial in range(3):
        bad = bytearray(comp)
        for pos in rng.integers(hdr, len(bad), 10):
            bad[int(pos)] ^= int(rng.integers(1, 256))
        bad = bytes(bad)
        st_o, _ = oracle.uncompress_status(bad)
        t0 = time.perf_counter()
        try:
            sm.uncompress(bad)
            st_g = 0
        except sm.SnappyError as exc:
            st_g = exc.code
        dt = time.perf_counter() - t0
        assert st_g == st_o, (trial, st_g, st_o)
        if st_o != 0:
            assert sm.last_uncompress_path() == 3
            # (the time includes the ~370 MB pageable upload; the in-order decode took about a
            # minute, so a generous bound still tells the paths apart -- ADVICE round 3)
            assert dt < 5.0, dt
        print("trial %d: status %d in %.3f s (path %d)" % (trial, st_g, dt, sm.last_uncompress_path()))


def sys_path_root():
    import sys
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)


def test_uncompress_origin_path_cases(sm, oracle, gpu_available):
    """The origin-pointer parallel decode (path 2) on streams built to stress it: deep copy
    chains (offset 1 runs over 300 KB: 18+ pointer-jumping rounds), copy-4 offsets past 64 KiB,
    overlapping copies of every offset 1..20, long literals between copies, and a stream whose
    every copy reaches exactly to the start of the output.  Output equals the oracle's."""
    from streams import build, random_ops
    rng = np.random.default_rng(77)
    cases = []
    # a 1-byte seed, then offset-1 copies: one chain through the whole output
    cases.append(build([("lit", b"x")] + [("copy", 1, 64)] * 5000))
    # copy-4: offsets beyond 64 KiB into a long random prefix
    pre = rng.integers(0, 256, 200_000, dtype=np.uint8).tobytes()
    ops = [("lit", pre)]
    for _ in range(6000):
        ops.append(("copy", int(rng.integers(65_536, 200_000)), int(rng.integers(4, 65))))
    cases.append(build(ops))
    # overlapping copies of small offsets, interleaved with literals (some long)
    ops = [("lit", rng.integers(0, 256, 64, dtype=np.uint8).tobytes())]
    for i in range(20_000):
        if i % 97 == 0:
            ops.append(("lit", rng.integers(0, 256, int(rng.integers(201, 2000)), dtype=np.uint8).tobytes()))
        ops.append(("copy", 1 + i % 20, int(rng.integers(1, 65))))
    cases.append(build(ops))
    # every copy reaches back to byte 0 (offset = produced)
    ops, size = [("lit", rng.integers(0, 256, 5000, dtype=np.uint8).tobytes())], 5000
    for _ in range(8000):
        ln = int(rng.integers(4, 65))
        ops.append(("copy", size, ln))
        size += ln
    cases.append(build(ops))
    cases.append(build(random_ops(rng, 1_500_000, max_off=65535, near=60_000)))
    try:
        for small in (False, True):  # path 2, then path 4 (the same origin pointers, device-chained)
            sm.set_small_decode(small)
            for s, e in cases:
                assert oracle.uncompress(s) == e
                assert sm.uncompress(s) == e
                assert sm.last_uncompress_path() == (4 if small and small_path(sm, s) else 2)
                assert sm.validate(s) == 0
    finally:
        sm.set_small_decode(True)
    assert sum(small_path(sm, s) for s, _ in cases) >= 3


def test_uncompress_small_streams_device_path(sm, oracle, libsnappy, gpu_available):
    """Path 4 (sm_api.hip small_uncompress; sm_decompress.hip k_stream_chain, k_origin_fill_dev,
    k_origin_resolve_hops): every corpus file in every compress mode and from libsnappy, streams
    at the path's size limits (4 KiB of output, one index chunk, 256 chunks), deep copy chains,
    and mutated streams -- output and status equal the oracle's (test/runtests.jl:8-24 round
    trips; internal.jl:411-466 errors, first in stream order)."""
    from streams import build, random_ops
    rng = np.random.default_rng(404)
    cases = []
    for f in ROUNDTRIP_FILES + ["sample-tweet.json"]:
        raw = read_testfile(f)
        cases += [(oracle.compress(raw), raw), (libsnappy.compress(raw), raw),
                  (sm.compress(raw, mode="fast"), raw), (sm.compress(raw, mode="dense"), raw)]
    text = _big_corpus(3_000_000)
    for n in (4095, 4096, 4097, 5000, 65535, 65536, 65537, 200_000):
        cases.append((oracle.compress(text[:n]), text[:n]))
    # bodies of exactly 1, 4 and 1024 index chunks of 1 KiB and one byte more
    for body in (1024, 1025, 4096, 4097, 1024 * 1024, 1024 * 1024 + 1):
        ops, left = [("lit", rng.integers(0, 256, 60, dtype=np.uint8).tobytes())], body - 61
        while left > 61:                      # copy-2 tags: 3 bytes for 60 bytes of output
            ops.append(("copy", 60, 60))
            left -= 3
        ops.append(("lit", rng.integers(0, 256, left - 1, dtype=np.uint8).tobytes()))
        st, ex = build(ops)
        assert len(st) - len(sm.encode32(len(ex))) == body
        cases.append((st, ex))
    cases.append(build([("lit", b"ab")] + [("copy", 2, 64)] * 4000))             # one period-2 run
    cases.append(build([("lit", b"q")] + [("copy", 1, 1)] * 20_000))             # 1-byte copies
    cases.append(build(random_ops(rng, 300_000, near=100)))                       # short offsets
    # long literals across index chunks, up to six in a row (deep chunk entries, deep-record
    # levels 0-3 and the walk past them), between runs of short copies
    ops, size = [("lit", rng.integers(0, 256, 50, dtype=np.uint8).tobytes())], 50
    for _ in range(120):
        for _ in range(int(rng.integers(1, 7))):
            ops.append(("lit", rng.integers(0, 256, int(rng.integers(70, 3000)), dtype=np.uint8).tobytes()))
            size += len(ops[-1][1])
        for _ in range(int(rng.integers(40, 160))):
            ops.append(("copy", int(rng.integers(1, min(2000, size) + 1)), int(rng.integers(4, 65))))
            size += ops[-1][2]
    cases.append(build(ops))
    assert small_path(sm, cases[-1][0])
    cases.append(build(random_ops(rng, 600_000, max_off=400_000, near=300_000)))  # copy-4 offsets
    for s, e in cases:
        assert oracle.uncompress(s) == e
        assert sm.uncompress(s) == e, len(e)
        assert sm.last_uncompress_path() == (4 if small_path(sm, s) else sm.last_uncompress_path())
    assert sum(small_path(sm, s) for s, _ in cases) >= len(cases) - 12
    # mutations: the reference's status (its first error), and its output when still valid
    for f in ("html", "alice29.txt", "urls.10K", "sample-tweet.json", "geo.protodata"):
        good = sm.compress(read_testfile(f), mode="fast")
        for _ in range(30):
            bad = bytearray(good)
            for _ in range(int(rng.integers(1, 4))):
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


def _chunk_of(sm, s):
    """sm_api.hip small_chunk(): 128-byte index chunks for bodies <= 16 KiB and <= 0.9 of the
    output, 512 for bodies <= 0.6 of the output and 256 KiB, else 1024."""
    size, hdr = sm.parse32(s)
    body = len(s) - hdr
    if body <= 16384 and body * 10 <= size * 9:
        return 128
    return 512 if body * 10 <= size * 6 and body <= 256 << 10 else 1024


def _fine_chunks(sm, s):
    return _chunk_of(sm, s) < 1024


def test_small_path_chunk_sizes_and_parallel_runs(sm, oracle, gpu_available):
    """Path 4's two index chunk sizes (sm_api.hip small_chunk) and the chain's parallel runs
    (sm_decompress.hip k_stream_chain: pointer-jumped chunk links, serial steps between): bodies
    of exactly 1, 2 and many 512-byte chunks, both sides of the size rule's bounds, long copy runs
    (runs of >= kMinRun links) broken by long literals (deep entries, then a new run), and
    mutations of such streams.  Output and status equal the oracle's."""
    from streams import build
    rng = np.random.default_rng(512)
    cases = []

    def copy_run(body, lit=60):  # copy-2 tags after one literal: a body of exactly `body` bytes
        ops, left = [("lit", rng.integers(0, 256, lit, dtype=np.uint8).tobytes())], body - lit - 1
        while left > 61:
            ops.append(("copy", 60, 60))
            left -= 3
        ops.append(("lit", rng.integers(0, 256, left - 1, dtype=np.uint8).tobytes()))
        return build(ops)

    for body in (512, 513, 1024, 1025, 4096 + 512, 256 << 10, (256 << 10) + 1):
        cases.append(copy_run(body))
    # runs broken by literal groups: ratio below and above the fine-chunk rule
    for lit_hi, groups, cp_lo, cp_hi in ((700, 60, 200, 900), (1500, 40, 200, 900), (4000, 30, 10, 60)):
        ops, size = [("lit", rng.integers(0, 256, 64, dtype=np.uint8).tobytes())], 64
        for _ in range(groups):
            for _ in range(int(rng.integers(1, 4))):
                ops.append(("lit", rng.integers(0, 256, int(rng.integers(65, lit_hi)), dtype=np.uint8).tobytes()))
                size += len(ops[-1][1])
            for _ in range(int(rng.integers(cp_lo, cp_hi))):
                ops.append(("copy", int(rng.integers(1, min(3000, size) + 1)), int(rng.integers(4, 65))))
                size += ops[-1][2]
        cases.append(build(ops))
    fine = [_fine_chunks(sm, s) for s, _ in cases]
    assert any(fine) and not all(fine)
    for s, e in cases:
        assert oracle.uncompress(s) == e
        assert sm.uncompress(s) == e, len(e)
        if small_path(sm, s):
            assert sm.last_uncompress_path() == 4
    assert sum(small_path(sm, s) for s, _ in cases) >= len(cases) - 2
    for s, _ in cases[-3:]:
        for _ in range(10):
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


def test_small_path_tiny_chunks(sm, oracle, gpu_available):
    """Path 4 with 128-byte index chunks (round 6): bodies of 1, 2 and many chunks up to the 16 KiB
    bound and past it, ratios on both sides of 0.9, copy runs across chunk boundaries, long
    literals that enter chunks deep (deep records at 128 bytes), and mutations: output and
    status equal the oracle's, and the chunk rule picks 128 where it says so."""
    from streams import build
    rng = np.random.default_rng(128)
    cases = []
    for body in (4000, 4096, 8000, 16384, 16385):
        for lit_share in (0.05, 0.3, 0.6):  # the literal bytes' share of the output
            ops, size, b = [], 0, 0
            while b < body - 80:
                if rng.random() < lit_share:
                    n = int(rng.integers(1, 300))
                    ops.append(("lit", rng.integers(0, 256, n, dtype=np.uint8).tobytes()))
                    size += n
                    b += n + (1 if n <= 60 else 2 if n <= 256 else 3)
                elif size >= 4:
                    L = int(rng.integers(4, 65))
                    ops.append(("copy", int(rng.integers(1, min(size, 2000) + 1)), L))
                    size += L
                    b += 3
                else:
                    ops.append(("lit", rng.integers(0, 256, 8, dtype=np.uint8).tobytes()))
                    size += 8
                    b += 9
            cases.append(build(ops))
    chunks = [_chunk_of(sm, s) for s, _ in cases]
    assert 128 in chunks and any(c != 128 for c in chunks), chunks
    for s, e in cases:
        assert oracle.uncompress(s) == e
        assert sm.uncompress(s) == e, len(e)
        if small_path(sm, s):
            assert sm.last_uncompress_path() == 4
    for s, _ in cases[::3]:
        for _ in range(6):
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


def test_host_path_piece_boundaries(sm, oracle, gpu_available):
    """The single-buffer host path's pipelining (sm_api.hip): inputs from 32 MiB upload in
    16 MiB pieces with per-piece compress kernels, outputs over 128 MiB download in pieces under
    the fragment decode.  Sizes just past each threshold, with partial last pieces."""
    base = _big_corpus(8 << 20)
    for n in ((32 << 20) + 12345, (128 << 20) + 7):
        raw = (base * (n // len(base) + 1))[:n]
        fast = sm.compress(raw, mode="fast")
        assert oracle.uncompress(fast) == raw
        assert sm.uncompress(fast) == raw
        assert sm.last_uncompress_path() == 1
        if n < (64 << 20):
            ref = sm.compress(raw, mode="reference")
            assert ref == oracle.compress(raw)
            assert sm.uncompress(ref) == raw


def test_single_calls_through_pinned_staging(sm, oracle, gpu_available):
    """The single-buffer calls' last kernel writes its result into the context's device-mapped
    pinned staging (sm_api.hip HostBuf::dp): back-to-back calls of equal sizes and different
    contents, alternating paths 0 and 4 and compress modes, never see a previous call's bytes or
    verdict words.  Includes a failing path-4 call (mutated stream: the fallback decides) between
    good ones, and output sizes not a multiple of 4 or 16."""
    rng = np.random.default_rng(0x57A6E)
    text = read_testfile("alice29.txt")
    for size in (4096 + 3, 65536 + 13, 150001):
        a = text[:size]
        b = bytes(reversed(text[:size]))
        lit = rng.integers(0, 256, size, dtype=np.uint8).tobytes()  # path 0 (mostly literals)
        streams = [(x, sm.compress(x, mode=m)) for x in (a, b, lit) for m in ("fast", "dense", "reference")]
        for x, c in streams:
            assert oracle.uncompress(c) == x
        for rep in range(3):
            for x, c in streams:
                assert sm.compress(x, mode="reference") == oracle.compress(x)
                assert sm.uncompress(c) == x
            x, c = streams[rep]
            bad = bytearray(c)
            bad[len(bad) // 2] ^= 0x5C
            bad = bytes(bad)
            assert _status(sm, bad) == oracle.uncompress_status(bad)


@pytest.mark.parametrize("mode", FAST_MODES)
def test_fast_mode_periodic_blocks(sm, oracle, gpu_available, mode):
    """Periodic blocks (sm_compress_sc.hip's resync on long matches: every row's first walk ends
    in a long extended copy, most of them covered by an earlier row's; the masked proposal and its
    plain-rule fallback must reach the same fixed point): periods 1..4096, some with mutations,
    batched and as single calls in parts; every stream decodes under the oracle, parts equal the
    whole-block parse, and a repeated launch gives the same bytes."""
    rng = np.random.default_rng(0x9E7)
    blocks = []
    for per in (1, 2, 3, 7, 16, 17, 31, 64, 100, 255, 256, 427, 1000, 1023, 4096):
        base = rng.integers(0, 256, per, dtype=np.uint8)
        blk = np.tile(base, 65536 // per + 1)[:65536].copy()
        blocks.append(blk.tobytes())
        mut = blk.copy()
        for q in rng.integers(0, 65536, 40):
            mut[q] = rng.integers(0, 256)
        blocks.append(mut.tobytes())
    out = sm.compress_batch(blocks, mode=mode)
    assert out == sm.compress_batch(blocks, mode=mode)
    for raw, comp in zip(blocks, out):
        assert oracle.uncompress(comp) == raw
        # (no literal fallback on low-entropy blocks: within 10% of the reference's size -- a
        # mutated constant block is 1.064x, copies of 64 split at other offsets than the reference's)
        assert len(comp) <= len(oracle.compress(raw)) * 1.10 + 64
    try:
        for raw in blocks[::3]:
            sm.set_split_compress(False)
            whole = sm.compress(raw, mode=mode)
            sm.set_split_compress(True)
            parts = sm.compress(raw, mode=mode)
            assert parts == whole
            assert oracle.uncompress(parts) == raw
    finally:
        sm.set_split_compress(True)


@pytest.mark.parametrize("mode", ["fast", "dense"])
def test_compress_in_parts_equals_whole_block_parse(sm, oracle, gpu_available, mode):
    """compress() of small inputs parses each 64 KiB fragment in parts on their own workgroups
    (sm_compress_sc.hip k_compress_sc_span: the table state before a part rebuilt by ds_max of
    every earlier position).  The bytes must equal the whole-fragment parse's, including fragments
    whose whole-block parse falls back to one literal (small random fragments: the parts gather
    writes that literal), fragments ending mid super-chunk, and every fragment count up to 64."""
    rng = np.random.default_rng(0x5BA7)
    text = read_testfile("alice29.txt") + read_testfile("html") + read_testfile("urls.10K")
    cases = []
    for n in (1, 17, 1023, 1024, 1025, 4096 + 7, 12836, 65535, 65536, 65537, 100000, 150001, 300000):
        cases.append(text[:n])
    cases.append((text * 7)[:(64 << 16)])          # 64 fragments: 4 parts each
    cases.append((text * 7)[:(33 << 16) + 5])      # 34 fragments: 4 parts each
    cases.append(rng.integers(0, 256, 5000, dtype=np.uint8).tobytes())       # parse expands: redo
    cases.append(rng.integers(0, 256, 200000, dtype=np.uint8).tobytes())     # screened literals
    mixed = bytearray(text[:70000])
    mixed[20000:50000] = rng.integers(0, 256, 30000, dtype=np.uint8).tobytes()
    cases.append(bytes(mixed))
    cases.append(bytes(rng.integers(0, 4, 90000, dtype=np.uint8)))            # long matches
    for name in ("html", "fireworks.jpeg", "paper-100k.pdf", "sample-tweet.json", "kppkn.gtb",
                 "geo.protodata", "smallrandom1.bin"):
        cases.append(read_testfile(name))
    try:
        for raw in cases:
            sm.set_split_compress(False)
            whole = sm.compress(raw, mode=mode)
            assert not sm.last_compress_split()
            sm.set_split_compress(True)
            parts = sm.compress(raw, mode=mode)
            assert sm.last_compress_split() == (len(raw) <= (4 << 20) and -(-len(raw) // 65536) <= 128)
            assert parts == whole, len(raw)
            assert oracle.uncompress(parts) == raw
    finally:
        sm.set_split_compress(True)
