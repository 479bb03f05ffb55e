"""CPU tests pinning the oracle (oracle/snappy_oracle.c) to the reference's own tests and
fixtures, plus libsnappy 1.1.8.  Mirrors test/runtests.jl testset by testset."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import ROOT, ROUNDTRIP_FILES, read_testfile

GOLDEN = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json")))

# test/runtests.jl:176-267 -- (a, b, limit, expected); None marks the @test_broken case (:225)
FML_KATS = [
    ("012345", "012345", 6, 6),
    ("01234567abc", "01234567abc", 11, 11),
    ("01234567abc", "01234567axc", 9, 9),
    ("01234567abc!", "01234567abc!", 11, 11),
    ("01234567abc!", "01234567abc?", 11, 11),
    ("01234567xxxxxxxx", "?1234567xxxxxxxx", 16, 0),
    ("01234567xxxxxxxx", "0?234567xxxxxxxx", 16, 1),
    ("01234567xxxxxxxx", "01237654xxxxxxxx", 16, 4),
    ("01234567xxxxxxxx", "0123456?xxxxxxxx", 16, 7),
    ("abcdefgh01234567xxxxxxxx", "abcdefgh?1234567xxxxxxxx", 24, 8),
    ("abcdefgh01234567xxxxxxxx", "abcdefgh0?234567xxxxxxxx", 24, 9),
    ("abcdefgh01234567xxxxxxxx", "abcdefgh01237654xxxxxxxx", 24, 12),
    ("abcdefgh01234567xxxxxxxx", "abcdefgh0123456?xxxxxxxx", 24, 15),
    ("01234567", "?1234567", 8, 0),
    ("01234567", "0?234567", 8, 1),
    ("01234567", "01?34567", 8, 2),
    ("01234567", "012?4567", 8, 3),
    ("01234567", "0123?567", 8, 4),
    ("01234567", "01234?67", 8, 5),
    ("01234567", "012345?7", 8, 6),
    ("01234567", "0123456?", 8, 7),
    ("01234567", "0123456?", 7, 7),
    ("01234567!", "0123456??", 7, 7),
    ("xxxxxxabcd", "xxxxxxabcd", 10, 10),
    ("xxxxxxabcd?", "xxxxxxabcd?", 10, 10),
    ("xxxxxxabcdef", "xxxxxxabcdef", 13, None),
    ("xxxxxxabcdef\0", "xxxxxxabcdef\0", 13, 13),
    ("xxxxxx0123abc!", "xxxxxx0123abc!", 12, 12),
    ("xxxxxx0123abc!", "xxxxxx0123abc?", 12, 12),
    ("xxxxxx0123abc", "xxxxxx0123axc", 13, 11),
    ("xxxxxx0123xxxxxxxx", "xxxxxx?123xxxxxxxx", 18, 6),
    ("xxxxxx0123xxxxxxxx", "xxxxxx0?23xxxxxxxx", 18, 7),
    ("xxxxxx0123xxxxxxxx", "xxxxxx0132xxxxxxxx", 18, 8),
    ("xxxxxx0123xxxxxxxx", "xxxxxx012?xxxxxxxx", 18, 9),
    ("xxxxxx0123", "xxxxxx?123", 10, 6),
    ("xxxxxx0123", "xxxxxx0?23", 10, 7),
    ("xxxxxx0123", "xxxxxx0132", 10, 8),
    ("xxxxxx0123", "xxxxxx012?", 10, 9),
    ("xxxxxxabcd0123xx", "xxxxxxabcd?123xx", 16, 10),
    ("xxxxxxabcd0123xx", "xxxxxxabcd0?23xx", 16, 11),
    ("xxxxxxabcd0123xx", "xxxxxxabcd0132xx", 16, 12),
    ("xxxxxxabcd0123xx", "xxxxxxabcd012?xx", 16, 13),
    ("xxxxxxabcd0123", "xxxxxxabcd?123", 14, 10),
    ("xxxxxxabcd0123", "xxxxxxabcd0?23", 14, 11),
    ("xxxxxxabcd0123", "xxxxxxabcd0132", 14, 12),
    ("xxxxxxabcd0123", "xxxxxxabcd012?", 14, 13),
]


def test_fml_kat_count():
    assert sum(1 for k in FML_KATS if k[3] is not None) == 45


@pytest.mark.parametrize("a,b,limit,expected", FML_KATS)
def test_find_match_length_kat(oracle, a, b, limit, expected):
    # test/runtests.jl:168-173: c = vcat(a, b); fml(c, 1, endof(a)+1, endof(a)+limit) (1-based)
    c = (a + b).encode("latin-1")
    got = oracle.find_match_length(c, 0, len(a), len(a) + limit - 1)
    if expected is None:
        assert got != 13  # @test_broken: the reference reads past the array (BoundsError)
    else:
        assert got == expected


@pytest.mark.parametrize("fname", sorted(GOLDEN["corpus"]))
def test_reference_mode_golden(oracle, fname):
    raw = read_testfile(fname)
    g = GOLDEN["corpus"][fname]
    out = oracle.compress(raw)
    assert len(raw) == g["n"]
    assert len(out) == g["c_reference"]
    assert hashlib.sha256(out).hexdigest() == g["sha256_reference"]


@pytest.mark.parametrize("fname", sorted(GOLDEN["corpus"]))
def test_compat_mode_equals_libsnappy(oracle, libsnappy, fname):
    raw = read_testfile(fname)
    assert oracle.compress(raw, compat=True) == libsnappy.compress(raw)


def test_q3_sixty_byte_literal(oracle, libsnappy):
    rng = np.random.default_rng(7)
    x = rng.integers(0, 256, 60, dtype=np.uint8).tobytes()
    ref = oracle.compress(x)
    assert ref[1:3] == bytes([0xF0, 59])            # Snappy.jl: len < 60 only (internal.jl:271)
    assert oracle.compress(x, compat=True) == libsnappy.compress(x)
    assert oracle.uncompress(ref) == x


@pytest.mark.parametrize("fname", ROUNDTRIP_FILES)
def test_roundtrip_corpus(oracle, libsnappy, fname):
    # test/runtests.jl:6-33
    raw = read_testfile(fname)
    a = oracle.compress(raw)
    assert a != raw
    assert oracle.uncompress(a) == raw
    assert libsnappy.uncompress(a) == raw            # independent decoder agrees


def test_alice29_snappy_decode_golden(oracle, libsnappy):
    # not produced by Snappy.jl, but decodes to alice29.txt
    comp = read_testfile("alice29.snappy")
    assert oracle.uncompress(comp) == read_testfile("alice29.txt")
    assert libsnappy.uncompress(comp) == read_testfile("alice29.txt")


def test_edge_strings_golden(oracle):
    from golden.make_golden import EDGE_STRINGS  # noqa
    for s, g in zip(EDGE_STRINGS, GOLDEN["edge_strings"]):
        out = oracle.compress(s)
        assert hashlib.sha256(out).hexdigest() == g["sha256_reference"]
        if "hex_reference" in g:
            assert out.hex() == g["hex_reference"]
        assert oracle.uncompress(out) == s


def test_tiny_strings_survey(oracle):
    # SURVEY.md 8(c)
    assert oracle.compress(b"").hex() == "00"
    assert oracle.compress(b"a").hex() == "010061"
    assert oracle.compress(b"ab").hex() == "02046162"
    assert oracle.compress(b"abc").hex() == "0308616263"


def dictionary_stream(rng, maxwords=1 << 16):
    # test/runtests.jl:37-43, seeded
    words = [rng.integers(0, 256, int(rng.integers(1, 17)), dtype=np.uint8).tobytes() for _ in range(64)]
    k = int(rng.integers(1, maxwords + 1))
    idx = rng.integers(0, 64, k)
    return b"".join(words[i] for i in idx)


def test_random_dictionary_roundtrips(oracle, libsnappy):
    rng = np.random.default_rng(0x5EED)
    for _ in range(20):
        raw = dictionary_stream(rng, 1 << 13)
        a = oracle.compress(raw)
        assert oracle.uncompress(a) == raw
        assert oracle.compress(raw, compat=True) == libsnappy.compress(raw)


def test_max_blowup(oracle):
    # test/runtests.jl:148-154 (seeded)
    rng = np.random.default_rng(3)
    raw = rng.integers(0, 2**32, 20000, dtype=np.uint32).tobytes()
    raw = raw + raw[::-1]
    a = oracle.compress(raw)
    assert oracle.uncompress(a) == raw


def test_varint_range(oracle):
    # test/runtests.jl:157-163
    for i in range(31):
        enc = oracle.encode32(1 << i)
        v, nxt = oracle.parse32(enc)
        assert v == 1 << i and nxt == len(enc)


CORRUPT_VARINTS = [bytes([0xF0]), bytes([0x80, 0x80, 0x80, 0x80, 0x80, 0x0A]), bytes([0xFB, 0xFF, 0xFF, 0xFF, 0x7F])]


@pytest.mark.parametrize("raw", CORRUPT_VARINTS)
def test_corrupt_varints(oracle, raw):
    # test/runtests.jl:100-111
    with pytest.raises(oracle.OracleError) as e:
        oracle.parse32(raw)
    assert e.value.code == 18
    st, _ = oracle.uncompress_status(raw)
    assert st == 18


def corrupted_cases(oracle):
    """test/runtests.jl:62-122 -- every case must be rejected."""
    cases = []
    src = b"making sure we don't crash with corrupted input"
    dst = bytearray(oracle.compress(src))
    assert len(dst) > 3
    dst[1] = (~dst[1]) & 0xFF
    dst[3] = dst[2]
    cases.append(bytes(dst))
    dst = bytearray(oracle.compress(b"A" * 100000))
    dst[0] = dst[1] = dst[2] = dst[3] = 0
    cases.append(bytes(dst))
    dst[0] = dst[1] = dst[2] = 0xFF
    dst[3] = 0x00
    cases.append(bytes(dst))
    for f in ("baddata1.snappy", "baddata2.snappy", "baddata3.snappy"):
        cases.append(read_testfile(f))
    cases.extend(CORRUPT_VARINTS)
    cases.append(bytes([0x40, 0x12, 0x00, 0x00]))
    cases.append(bytes([0x05, 0x12, 0x00, 0x00]))
    return cases


def test_corrupted_inputs_rejected(oracle, libsnappy):
    for f in ("baddata1.snappy", "baddata2.snappy", "baddata3.snappy"):
        assert oracle.uncompressed_length(read_testfile(f)) < (1 << 20)   # runtests.jl:96
    for c in corrupted_cases(oracle):
        st, out = oracle.uncompress_status(c)
        assert st != 0 and out is None
        assert libsnappy.uncompress(c) is None


def test_f6_leniencies(oracle, libsnappy):
    # a trailing byte after a valid stream is never parsed (internal.jl:416)
    good = oracle.compress(b"hello hello hello hello")
    assert oracle.uncompress(good + b"\x07") == b"hello hello hello hello"
    assert libsnappy.uncompress(good + b"\x07") is None
    assert oracle.uncompress(b"\x00\x00") == b""
    assert oracle.uncompress(b"\x00") == b""
    st, _ = oracle.uncompress_status(b"\x00\x00\x00")
    assert st == 21


def test_char_table_matches_reference(oracle):
    # all 256 CHAR_TABLE entries (src/internal.jl:47-80, extracted as data into golden.json)
    # against the table derived from the tag rules
    ref = GOLDEN["char_table"]
    assert [oracle.char_table(c) for c in range(256)] == ref


def test_hashtable_size(oracle):
    assert oracle.hashtable_size(0) == 256
    assert oracle.hashtable_size(257) == 512
    assert oracle.hashtable_size(16384) == 16384
    assert oracle.hashtable_size(10 ** 9) == 16384


def test_stream_builder_matches_oracle_decoder(oracle):
    """tests/streams.py (hand-built streams for the GPU decoder edge cases) agrees with the
    oracle decoder, so its expected outputs can be trusted."""
    from streams import build, random_ops
    rng = np.random.default_rng(77)
    for _ in range(20):
        stream, expect = build(random_ops(rng, int(rng.integers(1, 40000))))
        assert oracle.uncompress(stream) == expect
