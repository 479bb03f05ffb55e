"""CPU checks of the C-ABI boundary: the library loads, exports every symbol that
include/*.h declares, and the host-only format helpers (no device work) behave as the
reference's varint / maxlength functions.  No kernel is launched here."""
import ctypes
import glob
import os
import re
import subprocess

import pytest

from conftest import ROOT


def declared_symbols():
    syms = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"\b(sm_[a-z0-9_]+)\s*\(", src):
            syms.add(m.group(1))
    return syms


def test_header_declares_entry_points():
    syms = declared_symbols()
    for s in ("sm_compress", "sm_uncompress", "sm_compress_batch_device", "sm_uncompress_batch_device",
              "sm_max_compressed_length", "sm_uncompressed_length"):
        assert s in syms


def test_library_exports_every_declared_symbol(sm):
    lib = sm.lib()
    syms = declared_symbols()
    assert syms, "no declarations parsed"
    for s in sorted(syms):
        assert hasattr(lib, s), s
    assert set(sm.ABI_SYMBOLS) == syms


def test_exports_are_c_linkage(sm):
    out = subprocess.run(["nm", "-D", "--defined-only", sm.library_path()], capture_output=True, text=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    for s in declared_symbols():
        assert s in exported, s


def test_no_oracle_linkage(sm):
    # the product must not link or embed the test oracle
    out = subprocess.run(["nm", "-D", sm.library_path()], capture_output=True, text=True).stdout
    assert "smo_" not in out
    ldd = subprocess.run(["ldd", sm.library_path()], capture_output=True, text=True).stdout
    assert "oracle" not in ldd


def test_max_compressed_length(sm, oracle):
    for n in (0, 1, 6, 65536, 10 ** 6, 2 ** 32 - 1):
        assert sm.maxlength_compressed(n) == 32 + n + n // 6 == oracle.max_compressed_length(n)


def test_varint_roundtrip(sm, oracle):
    for i in range(32):
        v = (1 << i) - 1 if i else 0
        for val in (v, 1 << min(i, 31)):
            enc = sm.encode32(val)
            assert enc == oracle.encode32(val)
            assert sm.parse32(enc) == (val, len(enc))


@pytest.mark.parametrize("raw", [b"\xf0", b"\x80\x80\x80\x80\x80\x0a", b"\xfb\xff\xff\xff\x7f", b""])
def test_parse32_errors(sm, raw):
    with pytest.raises(sm.SnappyError) as e:
        sm.parse32(raw)
    assert e.value.code == 18
    assert str(e.value) == "Could not decode varint32."


def test_status_messages_match_reference_text(sm, oracle):
    for code, msg in oracle.MESSAGES.items():
        assert sm.status_message(code) == msg


def test_ctx_create_without_gpu_returns_null(sm):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    assert not sm.lib().sm_ctx_create(0)
    with pytest.raises(sm.SnappyError):
        sm.compress(b"abc")


@pytest.mark.parametrize("a,b,limit,expected", __import__("test_oracle").FML_KATS)
def test_find_match_length_kat_abi(sm, a, b, limit, expected):
    """The C ABI's find_match_length (host) on the reference's known-answer tests
    (test/runtests.jl:176-267); the @test_broken case reads past the array -> an error."""
    c = (a + b).encode("latin-1")
    if expected is None:
        with pytest.raises(sm.SnappyError):
            sm.find_match_length(c, 0, len(a), len(a) + limit - 1)
    else:
        assert sm.find_match_length(c, 0, len(a), len(a) + limit - 1) == expected


def test_mode_names_match_header(sm):
    """The Python mode names map to the header's SM_MODE_* values."""
    src = open(os.path.join(ROOT, "include", "snappy_mi355x.h")).read()
    enum = dict((k, int(v)) for k, v in re.findall(r"\b(SM_MODE_[A-Z_]+)\s*=\s*(\d+)", src))
    assert sm.MODES == {"reference": enum["SM_MODE_REFERENCE"], "fast": enum["SM_MODE_FAST"],
                        "dense": enum["SM_MODE_FAST_DENSE"]}
    with pytest.raises(ValueError):
        sm._mode("turbo")


def test_sharded_calls_reject_bad_contexts(sm):
    # argument checks happen on the host before any device work
    L = sm.lib()
    z = ctypes.c_void_p(0)
    none = (ctypes.c_void_p * 1)(None)
    assert L.sm_compress_batch_sharded(none, 1, z, z, z, 1, z, z, z, 1) == 33
    assert L.sm_compress_batch_sharded(None, 0, z, z, z, 1, z, z, z, 1) == 33
    assert L.sm_uncompress_batch_sharded(none, 1, z, z, z, 1, z, z, z, z, z) == 33
    assert L.sm_uncompress_batch_sharded(None, -1, z, z, z, 1, z, z, z, z, z) == 33
