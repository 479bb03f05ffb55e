"""The oracle under AddressSanitizer + UBSan (SURVEY.md §5 sanitizers; host code only -- GPU
sanitizers are unavailable on this pool).  oracle/asan_driver runs the restated compressor and
decoder over the whole test corpus plus the reference's corrupted streams (baddata1-3,
test/runtests.jl:64-71) and a seeded mutation fuzz of every compressed stream (flips,
truncations, extensions), each into exact-size heap buffers: an out-of-bounds access or UB aborts
the run."""
import os
import subprocess

import pytest

from conftest import ROOT, TESTDATA


@pytest.fixture(scope="module")
def asan_driver():
    d = os.path.join(ROOT, "oracle")
    r = subprocess.run(["make", "-s", "-C", d, "asan_driver"], capture_output=True, text=True)
    if r.returncode != 0:
        pytest.skip("cannot build the sanitizer driver here: " + r.stderr[-300:])
    return os.path.join(d, "asan_driver")


def test_oracle_under_asan_ubsan(asan_driver):
    files = sorted(os.path.join(TESTDATA, f) for f in os.listdir(TESTDATA))
    assert any(f.endswith("baddata1.snappy") for f in files)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([asan_driver, "-n", "120"] + files, capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "0 round-trip failures" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
