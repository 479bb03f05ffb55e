"""Host-side checks of formulas the kernels use (no GPU): compiled with gcc and run."""
import os
import subprocess

from conftest import ROOT


def test_swar_tag_sizes_equal_per_byte_definition(tmp_path):
    exe = tmp_path / "check_tag_sizes"
    subprocess.run(["gcc", "-O2", "-o", str(exe), os.path.join(ROOT, "tools", "check_tag_sizes.c")], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    assert out.startswith("bad 0,"), out


def test_kernel_register_budgets(tmp_path):
    """gfx950 resource usage of the hot kernels (hipcc -Rpass-analysis, no GPU needed):
    no VGPR spills in the fast compressor, and below the 128-VGPR ceiling that 16-wave
    workgroups allow -- a build of the two-chunk parse that landed exactly on 128 produced
    invalid streams; the decoder keeps 7 waves per SIMD."""
    import re
    csrc = os.path.join(ROOT, "snappy.jl_amd", "csrc")
    usage = {}
    for src in ("sm_compress_fast.hip", "sm_compress_sc.hip", "sm_decompress.hip"):
        out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fno-strict-aliasing",
                              "-fPIC", "-Rpass-analysis=kernel-resource-usage", "--cuda-device-only", "-c",
                              os.path.join(csrc, src), "-o", str(tmp_path / (src + ".o"))],
                             capture_output=True, text=True, check=True).stderr
        name = None
        for line in out.splitlines():
            m = re.search(r"Function Name: (\S+)", line)
            if m:
                name = m.group(1)
                usage[name] = {}
                continue
            m = re.search(r"remark:\s+(VGPRs|VGPRs Spill|Occupancy \[waves/SIMD\]): (\d+)", line)
            if m and name:
                usage[name][m.group(1)] = int(m.group(2))
    # sm_compress_fast.hip holds only the incompressible screen (the round-2 parse is gone)
    assert not [k for k in usage if "k_compress_fast" in k], usage.keys()
    scr = [k for k in usage if "k_literal_screen" in k]
    assert len(scr) == 1 and usage[scr[0]]["VGPRs Spill"] == 0, usage.get(scr[0] if scr else None)
    # the shipped fast compressor (sm_compress_sc.hip, fast and dense instances): 16-wave
    # workgroups, so at most 128 VGPRs, and at most 8 spilled dwords -- block-level values stored
    # once per block, outside the super-chunk loop (the lane index is laundered per super-chunk so
    # lane-derived addresses are not hoisted into the loop's registers: DESIGN.md 3.2)
    # (and the same parse in parts, k_compress_sc_span: fast and dense)
    sc = sorted(k for k in usage if "k_compress_sc" in k)
    assert len(sc) == 4, usage.keys()
    for k in sc:
        assert usage[k]["VGPRs"] <= 128 and usage[k]["VGPRs Spill"] <= 8, (k, usage[k])
    dec = [k for k in usage if k.endswith("k_decompressENS_14DecompressArgsE")]
    assert dec and usage[dec[0]]["Occupancy [waves/SIMD]"] >= 7, usage.get(dec[0] if dec else None)


def test_bench_visible_gpus_from_sysfs(monkeypatch):
    """bench.py counts GPUs without the GPU runtime (sysfs KFD topology), narrowed by the
    *_VISIBLE_DEVICES variables, and refuses to spawn ranks once the runtime is initialised."""
    import importlib
    import sys
    import types
    sys.path.insert(0, ROOT)
    bench = importlib.import_module("bench")
    n = bench.visible_gpus()
    assert n >= 0
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "")
    assert bench.visible_gpus() == 0
    monkeypatch.delenv("HIP_VISIBLE_DEVICES")
    fake = types.SimpleNamespace(cuda=types.SimpleNamespace(is_initialized=lambda: True))
    monkeypatch.setitem(sys.modules, "torch", fake)
    args = types.SimpleNamespace(gpus=2)
    assert bench.launch_ranks(args) == 2


def test_copy_tag_bytes_closed_form():
    """k_compress_sc's sc_copy_bytes: emit_copy!'s tag bytes (src/internal.jl:306-329) in closed
    form, 3 ((L - 1) >> 6) + (2 if ((L - 1) & 63) < 11 and offset < 2048 else 3), against the
    reference's piece loop for every copy length the kernel emits (4..255) and both offset classes."""
    def loop(off, L):
        b = 0
        while L >= 68:
            b, L = b + 3, L - 64
        if L > 64:
            b, L = b + 3, L - 60
        return b + (2 if (L < 12 and off < 2048) else 3)

    def closed(off, L):
        t = L - 1
        return 3 * (t >> 6) + (2 if ((t & 63) < 11 and off < 2048) else 3)

    for off in (1, 7, 2047, 2048, 30000, 65535):
        for L in range(4, 256):
            assert closed(off, L) == loop(off, L), (off, L)
