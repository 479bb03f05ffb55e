"""Host-side checks of formulas the kernels use (no GPU): compiled with gcc and run."""
import os
import subprocess

from conftest import ROOT


def test_swar_tag_sizes_equal_per_byte_definition(tmp_path):
    exe = tmp_path / "check_tag_sizes"
    subprocess.run(["gcc", "-O2", "-o", str(exe), os.path.join(ROOT, "tools", "check_tag_sizes.c")], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout
    assert out.startswith("bad 0,"), out
