"""bench.py's RCCL path on the GPU: the process-group code of the benchmark
-- init over `nccl` (RCCL), the u32 size all-gather inside every step, barriers, max over ranks
-- run at one rank with SM_BENCH_DIST=1 as a subprocess, config 5's 644 MiB stream included (its
fragment-size all-gather runs on nccl at world 1 too); its JSON line must report the backend and
world size the communicator saw, a gathered size table whose own slice matches the local sizes,
and bit-exact round trips."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_bench_rccl_one_rank(gpu_available):
    env = dict(os.environ)
    env["SM_BENCH_DIST"] = "1"
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "5", "--warmup", "2",
           "--no-cpu", "--no-random", "--blocks", "2000"]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    line = json.loads(lines[0])
    assert line["all_roundtrips_bit_exact"] is True
    assert line["n_gpus"] == 1
    rc = line["rccl"]
    assert rc["backend"] == "nccl" and rc["world"] == 1
    assert rc["sizes_gathered"] == 2000 and rc["own_slice_matches"] is True
    # config 5: the 644 MiB stream's fragment sizes all-gathered over RCCL (world 1 included,
    # dist.stream_offsets_device) and the stream decoded bit-exactly from that index
    assert line["large"]["roundtrip_bit_exact"] is True and line["large"]["stream_bytes"] > 0
    print("bench rccl line:", json.dumps(rc), line["value"])
