"""Benchmark: batched 64 KiB-block snappy compress + uncompress on MI355X (BASELINE.json).

Workload (BASELINE.json configs[1] + configs[2]): 10,000 blocks of
65,536 B, block i = the 64 KiB window at offset o_i ~ U[0, L-65536) of alice29 + asyoulik +
lcet10 + plrabn12 (L = 1,185,883), o_i from numpy default_rng(0x5EED + rank).  Inputs are
resident in HBM before timing starts.

One step = fast-mode batched compress of the 10K blocks (each an independent snappy stream
in a fixed 76,496-B slot) -> [N>1: RCCL all-gather of the u32 compressed sizes] -> batched
uncompress of those slots back into 64 KiB blocks.  value = (uncompressed bytes compressed +
uncompressed bytes decompressed) per second, summed over ranks (weak scaling: every rank
owns its own 10K blocks).  After timing, the round trip is checked bit-exactly on the device.

roofline: the dominant kernel's algorithmic HBM bytes per launch (compress: sum N read +
sum C written; uncompress: sum C read + sum N written) / its average duration from HIP events
on the launch stream, against 8.0 TB/s.  traffic: from profiles/<round>_pmc.json if present.
cpu_baseline: the oracle (C restatement of Snappy.jl, reference mode) on a bounded sample,
OpenMP over blocks on the host cores, rank 0 only.
"""
import argparse
import importlib.util
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
TESTDATA = os.path.join(ROOT, "tests", "golden", "testdata")
TEXTS = ["alice29.txt", "asyoulik.txt", "lcet10.txt", "plrabn12.txt"]
BLOCK = 65536
SLOT = 76496  # >= max_compressed_length(65536) = 76490, 16-B aligned
HBM_PEAK_GBPS = 8000.0
METRIC = "GB/s compressed+decompressed (batched blocks) at 1/2/4/8 GPUs; % HBM peak"  # BASELINE.json
ROUND = "r01"


def load_package():
    pkg_dir = os.path.join(ROOT, "snappy.jl_amd")
    spec = importlib.util.spec_from_file_location("snappy_jl_amd", os.path.join(pkg_dir, "__init__.py"),
                                                  submodule_search_locations=[pkg_dir])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["snappy_jl_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


# test/runtests.jl:8-24, the round-trip corpus; config 5 tiles it
ROUNDTRIP_FILES = ["alice29.txt", "asyoulik.txt", "html", "html_x_4", "kppkn.gtb", "lcet10.txt", "fireworks.jpeg",
                   "geo.protodata", "paper-100k.pdf", "plrabn12.txt", "urls.10K", "random1.bin", "random2.bin",
                   "random3.bin", "smallrandom1.bin"]
CONFIG5_BYTES = 675_282_944  # 644 MiB = exactly 10,304 blocks


def large_corpus(nbytes=CONFIG5_BYTES, seed=0x5EED + 5):
    """Config 5 ("large"): the 15 round-trip files (4,137,377 B) tiled, each tile rotated by a
    seeded offset, cut at nbytes.  One snappy stream of this is the single-stream workload."""
    corpus = np.frombuffer(b"".join(open(os.path.join(TESTDATA, f), "rb").read() for f in ROUNDTRIP_FILES),
                           dtype=np.uint8)
    rng = np.random.default_rng(seed)
    out = np.empty(nbytes, dtype=np.uint8)
    pos = 0
    while pos < nbytes:
        r = int(rng.integers(0, len(corpus)))
        n = min(len(corpus), nbytes - pos)
        k = min(n, len(corpus) - r)
        out[pos:pos + k] = corpus[r:r + k]
        out[pos + k:pos + n] = corpus[:n - k]
        pos += n
    return out


def text_blocks(nblk, seed):
    corpus = b"".join(open(os.path.join(TESTDATA, f), "rb").read() for f in TEXTS)
    arr = np.frombuffer(corpus, dtype=np.uint8)
    rng = np.random.default_rng(seed)
    offs = rng.integers(0, len(arr) - BLOCK, nblk)
    win = np.lib.stride_tricks.sliding_window_view(arr, BLOCK)
    return np.ascontiguousarray(win[offs])  # [nblk, 65536]


def random_blocks(nblk, seed):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, (nblk, BLOCK), dtype=np.uint8)


class Batch:
    """Device-resident batch: inputs, fixed compressed slots, decode targets."""

    def __init__(self, blocks_np, dev):
        nblk = blocks_np.shape[0]
        self.nblk = nblk
        self.d_in = torch.from_numpy(blocks_np.reshape(-1)).to(dev)
        self.in_off = (torch.arange(nblk, dtype=torch.int64, device=dev) * BLOCK)
        self.in_len = torch.full((nblk,), BLOCK, dtype=torch.int32, device=dev)
        self.d_comp = torch.empty(nblk * SLOT, dtype=torch.uint8, device=dev)
        self.comp_off = torch.arange(nblk, dtype=torch.int64, device=dev) * SLOT
        self.comp_len = torch.zeros(nblk, dtype=torch.int32, device=dev)
        self.d_dec = torch.empty(nblk * BLOCK, dtype=torch.uint8, device=dev)
        self.dec_cap = torch.full((nblk,), BLOCK, dtype=torch.int32, device=dev)
        self.dec_len = torch.zeros(nblk, dtype=torch.int32, device=dev)
        self.status = torch.zeros(nblk, dtype=torch.int32, device=dev)

    def compress(self, sm, mode):
        sm.compress_batch_device(self.d_in, self.in_off, self.in_len, self.d_comp, self.comp_off, self.comp_len,
                                 mode=mode)

    def uncompress(self, sm):
        sm.uncompress_batch_device(self.d_comp, self.comp_off, self.comp_len, self.d_dec, self.in_off, self.dec_cap,
                                   self.dec_len, self.status)

    def verify(self):
        ok = bool(torch.equal(self.d_dec, self.d_in)) and int(self.status.abs().sum()) == 0
        ok = ok and bool((self.dec_len == BLOCK).all())
        return ok


def config5_stream(sm, reps=3):
    """Config 5 as ONE stream through the single-buffer C entry points (sm_compress /
    sm_uncompress), host buffers allocated and touched once: PCIe-inclusive GB/s, best of reps."""
    import ctypes
    big = large_corpus()
    n = big.size
    L, ctx = sm.lib(), sm.context(0)
    cap = sm.maxlength_compressed(n)
    comp = np.zeros(cap, dtype=np.uint8)
    back = np.zeros(n, dtype=np.uint8)
    cl, bl = ctypes.c_size_t(0), ctypes.c_size_t(0)
    tc, td = [], []
    for _ in range(reps + 1):
        cl.value = cap
        t0 = time.perf_counter()
        st = L.sm_compress(ctx, big.ctypes.data, n, comp.ctypes.data, ctypes.byref(cl), 1)
        tc.append(time.perf_counter() - t0)
        bl.value = n
        t0 = time.perf_counter()
        st2 = L.sm_uncompress(ctx, comp.ctypes.data, cl.value, back.ctypes.data, ctypes.byref(bl))
        td.append(time.perf_counter() - t0)
    good = st == 0 and st2 == 0 and bl.value == n and bool(np.array_equal(back, big))
    return {"config5_stream_host_compress_GBps": round(n / min(tc[1:]) / 1e9, 3),
            "config5_stream_host_uncompress_GBps": round(n / min(td[1:]) / 1e9, 3),
            "config5_stream_ratio": round(cl.value / n, 5),
            "config5_stream_ok": good and sm.last_uncompress_path() == 1}


def time_kernel(fn, reps):
    """Average duration (ms) of fn's launches from HIP events on torch's current stream."""
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / reps


def cpu_baseline(blocks_np, seconds=10.0):
    """Oracle (Snappy.jl restated in C, reference mode) round trip on a bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    nthreads = int(os.environ.get("OMP_NUM_THREADS", "0")) or min(16, os.cpu_count() or 1)
    sample = np.ascontiguousarray(blocks_np[:512])
    nblk = sample.shape[0]
    inp = sample.reshape(-1)
    in_off = (np.arange(nblk, dtype=np.uint64) * BLOCK)
    in_len = np.full(nblk, BLOCK, dtype=np.uint32)
    comp = np.empty(nblk * SLOT, dtype=np.uint8)
    comp_off = np.arange(nblk, dtype=np.uint64) * SLOT
    comp_len = np.zeros(nblk, dtype=np.uint32)
    dec = np.empty(nblk * BLOCK, dtype=np.uint8)
    cap = np.full(nblk, BLOCK, dtype=np.uint32)
    dec_len = np.zeros(nblk, dtype=np.uint32)
    st = np.zeros(nblk, dtype=np.int32)

    def run(threads, budget):
        tc = td = 0.0
        reps = 0
        t_end = time.perf_counter() + budget
        while True:
            t0 = time.perf_counter()
            O.compress_batch(inp, in_off, in_len, comp, comp_off, comp_len, compat=False, nthreads=threads)
            t1 = time.perf_counter()
            O.uncompress_batch(comp, comp_off, comp_len, dec, in_off, cap, dec_len, st, nthreads=threads)
            t2 = time.perf_counter()
            tc += t1 - t0
            td += t2 - t1
            reps += 1
            if time.perf_counter() > t_end:
                break
        assert np.array_equal(dec, inp)
        nbytes = reps * inp.size
        return tc, td, nbytes, reps

    tc, td, nbytes, reps = run(nthreads, seconds)
    tc1, td1, nb1, _ = run(1, 3.0)
    return {
        "value": round(2 * nbytes / (tc + td) / 1e9, 4),
        "unit": "GB/s",
        "cores": nthreads,
        "kind": "port",
        "sample": "%d x 64 KiB text blocks (first %d of the workload), %d passes of reference-mode "
                  "compress + uncompress, oracle/snappy_oracle.c -O3, OpenMP over blocks" % (nblk, nblk, reps),
        "compress_GBps": round(nbytes / tc / 1e9, 4),
        "uncompress_GBps": round(nbytes / td / 1e9, 4),
        "single_thread_compress_GBps": round(nb1 / tc1 / 1e9, 4),
        "single_thread_uncompress_GBps": round(nb1 / td1 / 1e9, 4),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--blocks", type=int, default=10000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--extras", action="store_true", help="also time reference mode and random blocks")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    sm = load_package()
    sm.context(local_rank)

    blocks_np = text_blocks(args.blocks, 0x5EED + rank)
    batch = Batch(blocks_np, dev)
    sizes_all = None
    if world > 1:
        sizes_all = torch.zeros(world * args.blocks, dtype=torch.int32, device=dev)

    def step():
        batch.compress(sm, "fast")
        if world > 1:
            dist.all_gather_into_tensor(sizes_all, batch.comp_len)
        batch.uncompress(sm)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    ok = batch.verify()
    comp_bytes = int(batch.comp_len.to(torch.int64).sum())
    in_bytes = args.blocks * BLOCK

    # per-kernel durations (HIP events on the launch stream = torch current stream)
    reps = max(3, min(args.steps, 10))
    t_c = time_kernel(lambda: batch.compress(sm, "fast"), reps)
    t_d = time_kernel(lambda: batch.uncompress(sm), reps)
    c_bytes = in_bytes + comp_bytes + 4 * args.blocks
    d_bytes = comp_bytes + in_bytes
    kern = {"compress_fast": (t_c, c_bytes), "uncompress": (t_d, d_bytes)}
    dom = max(kern, key=lambda k: kern[k][0])
    dom_ms, dom_bytes = kern[dom]
    achieved = dom_bytes / (dom_ms * 1e-3) / 1e9
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", ROUND + "_pmc.json")
    if os.path.exists(pmc_path):
        try:
            traffic = json.load(open(pmc_path)).get(dom, {}).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    extras = {}
    if args.extras:
        # validation (the decoder's walk + checks, no output) of the fast streams
        # SM_MODE_FAST_DENSE: two chain candidates per position (smaller output, slower)
        t_dc = time_kernel(lambda: batch.compress(sm, "dense"), 3)
        extras["dense_compress_GBps"] = round(in_bytes / (t_dc * 1e-3) / 1e9, 3)
        extras["dense_ratio"] = round(int(batch.comp_len.to(torch.int64).sum()) / in_bytes, 5)
        t_dd = time_kernel(lambda: batch.uncompress(sm), 3)
        ok = ok and batch.verify()
        extras["dense_streams_uncompress_GBps"] = round(in_bytes / (t_dd * 1e-3) / 1e9, 3)
        batch.compress(sm, "fast")
        vst = torch.full_like(batch.status, -1)
        t_v = time_kernel(lambda: sm.validate_batch_device(batch.d_comp, batch.comp_off, batch.comp_len, vst), 3)
        ok = ok and int(vst.abs().sum()) == 0
        extras["validate_GBps"] = round(in_bytes / (t_v * 1e-3) / 1e9, 3)
        t_ref = time_kernel(lambda: batch.compress(sm, "reference"), 1)
        extras["reference_mode_compress_GBps"] = round(in_bytes / (t_ref * 1e-3) / 1e9, 3)
        # config 3 with the exact (Snappy.jl byte-identical) streams as input
        t_rd3 = time_kernel(lambda: batch.uncompress(sm), 3)
        ok = ok and batch.verify()
        extras["reference_streams_uncompress_GBps"] = round(in_bytes / (t_rd3 * 1e-3) / 1e9, 3)
        extras["reference_ratio"] = round(int(batch.comp_len.to(torch.int64).sum()) / in_bytes, 5)
        del batch
        torch.cuda.empty_cache()
        rb = Batch(random_blocks(args.blocks, 0x5EED + 1 + rank), dev)
        t_rc = time_kernel(lambda: rb.compress(sm, "fast"), 3)
        t_rd = time_kernel(lambda: rb.uncompress(sm), 3)
        rb_comp = int(rb.comp_len.to(torch.int64).sum())
        ok = ok and rb.verify()
        extras["random_compress_fast_GBps"] = round(in_bytes / (t_rc * 1e-3) / 1e9, 3)
        extras["random_uncompress_GBps"] = round(in_bytes / (t_rd * 1e-3) / 1e9, 3)
        extras["random_ratio"] = round(rb_comp / in_bytes, 5)
        t_rr = time_kernel(lambda: rb.compress(sm, "reference"), 1)
        extras["random_reference_compress_GBps"] = round(in_bytes / (t_rr * 1e-3) / 1e9, 3)

    if args.extras and rank == 0:
        extras.update(config5_stream(sm))
        ok = ok and extras["config5_stream_ok"]

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(blocks_np)

    value = 2.0 * in_bytes * args.steps * world / elapsed / 1e9
    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic: 64 KiB windows of the Calgary text files in tests/golden/testdata",
            "config": {
                "workload": "10K x 64 KiB text blocks: fast-mode compress + uncompress round trip per step",
                "blocks_per_gpu": args.blocks,
                "block_bytes": BLOCK,
                "parallelism": "dp%d (blocks sharded per rank, RCCL size all-gather)" % world,
            },
            "compress_GBps": round(in_bytes / (t_c * 1e-3) / 1e9, 3),
            "uncompress_GBps": round(in_bytes / (t_d * 1e-3) / 1e9, 3),
            "ratio": round(comp_bytes / in_bytes, 5),
            "roundtrip_bit_exact": ok,
            "roofline": {
                "kernel": dom,
                "bound": "hbm",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBPS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBPS, 5),
                "traffic": traffic,
                "algorithmic_bytes_per_launch": dom_bytes,
                "avg_launch_ms": round(dom_ms, 4),
            },
            "cpu_baseline": cpu,
        }
        line.update(extras)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
