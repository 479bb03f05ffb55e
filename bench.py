"""Benchmark: batched 64 KiB-block snappy compress + uncompress on MI355X (BASELINE.json).

`python bench.py --gpus N --steps K --warmup W`.  With N > 1 and no WORLD_SIZE in the
environment the script starts N ranks itself (torch.distributed.run, before any GPU call) and
exits with their status; under torchrun it checks WORLD_SIZE == N and that the node has N GPUs,
and exits non-zero otherwise.  One process per GPU, RCCL for the collectives.

Workloads (BASELINE.json configs):
* headline (`value`), configs 2+3: every rank owns 10,000 blocks of 65,536 B, block i = the
  64 KiB window at offset o_i ~ U[0, L-65536) of alice29 + asyoulik + lcet10 + plrabn12
  (L = 1,185,883), o_i from numpy default_rng(0x5EED + rank).  One step = fast-mode batched
  compress (each block an independent snappy stream in a fixed 76,496-B slot) -> [N > 1: RCCL
  all-gather of the u32 compressed sizes] -> batched uncompress back into 64 KiB blocks.
  value = (uncompressed bytes compressed + uncompressed bytes decompressed) / s summed over
  ranks: weak scaling.
* `random` (config 4): 10,000 uniform random blocks per rank (default_rng(0x5EED + 1 + rank)),
  the same step.
* `large` (config 5): ONE 644 MiB stream (the 15 round-trip corpus files tiled with seeded
  rotations, exactly 10,304 fragments), strong-scaled: rank r owns the contiguous fragments
  shard_range(10304, r, N).  One step = fast-mode compress of the rank's fragments (no headers,
  Q2 table size) -> RCCL all-gather of the u32 fragment sizes + exclusive scan = every
  fragment's global offset behind the varint header -> uncompress of the rank's fragments.
Inputs are resident in HBM before timing starts.  Every workload is timed over K steps between
a barrier + device synchronize on both sides, max over ranks, and its round trip is checked
bit-exactly on the device afterwards.

roofline: a kernel's algorithmic HBM bytes per launch (compress: sum N read + sum C written +
4 B of size per block; uncompress: sum C read + sum N written) / its median launch duration from
HIP events on the launch stream, against 8.0 TB/s.  traffic: profiles/<round>_pmc.json (rocprofv3
FETCH_SIZE/WRITE_SIZE passes) when present.  cpu_baseline (rank 0): the oracle (C restatement of
Snappy.jl, reference mode) and libsnappy 1.1.8, OpenMP over blocks on every core this process
may use, on a bounded sample of the headline workload.
"""
import argparse
import importlib.util
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
TESTDATA = os.path.join(ROOT, "tests", "golden", "testdata")
TEXTS = ["alice29.txt", "asyoulik.txt", "lcet10.txt", "plrabn12.txt"]
BLOCK = 65536
SLOT = 76496  # >= max_compressed_length(65536) = 76490, 16-B aligned
HBM_PEAK_GBPS = 8000.0
METRIC = "GB/s compressed+decompressed (batched blocks) at 1/2/4/8 GPUs; % HBM peak"  # BASELINE.json
ROUND = "r06"

# test/runtests.jl:8-24, the round-trip corpus; config 5 tiles it
ROUNDTRIP_FILES = ["alice29.txt", "asyoulik.txt", "html", "html_x_4", "kppkn.gtb", "lcet10.txt", "fireworks.jpeg",
                   "geo.protodata", "paper-100k.pdf", "plrabn12.txt", "urls.10K", "random1.bin", "random2.bin",
                   "random3.bin", "smallrandom1.bin"]
CONFIG5_BYTES = 675_282_944  # 644 MiB = exactly 10,304 blocks


def load_package():
    pkg_dir = os.path.join(ROOT, "snappy.jl_amd")
    spec = importlib.util.spec_from_file_location("snappy_jl_amd", os.path.join(pkg_dir, "__init__.py"),
                                                  submodule_search_locations=[pkg_dir])
    mod = importlib.util.module_from_spec(spec)
    sys.modules["snappy_jl_amd"] = mod
    spec.loader.exec_module(mod)
    return mod


def load_dist():
    spec = importlib.util.spec_from_file_location("snappy_jl_amd_dist", os.path.join(ROOT, "snappy.jl_amd", "dist.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


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


# ---- launching ranks ----------------------------------------------------------------------

def visible_gpus():
    """GPUs this process may use, without touching the GPU runtime: the KFD topology in sysfs
    (nodes with a GPU id), narrowed by HIP/ROCR/CUDA_VISIBLE_DEVICES when set."""
    n = 0
    root = "/sys/class/kfd/kfd/topology/nodes"
    try:
        for node in os.listdir(root):
            try:
                with open(os.path.join(root, node, "gpu_id")) as fh:
                    n += int(fh.read().strip() or "0") != 0
            except (OSError, ValueError):
                pass
    except OSError:
        return 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            n = min(n, len([x for x in v.split(",") if x.strip() != ""]))
    return n


def launch_ranks(args):
    """--gpus N > 1 without a launcher: start N ranks under torch.distributed.run.  The GPUs are
    counted from sysfs, and the script refuses to spawn from a process that has initialised the
    GPU runtime (a child must not inherit it)."""
    if "torch" in sys.modules and sys.modules["torch"].cuda.is_initialized():
        print("bench.py: the GPU runtime is already initialised; refusing to start ranks", file=sys.stderr)
        return 2
    ndev = visible_gpus()
    if ndev < args.gpus:
        print("bench.py: --gpus %d but only %d GPU(s) visible" % (args.gpus, ndev), file=sys.stderr)
        return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=%d" % args.gpus,
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


# ---- device workloads -----------------------------------------------------------------------

class Batch:
    """Device-resident batch of independent blocks: inputs, fixed compressed slots, decode targets."""

    def __init__(self, blocks_np, dev):
        import torch
        nblk = blocks_np.shape[0]
        self.nblk = nblk
        self.in_bytes = nblk * BLOCK
        self.d_in = torch.from_numpy(blocks_np.reshape(-1)).to(dev)
        self.in_off = torch.arange(nblk, dtype=torch.int64, device=dev) * BLOCK
        self.in_len = torch.full((nblk,), BLOCK, dtype=torch.int32, device=dev)
        self.d_comp = torch.empty(nblk * SLOT, dtype=torch.uint8, device=dev)
        self.comp_off = torch.arange(nblk, dtype=torch.int64, device=dev) * SLOT
        self.comp_len = torch.zeros(nblk, dtype=torch.int32, device=dev)
        self.d_dec = torch.empty(nblk * BLOCK, dtype=torch.uint8, device=dev)
        self.dec_cap = torch.full((nblk,), BLOCK, dtype=torch.int32, device=dev)
        self.dec_len = torch.zeros(nblk, dtype=torch.int32, device=dev)
        self.status = torch.zeros(nblk, dtype=torch.int32, device=dev)

    def compress(self, sm, mode="fast"):
        sm.compress_batch_device(self.d_in, self.in_off, self.in_len, self.d_comp, self.comp_off, self.comp_len,
                                 mode=mode)

    def uncompress(self, sm):
        sm.uncompress_batch_device(self.d_comp, self.comp_off, self.comp_len, self.d_dec, self.in_off, self.dec_cap,
                                   self.dec_len, self.status)

    def comp_bytes(self):
        import torch
        return int(self.comp_len.to(torch.int64).sum())

    def verify(self):
        import torch
        self.d_dec.fill_(0xAA)
        self.uncompress(load_package_cached())
        ok = bool(torch.equal(self.d_dec, self.d_in)) and int(self.status.abs().sum()) == 0
        return ok and bool((self.dec_len == self.in_len).all())


class StreamShard:
    """Config 5: this rank's fragments of ONE stream (no per-fragment header, table size of the
    whole stream), their compressed slots, the global index, and decode targets."""

    def __init__(self, stream_np, lo, hi, dev):
        import torch
        total = stream_np.size
        self.total = total
        self.lo, self.hi = lo, hi
        nf = hi - lo
        self.nfrag = nf
        a, b = lo * BLOCK, min(hi * BLOCK, total)
        self.in_bytes = b - a
        lens = np.minimum(BLOCK, total - np.arange(lo, hi, dtype=np.int64) * BLOCK)
        self.d_in = torch.from_numpy(np.ascontiguousarray(stream_np[a:b])).to(dev)
        self.in_off = torch.arange(nf, dtype=torch.int64, device=dev) * BLOCK
        self.in_len = torch.from_numpy(lens.astype(np.int32)).to(dev)
        self.d_comp = torch.empty(max(nf, 1) * SLOT, dtype=torch.uint8, device=dev)
        self.comp_off = torch.arange(nf, dtype=torch.int64, device=dev) * SLOT
        self.comp_len = torch.zeros(nf, dtype=torch.int32, device=dev)
        self.d_dec = torch.empty(max(self.in_bytes, 1), dtype=torch.uint8, device=dev)
        self.dec_len = torch.zeros(nf, dtype=torch.int32, device=dev)
        self.status = torch.zeros(nf, dtype=torch.int32, device=dev)
        self.offsets = None
        self.stream_len = None
        # the rank's byte range of the stream, materialised (sm_place_fragments_device): rank 0's
        # starts with the varint header; capacity = the worst case of its fragments
        self.header = lo == 0
        cap = int(sum(32 + int(x) + int(x) // 6 for x in lens)) + (5 if self.header else 0)
        self.d_stream = torch.zeros(max(cap, 1), dtype=torch.uint8, device=dev)
        self.loc_off = torch.zeros(max(nf, 1), dtype=torch.int64, device=dev)[:nf]
        self.place_status = torch.zeros(1, dtype=torch.int32, device=dev)

    def compress(self, sm):
        sm.compress_fragments_device(self.d_in, self.in_off, self.in_len, self.d_comp, self.comp_off, self.comp_len,
                                     self.total, mode="fast")

    def index(self, dist_mod, rank, world):
        self.offsets, self.stream_len = dist_mod.stream_offsets_device(self.comp_len, self.total, rank, world)

    def place(self, sm):
        """This rank's fragments at their global offsets (minus its range's start) in d_stream."""
        sm.place_fragments_device(self.d_comp, self.comp_off, self.comp_len, self.offsets, self.d_stream, self.total,
                                  self.header, d_local_off=self.loc_off, d_status=self.place_status)

    def range_bytes(self):
        """Bytes of this rank's materialised range (rank 0: the header included)."""
        import torch
        if self.nfrag == 0:
            return len_varint(self.total) if self.header else 0
        return int((self.loc_off[-1] + self.comp_len[-1].to(torch.int64)).item())

    def uncompress(self, sm):
        """The fragments decoded where they were placed: out of the materialised stream range."""
        sm.uncompress_fragments_device(self.d_stream, self.loc_off, self.comp_len, self.d_dec, self.in_off,
                                       self.in_len, self.dec_len, self.status)

    def verify(self, sm):
        import torch
        self.d_dec.fill_(0xAA)
        self.uncompress(sm)
        ok = bool(torch.equal(self.d_dec[: self.in_bytes], self.d_in)) and int(self.status.abs().sum()) == 0
        ok = ok and bool((self.dec_len == self.in_len).all())
        # the global index: a real stream length (not poisoned by an error mark, dist.py), and
        # offsets strictly increasing by this rank's sizes
        ok = ok and self.stream_len is not None and int(self.stream_len.item()) > 0
        ok = ok and int(self.place_status.item()) == 0
        if self.nfrag > 1 and self.offsets is not None:
            d = self.offsets[1:] - self.offsets[:-1]
            ok = ok and bool(torch.equal(d, self.comp_len[:-1].to(torch.int64)))
        return ok


def len_varint(v):
    n = 1
    while v >= 0x80:
        v >>= 7
        n += 1
    return n


_SM = None


def load_package_cached():
    global _SM
    if _SM is None:
        _SM = load_package()
    return _SM


def timed_steps(step, steps, warmup, world, dist, dev):
    # dist is None unless a process group is up (world > 1, or SM_BENCH_DIST=1)
    """W untimed steps, then K steps between barrier + synchronize on both sides; max over ranks."""
    import torch
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def kernel_ms(fn, reps):
    """Median launch duration (ms) of fn from HIP events on the launch stream (torch's current
    stream, which every sm.*_device call launches on)."""
    import torch
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    fn()
    torch.cuda.synchronize()
    for s, e in ev:
        s.record()
        fn()
        e.record()
    torch.cuda.synchronize()
    return float(np.median([s.elapsed_time(e) for s, e in ev]))


# compressed bytes each decode launch reads (set by main): the decoders' FETCH_SIZE splits into
# that stream, read once by coalesced 4-byte lanes (raw FETCH = 1/2 of the bytes, as the guide's
# wide reads), and far-copy sources and window reloads, 16-64-byte gathers whose raw FETCH is the
# 64-byte sectors they move (tools/probes/fetch_calib.hip, profiles/r06_fetch_calibration.txt)
DECODE_STREAM_BYTES = {}


def pmc_traffic(kernel):
    """HBM bytes per launch from the round's PMC file (rocprofv3 FETCH_SIZE/WRITE_SIZE passes, run
    separately from this process: counters cannot be collected inside a timed run), with where
    they came from: the file, the library build and commit the passes measured, and whether that
    build is the one this run loaded (a stale file is labelled, never silently reported)."""
    rel = os.path.join("profiles", ROUND + "_pmc.json")
    try:
        d = json.load(open(os.path.join(ROOT, rel)))
    except Exception:
        return None, {"file": rel, "present": False}
    lib = d.get("library")
    try:
        cur = load_package_cached().version()
    except Exception:
        cur = None
    src = {"file": rel, "library": lib, "commit": d.get("commit"), "this_run_library": cur,
           "same_build": bool(lib) and lib == cur}
    e = d.get(kernel, {})
    cstream = DECODE_STREAM_BYTES.get(kernel)
    if cstream is not None and "fetch_size_bytes_raw" in e:
        raw, wr = e["fetch_size_bytes_raw"], e["write_size_bytes"]
        rest = max(raw - cstream / 2.0, 0.0)
        src["calibrated"] = {"hbm_bytes_per_launch": round(cstream + rest + wr),
                             "stream_read": cstream, "gathers_and_reloads": round(rest), "written": wr,
                             "rule": "stream raw x2, gathers raw x1 (profiles/r06_fetch_calibration.txt); "
                                     "`traffic` applies x2 to all of FETCH (the guide's wide-read rule)"}
    return e.get("hbm_bytes_per_launch"), src


# the rocprof kernels behind each timed call (a fast-mode compress is the incompressible screen
# then the parse; avg_launch_ms is their sum, HIP events around the call)
ROCPROF_KERNELS = {
    "compress_fast": ["sm::k_literal_screen", "sm::k_compress_sc<0>"],
    "compress_fast_random": ["sm::k_literal_screen", "sm::k_compress_sc<0>"],
    "compress_fragments": ["sm::k_literal_screen", "sm::k_compress_sc<0>"],
    "uncompress": ["sm::k_decompress"],
    "uncompress_random": ["sm::k_decompress"],
    "uncompress_reference_streams": ["sm::k_decompress"],
}


def roofline(kernel, alg_bytes, ms):
    achieved = alg_bytes / (ms * 1e-3) / 1e9
    traffic, src = pmc_traffic(kernel)
    return {"kernel": kernel, "rocprof_kernels": ROCPROF_KERNELS.get(kernel), "bound": "hbm",
            "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBPS, 5), "traffic": traffic, "traffic_source": src,
            "algorithmic_bytes_per_launch": int(alg_bytes), "avg_launch_ms": round(ms, 4)}


# ---- CPU baseline ----------------------------------------------------------------------------

def cpu_quota():
    """CPUs the cgroup lets this process use (cgroup v2 cpu.max or v1 cfs quota), or None."""
    for path, parse in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                        ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", None)):
        try:
            if parse:
                q, per = parse(open(path).read())
                if q != "max":
                    return max(1, int(int(q) / int(per)))
            else:
                q = int(open(path).read())
                per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
                if q > 0:
                    return max(1, q // per)
        except (OSError, ValueError):
            pass
    return None


def cpu_cores():
    """Host threads for the CPU baseline: the CPUs this process may run on, capped by the cgroup
    quota and by OMP_NUM_THREADS when set (the GPU box sets it to the job's CPU share, 16 of
    the machine's 256; oversubscribing that share measured 0.9 GB/s instead of ~6)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    q = cpu_quota()
    if q:
        n = min(n, q)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(blocks_np, nblk=2048, reps=10, single_reps=3):
    """The oracle (Snappy.jl's algorithm restated in C, reference mode) and libsnappy 1.1.8, both
    OpenMP over blocks on every core this process may use, on the first nblk blocks of the
    headline workload; median over reps passes (single-thread figures: median over single_reps)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    threads = cpu_cores()
    sample = np.ascontiguousarray(blocks_np[:nblk])
    nblk = sample.shape[0]
    inp = sample.reshape(-1)
    in_off = np.arange(nblk, dtype=np.uint64) * BLOCK
    in_len = np.full(nblk, BLOCK, dtype=np.uint32)
    comp = np.empty(nblk * SLOT, dtype=np.uint8)
    comp_off = np.arange(nblk, dtype=np.uint64) * SLOT
    comp_cap = np.full(nblk, SLOT, dtype=np.uint32)
    comp_len = np.zeros(nblk, dtype=np.uint32)
    dec = np.empty(nblk * BLOCK, dtype=np.uint8)
    dec_len = np.zeros(nblk, dtype=np.uint32)
    st = np.zeros(nblk, dtype=np.int32)
    nbytes = inp.size

    def med(fn, n):
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts))

    def oracle_rates(th, n):
        tc = med(lambda: O.compress_batch(inp, in_off, in_len, comp, comp_off, comp_len, compat=False, nthreads=th), n)
        td = med(lambda: O.uncompress_batch(comp, comp_off, comp_len, dec, in_off, in_len, dec_len, st, nthreads=th), n)
        assert np.array_equal(dec, inp) and not st.any()
        return nbytes / tc / 1e9, nbytes / td / 1e9

    c_all, d_all = oracle_rates(threads, reps)
    c_one, d_one = oracle_rates(1, single_reps)
    res = {
        "value": round(2 / (1 / c_all + 1 / d_all), 4),
        "unit": "GB/s",
        "cores": threads,
        "kind": "port",
        "sample": "%d x 64 KiB text blocks (the first %d of the headline workload); reference-mode compress + "
                  "uncompress by oracle/snappy_oracle.c (-O3, OpenMP over blocks on %d threads = this job's CPU "
                  "share (affinity, cgroup quota, OMP_NUM_THREADS); os.cpu_count() = %d, %s); median of %d "
                  "passes" % (nblk, nblk, threads, os.cpu_count() or 0, cpu_model(), reps),
        "compress_GBps": round(c_all, 4),
        "uncompress_GBps": round(d_all, 4),
        "single_thread_compress_GBps": round(c_one, 4),
        "single_thread_uncompress_GBps": round(d_one, 4),
        "host_cpu": cpu_model(),
        "host_cpu_count": os.cpu_count(),
    }
    if O.libsnappy_batch() is not None:
        def lib_rates(th, n):
            tc = med(lambda: O.libsnappy_compress_batch(inp, in_off, in_len, comp, comp_off, comp_cap, comp_len, th), n)
            td = med(lambda: O.libsnappy_uncompress_batch(comp, comp_off, comp_len, dec, in_off, in_len, dec_len, th),
                     n)
            assert np.array_equal(dec, inp)
            return nbytes / tc / 1e9, nbytes / td / 1e9
        lc, ld = lib_rates(threads, reps)
        lc1, ld1 = lib_rates(1, single_reps)
        res["libsnappy_1.1.8"] = {
            "compress_GBps": round(lc, 4), "uncompress_GBps": round(ld, 4),
            "roundtrip_GBps": round(2 / (1 / lc + 1 / ld), 4), "threads": threads,
            "single_thread_compress_GBps": round(lc1, 4), "single_thread_uncompress_GBps": round(ld1, 4),
        }
        # README.md:37-45: Julia Snappy.jl is 3.8-48.7% slower than the libsnappy ccall, per file
        res["julia_estimate_single_thread"] = {
            "note": "ESTIMATE, not measured: libsnappy single-thread / (1.038 .. 1.487), the Julia/ccall "
                    "ratio range of the reference README.md:37-45",
            "compress_GBps": [round(lc1 / 1.487, 4), round(lc1 / 1.038, 4)],
            "uncompress_GBps": [round(ld1 / 1.487, 4), round(ld1 / 1.038, 4)],
        }
    return res


def config5_host_stream(sm, big, reps=3):
    """Config 5 as ONE stream through the single-buffer C entry points (sm_compress /
    sm_uncompress) from host buffers: PCIe-inclusive GB/s, best of reps."""
    import ctypes
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
    return {"host_compress_GBps": round(n / min(tc[1:]) / 1e9, 3),
            "host_uncompress_GBps": round(n / min(td[1:]) / 1e9, 3),
            "ratio": round(cl.value / n, 5),
            "ok": good and sm.last_uncompress_path() == 1}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)  # ~0.6 s timed on the headline: long enough for a busy sampler
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--blocks", type=int, default=10000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-large", action="store_true", help="skip the config-5 (644 MiB stream) workload")
    ap.add_argument("--no-random", action="store_true", help="skip the config-4 (random blocks) workload")
    ap.add_argument("--extras", action="store_true", help="also time dense/reference modes, validation and the "
                                                          "PCIe-inclusive single-stream entry points")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args))
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%d" % (args.gpus, world), file=sys.stderr)
        sys.exit(2)
    import torch
    ndev = torch.cuda.device_count()
    if ndev <= local_rank:
        print("bench.py: rank %d needs GPU %d but %d visible" % (rank, local_rank, ndev), file=sys.stderr)
        sys.exit(2)
    dist = None
    # SM_BENCH_DIST=1 (diagnostic): run the RCCL code path (process group, size all-gather,
    # barriers, max-over-ranks) even at one rank, to check it on a one-GPU box
    use_dist = world > 1 or os.environ.get("SM_BENCH_DIST") == "1"
    out_fd = 1
    if use_dist:
        # RCCL prints its version banner on stdout when a communicator comes up: keep stdout for
        # the one JSON line (written to the saved descriptor) and send everything else to stderr
        sys.stdout.flush()
        out_fd = os.dup(1)
        os.dup2(2, 1)
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if "MASTER_PORT" not in os.environ:
            with socket.socket() as s:
                s.bind(("127.0.0.1", 0))
                os.environ["MASTER_PORT"] = str(s.getsockname()[1])
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local_rank))
    dev = torch.device("cuda", local_rank)
    torch.cuda.set_device(dev)
    sm = load_package_cached()
    sm.context(local_rank)
    dmod = load_dist()
    reps = max(10, min(args.steps, 20))
    ok_all = True

    # ---- headline: configs 2 + 3, weak scaling -------------------------------------------
    blocks_np = text_blocks(args.blocks, 0x5EED + rank)
    batch = Batch(blocks_np, dev)
    sizes_all = torch.zeros(world * args.blocks, dtype=torch.int32, device=dev) if use_dist else None

    def step():
        batch.compress(sm)
        if use_dist:
            dist.all_gather_into_tensor(sizes_all, batch.comp_len)
        batch.uncompress(sm)

    elapsed = timed_steps(step, args.steps, args.warmup, world, dist, dev)
    headline_sizes = batch.comp_len.clone()
    comp_bytes = batch.comp_bytes()
    DECODE_STREAM_BYTES["uncompress"] = comp_bytes
    in_bytes = batch.in_bytes
    t_c = kernel_ms(lambda: batch.compress(sm), reps)
    t_d = kernel_ms(lambda: batch.uncompress(sm), reps)
    ok = batch.verify()
    ok_all &= ok
    c_bytes = in_bytes + comp_bytes + 4 * args.blocks
    d_bytes = comp_bytes + in_bytes
    kern = {"compress_fast": (t_c, c_bytes), "uncompress": (t_d, d_bytes)}
    dom = max(kern, key=lambda k: kern[k][0])
    value = 2.0 * in_bytes * args.steps * world / elapsed / 1e9

    # byte-identical (reference) mode on the same batch: Snappy.jl's own bytes (tests/ check
    # them against the oracle block for block); reported beside the headline, not in it
    t_ref = kernel_ms(lambda: batch.compress(sm, "reference"), 3)
    ref_comp = batch.comp_bytes()
    DECODE_STREAM_BYTES["uncompress_reference_streams"] = ref_comp
    # config 3's other half: the decode of the reference-mode (Snappy.jl's own)
    # streams of the same blocks, with its own roofline
    t_rd = kernel_ms(lambda: batch.uncompress(sm), reps)
    ref_mode = {"workload": "the headline's %d text blocks, byte-identical (reference) mode compress, and the "
                            "uncompress of those streams (config 3's reference-mode inputs)" % args.blocks,
                "compress_GBps": round(in_bytes / (t_ref * 1e-3) / 1e9, 3),
                "ratio": round(ref_comp / in_bytes, 5),
                "roundtrip_bit_exact": batch.verify()}
    ok_all &= ref_mode["roundtrip_bit_exact"]
    ref_streams = {"workload": "config 3: uncompress of the %d reference-mode (Snappy.jl byte-identical) streams of "
                               "the headline blocks, the stream set the oracle produces" % args.blocks,
                   "reference_streams_uncompress_GBps": round(in_bytes / (t_rd * 1e-3) / 1e9, 3),
                   "ratio": round(ref_comp / in_bytes, 5),
                   "roundtrip_bit_exact": ref_mode["roundtrip_bit_exact"],
                   "roofline": roofline("uncompress_reference_streams", ref_comp + in_bytes, t_rd)}
    batch.compress(sm, "fast")

    extras = {}
    if args.extras:
        extras.update(extra_modes(sm, batch, in_bytes))
    del batch
    torch.cuda.empty_cache()

    # ---- config 4: incompressible blocks ------------------------------------------------
    rnd = None
    if not args.no_random:
        rb = Batch(random_blocks(args.blocks, 0x5EED + 1 + rank), dev)

        def rstep():
            rb.compress(sm)
            rb.uncompress(sm)
        r_el = timed_steps(rstep, args.steps, args.warmup, world, dist, dev)
        rc_bytes = rb.comp_bytes()
        DECODE_STREAM_BYTES["uncompress_random"] = rc_bytes
        rt_c = kernel_ms(lambda: rb.compress(sm), reps)
        rt_d = kernel_ms(lambda: rb.uncompress(sm), reps)
        r_ok = rb.verify()
        ok_all &= r_ok
        rnd = {
            "workload": "config 4: %d x 64 KiB uniform random blocks per GPU (default_rng(0x5EED+1+rank)), "
                        "fast-mode compress + uncompress per step" % args.blocks,
            "GBps": round(2.0 * rb.in_bytes * args.steps * world / r_el / 1e9, 3),
            "ms_per_step": round(r_el / args.steps * 1e3, 4),
            "compress_GBps": round(rb.in_bytes / (rt_c * 1e-3) / 1e9, 3),
            "uncompress_GBps": round(rb.in_bytes / (rt_d * 1e-3) / 1e9, 3),
            "ratio": round(rc_bytes / rb.in_bytes, 6),
            "roundtrip_bit_exact": r_ok,
            "roofline": roofline("compress_fast_random", rb.in_bytes + rc_bytes + 4 * args.blocks, rt_c),
            "roofline_uncompress": roofline("uncompress_random", rb.in_bytes + rc_bytes, rt_d),
        }
        del rb
        torch.cuda.empty_cache()

    # ---- config 5: one 644 MiB stream, strong scaling --------------------------------------
    large = None
    big = None
    if not args.no_large:
        big = large_corpus()
        nfrag = (big.size + BLOCK - 1) // BLOCK
        lo, hi = dmod.shard_range(nfrag, rank, world)
        sh = StreamShard(big, lo, hi, dev)

        def lstep():
            sh.compress(sm)
            sh.index(dmod, rank, world)
            sh.place(sm)
            sh.uncompress(sm)
        l_el = timed_steps(lstep, args.steps, args.warmup, world, dist, dev)
        sh.index(dmod, rank, world)
        sh.place(sm)
        lt_c = kernel_ms(lambda: sh.compress(sm), reps)
        lt_p = kernel_ms(lambda: sh.place(sm), reps)
        lt_d = kernel_ms(lambda: sh.uncompress(sm), reps)
        l_ok = sh.verify(sm)
        lc_local = int(sh.comp_len.to(torch.int64).sum())
        # the stream's length read back from the materialised ranges (summed over ranks), which
        # must equal the all-gathered index's total
        rb = torch.tensor([sh.range_bytes()], dtype=torch.int64, device=dev)
        if dist is not None:
            dist.all_reduce(rb)
        stream_len = int(rb.item())
        l_ok = l_ok and stream_len == int(sh.stream_len.item())
        stream_sha = None
        if world == 1:  # the whole stream is rank 0's range: decode it through the single-buffer API
            import hashlib
            host = sh.d_stream[:stream_len].cpu().numpy()
            stream_sha = hashlib.sha256(host.tobytes()).hexdigest()
            back = sm.uncompress(host.tobytes())
            l_ok = l_ok and back == big.tobytes()
            del host, back
        ok_all &= l_ok
        per_rank_ms = l_el / args.steps * 1e3
        large = {
            "workload": "config 5: one %d-B (644 MiB) stream = %d fragments, %d..%d per GPU (contiguous shards); "
                        "per step: fast-mode fragment compress + RCCL all-gather of the u32 fragment sizes + "
                        "offset scan + the fragments placed at their stream offsets (sm_place_fragments_device; "
                        "rank 0 writes the varint header) + uncompress of the placed fragments"
                        % (big.size, nfrag, nfrag // world, (nfrag + world - 1) // world),
            "scaling": "strong",
            "GBps": round(2.0 * big.size * args.steps / l_el / 1e9, 3),
            "ms_per_step": round(per_rank_ms, 4),
            "fragments_rank0": hi - lo,
            "compress_GBps_per_gpu": round(sh.in_bytes / (lt_c * 1e-3) / 1e9, 3),
            "uncompress_GBps_per_gpu": round(sh.in_bytes / (lt_d * 1e-3) / 1e9, 3),
            "place_GBps_per_gpu": round(2 * lc_local / (lt_p * 1e-3) / 1e9, 3),
            "stream_bytes": stream_len,
            "stream_bytes_source": "the materialised ranges' lengths summed over ranks (= the gathered index total)",
            "stream_sha256": stream_sha,
            "ratio": round(stream_len / big.size, 5),
            "roundtrip_bit_exact": l_ok,
            "roofline": roofline("compress_fragments", sh.in_bytes + lc_local + 4 * sh.nfrag, lt_c),
        }
        del sh
        torch.cuda.empty_cache()

    if args.extras and rank == 0 and world == 1:
        extras["single_call"] = single_call_table(sm)
        if big is None:
            big = large_corpus()
        extras["config5_host_stream"] = config5_host_stream(sm, big)
        ok_all &= extras["config5_host_stream"]["ok"]

    rccl = None
    if use_dist:
        t = torch.tensor([0 if ok_all else 1], dtype=torch.int32, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ok_all = int(t.item()) == 0
        # what the communicator saw: its backend and size, and the gathered size table (every
        # rank's u32 compressed sizes; this rank's own slice must equal its local sizes)
        own = sizes_all[rank * args.blocks:(rank + 1) * args.blocks]
        rccl = {"backend": str(dist.get_backend()), "world": dist.get_world_size(),
                "sizes_gathered": int(sizes_all.numel()),
                "own_slice_matches": bool(torch.equal(own, headline_sizes))}
        ok_all &= rccl["own_slice_matches"]

    cpu = None
    if rank == 0 and not args.no_cpu:
        cpu = cpu_baseline(blocks_np)

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
                "workload": "configs 2+3: %d x 64 KiB text blocks per GPU, fast-mode compress + uncompress round "
                            "trip per step" % args.blocks,
                "blocks_per_gpu": args.blocks,
                "block_bytes": BLOCK,
                "parallelism": "dp%d (blocks sharded per rank, RCCL size all-gather)" % world,
            },
            "compress_GBps": round(in_bytes / (t_c * 1e-3) / 1e9, 3),
            "uncompress_GBps": round(in_bytes / (t_d * 1e-3) / 1e9, 3),
            "ratio": round(comp_bytes / in_bytes, 5),
            "roundtrip_bit_exact": ok,
            "all_roundtrips_bit_exact": ok_all,
            "roofline": roofline(dom, kern[dom][1], kern[dom][0]),
            "roofline_other": roofline(*[(k, v[1], v[0]) for k, v in kern.items() if k != dom][0]),
            "rccl": rccl,
            "random": rnd,
            "large": large,
            "reference_mode": ref_mode,
            "reference_streams_uncompress_GBps": ref_streams["reference_streams_uncompress_GBps"],
            "reference_streams": ref_streams,
            "cpu_baseline": cpu,
        }
        line.update(extras)
        sys.stdout.flush()
        os.write(out_fd, (json.dumps(line) + "\n").encode())
    if use_dist:
        dist.destroy_process_group()
    if not ok_all:
        sys.exit(3)


def extra_modes(sm, batch, in_bytes):
    """--extras: dense mode and its streams' decode, validation (the reference-mode streams'
    decode is in the default line: `reference_streams`)."""
    import torch
    out = {}
    t_dc = kernel_ms(lambda: batch.compress(sm, "dense"), 5)
    out["dense_compress_GBps"] = round(in_bytes / (t_dc * 1e-3) / 1e9, 3)
    out["dense_ratio"] = round(batch.comp_bytes() / in_bytes, 5)
    t_dd = kernel_ms(lambda: batch.uncompress(sm), 5)
    out["dense_streams_uncompress_GBps"] = round(in_bytes / (t_dd * 1e-3) / 1e9, 3)
    out["dense_ok"] = batch.verify()
    batch.compress(sm, "fast")
    vst = torch.full_like(batch.status, -1)
    t_v = kernel_ms(lambda: sm.validate_batch_device(batch.d_comp, batch.comp_off, batch.comp_len, vst), 5)
    out["validate_GBps"] = round(in_bytes / (t_v * 1e-3) / 1e9, 3)
    out["validate_ok"] = int(vst.abs().sum()) == 0
    return out


# test/benchmarks.jl:9-16 (the files) and README.md:37-45 (Julia 0.6 on a Mac, median of 10,000
# calls; MB = 2^20 B; compress rates per input byte, uncompress rates per COMPRESSED byte,
# test/benchmarks.jl:49,78)
REFERENCE_SINGLE_CALL = {
    "alice29.txt": ("txt", 243 * 2**20, 324 * 2**20),
    "html": ("html", 672 * 2**20, 288 * 2**20),
    "fireworks.jpeg": ("jpeg", 1.92 * 2**30, 6.73 * 2**30),
    "paper-100k.pdf": ("pdf", 3.43 * 2**30, 4.24 * 2**30),
    "urls.10K": ("urls", 357 * 2**20, 332 * 2**20),
    "sample-tweet.json": ("json", 744 * 2**20, 420 * 2**20),
}


def single_call_table(sm, min_s=0.25, max_calls=2000):
    """The drop-in single-buffer entry points (sm_compress / sm_uncompress: host buffers in and
    out, PCIe and launch latency included) on the reference's own benchmark files, timed the way
    test/benchmarks.jl times Snappy.jl: the median of repeated calls, compress rate per input
    byte, uncompress rate per compressed byte (of the stream the same mode produced).  Each row
    carries the reference's published Julia rate for the same file (README.md:37-45; other
    hardware) and the decode path the library took."""
    rows = {}
    for fname, (tag, ref_c, ref_d) in REFERENCE_SINGLE_CALL.items():
        data = open(os.path.join(TESTDATA, fname), "rb").read()
        row = {"file": fname, "bytes": len(data)}
        for mode in ("fast", "dense", "reference"):  # (dense: the sm_snappy_* entry points' default)
            comp = sm.compress(data, mode=mode)
            assert sm.uncompress(comp) == data

            def med(fn):
                ts, t_end = [], time.perf_counter() + min_s
                while len(ts) < 10 or (time.perf_counter() < t_end and len(ts) < max_calls):
                    t0 = time.perf_counter()
                    fn()
                    ts.append(time.perf_counter() - t0)
                return float(np.median(ts))
            tc = med(lambda: sm.compress(data, mode=mode))
            td = med(lambda: sm.uncompress(comp))
            row[mode] = {"compressed_bytes": len(comp),
                         "compress_us": round(tc * 1e6, 1), "compress_MBps": round(len(data) / tc / 2**20, 1),
                         "uncompress_us": round(td * 1e6, 1), "uncompress_MBps": round(len(comp) / td / 2**20, 1),
                         "uncompress_path": sm.last_uncompress_path()}
        row["julia_published_MBps"] = {"compress": round(ref_c / 2**20, 1), "uncompress": round(ref_d / 2**20, 1)}
        rows[tag] = row
    return {"workload": "single calls from host buffers on test/benchmarks.jl's files; MB/s with MB = 2^20 B; "
                        "uncompress per compressed byte; median over >= 10 calls; modes fast, dense (the snappy-c-shaped "
                        "entry points' default) and reference (Snappy.jl's bytes)",
            "files": rows}


if __name__ == "__main__":
    main()
