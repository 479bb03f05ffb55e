"""The sharded single-stream path (snappy.jl_amd/dist.py) with the HIP compressor in every rank.

World size 2 over gloo, both ranks on GPU 0 (the one-GPU box): each rank compresses its
contiguous fragments with sm_compress_fragments_device (table size of the whole stream, no
headers), the u32 sizes are all-gathered, each rank places its fragments at their stream offsets
with sm_place_fragments_device, and the concatenated ranges must
* equal the oracle's (= Snappy.jl's) stream byte for byte in reference mode;
* decode bit-exactly under the oracle in fast mode;
and stream_offsets_device (the bench's sync-free index) must give the same offsets."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT, load_package, read_testfile

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _gather_ranges(dist, world, rng):
    """Every rank's materialised byte range (a uint8 CPU tensor) to all ranks over gloo, in rank
    order (padded to the longest: gloo's all_gather takes equal shapes).  The ranges are
    contiguous in the stream, so their concatenation is the stream; nothing is placed here."""
    import torch
    n = torch.tensor([rng.numel()], dtype=torch.int64)
    ns = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(ns, n)
    m = max(int(x) for x in ns)
    pad = torch.zeros(m, dtype=torch.uint8)
    pad[: rng.numel()] = rng
    parts = [torch.zeros(m, dtype=torch.uint8) for _ in range(world)]
    dist.all_gather(parts, pad)
    return b"".join(parts[r][: int(ns[r])].numpy().tobytes() for r in range(world))


def _shard_and_place(sm, D, dist, world, rank, data_np, mode, dev):
    """One rank of the sharded stream, entirely through the product: its contiguous fragments by
    sm_compress_fragments_device, the global offsets from the all-gathered u32 sizes
    (stream_offsets_device; gloo: CPU tensors), the fragments placed at those offsets in its own
    device range by sm_place_fragments_device (rank 0: varint header first).  Returns the range
    (CPU) and the fragment count."""
    import torch
    sys.path.insert(0, ROOT)
    import bench
    total = data_np.size
    nfrag = (total + bench.BLOCK - 1) // bench.BLOCK
    lo, hi = D.shard_range(nfrag, rank, world)
    sh = bench.StreamShard(data_np, lo, hi, dev)
    sm.compress_fragments_device(sh.d_in, sh.in_off, sh.in_len, sh.d_comp, sh.comp_off, sh.comp_len, total,
                                 mode=mode)
    torch.cuda.synchronize()
    offs, tot = D.stream_offsets_device(sh.comp_len.to(torch.int64).cpu(), total, rank, world)
    sh.offsets = offs.to(dev)
    sh.place(sm)
    torch.cuda.synchronize()
    assert int(sh.place_status.item()) == 0
    rng = sh.d_stream[: sh.range_bytes()].cpu()
    # the placed fragments decode where they were placed (sm_uncompress_fragments_device)
    sh.stream_len = tot
    assert sh.verify(sm)
    return rng, hi - lo, int(tot.item())


def _worker(rank, world, port, fname, mode, q):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sm = load_package()
        from importlib import import_module
        D = import_module("snappy_jl_amd.dist")
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        data = np.frombuffer(read_testfile(fname), dtype=np.uint8)
        rng, _, total_c = _shard_and_place(sm, D, dist, world, rank, data, mode, dev)
        stream = _gather_ranges(dist, world, rng)
        assert len(stream) == total_c
        q.put((rank, stream))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fname", ["html_x_4", "urls.10K", "plrabn12.txt"])
@pytest.mark.parametrize("mode", ["reference", "fast"])
def test_sharded_stream_hip_compressor(oracle, gpu_available, fname, mode):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fname, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    raw = read_testfile(fname)
    assert outs[0] == outs[1]
    if mode == "reference":
        assert outs[0] == oracle.compress(raw)
    assert oracle.uncompress(outs[0]) == raw


def _config5_worker(rank, world, port, q):
    """One rank of the config-5 stream: its contiguous fragments compressed,
    indexed and placed at their global offsets by the product (_shard_and_place)."""
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        sm = load_package()
        from importlib import import_module
        D = import_module("snappy_jl_amd.dist")
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        big = bench.large_corpus()
        rng, nf, total_c = _shard_and_place(sm, D, dist, world, rank, big, "fast", dev)
        stream = _gather_ranges(dist, world, rng)
        assert len(stream) == total_c
        q.put((nf, stream if rank == 0 else None))
    finally:
        dist.destroy_process_group()


def test_config5_sharded_two_ranks(oracle, gpu_available):
    """The 644 MiB config-5 stream's 10,304 fragments sharded over two gloo ranks on GPU 0
    (5,152 each), each rank's fragments placed in its own device range by the product: the
    ranges' concatenation is byte-identical (SHA-256) to single-GPU sm_compress(fast) of the whole
    input and decodes under the oracle."""
    import hashlib
    import torch
    sys.path.insert(0, ROOT)
    import bench
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_config5_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in range(world)]
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert sorted(r[0] for r in res) == [5152, 5152]
    sharded = [r[1] for r in res if r[1] is not None][0]
    # the single-GPU stream of the same input through the single-buffer API (sm_compress, fast)
    sm = load_package()
    big = bench.large_corpus()
    single = sm.compress(big.tobytes(), mode="fast")
    assert hashlib.sha256(sharded).digest() == hashlib.sha256(single).digest()
    assert oracle.uncompress(sharded) == big.tobytes()
