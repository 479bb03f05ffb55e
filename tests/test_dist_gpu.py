"""The sharded single-stream path (snappy.jl_amd/dist.py) with the HIP compressor in every rank.

World size 2 over gloo, both ranks on GPU 0 (the one-GPU box): each rank compresses its
contiguous fragments with sm_compress_fragments_device (table size of the whole stream, no
headers), the u32 sizes are all-gathered, and the assembled stream must
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
        data = read_testfile(fname)

        def hip_fragments(frags, total):
            n = len(frags)
            lens = np.array([len(f) for f in frags], dtype=np.int32)
            buf = np.frombuffer(b"".join(frags), dtype=np.uint8).copy()
            d_in = torch.from_numpy(buf).to(dev)
            in_off = torch.from_numpy(np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)).to(dev)
            d_len = torch.from_numpy(lens).to(dev)
            slot = 76496
            d_out = torch.zeros(n * slot, dtype=torch.uint8, device=dev)
            o_off = torch.arange(n, dtype=torch.int64, device=dev) * slot
            o_len = torch.zeros(n, dtype=torch.int32, device=dev)
            sm.compress_fragments_device(d_in, in_off, d_len, d_out, o_off, o_len, total, mode=mode)
            torch.cuda.synchronize()
            out, ol = d_out.cpu().numpy(), o_len.cpu().numpy()
            return [out[i * slot: i * slot + int(ol[i])].tobytes() for i in range(n)]

        header, local, offs, total_c = D.compress_stream_sharded(data, rank, world, hip_fragments)
        # the bench's device-side index over the same sizes (gloo: CPU tensors)
        sizes = torch.tensor([len(x) for x in local], dtype=torch.int64)
        offs2, tot2 = D.stream_offsets_device(sizes, len(data), rank, world)
        assert offs2.tolist() == list(map(int, offs)) and int(tot2.item()) == total_c
        pieces = [None] * world
        dist.all_gather_object(pieces, list(zip(list(map(int, offs)), local)))
        allp = [p for rp in pieces for p in rp]
        q.put((rank, D.assemble(header, allp, total_c)))
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
    """One rank of the config-5 stream: its contiguous fragments through
    compress_fragments_device, the global offsets through stream_offsets_device (the gathered
    u32 sizes), its compressed bytes placed at those offsets."""
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
        nfrag = (big.size + bench.BLOCK - 1) // bench.BLOCK
        lo, hi = D.shard_range(nfrag, rank, world)
        sh = bench.StreamShard(big, lo, hi, dev)
        sh.compress(sm)
        torch.cuda.synchronize()
        sizes = sh.comp_len.to(torch.int64).cpu()  # gloo: the size all-gather on CPU tensors
        offs, total_c = D.stream_offsets_device(sizes, big.size, rank, world)
        comp = sh.d_comp.cpu().numpy()
        local = [(int(offs[i]), comp[i * bench.SLOT: i * bench.SLOT + int(sizes[i])].tobytes())
                 for i in range(hi - lo)]
        # the ranks' pieces to rank 0 as byte tensors (gloo all_gather needs equal shapes: pad)
        blob = np.frombuffer(b"".join(p for _, p in local), dtype=np.uint8)
        n = torch.tensor([blob.size], dtype=torch.int64)
        ns = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(ns, n)
        m = int(max(int(x) for x in ns))
        pad = torch.zeros(m, dtype=torch.uint8)
        pad[: blob.size] = torch.from_numpy(blob.copy())
        parts = [torch.zeros(m, dtype=torch.uint8) for _ in range(world)]
        dist.all_gather(parts, pad)
        first = torch.tensor([local[0][0]], dtype=torch.int64)
        firsts = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(firsts, first)
        if rank == 0:
            stream = bytearray(int(total_c.item()))
            hdr = D.varint32(big.size)
            stream[: len(hdr)] = hdr
            for r in range(world):
                o, k = int(firsts[r].item()), int(ns[r].item())
                stream[o: o + k] = parts[r][:k].numpy().tobytes()
            q.put((hi - lo, bytes(stream)))
        else:
            q.put((hi - lo, None))
    finally:
        dist.destroy_process_group()


def test_config5_sharded_two_ranks(oracle, gpu_available):
    """The 644 MiB config-5 stream's 10,304 fragments sharded over two gloo ranks on GPU 0
    (5,152 each): the assembled stream is byte-identical to the single-GPU fragment output and
    decodes under the oracle."""
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
    # the single-GPU fragment output of the same stream
    sm = load_package()
    dev = torch.device("cuda", 0)
    big = bench.large_corpus()
    sh = bench.StreamShard(big, 0, 10304, dev)
    sh.compress(sm)
    torch.cuda.synchronize()
    sizes = sh.comp_len.cpu().numpy().astype(np.int64)
    comp = sh.d_comp.cpu().numpy()
    hdr = bytes(sm.encode32(big.size))
    single = hdr + b"".join(comp[i * bench.SLOT: i * bench.SLOT + int(sizes[i])].tobytes() for i in range(10304))
    assert hashlib.sha256(sharded).digest() == hashlib.sha256(single).digest()
    assert oracle.uncompress(sharded) == big.tobytes()
