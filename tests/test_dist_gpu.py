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
