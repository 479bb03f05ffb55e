"""Multi-process (world_size 2, gloo, CPU) tests of the sharded path in snappy.jl_amd/dist.py.

The GPU kernels are replaced by the oracle (the checker) as each rank's compressor, so what is
under test is the distributed logic: shard ranges, the u32 size all-gather, the global offset
scan and the assembly -- sharded output must equal the single-process reference stream."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT, load_package, read_testfile


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _join(header, pieces_with_offsets, total_len):
    """The checker's concatenation of (offset, bytes) pieces behind the header (the product
    places them on the device: sm_place_fragments_device, tests/test_dist_gpu.py)."""
    buf = bytearray(total_len)
    buf[: len(header)] = header
    for off, piece in pieces_with_offsets:
        buf[int(off): int(off) + len(piece)] = piece
    return bytes(buf)


def _worker(rank, world, port, fname, q):
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle as O
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sm_dist = load_package().__dict__  # noqa: F841  (package import must work on every rank)
        from importlib import import_module
        D = import_module("snappy_jl_amd.dist")
        data = read_testfile(fname)

        def cfn(frags, total):
            return [O.compress_fragment(f, total) for f in frags]

        header, local, offs, total_c = D.compress_stream_sharded(data, rank, world, cfn)
        pieces = [None] * world
        dist.all_gather_object(pieces, list(zip(offs.tolist(), local)))
        allp = [p for rp in pieces for p in rp]
        stream = _join(header, allp, total_c)
        q.put((rank, stream))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("fname", ["html_x_4", "urls.10K", "smallrandom1.bin", "plrabn12.txt"])
def test_sharded_stream_equals_reference(oracle, fname):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, fname, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ref = oracle.compress(read_testfile(fname))
    for r in range(world):
        assert outs[r] == ref


def test_shard_range_partitions():
    D = load_package()
    from importlib import import_module
    D = import_module("snappy_jl_amd.dist")
    for n in (0, 1, 7, 10304, 10000):
        for w in (1, 2, 3, 8):
            rs = [D.shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(w - 1))
            sizes = [hi - lo for lo, hi in rs]
            assert max(sizes) - min(sizes) <= 1


def test_fragment_bounds_match_reference_loop():
    from importlib import import_module
    load_package()
    D = import_module("snappy_jl_amd.dist")
    # src/Snappy.jl:29 -- for i in 0:65536:n ; the empty tail fragment emits nothing
    for n in (0, 1, 65535, 65536, 65537, 675282944):
        offs, lens = D.fragment_bounds(n)
        assert lens.sum() == n
        assert (lens > 0).all()
        assert len(offs) == (n + 65535) // 65536
    assert D.varint32(675282944) == bytes.fromhex("80 80 80 c2 02".replace(" ", ""))


def _offsets_worker(rank, world, port, total, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        load_package()
        from importlib import import_module
        D = import_module("snappy_jl_amd.dist")
        nfrag = (total + 65535) // 65536
        lo, hi = D.shard_range(nfrag, rank, world)
        # stand-in fragment sizes, a function of the global fragment index
        local = torch.tensor([1000 + (7919 * i) % 5000 for i in range(lo, hi)], dtype=torch.int32)
        offs, tot = D.stream_offsets_device(local, total, rank, world)
        q.put((rank, offs.tolist(), int(tot.item())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_stream_offsets_device_world(world):
    """bench.py's config-5 index (the RCCL all-gather path, gloo here) equals the serial scan."""
    total = 675282944 // 64 + 12345  # 162 fragments, ragged tail
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_offsets_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    outs = {r: (o, t) for r, o, t in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    nfrag = (total + 65535) // 65536
    sizes = [1000 + (7919 * i) % 5000 for i in range(nfrag)]
    hl = 4  # varint(10563041)
    starts = list(hl + np.concatenate([[0], np.cumsum(sizes)[:-1]]))
    got = [x for r in range(world) for x in outs[r][0]]
    assert got == [int(x) for x in starts]
    assert all(outs[r][1] == hl + sum(sizes) for r in range(world))
