"""Multi-GPU sharding of the block codec: one process per GPU, torch.distributed (RCCL on
ROCm; gloo in the CPU tests).

The reference is single-threaded; its 64 KiB fragments are independent
(src/Snappy.jl:29-33, src/internal.jl:129,190 -- the table is reset and offsets are
block-relative), so the path shards with no data-path collective:

* batch mode (BASELINE configs 2-4): rank r owns its own contiguous run of independent
  blocks; nothing is exchanged.  `gather_sizes` is only needed when a global index of the
  compressed blocks is wanted.
* one large stream (config 5): fragments [lo, hi) of the stream go to each rank; each rank
  compresses its fragments (no per-fragment header, table size from the TOTAL length, Q2);
  one all-gather of the u32 fragment sizes gives every rank the global exclusive scan, i.e.
  where its fragments land after the varint(total) header (`stream_offsets_device`).  That
  all-gather is the only collective on the path (10,304 fragments x 4 B for 644 MiB).  Each
  rank then writes its fragments at those offsets into its byte range of the stream with
  sm_place_fragments_device (rank 0: the varint header first); the ranges are contiguous, so
  a D2H of each range at its offset (or a gather of the ranges) is the stream.

The per-rank compressor is injected (`compress_fn`) so that the CPU tests can run the
distributed logic with gloo, using the oracle as a stand-in for the GPU kernels.
"""
import numpy as np

BLOCK = 65536
SM_OUT_LEN_ERROR = 0xFFF00000  # include/snappy_mi355x.h: d_out_len error marks


def shard_range(nitems, rank, world):
    """Contiguous [lo, hi) of nitems for rank (the first nitems % world ranks get one more)."""
    base, extra = divmod(nitems, world)
    lo = rank * base + min(rank, extra)
    hi = lo + base + (1 if rank < extra else 0)
    return lo, hi


def fragment_bounds(total_len):
    """(offset, length) of every 64 KiB fragment of a stream (src/Snappy.jl:29)."""
    nfrag = (total_len + BLOCK - 1) // BLOCK
    offs = np.arange(nfrag, dtype=np.int64) * BLOCK
    lens = np.minimum(BLOCK, total_len - offs).astype(np.int64)
    return offs, lens


def varint32(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def gather_sizes(local_sizes, group=None):
    """All-gather per-rank u32 size vectors (ragged) -> one global int64 vector, rank order.

    local_sizes: 1-D torch tensor on the device of the process group's backend."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    n = torch.tensor([local_sizes.numel()], dtype=torch.int64, device=local_sizes.device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n, group=group)
    counts = [int(c.item()) for c in counts]
    m = max(counts) if counts else 0
    buf = torch.zeros(m, dtype=torch.int64, device=local_sizes.device)
    buf[: local_sizes.numel()] = local_sizes.to(torch.int64)
    parts = [torch.zeros_like(buf) for _ in range(world)]
    dist.all_gather(parts, buf, group=group)
    return torch.cat([p[:c] for p, c in zip(parts, counts)])


def collective_device(group=None):
    """Where a collective's tensors must live: the current GPU under nccl (RCCL), the CPU under
    gloo."""
    import torch
    import torch.distributed as dist
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def compress_stream_sharded(data, rank, world, compress_fn, group=None):
    """Compress one stream `data` (bytes) across `world` ranks.

    compress_fn(list_of_fragments, total_len) -> list of compressed fragments (no headers).
    Returns (header, local_fragments, global_offsets_of_local_fragments, total_compressed_len);
    header + all ranks' fragments written at their offsets is the snappy stream of `data` (on the
    device: sm_place_fragments_device writes them there, place_fragments_device in the package)."""
    import torch
    total = len(data)
    offs, lens = fragment_bounds(total)
    lo, hi = shard_range(len(offs), rank, world)
    frags = [data[int(o): int(o) + int(l)] for o, l in zip(offs[lo:hi], lens[lo:hi])]
    out = compress_fn(frags, total) if frags else []
    local = torch.tensor([len(x) for x in out], dtype=torch.int64, device=collective_device(group))
    sizes = gather_sizes(local, group).cpu().numpy()
    header = varint32(total)
    starts = len(header) + np.concatenate([[0], np.cumsum(sizes)[:-1]]) if len(sizes) else np.zeros(0, np.int64)
    return header, out, starts[lo:hi], int(len(header) + sizes.sum())


def stream_offsets_device(local_sizes, total_len, rank, world, group=None):
    """Device-side global index of a stream sharded by `shard_range` (config 5): all-gather the
    ranks' u32 fragment sizes (the only collective on the path; RCCL under nccl), then the
    exclusive scan behind the varint(total_len) header.  local_sizes: this rank's fragment
    sizes on the collective device.  Shard sizes are static (shard_range), so there is no host
    round trip: every rank pads to the largest shard.  Returns (global offsets of this rank's
    fragments, the stream's total length as a 1-element tensor) on local_sizes' device.

    The all-gather runs whenever a process group is up, world 1 included (so the RCCL path is
    the one measured at any world size).  A fragment whose size is a compressor error mark
    (>= SM_OUT_LEN_ERROR = 0xfff00000 as u32, i.e. negative as torch int32) poisons the result
    without a host round trip: the returned total is -1 on every rank."""
    import torch
    import torch.distributed as dist
    nfrag = (total_len + BLOCK - 1) // BLOCK
    bounds = [shard_range(nfrag, r, world) for r in range(world)]
    m = max(hi - lo for lo, hi in bounds)
    dev = local_sizes.device
    hl = len(varint32(total_len))
    if nfrag == 0:  # an empty stream: the header alone
        return torch.zeros(0, dtype=torch.int64, device=dev), torch.full((1,), hl, dtype=torch.int64, device=dev)
    if world == 1 and not (dist.is_available() and dist.is_initialized()):
        sizes = local_sizes.to(torch.int64)
    else:
        buf = torch.zeros(m, dtype=torch.int64, device=dev)
        buf[: local_sizes.numel()] = local_sizes.to(torch.int64)
        parts = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(parts, buf, group=group)
        sizes = torch.cat([p[: hi - lo] for p, (lo, hi) in zip(parts, bounds)])
    sizes = sizes & 0xFFFFFFFF  # (u32 sizes held in int32 tensors)
    bad = (sizes >= SM_OUT_LEN_ERROR).any()
    incl = torch.cumsum(sizes, 0)
    starts = hl + incl - sizes
    lo, hi = bounds[rank]
    total = torch.where(bad, torch.full((1,), -1, dtype=torch.int64, device=dev), incl[-1:] + hl)
    return starts[lo:hi], total
