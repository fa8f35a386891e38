"""Data-parallel sharding of LFB extraction: frames are independent, so each
rank (one process per GPU) takes a contiguous shard of the frame index range; no collective is on
the data path.  ``gather_rows`` assembles the full ``(N, C)`` feature bank on every rank (or only
to be written by rank 0) once extraction is done — one all_gather of the shards, padded to the
largest shard.  Works with any torch.distributed backend (RCCL on the GPU box, gloo in tests)."""
import torch
import torch.distributed as dist


def shard_range(n, rank, world):
    """[start, stop) of rank's contiguous shard; the first n % world ranks get one extra item."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    base, extra = divmod(n, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_rows(local, n_total, group=None):
    """All-gather per-rank row blocks (rank order) into one [n_total, C] tensor on every rank."""
    world = dist.get_world_size(group)
    sizes = [shard_range(n_total, r, world) for r in range(world)]
    cap = max(b - a for a, b in sizes)
    padded = local.new_zeros((cap,) + tuple(local.shape[1:]))
    padded[: local.shape[0]] = local
    bufs = [torch.empty_like(padded) for _ in range(world)]
    dist.all_gather(bufs, padded, group=group)
    return torch.cat([bufs[r][: b - a] for r, (a, b) in enumerate(sizes)], dim=0)
