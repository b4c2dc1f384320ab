"""Batch split across ranks: every cloud is independent and no operator
mixes clouds (e.g. query_ball_point_gpu indexes per batch, tf_grouping_g.cu:4-8), so the global
batch is split contiguously, B clouds per rank, with no collective in the data path. The only
collectives are the timing max and the per-cloud checksum gather, both outside the timed
region. Works with any torch.distributed backend (RCCL/"nccl" on the MI355X node, gloo in the
CPU tests)."""
import torch


def shard_ids(rank, world, per_rank):
    """Global cloud ids owned by `rank` (contiguous split)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    return list(range(rank * per_rank, (rank + 1) * per_rank))


def set_ids(rank, world, per_rank, set_index):
    """Global cloud ids of buffer set `set_index` on `rank`: the pipelined bench rotates over
    several buffer sets, each holding its own clouds, so set i of every rank is a contiguous
    global batch of world * per_rank clouds after the i batches before it."""
    return [set_index * world * per_rank + c for c in shard_ids(rank, world, per_rank)]


def min_over_ranks(value, device="cpu"):
    """all_reduce(MIN) of one float (e.g. a 0/1 parity flag) across ranks."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return float(t.item())


def max_over_ranks(value, device="cpu"):
    """all_reduce(MAX) of one float (the elapsed time) across ranks."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def cloud_checksums(outs, B):
    """Per-cloud float64 checksum of a step's outputs (each output has the batch first)."""
    return torch.stack([torch.stack([o[b].double().sum() for o in outs]).sum() for b in range(B)])


def gather_checksums(sums):
    """all_gather of the per-cloud checksums, concatenated in rank (= global cloud id) order."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return sums
    parts = [torch.zeros_like(sums) for _ in range(dist.get_world_size())]
    dist.all_gather(parts, sums)
    return torch.cat(parts)
