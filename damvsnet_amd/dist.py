"""Multi-GPU execution: one process per GPU over torch.distributed (backend "nccl" = RCCL on ROCm).

The unit of work is one reference view -> one depth map, and units are independent (each test
sample is its own ``__getitem__``, datasets/general_eval.py:111). Throughput therefore scales by
sharding the sample list over ranks — the reference's own pattern (DistributedSampler,
train.py:492-496) — with NO collective on the data path. Collectives are used only outside it:
a MAX of the per-rank elapsed time for benchmarking, and an optional gather of the finished
(small) depth/confidence maps to one rank.

Latency (one depth map over several GPUs) is a separate mode: damvsnet_amd/sharded.py shards each stage's cost
volume along the depth-hypothesis axis (north_star), re-shards it to row slabs for the U-Net (whose 3x3x3 kernels
and stride-2 levels couple all planes) with one all-to-all, exchanges slab halos per layer and all-gathers the
regressed rows. See DESIGN.md section 7 "Multi-GPU".
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_indices(n: int, rank: int, world_size: int):
    """Interleaved shard of range(n) (DistributedSampler order, no padding): every index exactly once."""
    return list(range(rank, n, world_size))


def max_over_ranks(x: float, device=None) -> float:
    rank, ws = world()
    if ws == 1:
        return float(x)
    t = torch.tensor([float(x)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_maps(local: dict, n: int, dst: int = 0):
    """Gather {index: tensor} from all ranks to ``dst``; returns the list ordered by index on dst
    (None elsewhere). Tensors travel as CPU copies (object gather): the maps are small and this runs
    once per batch, off the data path."""
    rank, ws = world()
    items = {i: t.detach().cpu() for i, t in local.items()}
    if ws == 1:
        return [items[i] for i in range(n)]
    bucket = [None] * ws if rank == dst else None
    dist.gather_object(items, bucket, dst=dst)
    if rank != dst:
        return None
    merged = {}
    for part in bucket:
        merged.update(part)
    if sorted(merged) != list(range(n)):
        raise RuntimeError("gathered indices %s do not cover 0..%d" % (sorted(merged), n - 1))
    return [merged[i] for i in range(n)]


def run_sharded(fn, n: int, gather: bool = True):
    """Run ``fn(index) -> tensor`` over this rank's shard of range(n); optionally gather to rank 0."""
    rank, ws = world()
    local = {i: fn(i) for i in shard_indices(n, rank, ws)}
    return gather_maps(local, n) if gather else local
