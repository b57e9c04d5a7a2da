"""One process per GPU under torch.distributed: static contig shards, no data-path collective.

Contigs are independent: a contig's result depends only on its own hits
and loci plus the read-only taxonomy. So rank r scores the r-th contiguous,
cost-balanced contig range on its own device. The only collectives are control traffic:
the result records (~100 B per contig) gathered to rank 0 for writing, and the barrier
plus max-over-ranks timing in bench.py. Backend "nccl" (RCCL) on the GPU box; the tests
drive the same code with "gloo" on CPU.
"""
from __future__ import annotations

import os

import numpy as np

from .engine import Results, contig_cost


def rank_env():
    """(rank, world, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def rank_bounds(cost, world):
    """Exactly `world` contiguous [a, b) ranges covering all contigs, with roughly equal
    summed cost. Trailing ranges may be empty when there are fewer contigs than ranks."""
    n = len(cost)
    cum = np.cumsum(np.asarray(cost, dtype=np.float64))
    total = cum[-1] if n else 0.0
    cuts = [0]
    for k in range(1, world):
        # the contig whose cumulative cost reaches the k-th target closes range k-1
        c = int(np.searchsorted(cum, total * k / world)) + 1 if n else 0
        cuts.append(min(max(c, cuts[-1]), n))
    cuts.append(n)
    return [(cuts[k], cuts[k + 1]) for k in range(world)]


def max_over_ranks(value, dist, device=None):
    """MAX of a float over all ranks (the bench's elapsed time)."""
    if dist is None:
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def score_ranked(batch, tax, params, score_shard, dist):
    """Score this rank's shard with `score_shard(sub_batch) -> Results` and gather all
    shards to rank 0. Returns the whole batch's Results on rank 0 and None elsewhere.
    Every rank must hold the same `batch` (they all parse the same input files)."""
    if dist is None:
        return score_shard(batch)
    rank, world = dist.get_rank(), dist.get_world_size()
    k2 = float(params.get("two_clade_threshold", 0.8)) if isinstance(params, dict) else 0.8
    bounds = rank_bounds(contig_cost(batch, k2), world)
    a, b = bounds[rank]
    try:
        local = score_shard(batch.slice(a, b))
    except Exception as exc:          # gathered first, so no rank blocks on a failed peer
        if hasattr(exc, "contigs"):
            exc.contigs = np.asarray(exc.contigs) + a   # shard-local -> batch contig index
        local = exc
    parts = [None] * world
    dist.all_gather_object(parts, local)
    for p in parts:
        if isinstance(p, Exception):
            raise p
    if rank != 0:
        return None
    return Results.concat(parts, [int(batch.hit_off[a0]) for a0, _ in bounds])
