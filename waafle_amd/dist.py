"""One process per GPU under torch.distributed: static contig shards, no data-path collective.

Contigs are independent: a contig's result depends only on its own hits
and loci plus the read-only taxonomy. So rank r scores the r-th contiguous,
cost-balanced contig range on its own device. The inputs are parsed once, on rank 0;
rank 0 sends every other rank its range's scoring arrays and the taxonomy tables as typed
arrays (host to host, a gloo group), and each rank sends its records back the same way.
The only other collectives are control traffic: a status word that carries a failing
shard's error to every rank, and the barrier plus max-over-ranks timing in bench.py.
"""
from __future__ import annotations

import os
import pickle
from types import SimpleNamespace

import numpy as np

from .engine import Results, contig_cost
from .inputs import HostBatch

# the arrays a shard needs for scoring (HostBatch fields), and the taxonomy tables
SHARD_FIELDS = ("contig_lengths", "hit_off", "hit_qlo", "hit_qhi", "hit_taxon", "hit_strand",
                "hit_score", "hit_scov", "hit_sysmask", "loc_off", "loc_start", "loc_end",
                "loc_strand")
TAX_FIELDS = ("parent", "depth", "sib_parent", "leaf_count")
_DTYPES = ("|i1", "|u1", "<i2", "<i4", "<u4", "<i8", "<f8")


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


def share_error(err, dist, group=None):
    """Rank 0's error (an exception, or None) on every rank: a status word, then the
    exception itself.  Every rank calls it before the scatter, so a parse or regroup failure
    on rank 0 ends every rank the same way instead of leaving the others in a recv."""
    if dist is None:
        return err
    import torch
    status = torch.tensor([0 if err is None else 1], dtype=torch.int64)
    dist.broadcast(status, 0, group=group)
    if not status.item():
        return None
    box = [err if dist.get_rank() == 0 else None]
    dist.broadcast_object_list(box, 0, group=group)
    return box[0]


def max_over_ranks(value, dist, device=None):
    """MAX of a float over all ranks (the bench's elapsed time)."""
    if dist is None:
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


# ---- typed arrays between two ranks (gloo: host memory, no pickling) ----------------------
def _send_arrays(arrs, dst, dist, group):
    import torch
    head = [len(arrs)]
    for a in arrs:
        head += [_DTYPES.index(a.dtype.str), int(a.size)]
    dist.send(torch.tensor([len(head)], dtype=torch.int64), dst, group=group)
    dist.send(torch.tensor(head, dtype=torch.int64), dst, group=group)
    for a in arrs:
        if a.size:
            dist.send(torch.from_numpy(np.ascontiguousarray(a).view(np.uint8).reshape(-1)), dst, group=group)


def _recv_arrays(src, dist, group):
    import torch
    n = torch.zeros(1, dtype=torch.int64)
    dist.recv(n, src, group=group)
    head = torch.zeros(int(n.item()), dtype=torch.int64)
    dist.recv(head, src, group=group)
    head = head.tolist()
    out = []
    for i in range(head[0]):
        dt = np.dtype(_DTYPES[head[1 + 2 * i]])
        size = head[2 + 2 * i]
        buf = torch.empty(size * dt.itemsize, dtype=torch.uint8)
        if size:
            dist.recv(buf, src, group=group)
        out.append(buf.numpy().view(dt).copy())
    return out


def _text(strings):
    return np.frombuffer("\n".join(strings).encode(), dtype=np.uint8).copy()


def _untext(blob, n):
    return blob.tobytes().decode().split("\n") if n else []


def _send_shard(sub, tax, a, b, dst, dist, group):
    arrs = [np.array([a, b, len(sub.contig_names), len(sub.systems), tax.root, tax.unknown,
                      len(tax.names)], np.int64)]
    arrs += [getattr(sub, f) for f in SHARD_FIELDS]
    arrs += [_text(sub.contig_names), _text(sub.systems)]
    arrs += [np.asarray(getattr(tax, f)) for f in TAX_FIELDS]
    _send_arrays(arrs, dst, dist, group)


def _recv_shard(dist, group):
    arrs = _recv_arrays(0, dist, group)
    a, b, n_names, n_sys, root, unknown, n_tax = arrs[0].tolist()
    f = dict(zip(SHARD_FIELDS, arrs[1:1 + len(SHARD_FIELDS)]))
    rest = arrs[1 + len(SHARD_FIELDS):]
    sub = HostBatch(contig_names=_untext(rest[0], n_names), systems=_untext(rest[1], n_sys), **f)
    tax = SimpleNamespace(names=range(n_tax), root=root, unknown=unknown,
                          **dict(zip(TAX_FIELDS, rest[2:])))
    return sub, tax, a, b


def score_ranked(batch, tax, params, score_shard, dist, group=None):
    """Score a batch over the ranks of `dist`: rank 0 holds the parsed batch and taxonomy
    (the others pass None), splits the contigs into cost-balanced ranges, sends each rank
    its range and the taxonomy tables; every rank runs `score_shard(sub_batch, tax, a, b)
    -> Results` on its range [a, b); the records come back to rank 0.  Returns the whole
    batch's Results on rank 0 and None elsewhere; a failing shard's error (its contigs as
    batch indices) is raised on every rank.  `group`: a gloo group for the host arrays
    (default: the default group, which must then be gloo)."""
    if dist is None:
        return score_shard(batch, tax, 0, batch.n_contigs)
    import torch
    rank, world = dist.get_rank(), dist.get_world_size()
    if rank == 0:
        k2 = float(params.get("two_clade_threshold", 0.8)) if isinstance(params, dict) else 0.8
        bounds = rank_bounds(contig_cost(batch, k2), world)
        for r in range(1, world):
            _send_shard(batch.slice(*bounds[r]), tax, bounds[r][0], bounds[r][1], r, dist, group)
        sub, a, b = batch.slice(*bounds[0]), bounds[0][0], bounds[0][1]
    else:
        sub, tax, a, b = _recv_shard(dist, group)
    try:
        local, err = score_shard(sub, tax, a, b), None
    except Exception as exc:          # reported to rank 0 first, so no rank blocks on a peer
        if hasattr(exc, "contigs"):
            exc.contigs = np.asarray(exc.contigs) + a   # shard-local -> batch contig index
        local, err = None, exc
    fields = list(Results.__dataclass_fields__)
    status = torch.zeros(1, dtype=torch.int64)        # 0 ok, else the first failing rank + 1
    first_err = None
    if rank == 0:
        parts = [local]
        if err is not None:
            status[0], first_err = 1, err
        for r in range(1, world):
            flag = torch.zeros(1, dtype=torch.int64)
            dist.recv(flag, r, group=group)
            if flag.item():
                blob = _recv_arrays(r, dist, group)[0]
                if first_err is None:
                    status[0], first_err = r + 1, pickle.loads(blob.tobytes())
                parts.append(None)
            else:
                parts.append(Results(**dict(zip(fields, _recv_arrays(r, dist, group)))))
    else:
        dist.send(torch.tensor([0 if err is None else 1], dtype=torch.int64), 0, group=group)
        if err is None:
            _send_arrays([getattr(local, f) for f in fields], 0, dist, group)
        else:   # (the error path only: the exception with its contig indices)
            _send_arrays([np.frombuffer(pickle.dumps(err), dtype=np.uint8).copy()], 0, dist, group)
    dist.broadcast(status, 0, group=group)
    if status.item():
        if rank == 0:
            box = [first_err]
        else:
            box = [None]
        dist.broadcast_object_list(box, 0, group=group)
        raise box[0]
    if rank != 0:
        return None
    return Results.concat(parts, [int(batch.hit_off[a0]) for a0, _ in bounds])
