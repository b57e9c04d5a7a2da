"""Host driver: HostBatch -> libwaafle_hip -> per-contig result records.

`score(batch, tax, params, gpus=N)` shards contigs over N devices (contiguous ranges
balanced by an estimated cost; contigs are independent, so there is no exchange step
and no collective) and runs one HIP context per device from its own host thread
(ctypes releases the GIL for the duration of wf_score).
"""
from __future__ import annotations

import ctypes as C
import threading
from dataclasses import dataclass

import numpy as np

from . import lib as L
from . import regroup

DIS_ONE = {"report-best": 0, "meld": 1}
DIS_TWO = {"report-best": 0, "jump": 1, "meld": 2}
LEVEL = {"off": 0, "lenient": 1, "strict": 2}
WEAK = {"ignore": 0, "penalize": 1, "assign-unknown": 2}
MODES = {"staged": L.MODE_STAGED, "level0": L.MODE_LEVEL0, "waves": L.MODE_WAVES}


def params_struct(p):
    """argparse-style dict (cli.param_dict) -> wf_params."""
    return L.WfParams(
        k1=float(p["one_clade_threshold"]), k2=float(p["two_clade_threshold"]),
        range=float(p["range"]), min_overlap=float(p["min_overlap"]),
        min_scov=float(p["min_scov"]), ambiguous_fraction=float(p["ambiguous_fraction"]),
        disambiguate_one=DIS_ONE[p["disambiguate_one"]],
        disambiguate_two=DIS_TWO[p["disambiguate_two"]],
        jump_taxonomy=int(p["jump_taxonomy"] or 0), allow_lca=int(bool(p["allow_lca"])),
        ambiguous_threshold=LEVEL[p["ambiguous_threshold"]],
        sister_penalty=LEVEL[p["sister_penalty"]],
        clade_genes=-1 if p["clade_genes"] is None else int(p["clade_genes"]),
        clade_leaves=-1 if p["clade_leaves"] is None else int(p["clade_leaves"]),
        weak_loci=WEAK[p["weak_loci"]], annotation_threshold=LEVEL[p["annotation_threshold"]],
        stranded=int(bool(p["stranded"])))


@dataclass
class Results:
    call: np.ndarray
    crit: np.ndarray
    rank: np.ndarray
    clade1: np.ndarray
    clade2: np.ndarray
    direction: np.ndarray
    iterations: np.ndarray
    synteny: np.ndarray
    n_meld1: np.ndarray
    n_meld2: np.ndarray
    meld: np.ndarray
    annot_hit: np.ndarray
    pair_evals: np.ndarray
    status: np.ndarray
    need_bytes: np.ndarray
    ppot_sum: np.ndarray = None    # sum of P_pot over the explain_two calls with pairs (B_k2)

    @classmethod
    def empty(cls, n, n_hits, n_loci, n_sys):
        return cls(call=np.zeros(n, np.int8), crit=np.zeros(n, np.float64),
                   rank=np.zeros(n, np.float64), clade1=np.zeros(n, np.int32),
                   clade2=np.zeros(n, np.int32), direction=np.zeros(n, np.int8),
                   iterations=np.zeros(n, np.int16), synteny=np.zeros(n_loci, np.uint8),
                   n_meld1=np.zeros(n, np.int32), n_meld2=np.zeros(n, np.int32),
                   meld=np.zeros(2 * n_hits + 2 * n, np.int32),
                   annot_hit=np.zeros(n_loci * n_sys, np.int32),
                   pair_evals=np.zeros(n, np.int64), status=np.zeros(n, np.int32),
                   need_bytes=np.zeros(n, np.int64), ppot_sum=np.zeros(n, np.int64))

    def struct(self):
        return L.WfResult(*[L.ptr(getattr(self, f)) for f, _ in L.WfResult._fields_])

    @classmethod
    def concat(cls, parts, hit_bases):
        out = {}
        for f in cls.__dataclass_fields__:
            out[f] = np.concatenate([getattr(p, f) for p in parts])
        # annotation winners are batch hit indices: rebase shard-local ones
        ann = [np.where(p.annot_hit >= 0, p.annot_hit + b, -1).astype(np.int32)
               for p, b in zip(parts, hit_bases)]
        out["annot_hit"] = np.concatenate(ann) if ann else np.zeros(0, np.int32)
        return cls(**out)


def hit_keys(b, min_scov):
    """wf_batch.hit_key of a host batch for this min_scov (packed once per batch and value:
    the level-0 triage then reads 20 bytes a hit instead of 32)."""
    cache = getattr(b, "_hit_keys", None)
    if cache is None or cache[0] != min_scov:
        cache = (min_scov, L.pack_hit_keys(b.hit_taxon, b.hit_strand, b.hit_scov, b.hit_sysmask, min_scov))
        b._hit_keys = cache
    return cache[1]


def batch_struct(b, min_scov=None):
    """wf_batch over a host batch; with min_scov, the packed hit_key too (which must stay
    alive for the call: it is cached on the batch)."""
    return L.WfBatch(
        n_contigs=b.n_contigs, n_systems=len(b.systems), n_hits=b.n_hits, n_loci=b.n_loci,
        max_hits=b.max_hits, max_loci=b.max_loci, device_resident=0, _pad=0,
        hit_off=L.ptr(b.hit_off), hit_qlo=L.ptr(b.hit_qlo), hit_qhi=L.ptr(b.hit_qhi),
        hit_taxon=L.ptr(b.hit_taxon), hit_strand=L.ptr(b.hit_strand),
        hit_score=L.ptr(b.hit_score), hit_scov=L.ptr(b.hit_scov),
        hit_sysmask=L.ptr(b.hit_sysmask), loc_off=L.ptr(b.loc_off),
        loc_start=L.ptr(b.loc_start), loc_end=L.ptr(b.loc_end), loc_strand=L.ptr(b.loc_strand),
        hit_key=None if min_scov is None or b.n_hits == 0 else L.ptr(hit_keys(b, min_scov)))


def taxonomy_struct(t):
    return L.WfTaxonomy(n=len(t.names), parent=L.ptr(t.parent), depth=L.ptr(t.depth),
                        sib_parent=L.ptr(t.sib_parent), leaf_count=L.ptr(t.leaf_count),
                        root=t.root, unknown=t.unknown)


def rebase_error(err, first):
    """A failure of a sub-batch starting at contig `first`: its failing-contig indices
    (WaafleHipError.contigs, relative to the sub-batch) made relative to the whole batch."""
    bad = getattr(err, "contigs", None)
    if bad is not None and len(bad):
        err.contigs = np.asarray(bad) + int(first)
    return err


class GpuScorer:
    """One libwaafle_hip context on one device.  `options`: {wf_option: value}
    (lib.OPT_*), e.g. {lib.OPT_ATT_LIMIT: n} to make wf_score split smaller batches.
    `host_keys`: pass the numpy-packed wf_batch.hit_key with the host arrays (a test form:
    the library packs it on the device faster than it checks a host one)."""

    def __init__(self, device=0, lds_bytes=None, mode=None, options=None, host_keys=False):
        self.host_keys = host_keys
        self.lib = L.load()
        h = C.c_void_p()
        rc = self.lib.wf_init(int(device), C.byref(h))
        if rc != L.WF_OK:
            raise L.WaafleHipError(rc, "wf_init(device={}) failed".format(device))
        self.h = h
        self.device = device
        if mode is not None:
            self._check(self.lib.wf_set_mode(self.h, MODES[mode] if isinstance(mode, str) else int(mode)))
        if lds_bytes:
            self._check(self.lib.wf_set_lds_bytes(self.h, int(lds_bytes)))
        for opt, val in (options or {}).items():
            self._check(self.lib.wf_set_option(self.h, int(opt), int(val)))

    def _check(self, rc):
        if rc != L.WF_OK:
            raise L.WaafleHipError(rc, self.lib.wf_last_error(self.h).decode())

    def set_taxonomy(self, tax):
        self._tables = tax
        self._tax = taxonomy_struct(tax)
        self._check(self.lib.wf_set_taxonomy(self.h, C.byref(self._tax)))

    def score(self, batch, params):
        """wf_score over the batch.  A batch whose hit-locus attachments exceed one call's
        limit (WF_E_TOOBIG: the device's 32-bit work indices, or WF_OPT_ATT_LIMIT) is
        scored in contig halves (contigs are independent, so the records are the same);
        a failing half reports its contigs relative to this batch.  A batch from an ungrouped
        blastout (hit_group) is scored as the reference scores it, run by run (regroup.py)."""
        if getattr(batch, "hit_group", None) is not None:
            batch = regroup.resolve(batch, self._tables.parent, params, lambda b: self.score(b, params))
        try:
            return self._score_once(batch, params)
        except L.WaafleHipError as err:
            if err.code != L.WF_E_TOOBIG or batch.n_contigs < 2:
                raise
        mid = batch.n_contigs // 2
        parts = []
        for a, b in ((0, mid), (mid, batch.n_contigs)):
            try:
                parts.append(self.score(batch.slice(a, b), params))
            except L.WaafleHipError as err:
                raise rebase_error(err, a)
        return Results.concat(parts, [0, int(batch.hit_off[mid])])

    def _score_once(self, batch, params):
        res = Results.empty(batch.n_contigs, batch.n_hits, batch.n_loci, len(batch.systems))
        # host arrays: no hit_key by default (the library packs it on the device in well under
        # a millisecond; a host key costs 4 B/hit more H2D and the library's host check of it
        # -- scope (ii) 0.25 -> 0.40 s at cfg4).  Device-resident callers pass it (bench.py).
        ms = float(params["min_scov"]) if self.host_keys else None
        bs, ps, rs = batch_struct(batch, ms), params_struct(params), res.struct()
        rc = self.lib.wf_score(self.h, C.byref(bs), C.byref(ps), C.byref(rs))
        if rc != L.WF_OK:
            bad = np.nonzero(res.status)[0]
            msg = self.lib.wf_last_error(self.h).decode()
            err = L.WaafleHipError(rc, msg)
            err.contigs = bad
            err.results = res
            raise err
        return res

    def score_details(self, batch, params):
        """wf_score with --write-details records on: (Results, {name: numpy array}) with the
        evaluated (contig, level) pairs and the per-level segment records
        (include/waafle_hip.h wf_details).  An ungrouped blastout (hit_group): the reference
        writes a contig's details at each of its evaluations, so the records come as
        {"parts": [(batch, records), ...]}, one per wf_score of regroup.resolve, each batch
        with its eval_key (details.render orders the rows by it)."""
        if getattr(batch, "hit_group", None) is not None:
            parts = []

            def one(b):
                res, det = self.score_details(b, params)
                parts.append((b, det))
                return res

            final = regroup.resolve(batch, self._tables.parent, params, one)
            res = one(final)
            return res, {"parts": parts}
        self._check(self.lib.wf_details_enable(self.h, 1))
        try:
            res = self.score(batch, params)
            d = L.WfDetails()
            self._check(self.lib.wf_details_read(self.h, C.byref(d)))

            def arr(ptr, n, dt):
                if n == 0:
                    return np.zeros(0, dtype=dt)
                ct = np.ctypeslib.as_ctypes_type(np.dtype(dt))
                return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ct)), shape=(n,)).copy()

            ne, ns = int(d.n_evals), int(d.n_segs)
            out = dict(eval_contig=arr(d.eval_contig, ne, np.int32),
                       eval_level=arr(d.eval_level, ne, np.int32),
                       seg_level=arr(d.seg_level, ns, np.int32),
                       seg_contig=arr(d.seg_contig, ns, np.int32),
                       seg_clade=arr(d.seg_clade, ns, np.int32),
                       seg_locus=arr(d.seg_locus, ns, np.int32),
                       seg_mean=arr(d.seg_mean, ns, np.float64),
                       seg_nspan=arr(d.seg_nspan, ns, np.int32),
                       span_off=arr(d.span_off, ns + 1, np.int64))
            out["spans"] = arr(d.spans, 2 * int(out["span_off"][-1]), np.int32)
            return res, out
        finally:
            self._check(self.lib.wf_details_enable(self.h, 0))

    def close(self):
        if getattr(self, "h", None):
            self.lib.wf_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def contig_cost(batch, k2=0.8):
    """Estimated work per contig for balancing shards:
    w = H + sum_loci len * P_c + G * P_pot^2, with P_c = distinct hit taxa of the contig and
    P_pot = distinct taxa with a hit scoring >= k2 (an upper bound of the clades whose best
    gene score reaches k2: a gene score is a mean of sites no higher than the best hit).
    The k2 term is the explain_two all-pairs search; it dominates skewed batches (cfg5
    stress contigs cost ~P_pot^2 * G where an ordinary contig costs ~H)."""
    N = batch.n_contigs
    H = np.diff(batch.hit_off).astype(np.float64)
    G = np.diff(batch.loc_off).astype(np.float64)
    if N == 0:
        return H
    lens = (np.abs(batch.loc_end.astype(np.int64) - batch.loc_start.astype(np.int64)) + 1).astype(np.float64)
    loc_contig = np.repeat(np.arange(N), np.diff(batch.loc_off))
    len_sum = np.bincount(loc_contig, weights=lens, minlength=N)
    hit_contig = np.repeat(np.arange(N, dtype=np.int64), np.diff(batch.hit_off))
    ntax = np.int64(max(int(batch.hit_taxon.max()) + 1, 1)) if batch.n_hits else np.int64(1)

    def distinct(mask):
        pairs = np.unique(hit_contig[mask] * ntax + batch.hit_taxon[mask].astype(np.int64))
        return np.bincount(pairs // ntax, minlength=N).astype(np.float64)

    p_c = distinct(np.ones(batch.n_hits, bool))
    p_pot = distinct(batch.hit_score >= k2)
    return H + len_sum * p_c + G * p_pot * p_pot + 1.0


def shard_bounds(cost, parts):
    """Contiguous ranges with ~equal summed cost."""
    n = len(cost)
    if parts <= 1 or n == 0:
        return [(0, n)]
    cum = np.cumsum(cost)
    total = cum[-1]
    cuts = [0]
    for k in range(1, parts):
        cuts.append(int(np.searchsorted(cum, total * k / parts)))
    cuts.append(n)
    cuts = sorted(set(min(max(c, 0), n) for c in cuts))
    return [(a, b) for a, b in zip(cuts[:-1], cuts[1:]) if b > a] or [(0, n)]


def score(batch, tax, params, gpus=1, lds_bytes=None, devices=None):
    """Score a batch on `gpus` devices: contiguous shards balanced by contig_cost, one
    context and host thread per shard.  `devices[k]` is shard k's device (default k); two
    shards may share a device (each context has its own stream and scratch)."""
    gpus = max(1, int(gpus))
    if gpus == 1:
        s = GpuScorer(devices[0] if devices else 0, lds_bytes)
        try:
            s.set_taxonomy(tax)
            return s.score(batch, params)
        finally:
            s.close()
    k2 = float(params.get("two_clade_threshold", 0.8)) if isinstance(params, dict) else 0.8
    bounds = shard_bounds(contig_cost(batch, k2), gpus)
    devs = list(devices) if devices else list(range(len(bounds)))
    if len(devs) < len(bounds):
        raise ValueError("devices: {} entries for {} shards".format(len(devs), len(bounds)))
    parts = [None] * len(bounds)
    errors = []

    def work(k, a, b):
        try:
            s = GpuScorer(devs[k], lds_bytes)
            try:
                s.set_taxonomy(tax)
                parts[k] = s.score(batch.slice(a, b), params)
            finally:
                s.close()
        except L.WaafleHipError as exc:   # re-raised on the main thread, batch-relative
            errors.append((k, rebase_error(exc, a)))
        except Exception as exc:
            errors.append((k, exc))

    threads = [threading.Thread(target=work, args=(k, a, b)) for k, (a, b) in enumerate(bounds)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    if errors:
        raise min(errors, key=lambda e: e[0])[1]   # the first failing shard
    return Results.concat(parts, [int(batch.hit_off[a]) for a, _ in bounds])
