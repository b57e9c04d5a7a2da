"""A blastout whose hits of one contig come in several separate runs (not grouped by query).

The reference scores every run as it reads it (orgscorer.py:941-960): `attach_hits` adds the
run's hits to the contig's site scores -- which earlier evaluations have already rolled up
(`raise_taxonomy`, :431-445) -- then the jumps (:955-957) and `evaluate_contig` (:566-583)
run again over the whole state, and the last evaluation is the one reported.  Locus
annotations carry over (:384-392: the same loci, the same running best score).

The state after an evaluation is a max envelope per clade, and rolling an envelope up is
the max over its children's, so that state is exactly the hits so far with each hit's
clade raised by the levels its run has been through: run g's hits enter evaluation e at
  ancestor^R(taxon),   R = sum over e' = g .. e-1 of (jumps + iterations(e') - 1)
(an evaluation of i iterations raises i - 1 times; a skipped contig, 0 iterations, none;
r__Root is its own parent, utils.py:386-387).  So the last evaluation is one ordinary
wf_score of the contig's whole hit list in file order with those clades, and the counts
come from scoring the earlier evaluations first -- one wf_score per extra run, over the
contigs that have it.  `resolve` returns that batch; every hit index (annotations, melds)
keeps its place in it.
"""
import numpy as np

from .lib import WaafleHipError


def _ancestors(parent, taxon, raises):
    """ancestor^raises(taxon), per hit."""
    out = taxon.astype(np.int32, copy=True)
    todo = np.nonzero(raises > 0)[0]
    r = raises[todo]
    step = 0
    while len(todo):
        out[todo] = parent[out[todo]]
        step += 1
        keep = r > step
        todo, r = todo[keep], r[keep]
    return out


def _ranges(a, b):
    """Concatenated [a[i], b[i]) index ranges (int64)."""
    a = np.asarray(a, np.int64)
    n = np.asarray(b, np.int64) - a
    tot = int(n.sum())
    if tot == 0:
        return np.zeros(0, np.int64)
    start = np.zeros(len(n), np.int64)
    np.cumsum(n[:-1], out=start[1:])
    return np.repeat(a - start, n) + np.arange(tot, dtype=np.int64)


def _with_hits(batch, contigs, hits, taxon):
    """A batch of `contigs` (ascending) holding the hits `hits` (ascending batch indices, all
    of them hits of those contigs) with clades `taxon` (one per entry of `hits`)."""
    from .inputs import HostBatch
    lo = batch.loc_off
    pos = np.searchsorted(contigs, np.searchsorted(batch.hit_off, hits, side="right") - 1)
    counts = np.bincount(pos, minlength=len(contigs))
    hit_off = np.zeros(len(contigs) + 1, np.int64)
    np.cumsum(counts, out=hit_off[1:])
    loc_idx = _ranges(lo[contigs], lo[contigs + 1])
    loc_off = np.zeros(len(contigs) + 1, np.int64)
    np.cumsum(np.diff(lo)[contigs], out=loc_off[1:])
    return HostBatch(
        contig_names=[batch.contig_names[c] for c in contigs],
        contig_lengths=batch.contig_lengths[contigs], hit_off=hit_off,
        hit_qlo=batch.hit_qlo[hits], hit_qhi=batch.hit_qhi[hits], hit_taxon=taxon,
        hit_strand=batch.hit_strand[hits], hit_score=batch.hit_score[hits],
        hit_scov=batch.hit_scov[hits], hit_sysmask=batch.hit_sysmask[hits], loc_off=loc_off,
        loc_start=batch.loc_start[loc_idx], loc_end=batch.loc_end[loc_idx],
        loc_strand=batch.loc_strand[loc_idx], loc_codes=[batch.loc_codes[i] for i in loc_idx],
        systems=batch.systems,
        annot_value_ids=None if batch.annot_value_ids is None else batch.annot_value_ids[hits],
        annot_values=batch.annot_values,
        hit_row=None if batch.hit_row is None else batch.hit_row[hits])


def _run_rows(batch, hits, pos, n, want):
    """Per contig (positions 0..n-1; `pos[i]` is the contig of batch hit `hits[i]`): the
    blastout row that starts its run number want[contig] -- the point in the file where the
    reference evaluates it (and writes its --write-details rows)."""
    g = batch.hit_group[hits]
    rows = batch.hit_row[hits] if batch.hit_row is not None else hits
    key = np.full(n, np.iinfo(np.int64).max, np.int64)
    first = np.nonzero(g == want[pos])[0]
    np.minimum.at(key, pos[first], np.asarray(rows)[first].astype(np.int64))
    return key


def resolve(batch, parent, params, score_fn):
    """-> the batch to score for the reference's records of an ungrouped blastout: each
    hit's clade raised as above (`batch` with hit_group dropped when every contig's hits are
    one run).  parent: the taxonomy's parent array (TaxonomyTables.parent); score_fn(batch)
    -> Results (one wf_score).  A failure of an earlier evaluation (e.g. WF_E_RUNAWAY: the
    reference dies there too) is raised with its contigs relative to `batch`.  Each batch
    scored and the one returned carry `eval_key`: per contig, the blastout row where the
    reference evaluates it (the start of the run it has just read), the order of
    --write-details rows.  Evaluation k touches only the hits of the contigs with more than k
    runs (the reference re-evaluates only the contig whose run it has just read)."""
    import dataclasses
    g = getattr(batch, "hit_group", None)
    if g is None:
        return batch
    if batch.n_hits == 0 or not np.any(g):
        return dataclasses.replace(batch, hit_group=None)
    N = batch.n_contigs
    hit_contig = np.repeat(np.arange(N), np.diff(batch.hit_off))
    runs = np.zeros(N, np.int64)
    np.maximum.at(runs, hit_contig, g.astype(np.int64) + 1)
    # (a negative --jump-taxonomy makes no jumps: range(negative), orgscorer.py:955-957)
    jumps = max(0, int((params.get("jump_taxonomy") if isinstance(params, dict) else 0) or 0))
    raises = np.zeros(batch.n_hits, np.int64)
    # the contigs of several runs, and their hits (batch indices, ascending)
    multi = np.nonzero(runs > 1)[0]
    mhits = _ranges(batch.hit_off[multi], batch.hit_off[multi + 1])
    mpos = np.repeat(np.arange(len(multi)), np.diff(batch.hit_off)[multi])
    for k in range(1, int(runs.max())):
        # evaluation k of the contigs with more than k runs: their runs 0 .. k-1
        keep = runs[multi] > k
        multi, mhits, mpos = multi[keep], mhits[keep[mpos]], np.cumsum(keep)[mpos[keep[mpos]]] - 1
        sel = multi
        seen = g[mhits] < k
        hits = mhits[seen]
        sub = _with_hits(batch, sel, hits, _ancestors(parent, batch.hit_taxon[hits], raises[hits]))
        sub.eval_key = _run_rows(batch, mhits, mpos, len(sel), np.full(len(sel), k - 1))
        try:
            res = score_fn(sub)
        except WaafleHipError as err:
            bad = getattr(err, "contigs", None)
            if bad is not None and len(bad):
                err.contigs = sel[np.asarray(bad)]
            raise
        per = jumps + np.maximum(res.iterations.astype(np.int64) - 1, 0)
        raises[hits] += per[mpos[seen]]
    out = dataclasses.replace(batch, hit_taxon=_ancestors(parent, batch.hit_taxon, raises),
                              hit_group=None)
    last = np.zeros(N, np.int64)
    np.maximum.at(last, hit_contig, g.astype(np.int64))
    out.eval_key = _run_rows(batch, np.arange(batch.n_hits), hit_contig, N, last)
    return out
