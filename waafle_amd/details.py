"""`--write-details` rows (orgscorer.py:766-812, 931-937) from the GPU's per-level records.

For every evaluated contig (blastout order) and roll-up level, write_details() prints one
row per clade on the contig: the gene scores (Contig.gene_scores, 3 decimals, '|' between
loci) and the gene spans (make_gene_spans_field).  The HIP path hands over, per level,
the contigs it evaluated and every (contig, clade, locus) segment with its exact numpy
mean and its nonzero-run boundaries (wf_details_read, include/waafle_hip.h); this module
only assembles and formats them:

  * iteration label: write_details is called with `iteration` before it is incremented,
    so roll-up level 0 and level 1 both print 1, level n >= 1 prints n (:566-583);
  * clades in name order (upstream iterates a set: PYTHONHASHSEED order);
  * --weak-loci assign-unknown: 'Unknown' = 1 - per-locus max over the other clades
    (:407-418), spans "None" unless a hit names 'Unknown' itself;
  * contigs without blastout rows are never evaluated (:943-948); contigs whose loci are
    all ignored are skipped (:958-960; no loci at all counts as all ignored);
  * an all-zero site array raises IndexError upstream (:785-789): DetailsError here.
"""
import gzip
import os

import numpy as np

HEADER = "CONTIG_NAME\tITERATION\tCLADE\tGENE_SCORES\tGENE_SPANS"
MISSING = "None"          # orgscorer.py:61
EMPTY = "--"              # utils.py:123, 139


class DetailsError(RuntimeError):
    pass


def _field(s):
    return s if s != "" else EMPTY


def render(batch, tax, params, det):
    """Rows (lists of 5 strings) in the reference's order.  det: one wf_score's records, or
    {"parts": [(batch, records), ...]} for an ungrouped blastout (engine.score_details):
    each evaluation's rows at the blastout row where the reference makes it."""
    if "parts" in det:
        keyed = []
        for b, d in det["parts"]:
            keyed.extend(_render_keyed(b, tax, params, d))
        keyed.sort(key=lambda kr: kr[0])
        return [r for _, rows in keyed for r in rows]
    return [r for _, rows in _render_keyed(batch, tax, params, det) for r in rows]


def _render_keyed(batch, tax, params, det):
    """[(order key, rows of one contig's evaluation)], in key order."""
    N = batch.n_contigs
    hit_off = np.asarray(batch.hit_off)
    loc_off = np.asarray(batch.loc_off)
    has_rows = hit_off[1:] > hit_off[:-1]
    first_row = np.full(N, np.iinfo(np.int64).max, dtype=np.int64)
    if batch.hit_row is not None and len(batch.hit_row):
        first_row[has_rows] = np.asarray(batch.hit_row)[hit_off[:-1][has_rows]]
    else:
        first_row[has_rows] = hit_off[:-1][has_rows]
    if getattr(batch, "eval_key", None) is not None:
        first_row = np.asarray(batch.eval_key, dtype=np.int64)
    unknown = int(tax.unknown)
    weak = params["weak_loci"]                       # cli.param_dict keys
    assign_unknown = weak == "assign-unknown"
    ignore = weak == "ignore"
    kmin = min(float(params["one_clade_threshold"]), float(params["two_clade_threshold"]))

    # segment records grouped by (contig, level)
    segs = {}
    sl, sc, scl, slo = det["seg_level"], det["seg_contig"], det["seg_clade"], det["seg_locus"]
    for i in range(len(sc)):
        segs.setdefault((int(sc[i]), int(sl[i])), []).append(i)
    evals = {}
    for c, lv in zip(det["eval_contig"].tolist(), det["eval_level"].tolist()):
        evals.setdefault(c, []).append(lv)

    def level_rows(c, lv, G):
        recs = segs.get((c, lv), [])
        scores, spans = {}, {}
        for i in recs:
            cl, g = int(scl[i]), int(slo[i])
            row = scores.setdefault(cl, np.zeros(G))
            row[g] = det["seg_mean"][i]
            n = int(det["seg_nspan"][i])
            if n < 0:
                raise DetailsError("IndexError in make_gene_spans_field: clade {} has an "
                                   "all-zero site array on contig {} (as upstream)".format(
                                       tax.names[cl], batch.contig_names[c]))
            a = int(det["span_off"][i])
            spans.setdefault(cl, {})[g] = ":".join(
                str(v) for v in det["spans"][2 * a:2 * (a + n)].tolist())
        if assign_unknown:
            top = np.zeros(G)
            for cl, row in scores.items():
                if cl != unknown:
                    top = np.maximum(top, row)
            scores[unknown] = 1 - top
        out = []
        for cl in sorted(scores, key=lambda x: tax.names[x]):
            sp = spans.get(cl, {})
            out.append([batch.contig_names[c], str(max(1, lv)), tax.names[cl],
                        _field("|".join("{:.3f}".format(v) for v in scores[cl])),
                        _field("|".join(sp.get(g, MISSING) for g in range(G)))])
        return out, scores

    keyed = []
    for c in sorted(np.nonzero(has_rows)[0].tolist(), key=lambda x: first_row[x]):
        G = int(loc_off[c + 1] - loc_off[c])
        if G == 0 or c not in evals:
            continue
        levels = sorted(evals[c])
        first, scores = level_rows(c, levels[0], G)
        if ignore:
            top = np.zeros(G)
            for cl, row in scores.items():
                if cl != unknown:
                    top = np.maximum(top, row)
            if not np.any(top >= kmin):
                continue                      # every locus ignored: not evaluated
        rows = list(first)
        for lv in levels[1:]:
            rows.extend(level_rows(c, lv, G)[0])
        keyed.append((int(first_row[c]), rows))
    return keyed


def write(rows, outdir, basename):
    path = os.path.join(outdir, basename + ".details.tsv.gz")
    with gzip.open(path, "wt") as fh:
        fh.write(HEADER + "\n")
        for r in rows:
            fh.write("\t".join(r) + "\n")
    return path
