"""Render the three waafle_orgscorer TSVs from device result records.

Restates orgscorer.py:750-894 and utils.py:122-143: rows in sorted contig-name
order, `{:.4f}` floats, empty fields as `--`, lineages joined by `|`, melded tails
as sorted unique `|`-paths joined by `; `, and one ANNOTATIONS:<SYSTEM> column per
transferred annotation system (sorted).
"""
import os

import numpy as np

from .lib import CALL_LGT, CALL_NO_LGT

FORMATS = {   # orgscorer.py:76-114
    "lgt": ["contig_name", "call", "contig_length", "min_max_score", "avg_max_score",
            "synteny", "direction", "clade_A", "clade_B", "lca", "melded_A", "melded_B",
            "taxonomy_A", "taxonomy_B", "loci"],
    "no_lgt": ["contig_name", "call", "contig_length", "min_score", "avg_score", "synteny",
               "clade", "melded", "taxonomy", "loci"],
    "unclassified": ["contig_name", "call", "contig_length", "loci"],
}
ANNOT_PREFIX = "ANNOTATIONS:"
MISSING = "None"


def _f(x):
    return "{:.4f}".format(x)


def _e(s):
    return s if s != "" else "--"


def _tails(tax, ids, lca_id):
    lca_name = tax.names[lca_id]
    items = set()
    for i in ids:
        t = tax.tail(int(i), lca_name)
        if t:
            items.add("|".join(t))
    return "; ".join(sorted(items))


def _annotation_fields(batch, res, bit, nsys):
    """Per contig: the ANNOTATIONS:<SYSTEM> field of system `bit` -- each locus's winning
    hit's value (orgscorer.py:384-392, 790-800) or "None", joined by "|" -- built with one
    table lookup per distinct value instead of one per locus."""
    L = batch.n_loci
    hits = res.annot_hit.reshape(-1, nsys)[:, bit] if L else np.zeros(0, np.int32)
    vid = np.full(L, -1, dtype=np.int64)
    m = hits >= 0
    if m.any():
        vid[m] = batch.annot_value_ids[hits[m], bit]
    table = batch.annot_values[bit]
    text = {int(i): table[int(i)] for i in np.unique(vid[m])} if m.any() else {}
    text[-1] = MISSING
    per_locus = [text[i] for i in vid.tolist()]
    lo = batch.loc_off.tolist()
    return [_e("|".join(per_locus[lo[c]:lo[c + 1]])) for c in range(batch.n_contigs)]


def render(batch, tax, res):
    """-> {kind: [header, row, ...]} (tab-joined strings)."""
    N = batch.n_contigs
    nsys = len(batch.systems)
    annot = res.annot_hit.reshape(-1, nsys) if nsys else None
    # systems that were transferred to at least one locus (orgscorer.py:824-828)
    used = [s for b, s in enumerate(batch.systems) if nsys and np.any(annot[:, b] >= 0)]
    used_bits = [batch.systems.index(s) for s in sorted(used)]
    out = {}
    for kind, cols in FORMATS.items():
        hdr = cols + [ANNOT_PREFIX + batch.systems[b] for b in used_bits]
        out[kind] = ["\t".join(c.upper() for c in hdr)]
    lo = batch.loc_off.tolist()
    ho = batch.hit_off.tolist()
    names = batch.contig_names
    calls = res.call.tolist()
    crit, rank = res.crit.tolist(), res.rank.tolist()
    c1s, c2s = res.clade1.tolist(), res.clade2.tolist()
    nm1s, nm2s = res.n_meld1.tolist(), res.n_meld2.tolist()
    dirs = res.direction.tolist()
    lengths = batch.contig_lengths.tolist()
    syn = res.synteny.tobytes().decode("latin-1")
    meld = res.meld
    fields = batch.loci_fields
    codes = batch.loc_codes
    ann = [_annotation_fields(batch, res, b, nsys) for b in used_bits]
    tnames = tax.names
    lin_cache, tail_cache = {}, {}

    def lin(i):
        s = lin_cache.get(i)
        if s is None:
            s = lin_cache[i] = _e("|".join(tax.lineage(i)))
        return s

    def tails(ids, c):
        key = (c, tuple(sorted(ids.tolist())))
        s = tail_cache.get(key)
        if s is None:
            s = tail_cache[key] = _e(_tails(tax, ids, c))
        return s

    lgt, no_lgt, uncl = out["lgt"], out["no_lgt"], out["unclassified"]
    for c in sorted(range(N), key=names.__getitem__):
        l0, l1 = lo[c], lo[c + 1]
        loci = _e(fields[c] if fields is not None else "|".join(codes[l0:l1]))
        call = calls[c]
        length = str(lengths[c])
        if call == CALL_NO_LGT:
            c1 = c1s[c]
            mbase = 2 * ho[c] + 2 * c
            vals = [names[c], "no_lgt", length, _f(crit[c]), _f(rank[c]), _e(syn[l0:l1]),
                    _e(tnames[c1]), tails(meld[mbase:mbase + nm1s[c]], c1), lin(c1), loci]
            dest = no_lgt
        elif call == CALL_LGT:
            a, b = c1s[c], c2s[c]
            mbase = 2 * ho[c] + 2 * c
            n1, n2 = nm1s[c], nm2s[c]
            vals = [names[c], "lgt", length, _f(crit[c]), _f(rank[c]), _e(syn[l0:l1]),
                    "B>A" if dirs[c] else "A?B", _e(tnames[a]), _e(tnames[b]),
                    _e(tax.lca([a, b])), tails(meld[mbase:mbase + n1], a),
                    tails(meld[mbase + n1:mbase + n1 + n2], b), lin(a), lin(b), loci]
            dest = lgt
        else:
            vals = [names[c], "unclassified", length, loci]
            dest = uncl
        for col in ann:
            vals.append(col[c])
        dest.append("\t".join(vals))
    return out


def write(rows, outdir, basename):
    for kind in ("lgt", "no_lgt", "unclassified"):
        with open(os.path.join(outdir, "{}.{}.tsv".format(basename, kind)), "w") as fh:
            fh.write("\n".join(rows[kind]) + "\n")
