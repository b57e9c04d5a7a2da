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
    lo = batch.loc_off
    ho = batch.hit_off
    names = batch.contig_names
    for c in sorted(range(N), key=lambda i: names[i]):
        l0, l1 = int(lo[c]), int(lo[c + 1])
        loci = _e(batch.loci_fields[c] if batch.loci_fields is not None
                  else "|".join(batch.loc_codes[l0:l1]))
        call = int(res.call[c])
        length = str(int(batch.contig_lengths[c]))
        if call == CALL_NO_LGT:
            kind = "no_lgt"
            c1 = int(res.clade1[c])
            mbase = 2 * int(ho[c]) + 2 * c
            meld = res.meld[mbase:mbase + int(res.n_meld1[c])]
            vals = [names[c], "no_lgt", length, _f(res.crit[c]), _f(res.rank[c]),
                    _e(res.synteny[l0:l1].tobytes().decode()), _e(tax.names[c1]),
                    _e(_tails(tax, meld, c1)), _e("|".join(tax.lineage(c1))), loci]
        elif call == CALL_LGT:
            kind = "lgt"
            a, b = int(res.clade1[c]), int(res.clade2[c])
            mbase = 2 * int(ho[c]) + 2 * c
            n1, n2 = int(res.n_meld1[c]), int(res.n_meld2[c])
            m1 = res.meld[mbase:mbase + n1]
            m2 = res.meld[mbase + n1:mbase + n1 + n2]
            vals = [names[c], "lgt", length, _f(res.crit[c]), _f(res.rank[c]),
                    _e(res.synteny[l0:l1].tobytes().decode()),
                    "B>A" if res.direction[c] else "A?B", _e(tax.names[a]), _e(tax.names[b]),
                    _e(tax.lca([a, b])), _e(_tails(tax, m1, a)), _e(_tails(tax, m2, b)),
                    _e("|".join(tax.lineage(a))), _e("|".join(tax.lineage(b))), loci]
        else:
            kind = "unclassified"
            vals = [names[c], "unclassified", length, loci]
        for bit in used_bits:
            items = []
            for l in range(l0, l1):
                h = int(annot[l, bit])
                if h < 0:
                    items.append(MISSING)
                else:
                    items.append(batch.annot_values[bit][int(batch.annot_value_ids[h, bit])])
            vals.append(_e("|".join(items)))
        out[kind].append("\t".join(vals))
    return out


def write(rows, outdir, basename):
    for kind in ("lgt", "no_lgt", "unclassified"):
        with open(os.path.join(outdir, "{}.{}.tsv".format(basename, kind)), "w") as fh:
            fh.write("\n".join(rows[kind]) + "\n")
