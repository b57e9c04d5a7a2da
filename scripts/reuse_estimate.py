"""How often a roll-up segment's mean could be carried over from the level below (CPU only).

A segment (clade P, locus g) at level L keeps its level-(L-1) mean exactly when all of its
attachments had one clade at level L-1 (the same attachment set, so the same envelope).
This counts, on one 10,000-contig chunk of the cfg4 synthetic set (every contig, hits at
species level, parents by make_taxonomy's rule), the multi-attachment segments per contig
at levels 1-4 -- the ones whose means cost the roll-up launches most -- and the share of
them that are unchanged from the level below.  (DESIGN.md §9 quotes the result.)

    python scripts/reuse_estimate.py
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from waafle_amd import synth
    spec = synth.CONFIGS["cfg4"]
    d = synth.generate_chunk("cfg4", 0)
    n = d.n_contigs
    s = spec["clades"]
    counts = [1, 2, 4, max(1, s // 48), max(1, s // 16), max(1, s // 4), s]   # make_taxonomy
    anc = [d.hit_clade.astype(np.int64)]
    lv = len(counts) - 1
    for _ in range(4):
        anc.append(anc[-1] * counts[lv - 1] // counts[lv])
        lv -= 1
    for L in range(1, 5):
        seg = (d.hit_contig.astype(np.int64) * 64 + d.hit_gene) * (s + 1) + anc[L]
        order = np.argsort(seg, kind="stable")
        key, child = seg[order], anc[L - 1][order]
        starts = np.r_[0, np.nonzero(np.diff(key))[0] + 1]
        sizes = np.diff(np.r_[starts, len(key)])
        multi = sizes >= 2
        # unchanged: one child clade over the segment (its min and max child ids agree)
        cmin = np.minimum.reduceat(child, starts)
        cmax = np.maximum.reduceat(child, starts)
        same = cmin == cmax
        print("level {}: segments/contig {:.1f}, multi-attachment {:.1f} ({:.1f} attachments), "
              "unchanged from level {} {:.1%}".format(L, len(starts) / n, multi.sum() / n,
                                                     sizes[multi].sum() / n, L - 1,
                                                     same[multi].mean() if multi.any() else 0.0))


if __name__ == "__main__":
    main()
