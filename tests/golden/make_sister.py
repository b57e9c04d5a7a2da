"""Sister-penalty fixtures with taxa missing from the taxonomy file (build container only).

`check_sister_penalty` (waafle_orgscorer.py:717-744) penalises a locus by
`Taxonomy.get_sisters(clade) = children(parent(clade)) - {clade}` (utils.py:428-434).  A
hit taxon that is not listed in the taxonomy file has parent r__Root
(`get_parent`, utils.py:386-387) but is nobody's listed child, so its sisters are
r__Root's listed children, while no clade counts it as a sister.  These contigs make
the two-clade option depend on exactly that:

  unl_b    unlisted X on genes 1, 2, 4 and listed s__Y on gene 3 (B>A, recipient s__Y);
           root child k__C scores 0.60 on gene 3 (a B locus, X's sister via r__Root)
  unl_b85  the same with k__C at 0.85 (fails --sister-penalty lenient as well)
  unl_ok   the same without k__C (the LGT call stands)
  lst_b    listed s__Y on genes 1, 2, 4, unlisted X on gene 3: swapped, sisters of s__Y
           (s__Z at 0.60 on gene 3)
  unl_ab   unlisted U1 on genes 1, 2 and unlisted U2 on genes 3, 4 (A?B: both sides
           checked); root child k__B at 0.60 on gene 1 (an A locus, U2's sister)
  unl_sib  unlisted X vs listed s__Y, and root child k__B (not a hit on any B locus) at
           0.90 on gene 3 plus k__C at 0.55 on gene 2 (A locus: not checked, B>A)

Each case is run by make_golden.make_case (reference under two hash seeds and sorted
clade order).  Run:  python tests/golden/make_sister.py
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden  # noqa: E402

INPUTS = os.path.join(HERE, "sister_inputs")
GENES = [(1, 300), (401, 700), (801, 1100), (1201, 1500)]
TAXONOMY = [("k__B", "r__Root"), ("k__C", "r__Root"), ("p__P", "k__B"), ("g__G", "p__P"),
            ("s__Y", "g__G"), ("s__Z", "g__G"), ("s__Q", "g__G")]
# contig -> [(taxon, gene index, pident)]
CONTIGS = {
    "unl_b": [("s__X", 0, 95), ("s__X", 1, 95), ("s__X", 3, 95), ("s__Y", 2, 95), ("k__C", 2, 60)],
    "unl_b85": [("s__X", 0, 95), ("s__X", 1, 95), ("s__X", 3, 95), ("s__Y", 2, 95), ("k__C", 2, 85)],
    "unl_ok": [("s__X", 0, 95), ("s__X", 1, 95), ("s__X", 3, 95), ("s__Y", 2, 95)],
    "lst_b": [("s__Y", 0, 95), ("s__Y", 1, 95), ("s__Y", 3, 95), ("s__X", 2, 95), ("s__Z", 2, 60)],
    "unl_ab": [("s__U1", 0, 95), ("s__U1", 1, 95), ("s__U2", 2, 95), ("s__U2", 3, 95),
               ("k__B", 0, 60)],
    "unl_sib": [("s__X", 0, 95), ("s__X", 1, 95), ("s__X", 3, 95), ("s__Y", 2, 95),
                ("k__B", 2, 90), ("k__C", 1, 55)],
}
FLAG_SETS = [[], ["--sister-penalty", "lenient"], ["--sister-penalty", "off"]]


def write_inputs():
    os.makedirs(INPUTS, exist_ok=True)
    stem = os.path.join(INPUTS, "sister")
    with open(stem + ".taxonomy.tsv", "w") as fh:
        fh.writelines("{}\t{}\n".format(c, p) for c, p in TAXONOMY)
    with open(stem + ".fna", "w") as fh:
        for name in CONTIGS:
            fh.write(">{}\n{}\n".format(name, "N" * 1600))
    with open(stem + ".gff", "w") as fh:
        for name in CONTIGS:
            for s, e in GENES:
                fh.write("{}\thand\tgene\t{}\t{}\t.\t+\t0\t.\n".format(name, s, e))
    with open(stem + ".blastout", "w") as fh:
        k = 0
        for name, hits in CONTIGS.items():
            for taxon, g, pident in sorted(hits, key=lambda h: (GENES[h[1]][0], h[0])):
                s, e = GENES[g]
                fh.write("{}\tH{}|{}|KO=K{}\t1600\t300\t300\t{}\t{}\t1\t300\t{:.3f}\t300\t0\t0.0\t500\tplus\n"
                         .format(name, k, taxon, k, s, e, float(pident)))
                k += 1
    return [stem + e for e in (".fna", ".blastout", ".gff", ".taxonomy.tsv")]


def main():
    import tempfile
    inputs = write_inputs()
    with tempfile.TemporaryDirectory() as tmp:
        for flags in FLAG_SETS:
            name = "sister_{}".format(make_golden.flag_tag(flags))
            make_golden.make_case(name, inputs, flags, dict(kind="files", dir="sister_inputs", stem="sister"),
                                  tmp, dump_scores=True)


if __name__ == "__main__":
    main()
