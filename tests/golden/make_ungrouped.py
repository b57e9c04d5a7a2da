"""Fixtures of a blastout NOT grouped by query (build container only).

The reference reads the blastout as runs of consecutive rows with one qseqid
(utils.py:255-270) and scores each run as it comes (orgscorer.py:941-960): a contig
whose hits come in several runs is attached, rolled up and evaluated once per run,
every run on top of the state the previous evaluations left (site scores already
raised, annotations kept), and the last evaluation is what it writes.  These cases
take the seeded synthetic contigs (`waafle_amd.synth`, syn_small's shape) and split
contig i's hits, in file order, into runs by i % 5:
  0  one run (grouped)
  1  first half | second half        (run 1 usually leaves loci without hits)
  2  even rows | odd rows            (run 1 usually covers every locus)
  3  three runs: rows mod 3
  4  the last row alone in run 2
The runs are written round by round: every contig's run 1 (FASTA order), then every
run 2, then every run 3.  GFF and FASTA stay as generated.  Each case is run by
make_golden.make_case (reference under two hash seeds and sorted clade order).
Run:  python tests/golden/make_ungrouped.py
"""
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, REPO)
import make_golden  # noqa: E402
from waafle_amd import synth  # noqa: E402

INPUTS = os.path.join(HERE, "ungrouped_inputs")
PARAMS = dict(n=120, genes=6, clades=24, seed=31, lgt_frac=0.3, decoys=3)
FLAG_SETS = [[], ["--jump-taxonomy", "1"], ["--weak-loci", "assign-unknown"],
             ["--weak-loci", "penalize"]]


def split_runs(i, rows):
    style = i % 5
    n = len(rows)
    if style == 0 or n < 2:
        return [rows]
    if style == 1:
        return [rows[:n // 2], rows[n // 2:]]
    if style == 2:
        return [rows[0::2], rows[1::2]]
    if style == 3 and n >= 3:
        return [rows[0::3], rows[1::3], rows[2::3]]
    return [rows[:-1], rows[-1:]]


def write_inputs():
    with tempfile.TemporaryDirectory() as tmp:
        synth.write_text(synth.generate(**PARAMS), tmp, "u")
        os.makedirs(INPUTS, exist_ok=True)
        stem = os.path.join(INPUTS, "ungrouped")
        for ext in (".fna", ".gff", ".taxonomy.tsv"):
            with open(os.path.join(tmp, "u" + ext)) as src, open(stem + ext, "w") as dst:
                dst.write(src.read())
        order, by = [], {}
        with open(os.path.join(tmp, "u.blastout")) as fh:
            for line in fh:
                q = line.split("\t", 1)[0]
                if q not in by:
                    order.append(q)
                    by[q] = []
                by[q].append(line)
    rounds = [[], [], []]
    for i, q in enumerate(order):
        for r, run in enumerate(split_runs(i, by[q])):
            rounds[r].append(run)
    with open(stem + ".blastout", "w") as fh:
        for rnd in rounds:
            for run in rnd:
                fh.writelines(run)
    return [stem + e for e in (".fna", ".blastout", ".gff", ".taxonomy.tsv")]


def main():
    inputs = write_inputs()
    with tempfile.TemporaryDirectory() as tmp:
        for flags in FLAG_SETS:
            name = "ungrouped_{}".format(make_golden.flag_tag(flags))
            make_golden.make_case(name, inputs, flags,
                                  dict(kind="files", dir="ungrouped_inputs", stem="ungrouped"),
                                  tmp, dump_scores=True)


if __name__ == "__main__":
    main()
