"""Regenerate the --write-details fixtures tests/golden/details_*.json.gz (build container only).

Runs the reference `waafle_orgscorer --write-details` through ref_runner.py in "sorted"
mode (contig clade sets iterate in name order, the order this build writes; upstream
the row order within one contig and iteration follows PYTHONHASHSEED).  ref_runner opens
the details file in text mode, which is the only change: upstream raises on Python 3
when write_details() prints to the binary GzipFile.  Each fixture holds the case's input
recipe, its flags and the reference's details TSV text.

    python tests/golden/make_details.py [ungrouped]     (ungrouped: only those cases)
"""
import gzip
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
from waafle_amd import synth  # noqa: E402
from make_golden import DEMO, DEMO_INPUTS, flag_tag  # noqa: E402

# (--min-overlap 0 attaches hits with empty site ranges: a clade whose sites at a locus are
# all zero makes make_gene_spans_field raise IndexError upstream, orgscorer.py:785-789.)
CASES = [
    ("homology", []), ("prodigal", []), ("prodigal", ["--jump-taxonomy", "1"]),
    ("prodigal", ["--weak-loci", "assign-unknown"]), ("prodigal", ["--weak-loci", "penalize"]),
    ("prodigal", ["-k1", "0.9", "-k2", "0.8"]),
]
SYNTH = [("syn_small", dict(n=120, genes=6, clades=24, seed=11, lgt_frac=0.3, decoys=3),
          [[], ["--weak-loci", "assign-unknown"], ["--weak-loci", "penalize"]]),
         ("syn_short", dict(n=80, genes=8, clades=60, seed=7, short_frac=0.25, decoys=8),
          [[], ["--min-gene-length", "100"]])]
# the blastout of tests/golden/make_ungrouped.py (a contig's hits in 1-3 separate runs: the
# reference writes a contig's rows once per run, each time it evaluates it)
UNGROUPED = [[], ["--jump-taxonomy", "1"], ["--weak-loci", "penalize"]]


def run(inputs, flags, outdir):
    os.makedirs(outdir, exist_ok=True)
    cmd = [sys.executable, os.path.join(HERE, "ref_runner.py"), "sorted",
           os.path.join(outdir, "dump.json")] + inputs + \
          ["--outdir", outdir, "--basename", "case", "--quiet", "--write-details"] + flags
    subprocess.run(cmd, check=True, env=dict(os.environ, PYTHONDONTWRITEBYTECODE="1",
                                             PYTHONHASHSEED="0"), stderr=subprocess.DEVNULL)
    with gzip.open(os.path.join(outdir, "case.details.tsv.gz"), "rt") as fh:
        return fh.read()


def save(name, flags, recipe, text):
    with gzip.open(os.path.join(HERE, "details_" + name + ".json.gz"), "wt") as fh:
        json.dump(dict(case=name, flags=flags, recipe=recipe, details=text), fh, sort_keys=True)
    print("{:50s} rows={}".format(name, text.count("\n") - 1))


def main():
    only_ungrouped = sys.argv[1:] == ["ungrouped"]
    with tempfile.TemporaryDirectory() as tmp:
        d = os.path.join(HERE, "ungrouped_inputs")
        inputs = [os.path.join(d, "ungrouped" + e) for e in (".fna", ".blastout", ".gff", ".taxonomy.tsv")]
        for flags in UNGROUPED:
            name = "ungrouped_{}".format(flag_tag(flags))
            save(name, flags, dict(kind="files", dir="ungrouped_inputs", stem="ungrouped"),
                 run(inputs, flags, os.path.join(tmp, name)))
        if only_ungrouped:
            return
        for kind, flags in CASES:
            name = "demo_{}_{}".format(kind, flag_tag(flags))
            inputs = [os.path.join(DEMO, r) for r in DEMO_INPUTS[kind]]
            save(name, flags, dict(kind="demo", gff=kind), run(inputs, flags, os.path.join(tmp, name)))
        for case, params, flag_sets in SYNTH:
            sub = os.path.join(tmp, case)
            synth.write_text(synth.generate(**params), sub, "synth")
            inputs = [os.path.join(sub, "synth" + e)
                      for e in (".fna", ".blastout", ".gff", ".taxonomy.tsv")]
            for flags in flag_sets:
                name = "{}_{}".format(case, flag_tag(flags))
                save(name, flags, dict(kind="synth", params=params),
                     run(inputs, flags, os.path.join(tmp, name)))


if __name__ == "__main__":
    main()
