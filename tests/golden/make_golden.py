"""Regenerate the committed golden fixtures under tests/golden/ (build container only).

For every case it runs the reference `waafle_orgscorer` (via ref_runner.py) three
times: PYTHONHASHSEED=0 and =1 as shipped, and once with sorted clade iteration.
The fixture `<case>.json.gz` holds
  * the sorted-mode TSV texts (the target for the oracle and the HIP path),
  * the sorted-mode decision dump (crit/rank float64 hex, clades, synteny, ok),
  * `ties`: contigs whose output rows differ between the three runs (exact rank
    ties resolved by set order -- compared as "output in outcome set"),
  * `alt_rows`: those contigs' rows from the hash-seeded runs,
  * the case's input recipe (demo file names or synthetic generator parameters),
    so tests can rebuild inputs without the reference.

Inputs are the reference's demo files (read here, never copied) and the seeded
synthetic generator `waafle_amd.synth`.  Run:  python tests/golden/make_golden.py
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

DEMO = "/root/reference/demo"
DEMO_INPUTS = {
    "homology": ["input/demo_contigs.fna", "output/demo_contigs.blastout",
                 "output/demo_contigs.gff", "input/demo_taxonomy.tsv"],
    "prodigal": ["input/demo_contigs.fna", "output/demo_contigs.blastout",
                 "output_prodigal/demo_contigs.prodigal.gff", "input/demo_taxonomy.tsv"],
}

FLAG_MATRIX = [
    [], ["-k1", "0.9", "-k2", "0.8"], ["-k1", "0.3", "-k2", "0.6"],
    ["-k1", "0.95", "-k2", "0.7"], ["--weak-loci", "assign-unknown"],
    ["--weak-loci", "penalize"], ["--min-overlap", "0"], ["--stranded"],
    ["--disambiguate-one", "report-best"], ["--disambiguate-two", "report-best"],
    ["--disambiguate-two", "jump"], ["--range", "0.2"], ["--range", "0"],
    ["--jump-taxonomy", "1"], ["--jump-taxonomy", "3"], ["--allow-lca"],
    ["--ambiguous-fraction", "0.5"], ["--ambiguous-threshold", "off"],
    ["--ambiguous-threshold", "strict"], ["--sister-penalty", "lenient"],
    ["--sister-penalty", "off"], ["--clade-genes", "2"], ["--clade-leaves", "2"],
    ["--annotation-threshold", "off"], ["--annotation-threshold", "strict"],
    ["--min-gene-length", "600"], ["--min-scov", "0.9"],
    ["--sister-penalty", "off", "--ambiguous-threshold", "strict"],
    ["-k1", "0.9", "--weak-loci", "assign-unknown", "--range", "0.1"],
]

SYNTH = {
    # case: (generator kwargs, flag sets)
    "syn_cfg2": (dict(n=300, genes=8, clades=200, seed=2),
                 [[], ["--weak-loci", "assign-unknown"], ["-k1", "0.9"],
                  ["--jump-taxonomy", "1"], ["--disambiguate-two", "report-best"]]),
    "syn_cfg3": (dict(n=200, genes=12, clades=1000, seed=3), [[], ["-k1", "0.95", "-k2", "0.85"]]),
    "syn_cfg4": (dict(n=200, genes=10, clades=2000, seed=4), [[]]),
    "syn_small": (dict(n=300, genes=6, clades=24, seed=11, lgt_frac=0.3, decoys=3),
                  [[], ["--weak-loci", "assign-unknown"], ["--sister-penalty", "lenient"],
                   ["-k1", "0.8", "-k2", "0.7"], ["--clade-leaves", "3", "--clade-genes", "2"],
                   ["--min-overlap", "0"], ["--stranded"]]),
    "syn_short": (dict(n=200, genes=8, clades=60, seed=7, short_frac=0.25, decoys=8),
                  [[], ["--min-gene-length", "100"]]),
    "syn_stress": (dict(n=3, genes=20, clades=600, seed=5, stress=True), [[]]),
    # size-dependent device paths (round 2): full cfg5 stress contigs (5000 clades, ~5000
    # attachments: device radix sort + mask-class explain_two), > 4096 attachments with a
    # small potential set, and > 64 / > 128 loci (non-mask two-clade test, HBM loci)
    "syn_cfg5": (dict(n=2, genes=20, clades=5000, seed=5, stress=True), [[]]),
    "syn_bigatt": (dict(n=2, genes=10, clades=100, seed=21, decoys=600, lgt_frac=0.5),
                   [[], ["-k1", "0.9"]]),
    "syn_loci70": (dict(n=4, genes=70, clades=60, seed=22, decoys=4, lgt_frac=0.75),
                   [[], ["--weak-loci", "assign-unknown"], ["-k1", "0.9"],
                    ["-k1", "0.9", "--weak-loci", "assign-unknown"]]),
    "syn_loci150": (dict(n=3, genes=150, clades=80, seed=23, decoys=3, lgt_frac=0.75),
                    [[], ["-k1", "0.9"]]),
}


def flag_tag(flags):
    return "default" if not flags else "_".join(f.lstrip("-").replace(".", "p") for f in flags)


def run_ref(mode, inputs, flags, outdir, env_extra):
    os.makedirs(outdir, exist_ok=True)
    dump = os.path.join(outdir, "dump.json")
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", **env_extra)
    cmd = [sys.executable, os.path.join(HERE, "ref_runner.py"), mode, dump] + inputs + \
          ["--outdir", outdir, "--basename", "case", "--quiet"] + flags
    subprocess.run(cmd, check=True, env=env, stderr=subprocess.DEVNULL)
    texts = {}
    for kind in ("lgt", "no_lgt", "unclassified"):
        with open(os.path.join(outdir, "case.{}.tsv".format(kind))) as fh:
            texts[kind] = fh.read()
    with open(dump) as fh:
        return texts, json.load(fh)


def rows_by_contig(texts):
    out = {}
    for kind, text in texts.items():
        for line in text.splitlines()[1:]:
            out[line.split("\t", 1)[0]] = (kind, line)
    return out


def make_case(name, inputs, flags, recipe, tmp, dump_scores):
    env = {"REF_DUMP_SCORES": "1" if dump_scores else "0"}
    runs = {}
    for tag, mode, seed in (("sorted", "sorted", "0"), ("h0", "hash", "0"), ("h1", "hash", "1")):
        texts, dump = run_ref(mode, inputs, flags, os.path.join(tmp, name, tag),
                              dict(env, PYTHONHASHSEED=seed))
        runs[tag] = (texts, dump)
    base = rows_by_contig(runs["sorted"][0])
    ties, alt = [], {}
    for tag in ("h0", "h1"):
        other = rows_by_contig(runs[tag][0])
        for contig, row in other.items():
            if base.get(contig) != row:
                if contig not in ties:
                    ties.append(contig)
                alt.setdefault(contig, [])
                if list(row) not in alt[contig]:
                    alt[contig].append(list(row))
    fixture = dict(case=name, flags=flags, recipe=recipe, tsv=runs["sorted"][0],
                   dump=runs["sorted"][1], ties=sorted(ties), alt_rows=alt)
    path = os.path.join(HERE, name + ".json.gz")
    with gzip.open(path, "wt") as fh:
        json.dump(fixture, fh, sort_keys=True)
    n = {k: v.count("\n") - 1 for k, v in runs["sorted"][0].items()}
    print("{:55s} lgt/no_lgt/unclassified={}/{}/{} ties={}".format(
        name, n["lgt"], n["no_lgt"], n["unclassified"], len(ties)))


def main():
    only = set(sys.argv[1:])
    with tempfile.TemporaryDirectory() as tmp:
        for gff_kind, rel in DEMO_INPUTS.items():
            inputs = [os.path.join(DEMO, r) for r in rel]
            for flags in FLAG_MATRIX:
                if gff_kind == "homology" and flags not in (
                        [], ["--sister-penalty", "off", "--ambiguous-threshold", "strict"],
                        ["--min-overlap", "0"], ["--weak-loci", "assign-unknown"],
                        ["--jump-taxonomy", "1"], ["-k1", "0.95", "-k2", "0.7"]):
                    continue
                name = "demo_{}_{}".format(gff_kind, flag_tag(flags))
                if only and name not in only:
                    continue
                make_case(name, inputs, flags, dict(kind="demo", gff=gff_kind), tmp,
                          dump_scores=not flags)
        for base, (kw, flag_sets) in SYNTH.items():
            sdir = os.path.join(tmp, "inputs", base)
            data = synth.generate(**kw)
            inputs = synth.write_text(data, sdir, "synth")
            for flags in flag_sets:
                name = "{}_{}".format(base, flag_tag(flags))
                if only and name not in only:
                    continue
                make_case(name, inputs, flags, dict(kind="synth", params=kw), tmp,
                          dump_scores=(not flags and kw["n"] <= 300
                                       and kw["clades"] * kw["genes"] <= 20000))
        tie_dir = os.path.join(HERE, "tie_inputs")
        inputs = [os.path.join(tie_dir, f) for f in
                  ("tie.fna", "tie.blastout", "tie.gff", "tie.taxonomy.tsv")]
        for flags in ([], ["--disambiguate-one", "report-best"]):
            name = "tie_{}".format(flag_tag(flags))
            if only and name not in only:
                continue
            make_case(name, inputs, flags, dict(kind="files", dir="tie_inputs"), tmp,
                      dump_scores=True)


if __name__ == "__main__":
    main()
