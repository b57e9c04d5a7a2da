"""Regenerate the waafle_junctions / waafle_qc fixtures (build container only).

Inputs: a seeded synthetic contig set (waafle_amd.synth, the syn_small recipe of
make_golden.py) rendered as FASTA + GFF, seeded synthetic read alignments over it
(waafle_amd.synth_reads, SAM), and the reference's own `.lgt.tsv` for that set (the
committed syn_small_* orgscorer fixtures).  For each case this runs, from /root/reference:

  * `waafle_junctions <fna> <gff> --sam <sam> [--min-overlap-sites N]
     --write-detailed-output`  -> .junctions.tsv, .gene_hits.tsv, .site_hits.tsv.gz
    (the .site_hits.tsv.gz writer passes text to a binary GzipFile on Python 3 and
    raises, waafle_junctions.py:323-345 + utils.py:60-72; the runner opens that one
    file in text mode, everything written is still the reference's own code);
  * `waafle_qc <lgt.tsv> <junctions.tsv> [--min-junction-hits N]` -> .qc_pass + stderr.

The fixture `junc_<case>.json.gz` stores the recipe, flags and the reference's outputs.
Run:  python tests/golden/make_junctions.py
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
from waafle_amd import synth, synth_reads  # noqa: E402

RUNNER = r'''
import gzip, sys
sys.dont_write_bytecode = True
sys.path.insert(0, "/root/reference")
from waafle import utils as wu
import waafle.waafle_junctions as wj
opener = wu.try_open
def try_open(path, *args):
    if path.endswith(".gz") and args == ("w",):
        return gzip.open(path, "wt")
    return opener(path, *args)
wu.try_open = try_open
sys.argv = ["waafle_junctions"] + sys.argv[1:]
wj.main()
'''

SETS = {
    # name: (synth.generate kwargs, orgscorer golden holding its .lgt.tsv, read kwargs)
    "small": (dict(n=300, genes=6, clades=24, seed=11, lgt_frac=0.3, decoys=3),
              "syn_small_default", dict(pairs_per_kb=4.0, seed=101)),
    "short": (dict(n=200, genes=8, clades=60, seed=7, short_frac=0.25, decoys=8),
              "syn_short_default", dict(pairs_per_kb=2.0, seed=102, insert=(100, 900))),
}
CASES = [
    ("small", [], []),
    ("small", ["--min-overlap-sites", "1"], ["--min-junction-hits", "5"]),
    ("small", ["--min-overlap-sites", "80"], ["--min-junction-hits", "0"]),
    ("short", [], []),
    ("short", ["--min-overlap-sites", "200"], ["--min-junction-hits", "1"]),
    # <= 0: every locus counts as hit (overlap 0 >= 0), including loci right of the pair
    ("small", ["--min-overlap-sites", "0"], []),
    ("short", ["--min-overlap-sites", "-3"], ["--min-junction-hits", "2"]),
]


def tag(flags):
    def one(f):   # "--flag" -> "flag", "-3" -> "m3"
        return "m" + f[1:] if f[:1] == "-" and f[1:2].isdigit() else f.lstrip("-").replace(".", "p")
    return "default" if not flags else "_".join(one(f) for f in flags)


def main(outdir=HERE):
    env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", PYTHONHASHSEED="0")
    with tempfile.TemporaryDirectory() as tmp:
        for set_name, jflags, qflags in CASES:
            gen, golden, reads = SETS[set_name]
            d = os.path.join(tmp, set_name)
            os.makedirs(d, exist_ok=True)
            data = synth.generate(**gen)
            fna, _, gff, _ = synth.write_text(data, d, "synth")
            sam = synth_reads.write_sam(data, os.path.join(d, "reads.sam"), **reads)
            with gzip.open(os.path.join(HERE, golden + ".json.gz"), "rt") as fh:
                lgt_text = json.load(fh)["tsv"]["lgt"]
            lgt = os.path.join(d, "synth.lgt.tsv")
            with open(lgt, "w") as fh:
                fh.write(lgt_text)
            out = os.path.join(d, "out_" + tag(jflags))
            os.makedirs(out, exist_ok=True)
            run = subprocess.run([sys.executable, "-c", RUNNER, fna, gff, "--sam", sam,
                                  "--outdir", out, "--basename", "case",
                                  "--write-detailed-output"] + jflags,
                                 env=env, capture_output=True, text=True, check=True)
            texts = {}
            for ext in (".junctions.tsv", ".gene_hits.tsv"):
                with open(os.path.join(out, "case" + ext)) as fh:
                    texts[ext] = fh.read()
            with gzip.open(os.path.join(out, "case.site_hits.tsv.gz"), "rt") as fh:
                texts[".site_hits.tsv"] = fh.read()
            qc_out = os.path.join(out, "case.qc_pass")
            qrun = subprocess.run([sys.executable, "-m", "waafle.waafle_qc", lgt,
                                   os.path.join(out, "case.junctions.tsv"), "--outfile",
                                   qc_out] + qflags, env=dict(env, PYTHONPATH="/root/reference"),
                                  capture_output=True, text=True)
            qc_text = None
            if os.path.exists(qc_out):
                with open(qc_out) as fh:
                    qc_text = fh.read()
            name = "junc_{}_{}_{}".format(set_name, tag(jflags), tag(qflags))
            fx = dict(case=name, recipe=dict(generate=gen, reads=reads, lgt_golden=golden),
                      junction_flags=jflags, qc_flags=qflags, junctions=texts[".junctions.tsv"],
                      gene_hits=texts[".gene_hits.tsv"], site_hits=texts[".site_hits.tsv"],
                      junctions_stderr=run.stderr, qc_returncode=qrun.returncode,
                      qc_stderr=qrun.stderr, qc_pass=qc_text)
            with gzip.open(os.path.join(outdir, name + ".junc.json.gz"), "wt") as fh:
                json.dump(fx, fh, sort_keys=True)
            print("{:50s} junction rows {:5d}  qc rc {} kept {}".format(
                name, texts[".junctions.tsv"].count("\n") - 1, qrun.returncode,
                None if qc_text is None else qc_text.count("\n") - 1))


if __name__ == "__main__":
    main(*sys.argv[1:2])
