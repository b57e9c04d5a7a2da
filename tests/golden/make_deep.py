"""Deep-taxonomy fixtures: roll-up depth and the runaway guard (build container only).

`evaluate_contig` raises a contig's clades one level per iteration and dies with
"Runaway taxonomic recursion" once the iteration counter passes 100
(waafle_orgscorer.py:566-583, the die at :580-581).  These inputs reach that guard
without a cyclic taxonomy (a cycle never reaches r__Root, so Taxonomy.get_lineage at
utils.py:392-399 would not terminate upstream):

  * every contig has two 300 bp genes; gene 1 is hit only by leaf A_<tag>, gene 2 only by
    leaf B_<tag> (pident 90, full coverage), and -k2 0.95 keeps explain_two empty, so
    neither option is OK until A's and B's lineages meet;
  * A and B hang under two separate chains of depth D from r__Root, so they meet at
    r__Root after D raises (iteration D + 1).

Cases (each run separately, because a die ends the whole run):
  deep_ok     : D = 40 (one-clade call at r__Root after 40 raises, beyond the 16-level
                lineage table), D = 99 (the last depth that passes: iteration 100), and a
                mixed pair (A at depth 120, B at depth 5: B reaches r__Root first and the
                loop stops with the contig unclassified, iteration 6);
  deep_d100   : D = 100 -> the 100th raise makes iteration 101 -> die;
  deep_d130   : D = 130 -> die at the same point.
The fixture stores the reference's TSVs, or its exit status and stderr.
Run:  python tests/golden/make_deep.py
"""
import gzip
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
INPUTS = os.path.join(HERE, "deep_inputs")
CASES = {"deep_ok": [("d40", 40, 40), ("d99", 99, 99), ("mixed", 120, 5)],
         "deep_d100": [("d100", 100, 100)],
         "deep_d130": [("d130", 130, 130)]}
FLAGS = ["-k2", "0.95"]


def write_inputs(case, contigs):
    d = os.path.join(INPUTS, case)
    os.makedirs(d, exist_ok=True)
    tax, fna, gff, blast = [], [], [], []
    for tag, da, db in contigs:
        for side, depth in (("A", da), ("B", db)):
            prev = "r__Root"
            for k in range(1, depth):
                node = "x__{}{}_{}".format(side, tag, k)
                tax.append((node, prev))
                prev = node
            tax.append(("s__{}_{}".format(side, tag), prev))
        name = "contig_" + tag
        fna.append(">{}\n{}\n".format(name, "N" * 700))
        gff.append("{}\tdeep\tgene\t11\t310\t.\t+\t0\t.\n".format(name))
        gff.append("{}\tdeep\tgene\t381\t680\t.\t-\t0\t.\n".format(name))
        for i, (qs, side) in enumerate(((11, "A"), (381, "B"))):
            blast.append("{}\tG{}|s__{}_{}|KO=K{}\t700\t300\t300\t{}\t{}\t1\t300\t90.0\t270\t0\t0.0"
                         "\t500\tplus\n".format(name, i, side, tag, i, qs, qs + 299))
    paths = [os.path.join(d, "deep" + e) for e in (".fna", ".blastout", ".gff", ".taxonomy.tsv")]
    for p, lines in zip(paths, (fna, blast, gff, ["{}\t{}\n".format(c, p) for c, p in tax])):
        with open(p, "w") as fh:
            fh.writelines(lines)
    return paths


def main():
    for case, contigs in CASES.items():
        paths = write_inputs(case, contigs)
        with tempfile.TemporaryDirectory() as tmp:
            env = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", PYTHONHASHSEED="0",
                       PYTHONPATH="/root/reference")
            cmd = [sys.executable, "-m", "waafle.waafle_orgscorer"] + paths + \
                  ["--outdir", tmp, "--basename", "case", "--quiet"] + FLAGS
            run = subprocess.run(cmd, env=env, capture_output=True, text=True)
            fx = dict(case=case, flags=FLAGS, recipe=dict(kind="files", dir="deep_inputs/" + case,
                                                          stem="deep"),
                      returncode=run.returncode, stderr=run.stderr, tsv=None)
            if run.returncode == 0:
                fx["tsv"] = {}
                for kind in ("lgt", "no_lgt", "unclassified"):
                    with open(os.path.join(tmp, "case.{}.tsv".format(kind))) as fh:
                        fx["tsv"][kind] = fh.read()
        with gzip.open(os.path.join(HERE, case + ".runaway.json.gz"), "wt") as fh:
            json.dump(fx, fh, sort_keys=True)
        print(case, "rc", run.returncode, run.stderr.strip().splitlines()[-2:] if run.returncode else
              {k: v.count("\n") - 1 for k, v in fx["tsv"].items()})


if __name__ == "__main__":
    main()
