"""What a blastout not grouped by contig costs the CLI (scope iii): the cfg2 text as generated
and the same rows with every 4th contig's hits split into two runs, the second halves moved
to the end of the file (so 25% of the contigs are evaluated twice, regroup.py).  Prints one
JSON object: wall time and the CLI's phase line for both files, and whether the two runs'
TSVs differ (they should: the reference scores a split contig differently).

    python scripts/ungrouped_cost.py [--config cfg2] [--out FILE]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def split_file(src, dst, every=4):
    order, by = [], {}
    with open(src) as fh:
        for line in fh:
            q = line.split("\t", 1)[0]
            if q not in by:
                order.append(q)
                by[q] = []
            by[q].append(line)
    late = []
    with open(dst, "w") as fh:
        for i, q in enumerate(order):
            rows = by[q]
            if i % every == 1 and len(rows) > 1:
                fh.writelines(rows[:len(rows) // 2])
                late.append(rows[len(rows) // 2:])
            else:
                fh.writelines(rows)
        for rows in late:
            fh.writelines(rows)
    return len(late)


def run_cli(paths, outdir):
    os.makedirs(outdir, exist_ok=True)
    cmd = [sys.executable, "-m", "waafle_amd.orgscorer"] + paths + ["--outdir", outdir, "--basename", "x"]
    t0 = time.perf_counter()
    run = subprocess.run(cmd, capture_output=True, text=True, cwd=REPO, timeout=900)
    wall = time.perf_counter() - t0
    if run.returncode != 0:
        raise SystemExit(run.stderr[-3000:])
    phases = [l for l in run.stderr.splitlines() if l.startswith("Finished successfully")]
    texts = {}
    for kind in ("lgt", "no_lgt", "unclassified"):
        with open(os.path.join(outdir, "x.{}.tsv".format(kind))) as fh:
            texts[kind] = fh.read()
    return wall, phases[-1] if phases else None, texts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from waafle_amd import synth
    with tempfile.TemporaryDirectory() as tmp:
        paths, n, nh = synth.write_text_chunked(a.config, tmp, "e2e", workers=8)
        ug = os.path.join(tmp, "ungrouped.blastout")
        nsplit = split_file(paths[1], ug)
        g_wall, g_ph, g_tx = run_cli(paths, os.path.join(tmp, "g"))
        u_wall, u_ph, u_tx = run_cli([paths[0], ug, paths[2], paths[3]], os.path.join(tmp, "u"))
    diff = sum(1 for k in g_tx for x, y in zip(g_tx[k].splitlines(), u_tx[k].splitlines()) if x != y)
    out = {"config": a.config, "contigs": n, "hits": nh, "split_contigs": nsplit,
           "grouped": {"wall_s": g_wall, "phases": g_ph},
           "ungrouped": {"wall_s": u_wall, "phases": u_ph},
           "rows_differing": diff,
           "scope": "text files -> native ingest -> wf_score (1 GPU; ungrouped: one extra wf_score "
                    "over the split contigs' first runs, regroup.py) -> 3 TSVs, one process"}
    line = json.dumps(out)
    print(line)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(line + "\n")


if __name__ == "__main__":
    main()
