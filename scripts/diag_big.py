"""Diagnostic: the HBM decision tier (small decision arena) against the default arena on a
cfg4 contig range, with the oracle on the contigs where they differ.

    python scripts/diag_big.py [N_CONTIGS] [LDS_BYTES] > gpurun_out/diag.json
"""
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

from waafle_amd import cli, engine, synth  # noqa: E402

FIELDS = ("call", "crit", "rank", "clade1", "clade2", "direction", "n_meld1", "n_meld2",
          "iterations", "status", "pair_evals")


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
    lds = int(sys.argv[2]) if len(sys.argv) > 2 else 16384
    batch, tax = synth.generate_batch("cfg4", 0, n, workers=16)
    params = cli.param_dict(cli.parse_flags([]))
    out = {"contigs": n, "lds_bytes": lds}
    res = {}
    for tag, kw in (("default", {}), ("small", {"lds_bytes": lds}), ("staged", {"mode": "staged"})):
        s = engine.GpuScorer(0, **kw)
        s.set_taxonomy(tax)
        res[tag] = s.score(batch, params)
        s.close()
        out["status_" + tag] = {int(k): int(v) for k, v in zip(*np.unique(res[tag].status, return_counts=True))}
    diff = np.zeros(n, bool)
    for f in FIELDS:
        a, b = getattr(res["default"], f), getattr(res["small"], f)
        if f in ("crit", "rank"):
            a, b = a.view(np.int64), b.view(np.int64)
        diff |= a != b
    idx = np.nonzero(diff)[0]
    out["n_diff"] = int(idx.size)
    rows = []
    for c in idx[:12].tolist():
        rows.append({"c": c, **{t: {f: (float(getattr(r, f)[c]) if f in ("crit", "rank") else int(getattr(r, f)[c]))
                                    for f in FIELDS} for t, r in res.items()},
                     "hits": int(batch.hit_off[c + 1] - batch.hit_off[c]),
                     "loci": int(batch.loc_off[c + 1] - batch.loc_off[c])})
    if idx.size:
        from oracle import orgscorer_oracle as orc          # the checker
        from oracle_bridge import oracle_hits_from_batch, oracle_loci_from_batch
        chunk = synth.chunk_size("cfg4")
        for row in rows[:6]:
            c = row["c"]
            data = synth.generate_chunk("cfg4", c // chunk)      # names for the oracle
            b2, t2 = synth.to_batch(data, with_codes=False)
            sub = b2.slice(c % chunk, c % chunk + 1)
            try:
                contigs = orc.score_contigs(dict(zip(sub.contig_names, sub.contig_lengths.tolist())),
                                            oracle_loci_from_batch(sub), oracle_hits_from_batch(sub, t2),
                                            orc.Taxonomy(data.tax.edges), orc.Params(**params))
            except BaseException as exc:        # the reference's die / numpy errors
                row["oracle"] = repr(exc)
                continue
            k = next(iter(contigs.values()))
            row["oracle"] = {"one": None if k.best_one is None else [k.best_one.crit, k.best_one.rank],
                             "two": None if k.best_two is None else [k.best_two.crit, k.best_two.rank]}
    out["rows"] = rows
    print(json.dumps(out, default=str))


if __name__ == "__main__":
    main()
