"""A/B of two library builds on the same synthetic batch (e.g. a kernel change against the
build before it): `dump OUT.npz [config] [contigs]` scores the batch with the library
WAAFLE_HIP_LIB names (default: the in-tree one) and saves every result field; `compare A B`
reports the fields that differ."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))

FIELDS = ("call", "crit", "rank", "clade1", "clade2", "direction", "synteny", "n_meld1", "n_meld2",
          "annot_hit", "pair_evals", "ppot_sum", "iterations", "status")


def dump(out, config="cfg5", n=6250):
    from waafle_amd import engine, synth, cli
    batch, tax = synth.generate_batch(config, 0, int(n))
    params = cli.param_dict(cli.parse_flags([]))
    s = engine.GpuScorer(0)
    s.set_taxonomy(tax)
    r = s.score(batch, params)
    again = s.score(batch, params)
    s.close()
    same = all(np.array_equal(getattr(r, f), getattr(again, f)) for f in FIELDS)
    np.savez(out, **{f: getattr(r, f) for f in FIELDS})
    print(out, "contigs", batch.n_contigs, "lgt", int((r.call == 2).sum()), "repeat-identical", same, flush=True)


def compare(a, b):
    A, B = np.load(a), np.load(b)
    bad = [f for f in FIELDS if not np.array_equal(A[f], B[f])]
    for f in bad:
        d = np.nonzero(A[f] != B[f])[0] if A[f].shape == B[f].shape else []
        print("DIFF", f, len(d), "first", d[:10])
    print("identical" if not bad else "differ")
    return 0 if not bad else 1


if __name__ == "__main__":
    if sys.argv[1] == "dump":
        dump(*sys.argv[2:])
    else:
        sys.exit(compare(sys.argv[2], sys.argv[3]))
