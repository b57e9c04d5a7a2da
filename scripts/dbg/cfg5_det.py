"""Debug: the cfg5 6,250-contig share generated as the k2 leg and as --config cfg5 --contigs 6250
give the same inputs and the same records; two passes give the same records."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
from waafle_amd import synth, cli, engine
a, ta = synth.generate_batch("cfg5", 0, 6250, workers=16)
b, tb = synth.generate_batch("cfg5", 0, 6250, workers=16, n_total=6250)
for f in ("hit_off", "hit_qlo", "hit_qhi", "hit_taxon", "hit_score", "hit_scov", "loc_off", "loc_start"):
    print(f, np.array_equal(getattr(a, f), getattr(b, f)))
print("tax", list(ta.names) == list(tb.names))
p = cli.param_dict(cli.parse_flags([]))
s = engine.GpuScorer(0)
s.set_taxonomy(ta)
r1 = s.score(a, p)
r2 = s.score(a, p)
r3 = s.score(b, p)
for f in ("call", "crit", "rank", "clade1", "clade2", "iterations", "pair_evals", "ppot_sum"):
    x, y, z = getattr(r1, f), getattr(r2, f), getattr(r3, f)
    print(f, int((x != y).sum()), int((x != z).sum()))
print("lgt", int((r1.call == 2).sum()), int((r3.call == 2).sum()))
