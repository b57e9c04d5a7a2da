"""Debug: GPU ppot_sum vs the oracle's per-level pools on the -k1 0.9 synthetic case."""
import os, sys, tempfile
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import numpy as np
from waafle_amd import synth, cli, inputs, engine, lib
from oracle import orgscorer_oracle as orc
from oracle_bridge import oracle_results
flags = ["-k1", "0.9"]
tmp = tempfile.mkdtemp()
data = synth.generate(n=600, genes=12, clades=1000, seed=31)
paths = synth.write_text(data, tmp, "s")
args = cli.parse_flags(flags)
batch, tax = inputs.load_inputs(*paths, args.min_gene_length, warn=None)
pools = {}
orig = orc.two_clade
def spy(C, t):
    p = C.p
    pool = [c for c in orc._ordered(C.clades) if max(C.genes[c]) >= p.k2]
    pools.setdefault(id(C), []).append(len(pool))
    return orig(C, t)
orc.two_clade = spy
contigs, _ = orc.run(*paths, orc.Params(**cli.param_dict(args)))
want = oracle_results(contigs, batch, tax)
for form, kw in (("level0", {}), ("staged", dict(mode="staged")), ("notriage", dict(options={lib.OPT_TRIAGE: 0}))):
    s = engine.GpuScorer(0, **kw)
    s.set_taxonomy(tax)
    got = s.score(batch, cli.param_dict(args))
    s.close()
    bad = np.nonzero(got.ppot_sum != want.ppot_sum)[0]
    print(form, "mismatch", len(bad), "pair_evals mismatch", int((got.pair_evals != want.pair_evals).sum()))
    for c in bad[:6]:
        C = contigs[batch.contig_names[c]]
        print("  c", c, "gpu", int(got.ppot_sum[c]), "oracle", int(want.ppot_sum[c]), "pools", pools.get(id(C)),
              "pairs", int(got.pair_evals[c]), int(want.pair_evals[c]), "iters", int(got.iterations[c]), int(want.iterations[c]))
