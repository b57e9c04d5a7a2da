"""bench.py's SURVEY 8(d) op count (OPS_site, the `ops_roofline` object): its numpy attachment
rule and level walk against a per-hit, per-locus Python loop over the oracle's overlap rule,
with the oracle's own evaluated levels."""
import importlib.util
import os

import numpy as np
import pytest

from oracle import orgscorer_oracle as orc
from oracle_bridge import oracle_hits_from_batch, oracle_loci_from_batch, oracle_results
from waafle_amd import cli, synth

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load_bench():
    spec = importlib.util.spec_from_file_location("bench", os.path.join(REPO, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def brute_ops(batch, parent, pdict, iters):
    total = 0
    for c in range(batch.n_contigs):
        loci = range(int(batch.loc_off[c]), int(batch.loc_off[c + 1]))
        pairs = set()
        for h in range(int(batch.hit_off[c]), int(batch.hit_off[c + 1])):
            if not batch.hit_scov[h] >= pdict["min_scov"]:
                continue
            for g in loci:
                if pdict["stranded"] and batch.hit_strand[h] != batch.loc_strand[g]:
                    continue
                if orc.overlap_fraction(int(batch.hit_qlo[h]), int(batch.hit_qhi[h]), int(batch.loc_start[g]),
                                        int(batch.loc_end[g])) >= pdict["min_overlap"]:
                    cl = int(batch.hit_taxon[h])
                    for _ in range(max(0, pdict["jump_taxonomy"] or 0)):
                        cl = int(parent[cl])
                    pairs.add((cl, g))
        for _ in range(max(1, int(iters[c]))):
            total += sum(abs(int(batch.loc_end[g]) - int(batch.loc_start[g])) + 1 for _, g in pairs)
            pairs = {(int(parent[cl]), g) for cl, g in pairs}
    return total


@pytest.mark.parametrize("flags", [[], ["--stranded", "--min-overlap", "0.5"], ["--jump-taxonomy", "1"],
                                   ["--min-overlap", "0"]],
                         ids=["default", "stranded", "jump", "min-overlap-0"])
def test_ops_site_matches_bruteforce(flags):
    data = synth.generate(n=40, genes=6, clades=30, decoys=6, lgt_frac=0.5, seed=23)
    batch, tax = synth.to_batch(data)
    pdict = cli.param_dict(cli.parse_flags(flags))
    contigs = orc.score_contigs(dict(zip(batch.contig_names, batch.contig_lengths.tolist())),
                                oracle_loci_from_batch(batch), oracle_hits_from_batch(batch, tax),
                                orc.Taxonomy(data.tax.edges), orc.Params(**pdict))
    iters = oracle_results(contigs, batch, tax).iterations
    assert (iters > 1).any()
    bench = load_bench()
    got, sampled = bench.ops_site(batch, tax.parent, pdict, iters)
    assert sampled == batch.n_contigs
    assert got == brute_ops(batch, tax.parent, pdict, iters)
    # a sample: the first contigs within the pair budget, scaled by contigs
    part, s = bench.ops_site(batch, tax.parent, pdict, iters, pair_budget=int(np.diff(batch.hit_off)[:10].dot(
        np.diff(batch.loc_off)[:10])))
    assert s == 10
    assert part == brute_ops(batch.slice(0, 10), tax.parent, pdict, iters[:10]) * batch.n_contigs / 10
