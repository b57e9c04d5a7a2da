"""Host-side product logic on CPU: parsing/packing, taxonomy interning, sharding and
TSV rendering, driven by oracle decisions (the GPU supplies them in production)."""
import numpy as np
import pytest

import golden_cases as gc
from oracle_bridge import oracle_results, run_oracle
from waafle_amd import cli, engine, inputs, output, synth
from waafle_amd.taxonomy import TaxonomyTables, TaxonomyError

CASES = gc.case_names()


def load(fx, tmp_path):
    paths = gc.materialize(fx, tmp_path)
    args = cli.parse_flags(fx["flags"])
    batch, tax = inputs.load_inputs(*paths, args.min_gene_length, warn=None)
    return paths, batch, tax


@pytest.mark.parametrize("name", CASES)
def test_render_from_oracle_decisions_matches_goldens(name, tmp_path):
    fx = gc.load(name)
    paths, batch, tax = load(fx, tmp_path)
    contigs, _ = run_oracle(paths, fx["flags"])
    res = oracle_results(contigs, batch, tax)
    rows = output.render(batch, tax, res)
    texts = {k: "\n".join(v) + "\n" for k, v in rows.items()}
    assert gc.compare_tsv(fx, texts) == []


def test_packed_scores_match_oracle_hits(tmp_path):
    fx = gc.load("demo_prodigal_default")
    paths, batch, tax = load(fx, tmp_path)
    from oracle import orgscorer_oracle as orc
    rows = list(orc._tsv_rows(paths[1]))
    for i in range(batch.n_hits):
        h = orc.BlastHit(rows[int(batch.hit_row[i])])
        assert batch.hit_score[i] == h.score and batch.hit_scov[i] == h.scov_mod
        assert tax.names[batch.hit_taxon[i]] == h.taxon
        assert batch.hit_qlo[i] == min(h.qstart, h.qend)
        assert batch.hit_strand[i] == (1 if h.strand == "-" else 0)


def test_synth_text_and_binary_agree(tmp_path):
    data = synth.generate(n=40, genes=6, clades=30, seed=3, short_frac=0.1)
    paths = synth.write_text(data, str(tmp_path), "s")
    batch, tax = inputs.load_inputs(*paths, 200.0, warn=None)
    direct, dtax = synth.to_batch(data, 200.0)
    assert tax.names == dtax.names
    for f in ("hit_off", "hit_qlo", "hit_qhi", "hit_taxon", "hit_strand", "hit_score",
              "hit_scov", "hit_sysmask", "loc_off", "loc_start", "loc_end", "loc_strand"):
        np.testing.assert_array_equal(getattr(batch, f), getattr(direct, f), err_msg=f)


def test_shard_concat_roundtrip(tmp_path):
    fx = gc.load("syn_cfg2_default")
    paths, batch, tax = load(fx, tmp_path)
    contigs, _ = run_oracle(paths, fx["flags"])
    full = oracle_results(contigs, batch, tax)
    bounds = engine.shard_bounds(engine.contig_cost(batch), 3)
    assert bounds[0][0] == 0 and bounds[-1][1] == batch.n_contigs and len(bounds) == 3
    parts = []
    for a, b in bounds:
        sub = batch.slice(a, b)
        r = oracle_results(contigs, sub, tax)
        parts.append(r)
    merged = engine.Results.concat(parts, [int(batch.hit_off[a]) for a, _ in bounds])
    for f in full.__dataclass_fields__:
        np.testing.assert_array_equal(getattr(full, f), getattr(merged, f), err_msg=f)


def test_taxonomy_tables():
    edges = [("k__A", "r__Root"), ("g__B", "k__A"), ("s__C", "g__B"), ("s__D", "g__B")]
    t = TaxonomyTables(edges, extra_names={"s__X"})
    assert t.names == sorted(t.names)
    i = t.index
    assert t.parent[i["s__C"]] == i["g__B"] and t.parent[i["s__X"]] == i["r__Root"]
    assert t.depth[i["s__C"]] == 3 and t.depth[i["r__Root"]] == 0 and t.depth[i["s__X"]] == 1
    assert t.sib_parent[i["s__C"]] == i["g__B"] and t.sib_parent[i["s__X"]] == -1
    assert t.leaf_count[i["g__B"]] == 2 and t.leaf_count[i["r__Root"]] == 2
    assert t.lca([i["s__C"], i["s__D"]]) == "g__B"
    assert t.tail(i["s__C"], "k__A") == ["g__B", "s__C"]
    with pytest.raises(TaxonomyError):
        TaxonomyTables([("a", "b"), ("b", "a")])
    with pytest.raises(TaxonomyError):
        TaxonomyTables([("s__C", "g__B"), ("s__C", "g__Z")])


def test_ungrouped_blastout_keeps_its_runs(tmp_path):
    fx = gc.load("tie_default")
    paths = gc.materialize(fx, tmp_path)
    lines = open(paths[1]).read().splitlines()
    bad = tmp_path / "bad.blastout"
    bad.write_text("\n".join([lines[0], lines[4], lines[1]]) + "\n")
    b, _ = inputs.load_inputs(paths[0], str(bad), paths[2], paths[3], 200.0, warn=None)
    q = [ln.split("\t", 1)[0] for ln in (lines[0], lines[4], lines[1])]
    assert q[0] == q[2] != q[1]
    c = b.contig_names.index(q[0])
    h0, h1 = int(b.hit_off[c]), int(b.hit_off[c + 1])
    assert b.hit_group[h0:h1].tolist() == [0, 1] and b.hit_row[h0:h1].tolist() == [0, 2]


def test_regroup_raises_each_run_by_the_levels_it_has_been_through():
    """regroup.resolve: run g's hits enter the last evaluation at ancestor^R(taxon),
    R = sum over the evaluations since g of (jumps + iterations - 1) (orgscorer.py:941-960)."""
    from waafle_amd import regroup
    from waafle_amd.engine import Results
    parent = np.array([0, 0, 1, 2, 3, 4, 5, 6, 7, 8], dtype=np.int32)   # a chain, 0 the root
    H = 6
    z = np.zeros(H, np.int32)
    b = inputs.HostBatch(
        contig_names=["a", "b"], contig_lengths=np.array([900, 900]), hit_off=np.array([0, 4, 6]),
        hit_qlo=z + 1, hit_qhi=z + 300, hit_taxon=z + 9, hit_strand=z.astype(np.int8),
        hit_score=np.ones(H), hit_scov=np.ones(H), hit_sysmask=z.astype(np.uint32),
        loc_off=np.array([0, 1, 2]), loc_start=np.array([1, 1], np.int32),
        loc_end=np.array([300, 300], np.int32), loc_strand=np.zeros(2, np.int8),
        loc_codes=["1:300:+"] * 2,
        hit_group=np.array([0, 0, 1, 2, 0, 1], np.int32))    # contig a: runs 0,0,1,2; b: 0,1
    calls = []

    keys = []

    def score_fn(sub):
        calls.append((sub.n_contigs, sub.hit_off.tolist(), sub.hit_taxon.tolist()))
        keys.append(sub.eval_key.tolist())
        res = Results.empty(sub.n_contigs, sub.n_hits, sub.n_loci, 0)
        res.iterations[:] = [3, 1][:sub.n_contigs] if len(calls) == 1 else [2]
        return res

    out = regroup.resolve(b, parent, {"jump_taxonomy": 1}, score_fn)
    # evaluation 1: both contigs, their run-0 hits; evaluation 2: contig 0's runs 0-1
    assert calls[0] == (2, [0, 2, 3], [9, 9, 9])
    assert calls[1] == (1, [0, 3], [6, 6, 9])           # run 0 raised 1 + 2 = 3 levels
    # contig 0: run 0 raised 3 + (1 + 1) = 5, run 1 raised 2, run 2 none; contig 1: run 0 1
    assert out.hit_taxon.tolist() == [4, 4, 7, 9, 8, 9]
    # where the reference evaluates (and writes --write-details rows): the first row of the
    # run just read -- evaluation 1 at run 0, evaluation 2 at run 1, the last at the last run
    assert keys == [[0, 4], [2]] and out.eval_key.tolist() == [3, 5]
    assert out.hit_group is None and b.hit_group is not None


def _chain_batch(hit_group, jumps_taxon=9):
    z = np.zeros(len(hit_group), np.int32)
    H = len(hit_group)
    return inputs.HostBatch(
        contig_names=["a"], contig_lengths=np.array([900]), hit_off=np.array([0, H]),
        hit_qlo=z + 1, hit_qhi=z + 300, hit_taxon=z + jumps_taxon, hit_strand=z.astype(np.int8),
        hit_score=np.ones(H), hit_scov=np.ones(H), hit_sysmask=z.astype(np.uint32),
        loc_off=np.array([0, 1]), loc_start=np.array([1], np.int32),
        loc_end=np.array([300], np.int32), loc_strand=np.zeros(1, np.int8),
        loc_codes=["1:300:+"], hit_group=np.asarray(hit_group, np.int32))


def test_regroup_negative_jump_makes_no_jumps():
    """--jump-taxonomy -1 on a split blastout: range(-1) is empty upstream (orgscorer.py:
    955-957), so each evaluation raises by iterations - 1 only (wf_api.cpp clamps the same)."""
    from waafle_amd import regroup
    from waafle_amd.engine import Results
    parent = np.array([0, 0, 1, 2, 3, 4, 5, 6, 7, 8], dtype=np.int32)

    def score_fn(sub):
        res = Results.empty(sub.n_contigs, sub.n_hits, sub.n_loci, 0)
        res.iterations[:] = 2
        return res
    for j in (-1, -5, 0):
        out = regroup.resolve(_chain_batch([0, 1, 2]), parent, {"jump_taxonomy": j}, score_fn)
        assert out.hit_taxon.tolist() == [7, 8, 9], j


def test_regroup_all_zero_groups_and_details_do_not_recurse():
    """hit_group present but all zero (one run per contig, e.g. after HostBatch.slice):
    resolve returns the batch without hit_group, so score_details' second call ends."""
    from waafle_amd import regroup
    b = _chain_batch([0, 0, 0])
    out = regroup.resolve(b, np.zeros(10, np.int32), {}, lambda s: 1 / 0)
    assert out.hit_group is None and out.hit_taxon.tolist() == [9, 9, 9]
    assert regroup.resolve(out, np.zeros(10, np.int32), {}, lambda s: 1 / 0) is out


def test_regroup_one_run_per_hit_costs_only_the_split_contig():
    """A blastout sorted by subject can give one contig one run per hit: evaluation k then
    touches only the contigs with more than k runs, not every hit of the batch."""
    import time
    from waafle_amd import regroup
    from waafle_amd.engine import Results
    R, other = 400, 200_000                       # one contig of 400 runs, one of 200 k hits
    H = R + other
    z = np.zeros(H, np.int32)
    g = np.concatenate([np.arange(R), np.zeros(other)]).astype(np.int32)
    b = inputs.HostBatch(
        contig_names=["a", "b"], contig_lengths=np.array([900, 900]), hit_off=np.array([0, R, H]),
        hit_qlo=z + 1, hit_qhi=z + 300, hit_taxon=z + 9, hit_strand=z.astype(np.int8),
        hit_score=np.ones(H), hit_scov=np.ones(H), hit_sysmask=z.astype(np.uint32),
        loc_off=np.array([0, 1, 2]), loc_start=np.array([1, 1], np.int32),
        loc_end=np.array([300, 300], np.int32), loc_strand=np.zeros(2, np.int8),
        loc_codes=["1:300:+"] * 2, hit_group=g)
    parent = np.array([0, 0, 1, 2, 3, 4, 5, 6, 7, 8], dtype=np.int32)
    seen = []

    def score_fn(sub):
        seen.append(sub.n_hits)
        res = Results.empty(sub.n_contigs, sub.n_hits, sub.n_loci, 0)
        res.iterations[:] = 1
        return res
    t0 = time.perf_counter()
    out = regroup.resolve(b, parent, {"jump_taxonomy": 0}, score_fn)
    dt = time.perf_counter() - t0
    assert seen == list(range(1, R))              # evaluation k: contig a's first k hits
    assert out.hit_taxon.tolist() == [9] * H
    assert dt < 5.0, dt                           # O(runs x the split contig), not O(runs x H)
