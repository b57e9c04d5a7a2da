"""GPU checks at BASELINE.json's full sizes (cfg4: 1,000,000 contigs; cfg5: the 6,250-contig
per-GPU share of the 50,000-contig stress set) and of the size-dependent host paths (batch
splitting, the decision arena).  Size-independent properties: determinism, shard
invariance, option invariance, and the reference's own fixtures embedded in a full batch;
plus an oracle sample where the oracle finishes in seconds."""
import numpy as np
import pytest

import golden_cases as gc
from oracle import orgscorer_oracle as orc
from oracle_bridge import oracle_hits_from_batch, oracle_loci_from_batch, oracle_results
from waafle_amd import cli, engine, inputs, lib, output, synth
from waafle_amd.inputs import HostBatch

pytestmark = pytest.mark.gpu

PARAMS = cli.param_dict(cli.parse_flags([]))
SCALARS = ("call", "crit", "rank", "clade1", "direction", "iterations", "n_meld1", "n_meld2",
           "pair_evals", "ppot_sum", "status")


def meld_keys(res, batch):
    """Sorted (contig, part, clade) triples of every melded clade (order-free per contig)."""
    N = batch.n_contigs
    base = 2 * batch.hit_off[:-1] + 2 * np.arange(N, dtype=np.int64)
    keys = []
    for part, (start, n) in enumerate(((base, res.n_meld1),
                                       (base + res.n_meld1, res.n_meld2))):
        n = n.astype(np.int64)
        c = np.repeat(np.arange(N, dtype=np.int64), n)
        pos = np.repeat(start.astype(np.int64), n) + (np.arange(n.sum()) - np.repeat(np.cumsum(n) - n, n))
        keys.append((c * 2 + part) * (1 << 31) + res.meld[pos].astype(np.int64))
    return np.sort(np.concatenate(keys))


def assert_same(got, want, batch):
    """Field-by-field equality (crit/rank as bits; clade2 on LGT rows; synteny on classified
    contigs; melds as sets), vectorised for million-contig batches."""
    bad = []
    for f in SCALARS:
        a, b = getattr(got, f), getattr(want, f)
        if f in ("crit", "rank"):
            a, b = a.view(np.int64), b.view(np.int64)
        if f == "iterations":
            a, b = a[want.call != 0], b[want.call != 0]
        d = np.nonzero(a != b)[0]
        if len(d):
            bad.append((f, d[:5].tolist()))
    lgt = want.call == 2
    if not np.array_equal(got.clade2[lgt], want.clade2[lgt]):
        bad.append("clade2")
    keep = np.repeat(want.call != 0, np.diff(batch.loc_off))
    if not np.array_equal(got.synteny[keep], want.synteny[keep]):
        bad.append("synteny")
    if not np.array_equal(got.annot_hit, want.annot_hit):
        bad.append("annot_hit")
    if not np.array_equal(meld_keys(got, batch), meld_keys(want, batch)):
        bad.append("meld")
    assert bad == []


def concat_batches(parts):
    """Contigs of several batches (same taxonomy) as one batch."""
    def cat(f):
        return np.concatenate([getattr(p, f) for p in parts])
    hoff, loff = [np.zeros(1, np.int64)], [np.zeros(1, np.int64)]
    for p in parts:
        hoff.append(p.hit_off[1:] + hoff[-1][-1])
        loff.append(p.loc_off[1:] + loff[-1][-1])
    return HostBatch(
        contig_names=sum((list(p.contig_names) or ["c{}_{}".format(i, j) for j in range(p.n_contigs)]
                          for i, p in enumerate(parts)), []),
        contig_lengths=cat("contig_lengths"), hit_off=np.concatenate(hoff),
        hit_qlo=cat("hit_qlo"), hit_qhi=cat("hit_qhi"), hit_taxon=cat("hit_taxon"),
        hit_strand=cat("hit_strand"), hit_score=cat("hit_score"), hit_scov=cat("hit_scov"),
        hit_sysmask=cat("hit_sysmask"), loc_off=np.concatenate(loff),
        loc_start=cat("loc_start"), loc_end=cat("loc_end"), loc_strand=cat("loc_strand"),
        systems=parts[0].systems)


def slice_results(res, batch, a, b):
    h0, h1 = int(batch.hit_off[a]), int(batch.hit_off[b])
    l0, l1 = int(batch.loc_off[a]), int(batch.loc_off[b])
    nsys = len(batch.systems)
    out = {}
    for f in engine.Results.__dataclass_fields__:
        v = getattr(res, f)
        if f == "synteny":
            out[f] = v[l0:l1]
        elif f == "annot_hit":
            w = v[l0 * nsys:l1 * nsys]
            out[f] = np.where(w >= 0, w - h0, -1).astype(np.int32)
        elif f == "meld":
            out[f] = v[2 * h0 + 2 * a:2 * h1 + 2 * b]
        else:
            out[f] = v[a:b]
    return engine.Results(**out)


def score(batch, tax, **kw):
    s = engine.GpuScorer(0, **kw)
    try:
        s.set_taxonomy(tax)
        return s.score(batch, PARAMS)
    finally:
        s.close()


def oracle_chunk_sample(name, k, n, tax):
    """The oracle's records for the first n contigs of chunk k of a chunked config (the
    chunk regenerated with its names and annotations; same taxonomy ids as the batch)."""
    data = synth.generate_chunk(name, k)
    b, t = synth.to_batch(data, with_codes=False)
    assert list(t.names) == list(tax.names)
    sub = b.slice(0, n)
    contigs = orc.score_contigs(dict(zip(sub.contig_names, sub.contig_lengths.tolist())),
                                oracle_loci_from_batch(sub), oracle_hits_from_batch(sub, t),
                                orc.Taxonomy(data.tax.edges), orc.Params(**PARAMS))
    return sub, oracle_results(contigs, sub, t)


def test_attachment_limit_splits_batch_like_unsplit():
    """WF_OPT_ATT_LIMIT makes wf_score return WF_E_TOOBIG for a batch whose staged
    attachments exceed the limit (the staged form: every contig's attachments go to HBM;
    the wave forms keep theirs in LDS); GpuScorer.score then scores contig halves
    (recursively): the records equal the unsplit call's field by field (annotation winners
    rebased, meld slots in place)."""
    data = synth.generate(n=3000, genes=8, clades=200, seed=81)
    batch, tax = synth.to_batch(data)
    want = score(batch, tax)
    s = engine.GpuScorer(0, mode="staged", options={lib.OPT_ATT_LIMIT: 20000})
    s.set_taxonomy(tax)
    with pytest.raises(lib.WaafleHipError) as ei:
        s._score_once(batch, PARAMS)
    assert ei.value.code == lib.WF_E_TOOBIG
    got = s.score(batch, PARAMS)
    s.close()
    assert_same(got, want, batch)


def test_attachment_limit_default_mode_oversized_contigs():
    """The default form (WF_MODE_LEVEL0) with contigs past the wave slice's capacity
    (8 genes x 71 hits = 568 attachments > 512): the wave form hands them to the staged
    kernels, whose attachments then exceed a low WF_OPT_ATT_LIMIT -> WF_E_TOOBIG; the split
    records equal the unsplit call's (the path the full 50,000-contig cfg5 batch takes)."""
    small = synth.generate(n=600, genes=8, clades=200, seed=83)
    big = synth.generate(n=120, genes=8, clades=200, seed=83, decoys=70)
    (b1, tax), (b2, tax2) = synth.to_batch(small), synth.to_batch(big)
    assert list(tax.names) == list(tax2.names)
    batch = concat_batches([b1, b2, b1.slice(0, 200)])
    assert batch.max_hits > 512
    want = score(batch, tax)
    assert not want.status.any()
    s = engine.GpuScorer(0, options={lib.OPT_ATT_LIMIT: 20000})
    s.set_taxonomy(tax)
    with pytest.raises(lib.WaafleHipError) as ei:
        s._score_once(batch, PARAMS)
    assert ei.value.code == lib.WF_E_TOOBIG
    got = s.score(batch, PARAMS)
    s.close()
    assert_same(got, want, batch)
    staged = score(batch, tax, mode="staged")
    assert_same(staged, want, batch)


def test_option_validation():
    s = engine.GpuScorer(0)
    for opt, val in ((lib.OPT_ATT_LIMIT, 0), (lib.OPT_ATT_LIMIT, 1 << 31), (lib.OPT_SPARSE_BIG, 4),
                     (lib.OPT_SPARSE_BIG, 0), (lib.OPT_SPARSE_BIG, 1), (lib.OPT_TRIAGE, 2),
                     (lib.OPT_WAVE_TWO, 0), (99, 1)):   # (SPARSE_BIG 0, 1 and WAVE_TWO 0: retired)
        assert s.lib.wf_set_option(s.h, opt, val) == lib.WF_E_BADINPUT
    s.close()


@pytest.fixture(scope="module")
def cfg4_full():
    batch, tax = synth.generate_batch("cfg4")
    assert batch.n_contigs == 1_000_000
    return batch, tax


def test_cfg4_full_size(cfg4_full):
    """cfg4 at full size (1 M contigs, 210 M hits, one call): no contig errors, the same
    records on a second pass, from four cost-balanced shards, with a 16 KB decision arena
    (round 2: WF_DEC_LDS=16384 produced WF_E_EMPTYMASK at this shape), with the dense
    workgroup decision's arena, with every staged decision in the segment-table form, and
    without the triage; and the oracle's records on a 200-contig sample."""
    batch, tax = cfg4_full
    s = engine.GpuScorer(0)
    s.set_taxonomy(tax)
    a = s.score(batch, PARAMS)
    assert not a.status.any()
    assert (a.call == 2).sum() > 0 and (a.call == 1).sum() > 0 and (a.iterations > 1).sum() > 0
    assert_same(s.score(batch, PARAMS), a, batch)
    bounds = engine.shard_bounds(np.ones(batch.n_contigs), 4)   # homogeneous generator
    parts = [s.score(batch.slice(x, y), PARAMS) for x, y in bounds]
    s.close()
    assert_same(engine.Results.concat(parts, [int(batch.hit_off[x]) for x, _ in bounds]), a, batch)
    for kw in (dict(lds_bytes=16384), dict(options={lib.OPT_SPARSE_BIG: 2}),
               dict(options={lib.OPT_TRIAGE: 0})):
        c = score(batch, tax, **kw)
        assert not c.status.any(), kw
        assert_same(c, a, batch)
    k = 70                                           # contigs 700,000 .. 700,199
    sub, want = oracle_chunk_sample("cfg4", k, 200, tax)
    c0 = k * synth.chunk_size("cfg4")
    assert_same(slice_results(a, batch, c0, c0 + 200), want, sub)


def test_cfg3_full_size():
    """BASELINE config 3 at full size (100,000 contigs x 12 genes x 1,000 clades, 25 M hits,
    the full taxonomy roll-up): no contig errors, deterministic, equal in the staged form
    (which evaluates every segment mean) and from four cost-balanced shards, and equal to the
    oracle on a 300-contig sample (contigs are independent)."""
    batch, tax = synth.generate_batch("cfg3")
    assert batch.n_contigs == 100_000
    s = engine.GpuScorer(0)
    s.set_taxonomy(tax)
    a = s.score(batch, PARAMS)
    assert not a.status.any()
    assert (a.call == 2).sum() > 0 and (a.call == 1).sum() > 0 and (a.iterations > 2).sum() > 0
    assert_same(s.score(batch, PARAMS), a, batch)
    bounds = engine.shard_bounds(engine.contig_cost(batch), 4)
    parts = [s.score(batch.slice(x, y), PARAMS) for x, y in bounds]
    s.close()
    assert len(parts) == 4
    assert_same(engine.Results.concat(parts, [int(batch.hit_off[x]) for x, _ in bounds]), a, batch)
    staged = score(batch, tax, mode="staged")
    assert not staged.status.any()
    assert_same(staged, a, batch)
    k = 3                                            # 300 contigs of chunk 3
    sub, want = oracle_chunk_sample("cfg3", k, 300, tax)
    c0 = k * synth.chunk_size("cfg3")
    assert_same(slice_results(a, batch, c0, c0 + 300), want, sub)


@pytest.mark.parametrize("genes,decoys", [(20, 240), (70, 70)], ids=["packed", "wide-loci"])
def test_stress_front_end_matches_five_launch_form(genes, decoys):
    """k_front_radix -- the > 4,096-attachment contigs' sort, segments and exact means in one
    LDS-resident launch per level, segment offsets by decoupled look-back -- against the
    five-launch form the --write-details path keeps (k_sort_radix, k_seg_build_wide,
    k_seg_rec, the leaf-count scan, k_leaf_expand), on decoy-heavy contigs whose segments
    take every mean path (one run; 2..4 overlapping attachments: the leaf kernels; 5..64:
    k_seg_wave; more: the leaf kernels), at level 0 and the roll-up levels; and the oracle's
    records on 3 of them.  20 loci: the packed sort words (contig-local clade ranks); 70 loci
    (lb = 7): the key + index buffers."""
    data = synth.generate(n=48, genes=genes, clades=300, decoys=decoys, lgt_frac=0.5, seed=17)
    batch, tax = synth.to_batch(data)
    assert batch.max_hits > 4096
    per_seg = np.unique(data.hit_contig * 1_000_000 + data.hit_clade * 100 + data.hit_gene,
                        return_counts=True)[1]
    assert (per_seg == 1).any() and ((per_seg >= 2) & (per_seg <= 4)).any() and (per_seg >= 5).any()
    s = engine.GpuScorer(0)
    s.set_taxonomy(tax)
    fused = s.score(batch, PARAMS)
    five, _ = s.score_details(batch, PARAMS)
    s.close()
    assert not fused.status.any()
    assert (fused.iterations > 1).any()
    assert_same(fused, five, batch)
    sub = batch.slice(0, 3)
    contigs = orc.score_contigs(dict(zip(sub.contig_names, sub.contig_lengths.tolist())),
                                oracle_loci_from_batch(sub), oracle_hits_from_batch(sub, tax),
                                orc.Taxonomy(data.tax.edges), orc.Params(**PARAMS))
    assert_same(slice_results(fused, batch, 0, 3), oracle_results(contigs, sub, tax), sub)


def test_cfg5_shard_and_embedded_fixture(tmp_path):
    """The cfg5 per-GPU share at 8 GPUs (6,250 stress contigs, ~31 M hits, 5,000 clades):
    equal to its two halves and to the all-segment-table staged form; the reference-generated
    syn_cfg5 fixture contigs (same taxonomy) placed in front of the shard give the
    fixture's TSV rows."""
    batch, tax = synth.generate_batch("cfg5", 0, 6250)
    whole = score(batch, tax)
    assert not whole.status.any()
    assert (whole.pair_evals > 5_000_000).all()     # the stress shape: ~4,400 potential clades
    assert (whole.call != 0).all() and (whole.call == 2).sum() > 2000   # r02: 56% LGT, rest genus
    mid = 3125
    halves = [score(batch.slice(0, mid), tax), score(batch.slice(mid, 6250), tax)]
    assert_same(engine.Results.concat(halves, [0, int(batch.hit_off[mid])]), whole, batch)
    sparse = score(batch.slice(0, 400), tax, mode="staged", options={lib.OPT_SPARSE_BIG: 2})
    assert_same(sparse, slice_results(whole, batch, 0, 400), batch.slice(0, 400))
    # the fixture's contigs in front of the shard
    fx = gc.load("syn_cfg5_default")
    paths = gc.materialize(fx, tmp_path)
    gb, gtax = inputs.load_inputs(*paths, 200.0, warn=None)
    assert list(gtax.names) == list(tax.names)
    both = concat_batches([gb, batch])
    res = score(both, tax)
    own = slice_results(res, both, 0, gb.n_contigs)
    rows = output.render(gb, gtax, own)
    texts = {k: "\n".join(v) + "\n" for k, v in rows.items()}
    assert gc.compare_tsv(fx, texts) == []
    assert_same(slice_results(res, both, gb.n_contigs, both.n_contigs), whole, batch)


FORM_FLAGS = [[], ["--sister-penalty", "lenient"], ["--sister-penalty", "off"],
              ["-k1", "0.6", "-k2", "0.7"], ["-k1", "0.9"], ["--ambiguous-threshold", "strict", "--range", "0.1"],
              ["--ambiguous-threshold", "off"], ["--disambiguate-two", "report-best"],
              ["--weak-loci", "penalize"], ["--annotation-threshold", "strict"], ["--range", "0"],
              ["--clade-genes", "2", "--clade-leaves", "2"]]


@pytest.fixture(scope="module")
def lgt_heavy():
    """3,000 contigs with 30% LGT candidates and 20 decoys per gene over 300 clades: many
    explain_two hand-overs and roll-ups (the pruned passes' inputs)."""
    data = synth.generate(n=3000, genes=10, clades=300, decoys=20, lgt_frac=0.3, seed=57)
    return synth.to_batch(data)


@pytest.mark.parametrize("flags", FORM_FLAGS, ids=[" ".join(f) or "default" for f in FORM_FLAGS])
def test_pruned_forms_agree_with_staged(lgt_heavy, flags):
    """The default LEVEL0 form -- the triage, the first form's bounds (one-attachment upper
    bounds, lower bounds for the unmasked loci and for pass 4), candidate-pair members' rows
    only, the compact hand-over -- against the staged form, which evaluates every segment
    mean and decides from whole tables, over flag sets that move every threshold those
    shortcuts compare with (k1, k2, kmin, the sister and ambiguity thresholds, --range)."""
    batch, tax = lgt_heavy
    params = cli.param_dict(cli.parse_flags(flags))
    got = {}
    for form, kw in (("level0", {}), ("notriage", dict(options={lib.OPT_TRIAGE: 0})), ("staged", dict(mode="staged"))):
        s = engine.GpuScorer(0, **kw)
        try:
            s.set_taxonomy(tax)
            got[form] = s.score(batch, params)
        finally:
            s.close()
    assert (got["staged"].call == 2).sum() > 100           # (the shortcuts' inputs are there)
    assert_same(got["level0"], got["staged"], batch)
    assert_same(got["notriage"], got["staged"], batch)


@pytest.mark.parametrize("flags", [[], ["--min-scov", "0.9"], ["--stranded"]],
                         ids=["default", "min-scov_0p9", "stranded"])
def test_packed_hit_key_equals_library_packed_and_is_checked(flags):
    """wf_batch.hit_key (ABI 6): the caller's packed words (numpy, lib.pack_hit_keys) and the
    library's own packing (hit_key NULL: k_pack_keys before the triage) give the same
    records; a host batch whose key disagrees with its arrays (packed for another
    --min-scov) is refused with WF_E_BADINPUT before any launch."""
    data = synth.generate(n=2000, genes=8, clades=200, seed=91)
    batch, tax = synth.to_batch(data)
    params = cli.param_dict(cli.parse_flags(flags))
    s = engine.GpuScorer(0)
    s.set_taxonomy(tax)
    got = s.score(batch, params)                               # hit_key NULL
    res = engine.Results.empty(batch.n_contigs, batch.n_hits, batch.n_loci, len(batch.systems))
    bs, rs = engine.batch_struct(batch, float(params["min_scov"])), res.struct()
    ps = engine.params_struct(params)
    import ctypes as C
    assert s.lib.wf_score(s.h, C.byref(bs), C.byref(ps), C.byref(rs)) == lib.WF_OK
    assert_same(res, got, batch)
    stale = engine.hit_keys(batch, float(params["min_scov"]) + 0.07).copy()
    bs = engine.batch_struct(batch)
    bs.hit_key = lib.ptr(stale)
    if (stale != engine.hit_keys(batch, float(params["min_scov"]))).any():
        assert s.lib.wf_score(s.h, C.byref(bs), C.byref(ps), C.byref(rs)) == lib.WF_E_BADINPUT
        assert b"hit_key" in s.lib.wf_last_error(s.h)
    s.close()
