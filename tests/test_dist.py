"""N>1 plumbing on CPU: two gloo ranks run the product's sharding / gather / timing code
(waafle_amd.dist) with the oracle standing in for the device scorer (test-only)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from waafle_amd import dist as wdist
from waafle_amd import engine, lib as L

WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _oracle_scorer(data, tax):
    from oracle import orgscorer_oracle as orc
    from oracle_bridge import oracle_hits_from_batch, oracle_loci_from_batch, oracle_results
    from waafle_amd import cli
    params = orc.Params(**cli.param_dict(cli.parse_flags([])))
    otax = orc.Taxonomy(data.tax.edges)

    def score(sub):
        lengths = dict(zip(sub.contig_names, sub.contig_lengths.tolist()))
        contigs = orc.score_contigs(lengths, oracle_loci_from_batch(sub),
                                    oracle_hits_from_batch(sub, tax), otax, params)
        return oracle_results(contigs, sub, tax)
    return score


def _worker(rank, port, outdir, fail_rank):
    import torch.distributed as dist
    from waafle_amd import synth
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        data = synth.generate(n=40, genes=5, clades=30, seed=7)
        batch, tax = synth.to_batch(data, with_codes=False)
        inner = _oracle_scorer(data, tax)

        def score(sub, stax, a, b):
            assert sub.n_contigs == b - a and np.array_equal(sub.hit_qlo, batch.slice(a, b).hit_qlo)
            assert list(stax.parent) == list(tax.parent)
            sub = batch.slice(a, b)                   # (the oracle reads names and annotations)
            if rank == fail_rank:
                err = L.WaafleHipError(L.WF_E_RUNAWAY, "runaway")
                err.contigs = np.array([1])
                raise err
            return inner(sub)
        try:
            res = wdist.score_ranked(batch if rank == 0 else None, tax if rank == 0 else None,
                                     None, score, dist)
            outcome = "ok"
        except L.WaafleHipError as exc:
            res, outcome = None, "err:{}:{}".format(exc.code, list(exc.contigs))
        t = wdist.max_over_ranks(1.0 + rank, dist)
        if rank == 0:
            full = inner(batch) if res is not None else None
            np.savez(os.path.join(outdir, "r0.npz"), outcome=outcome, tmax=t,
                     **({} if res is None else {
                         "got_" + f: getattr(res, f) for f in res.__dataclass_fields__}),
                     **({} if full is None else {
                         "want_" + f: getattr(full, f) for f in full.__dataclass_fields__}))
    finally:
        dist.destroy_process_group()


def _run(tmp_path, fail_rank=-1):
    mp.start_processes(_worker, args=(_free_port(), str(tmp_path), fail_rank), nprocs=WORLD,
                       join=True, start_method="spawn")
    return np.load(os.path.join(tmp_path, "r0.npz"))


def test_rank_bounds_cover_and_balance():
    cost = np.array([5, 1, 1, 1, 1, 1, 5, 1], np.float64)
    b = wdist.rank_bounds(cost, 2)
    assert b[0][0] == 0 and b[-1][1] == len(cost) and b[0][1] == b[1][0]
    assert wdist.rank_bounds(cost[:1], 4) == [(0, 1), (1, 1), (1, 1), (1, 1)]
    assert wdist.rank_bounds(np.zeros(0), 3) == [(0, 0)] * 3


def test_two_rank_gloo_shards_match_unsharded(tmp_path):
    r = _run(tmp_path)
    assert str(r["outcome"]) == "ok"
    assert float(r["tmax"]) == 2.0                    # max over ranks, not rank 0's value
    for f in engine.Results.__dataclass_fields__:
        np.testing.assert_array_equal(r["got_" + f], r["want_" + f], err_msg=f)


def test_two_rank_gloo_error_reaches_every_rank(tmp_path):
    r = _run(tmp_path, fail_rank=1)
    # rank 1's shard-local contig 1 is reported as a batch contig index (>= its shard base)
    kind, code, contigs = str(r["outcome"]).split(":")
    assert kind == "err" and int(code) == L.WF_E_RUNAWAY
    assert eval(contigs)[0] > 1


def test_oversized_batch_is_scored_in_halves():
    """GpuScorer.score splits a batch the device rejects as too large (32-bit attachment
    indices) into contig halves and concatenates the records (meld slots, rebased
    annotation winners): the result equals the unsplit one.  The oracle stands in for
    the device (test-only), rejecting batches of more than 7 contigs."""
    from waafle_amd import synth
    data = synth.generate(n=30, genes=5, clades=30, seed=11)
    batch, tax = synth.to_batch(data, with_codes=False)
    inner = _oracle_scorer(data, tax)
    calls = []

    def fake_once(self, sub, params):
        calls.append(sub.n_contigs)
        if sub.n_contigs > 7:
            raise L.WaafleHipError(L.WF_E_TOOBIG, "too many hit-locus attachments (split it)")
        return inner(sub)

    s = engine.GpuScorer.__new__(engine.GpuScorer)
    s._score_once = fake_once.__get__(s)
    got = s.score(batch, None)
    want = inner(batch)
    assert max(calls) == 30 and min(calls) <= 7
    for f in engine.Results.__dataclass_fields__:
        a, b = getattr(got, f), getattr(want, f)
        assert np.array_equal(a, b, equal_nan=a.dtype.kind == "f"), f


def test_split_half_failure_names_batch_contig():
    """A contig failing inside the second half of a split batch is reported by its index
    in the whole batch (the half-relative index named the wrong contig)."""
    from waafle_amd import synth
    data = synth.generate(n=20, genes=5, clades=30, seed=12)
    batch, tax = synth.to_batch(data, with_codes=False)
    inner = _oracle_scorer(data, tax)
    bad_name = batch.contig_names[13]

    def fake_once(self, sub, params):
        if sub.n_contigs > 6:
            raise L.WaafleHipError(L.WF_E_TOOBIG, "too many hit-locus attachments (split it)")
        if bad_name in sub.contig_names:
            err = L.WaafleHipError(L.WF_E_RUNAWAY, "runaway")
            err.contigs = np.array([list(sub.contig_names).index(bad_name)])
            raise err
        return inner(sub)

    s = engine.GpuScorer.__new__(engine.GpuScorer)
    s._score_once = fake_once.__get__(s)
    with pytest.raises(L.WaafleHipError) as ei:
        s.score(batch, None)
    assert ei.value.code == L.WF_E_RUNAWAY
    assert list(ei.value.contigs) == [13]


def test_other_errors_do_not_split():
    from waafle_amd import synth
    data = synth.generate(n=10, genes=5, clades=30, seed=13)
    batch, _ = synth.to_batch(data, with_codes=False)
    calls = []

    def fake_once(self, sub, params):
        calls.append(sub.n_contigs)
        raise L.WaafleHipError(L.WF_E_BADINPUT, "too many hit-locus attachments")

    s = engine.GpuScorer.__new__(engine.GpuScorer)
    s._score_once = fake_once.__get__(s)
    with pytest.raises(L.WaafleHipError):
        s.score(batch, None)
    assert calls == [10]                       # the code decides, not the message text


def test_cli_two_ranks_rank0_parse_failure_ends_every_rank(tmp_path):
    """A parse failure on rank 0 (the only rank that reads the inputs) reaches every rank
    before the scatter (dist.share_error): both ranks exit "EXITING.", rank 0 with the
    reference's LETHAL ERROR line, and no rank waits in a recv.  CPU only (gloo)."""
    import subprocess
    import sys
    import golden_cases as gc
    paths = gc.materialize(gc.load("tie_default"), tmp_path)
    bad = tmp_path / "bad.blastout"
    bad.write_text("contig_1\tnot-enough-columns\n")
    out = tmp_path / "out"
    out.mkdir()
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", CUDA_VISIBLE_DEVICES="",
               HIP_VISIBLE_DEVICES="")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           "-m", "waafle_amd.orgscorer", paths[0], str(bad), paths[2], paths[3],
           "--outdir", str(out)]
    run = subprocess.run(cmd, capture_output=True, text=True, timeout=300,
                         cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))), env=env)
    assert run.returncode != 0
    assert run.stderr.count("LETHAL ERROR") == 1, run.stderr[-2000:]
    assert run.stderr.count("EXITING.") >= 2, run.stderr[-2000:]
    assert "Connection closed" not in run.stderr and "Gloo" not in run.stderr.split("LETHAL")[0]
