"""The N > 1 path with the real HIP scorer: two fresh rank processes (gloo for the control
traffic, both ranks on device 0 through a device override), each scoring its
`dist.rank_bounds` shard with `engine.GpuScorer`; rank 0 gathers the records
(`dist.score_ranked`, what the CLI runs under torch.distributed.run) and they must equal a
one-call result field by field.  Also the bench's N > 1 branch (per-rank passes, the k2 leg's
all_reduce, max over ranks) run once as two ranks on device 0.

The GPU is initialised only inside the children (start method "spawn": fresh interpreters).
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORLD = 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, port, outdir):
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    from waafle_amd import cli, dist as wdist, engine, synth
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        data = synth.generate(n=3000, genes=8, clades=200, seed=61, lgt_frac=0.2)
        batch, tax = synth.to_batch(data)
        params = cli.param_dict(cli.parse_flags([]))
        scorer = engine.GpuScorer(0)          # the device override: every rank on device 0
        try:
            scorer.set_taxonomy(tax)
            got = wdist.score_ranked(batch if rank == 0 else None, tax if rank == 0 else None, params,
                                     lambda sub, stax, a, b: scorer.score(sub, params), dist)
            if rank == 0:
                want = scorer.score(batch, params)
                np.savez(os.path.join(outdir, "ranked.npz"),
                         **{"got_" + f: getattr(got, f) for f in engine.Results.__dataclass_fields__},
                         **{"want_" + f: getattr(want, f) for f in engine.Results.__dataclass_fields__})
        finally:
            scorer.close()
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_two_ranks_one_device_match_one_call(tmp_path):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, port, str(tmp_path))) for r in range(WORLD)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    for p in procs:
        if p.is_alive():
            p.kill()
    assert [p.exitcode for p in procs] == [0] * WORLD
    z = np.load(str(tmp_path / "ranked.npz"))
    from waafle_amd import engine
    for f in engine.Results.__dataclass_fields__:
        a, b = z["got_" + f], z["want_" + f]
        if a.dtype == np.float64:
            a, b = a.view(np.int64), b.view(np.int64)
        assert np.array_equal(a, b), f
    assert (z["want_call"] == 2).sum() > 0 and (z["want_call"] == 1).sum() > 0


def test_bench_two_ranks_on_one_device(tmp_path):
    """bench.py's N > 1 branch under torch.distributed.run with gloo and --device-map 0,0:
    one JSON line from rank 0, labelled as a rehearsal (not a scaling number); the headline
    splits the configuration's contigs over the ranks (strong scaling), `weak` gives every
    rank its own, and the k2 leg's HBM fraction is per GPU."""
    out = tmp_path / "bench2.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--contigs", "20000", "--k2-contigs", "200", "--k2-steps", "1", "--cpu-sample", "0",
           "--e2e=", "--pcie", "0", "--backend", "gloo", "--device-map", "0,0"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    run = subprocess.run(cmd, capture_output=True, text=True, timeout=420, cwd=REPO, env=env)
    assert run.returncode == 0, run.stderr[-3000:]
    lines = [l for l in run.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    out.write_text(lines[0])
    # strong scaling: the 20,000 contigs split 10,000 / 10,000; weak: each rank its own 20,000
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert d["config"]["contigs_total"] == 20000 and d["config"]["contigs_per_gpu"] == 10000
    assert d["ranks"]["backend"] == "gloo" and d["ranks"]["devices"] == [0, 0]
    assert "not a scaling number" in d["ranks"]["note"]
    assert d["calls"]["lgt"] + d["calls"]["no_lgt"] + d["calls"]["unclassified"] == 20000
    assert abs(d["value"] - 20000 / (d["ms_per_step"] * 1e-3)) <= 1e-6 * d["value"]
    w = d["weak"]
    assert w["scaling"] == "weak" and w["contigs_total"] == 40000 and w["contigs_per_gpu"] == 20000
    # the k2 leg: per-GPU fraction = all ranks' bytes / slowest explain_two time / (2 x peak)
    k = d["k2"]
    assert k["contigs"] == 400
    want = k["b_k2_bytes"] / (k["explain_two_ms_per_pass"] * 1e-3) / 1e9 / 2 / k["hbm"]["peak_GBs"]
    assert abs(k["hbm"]["frac"] - want) <= 1e-9 * max(want, 1e-30)
    if os.environ.get("WAAFLE_KEEP_BENCH2"):
        with open(os.environ["WAAFLE_KEEP_BENCH2"], "w") as fh:
            fh.write(lines[0] + "\n")


def test_cli_two_ranks_one_device_match_one_rank(tmp_path):
    """The drop-in CLI under torch.distributed.run as 2 ranks on device 0 (WAAFLE_DEVICE_MAP):
    the inputs are parsed once, on rank 0, which sends rank 1 its cost-balanced contig range
    as typed arrays; each rank scores exactly its shard's hits; the TSVs are byte-identical
    to a one-rank run."""
    import re
    from waafle_amd import cli, dist as wdist, engine, inputs, synth
    data = synth.generate(n=600, genes=8, clades=200, seed=63, lgt_frac=0.2)
    paths = synth.write_text(data, str(tmp_path / "in"))
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", WAAFLE_DEVICE_MAP="0,0")
    one, two = tmp_path / "one", tmp_path / "two"
    one.mkdir()
    two.mkdir()
    r1 = subprocess.run([sys.executable, "-m", "waafle_amd.orgscorer"] + paths + ["--outdir", str(one)],
                        capture_output=True, text=True, timeout=300, cwd=REPO, env=env)
    assert r1.returncode == 0, r1.stderr[-2000:]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "-m",
           "waafle_amd.orgscorer"] + paths + ["--outdir", str(two)]
    r2 = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=REPO, env=env)
    assert r2.returncode == 0, r2.stderr[-3000:]
    for kind in ("lgt", "no_lgt", "unclassified"):
        a = (one / "synth.{}.tsv".format(kind)).read_bytes()
        b = (two / "synth.{}.tsv".format(kind)).read_bytes()
        assert a == b, kind
    # each rank scored exactly its shard's hits (rank 0 parsed; rank 1 received its range)
    batch, _ = inputs.load_inputs(*paths, 200.0, warn=None)
    params = cli.param_dict(cli.parse_flags([]))
    bounds = wdist.rank_bounds(engine.contig_cost(batch, params["two_clade_threshold"]), 2)
    seen = {int(m.group(1)): (int(m.group(2)), int(m.group(3)), int(m.group(4).replace(",", "")))
            for m in re.finditer(r"rank (\d+): contigs (\d+)\.\.(\d+) \(([\d,]+) hits\)", r2.stderr)}
    assert sorted(seen) == [0, 1]
    for r, (a, b) in enumerate(bounds):
        assert seen[r] == (a, b, int(batch.hit_off[b] - batch.hit_off[a]))
    assert 0 < bounds[0][1] < batch.n_contigs


def test_ungrouped_blastout_cli_one_and_two_ranks(tmp_path):
    """A blastout not grouped by query (tests/golden/make_ungrouped.py): the CLI on one rank
    and as 2 ranks on device 0 (rank 0 scores the earlier runs, regroup.py, before the
    split) writes the reference's TSVs; engine.score in two shards on one device agrees."""
    import golden_cases as gc
    from waafle_amd import cli, engine, inputs
    for case in ("ungrouped_default", "ungrouped_jump-taxonomy_1"):
        fx = gc.load(case)
        paths = gc.materialize(fx, tmp_path)
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", WAAFLE_DEVICE_MAP="0,0")
        one, two = tmp_path / (case + "_one"), tmp_path / (case + "_two")
        one.mkdir()
        two.mkdir()
        r1 = subprocess.run([sys.executable, "-m", "waafle_amd.orgscorer"] + paths +
                            ["--outdir", str(one), "--basename", "u", "--quiet"] + fx["flags"],
                            capture_output=True, text=True, timeout=300, cwd=REPO, env=env)
        assert r1.returncode == 0, r1.stderr[-2000:]
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "-m",
               "waafle_amd.orgscorer"] + paths + ["--outdir", str(two), "--basename", "u",
                                                  "--quiet"] + fx["flags"]
        r2 = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=REPO, env=env)
        assert r2.returncode == 0, r2.stderr[-3000:]
        texts = {}
        for kind in ("lgt", "no_lgt", "unclassified"):
            texts[kind] = (one / "u.{}.tsv".format(kind)).read_text()
            assert (two / "u.{}.tsv".format(kind)).read_text() == texts[kind], kind
        assert gc.compare_tsv(fx, texts) == []
        args = cli.parse_flags(fx["flags"])
        batch, tax = inputs.load_inputs(*paths, args.min_gene_length, warn=None)
        assert batch.hit_group is not None
        params = cli.param_dict(args)
        a = engine.score(batch, tax, params, gpus=1)
        b = engine.score(batch, tax, params, gpus=2, devices=[0, 0])
        for f in ("call", "crit", "rank", "clade1", "clade2", "iterations", "annot_hit"):
            assert np.array_equal(getattr(a, f), getattr(b, f)), f


def test_bench_one_gpu_share_projection(tmp_path):
    """bench.py at N = 1 times every strong-scaling share of the workload alone on the GPU
    (`strong_share_projection`): N shares per N covering the contigs, projected value = the
    contigs / the slowest share's pass, efficiency = t(whole) / (N x slowest share)."""
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--steps", "2", "--warmup", "1",
           "--contigs", "20000", "--k2-contigs", "0", "--cpu-sample", "0", "--e2e=", "--pcie", "0",
           "--shares", "2,4"]
    run = subprocess.run(cmd, capture_output=True, text=True, timeout=420, cwd=REPO)
    assert run.returncode == 0, run.stderr[-3000:]
    d = json.loads([l for l in run.stdout.splitlines() if l.startswith("{")][0])
    p = d["strong_share_projection"]
    assert abs(p["t_whole_ms"] - d["ms_per_step"]) <= 1e-6 * d["ms_per_step"]
    for n in (2, 4):
        q = p["per_n"][str(n)]
        assert len(q["shares_ms"]) == n and q["contigs_per_gpu"] in (20000 // n, 20000 // n + 1)
        t = max(q["shares_ms"])
        assert q["ms_slowest_share"] == pytest.approx(t, rel=1e-3)
        assert q["projected_value"] == pytest.approx(20000 / (t * 1e-3), rel=1e-3)
        assert q["projected_efficiency"] == pytest.approx(d["ms_per_step"] / (n * t), rel=1e-3)
