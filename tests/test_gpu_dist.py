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
            got = wdist.score_ranked(batch, tax, params, lambda sub: scorer.score(sub, params), dist)
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
