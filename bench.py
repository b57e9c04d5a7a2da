"""Benchmark: contigs scored/sec (+ k2 clade-pair evals/sec) on MI355X.

Workload (BASELINE.json configs[3], the north-star configuration): synthetic 1,000,000
contigs x 10 genes x 2000 clades, 20 decoy hits per gene (210 M hits), default
waafle_orgscorer parameters, roll-up enabled, on one MI355X (it fits: ~7 GB of hits).
One step = one wf_score pass over the whole batch with inputs already resident in HBM.
For N GPUs (torch.distributed.run, one process per GPU) the SAME 1M-contig batch is split
into N contiguous contig ranges (strong scaling; dist.rank_bounds over the per-contig cost,
uniform for this homogeneous generator); contigs are independent, so there is no
data-path collective -- only the barrier and the max-over-ranks timing.

Each rank generates only its own contig range: the generator draws every 10k-contig
chunk from its own seed (synth.generate_batch), in parallel worker processes, before the
GPU is touched.  cfg2 / cfg3 / cfg5 stay available with --config.

Extra keys on the line (rank 0, N=1): `cpu_baseline` (the oracle port on 1 core and on
disjoint shards in parallel processes, a bounded sample of the same workload),
`pcie_inclusive` (scope ii: host arrays -> wf_score host mode -> host results),
`cli_end_to_end` (scope iii: text files -> `python -m waafle_amd.orgscorer` -> TSVs, cfg2),
`k2` (the isolated explain_two kernel at cfg5, from profiles/ when present).

    python bench.py [--gpus N --steps K --warmup W] [--config cfg2|cfg3|cfg4|cfg5]
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
PROFILES = os.path.join(REPO, "profiles")


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="cfg4")
    ap.add_argument("--contigs", type=int, default=None, help="override total contigs")
    ap.add_argument("--lds-bytes", type=int, default=None)
    ap.add_argument("--mode", default=None, choices=["level0", "waves", "staged"],
                    help="execution form (wf_set_mode; default: the library's, level0)")
    ap.add_argument("--cpu-sample", type=int, default=5000,
                    help="contigs timed on the CPU oracle, 1 core (rank 0, N=1); 0 disables")
    ap.add_argument("--cpu-shard", type=int, default=600,
                    help="contigs per process of the parallel CPU leg; 0 disables")
    ap.add_argument("--e2e", default="cfg2", help="CLI end-to-end config ('' disables)")
    ap.add_argument("--pcie", type=int, default=1, help="time the host-array scope")
    ap.add_argument("--traffic-json", default=None)
    ap.add_argument("--k2-json", default=os.path.join(PROFILES, "r02_k2_cfg5.json"))
    return ap.parse_args()


def algorithmic_bytes(batch):
    """24 B/hit + 12 B/locus + 16 B/contig offsets + 80 B/contig result."""
    N = batch.n_contigs
    return 24 * batch.n_hits + 12 * batch.n_loci + 16 * (N + 1) + 80 * N


def k2_algorithmic(pair_evals, batch):
    """SURVEY §8(d) counts for the isolated explain_two kernel, from the per-contig
    reference-equivalent pair counts P_pot(P_pot-1)/2: B_k2 = sum P_pot*G*8 (the S rows
    of the potential clades) and OPS_pair = sum pairs*G (this rank only)."""
    sel = pair_evals > 0
    p = pair_evals[sel].astype(np.float64)
    ppot = np.rint((1.0 + np.sqrt(1.0 + 8.0 * p)) / 2.0)
    g = np.diff(batch.loc_off)[sel].astype(np.float64)
    return {"contigs_explain_two": int(sel.sum()), "p_pot_max": int(ppot.max()) if p.size else 0,
            "b_k2_bytes": float((ppot * g * 8.0).sum()), "ops_pair": float((p * g).sum()),
            "pairs": float(p.sum())}


def host_cpus():
    """(threads usable by this job, CPU model string)."""
    n = len(os.sched_getaffinity(0))
    cap = os.environ.get("OMP_NUM_THREADS")
    if cap and cap.isdigit():
        n = min(n, int(cap))
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return max(1, n), model


# ---- CPU baseline (the oracle port; never the measured product path) -------------------
_CPU = {}


def _oracle_contigs(a, b):
    """Score contigs [a, b) of the sample batch with the oracle; returns seconds."""
    from oracle import orgscorer_oracle as orc
    from oracle_bridge import oracle_hits_from_batch, oracle_loci_from_batch
    sub = _CPU["batch"].slice(a, b)
    hits = oracle_hits_from_batch(sub, _CPU["tax"])
    loci = oracle_loci_from_batch(sub)
    lengths = dict(zip(sub.contig_names, sub.contig_lengths.tolist()))
    t0 = time.perf_counter()
    orc.score_contigs(lengths, loci, hits, _CPU["otax"], _CPU["params"])
    return time.perf_counter() - t0


def cpu_baseline(config, n_one, n_shard):
    """The oracle (Python/numpy restatement of waafle_orgscorer) on chunk 0 of the same
    workload, inputs pre-parsed (same scope as the GPU value): one core, then P processes
    on disjoint contig shards (fork), rate = contigs / slowest shard."""
    from oracle import orgscorer_oracle as orc
    from waafle_amd import cli, synth
    sys.path.insert(0, os.path.join(REPO, "tests"))
    data = synth.generate_chunk(config, 0)
    batch, tax = synth.to_batch(data, with_codes=False)
    _CPU.update(batch=batch, tax=tax, otax=orc.Taxonomy(data.tax.edges),
                params=orc.Params(**cli.param_dict(cli.parse_flags([]))))
    cores, model = host_cpus()
    n_one = min(n_one, batch.n_contigs)
    dt = _oracle_contigs(0, n_one)
    out = {"value": n_one / dt, "unit": "contigs/s", "cores": 1, "kind": "port",
           "cpu_model": model,
           "sample": "contigs 0..{} of the {} workload (chunk 0), oracle (Python/numpy "
                     "restatement of waafle_orgscorer) on 1 host core, inputs pre-parsed; "
                     "{:.1f} s".format(n_one, config, dt)}
    P = min(cores, batch.n_contigs // max(n_shard, 1)) if n_shard else 0
    if P >= 2:
        import multiprocessing as mp
        shards = [(i * n_shard, (i + 1) * n_shard) for i in range(P)]
        t0 = time.perf_counter()
        pool = mp.get_context("fork").Pool(P)      # close + join (see synth.generate_batch)
        try:
            secs = pool.starmap(_oracle_contigs, shards)
        finally:
            pool.close()
            pool.join()
        wall = time.perf_counter() - t0
        out["parallel"] = {"value": P * n_shard / max(secs), "unit": "contigs/s", "cores": P,
                           "kind": "port", "slowest_shard_s": max(secs), "wall_s": wall,
                           "sample": "{} processes x {} disjoint contigs of chunk 0, "
                                     "rate = contigs / slowest shard".format(P, n_shard)}
    return out


# ---- scope (iii): CLI text -> TSV ---------------------------------------------------------
def cli_end_to_end(config):
    """`python -m waafle_amd.orgscorer` on the text rendering of a config (native ingest,
    one GPU, TSV writer): wall clock of the whole process, and the CLI's own phase split."""
    from waafle_amd import synth
    data = synth.generate_config(config)
    with tempfile.TemporaryDirectory() as tmp:
        paths = synth.write_text(data, tmp, "e2e")
        cmd = [sys.executable, "-m", "waafle_amd.orgscorer"] + paths + ["--outdir", tmp]
        t0 = time.perf_counter()
        run = subprocess.run(cmd, capture_output=True, text=True, cwd=REPO, timeout=600)
        wall = time.perf_counter() - t0
    if run.returncode != 0:
        return {"error": run.stderr.strip().splitlines()[-3:]}
    phases = [l for l in run.stderr.splitlines() if l.startswith("Finished successfully")]
    return {"config": config, "contigs": data.n_contigs, "hits": data.n_hits,
            "value": data.n_contigs / wall, "unit": "contigs/s", "wall_s": wall,
            "phases": phases[-1] if phases else None,
            "scope": "text files -> native ingest -> wf_score (1 GPU) -> 3 TSVs, one process "
                     "incl. interpreter start and GPU init"}


def main():
    args = parse_args()
    from waafle_amd import dist as wdist
    from waafle_amd import synth
    rank, world, local = wdist.rank_env()
    cores, _ = host_cpus()

    # ---- generate this rank's contig range BEFORE touching the GPU (fork-safe) ----
    n_total = args.contigs or synth.CONFIGS[args.config]["n"]
    a, b = wdist.rank_bounds(np.ones(n_total), world)[rank]    # uniform expected cost
    t_gen = time.perf_counter()
    batch, tax = synth.generate_batch(args.config, a, b, workers=max(1, min(16, cores // world)),
                                      n_total=n_total)
    t_gen = time.perf_counter() - t_gen
    # CPU legs before the GPU is initialised: the parallel leg forks worker processes, and
    # the end-to-end leg is its own process that initialises the GPU itself
    cpu_line = e2e_line = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        cpu_line = cpu_baseline(args.config, args.cpu_sample, args.cpu_shard)
    if rank == 0 and world == 1 and args.e2e:
        e2e_line = cli_end_to_end(args.e2e)

    import torch
    from waafle_amd import cli, engine, lib as L
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    N, NH, NL = batch.n_contigs, batch.n_hits, batch.n_loci
    pdict = cli.param_dict(cli.parse_flags([]))
    params = engine.params_struct(pdict)
    so = L.load()
    h = C.c_void_p()
    assert so.wf_init(local, C.byref(h)) == 0, "wf_init failed"

    def chk(rc):
        if rc:
            raise RuntimeError(so.wf_last_error(h).decode())
    if args.lds_bytes:
        chk(so.wf_set_lds_bytes(h, args.lds_bytes))
    if args.mode:
        chk(so.wf_set_mode(h, engine.MODES[args.mode]))
    tstruct = engine.taxonomy_struct(tax)
    chk(so.wf_set_taxonomy(h, C.byref(tstruct)))
    stream = torch.cuda.current_stream(dev)
    chk(so.wf_set_stream(h, C.c_void_p(stream.cuda_stream)))

    d = {}
    for f in ("hit_off", "hit_qlo", "hit_qhi", "hit_taxon", "hit_strand", "hit_score",
              "hit_scov", "hit_sysmask", "loc_off", "loc_start", "loc_end", "loc_strand"):
        arr = getattr(batch, f)
        if arr.dtype == np.uint32:
            arr = arr.view(np.int32)
        d[f] = torch.from_numpy(np.ascontiguousarray(arr)).to(dev)
    out = {
        "call": torch.empty(N, dtype=torch.int8, device=dev),
        "crit": torch.empty(N, dtype=torch.float64, device=dev),
        "rank": torch.empty(N, dtype=torch.float64, device=dev),
        "clade1": torch.empty(N, dtype=torch.int32, device=dev),
        "clade2": torch.empty(N, dtype=torch.int32, device=dev),
        "direction": torch.empty(N, dtype=torch.int8, device=dev),
        "iterations": torch.empty(N, dtype=torch.int16, device=dev),
        "synteny": torch.empty(max(NL, 1), dtype=torch.uint8, device=dev),
        "n_meld1": torch.empty(N, dtype=torch.int32, device=dev),
        "n_meld2": torch.empty(N, dtype=torch.int32, device=dev),
        "meld": torch.empty(2 * NH + 2 * N, dtype=torch.int32, device=dev),
        "annot_hit": torch.empty(max(NL, 1), dtype=torch.int32, device=dev),
        "pair_evals": torch.empty(N, dtype=torch.int64, device=dev),
        "status": torch.empty(N, dtype=torch.int32, device=dev),
        "need_bytes": torch.empty(N, dtype=torch.int64, device=dev),
    }
    bs = L.WfBatch(n_contigs=N, n_systems=1, n_hits=NH, n_loci=NL, max_hits=batch.max_hits,
                   max_loci=batch.max_loci, device_resident=1, _pad=0,
                   **{f: C.c_void_p(d[f].data_ptr()) for f in d})
    rs = L.WfResult(**{f: C.c_void_p(out[f].data_ptr()) for f, _ in L.WfResult._fields_})

    def step():
        chk(so.wf_score(h, C.byref(bs), C.byref(params), C.byref(rs)))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    status = out["status"].cpu().numpy()
    assert not status.any(), "contig status errors: {}".format(np.unique(status))
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    chk(so.wf_timing_enable(h, 1))
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    tm = L.WfTiming()
    chk(so.wf_timing_read(h, C.byref(tm)))
    elapsed = wdist.max_over_ranks(t1 - t0, dist, dev)

    calls = out["call"].cpu().numpy()
    pe = out["pair_evals"].cpu().numpy()
    pairs = float(pe.sum())
    k2_counts = k2_algorithmic(pe, batch)
    iters = out["iterations"].cpu().numpy()
    if dist:          # whole-job counts
        import torch as T
        v = T.tensor([pairs, float((calls == 2).sum()), float((calls == 1).sum()),
                      float((calls == 0).sum()), float((iters > 1).sum())], dtype=T.float64,
                     device=dev)
        dist.all_reduce(v)
        pairs, n_lgt, n_no, n_un, n_up = v.tolist()
    else:
        n_lgt, n_no, n_un, n_up = ((calls == 2).sum(), (calls == 1).sum(), (calls == 0).sum(),
                                   (iters > 1).sum())
    ms_step = elapsed / args.steps * 1e3
    value = n_total / (elapsed / args.steps)
    pass_ms = tm.pass_ms / max(1, tm.passes)
    b_alg = algorithmic_bytes(batch)
    achieved = b_alg / (pass_ms * 1e-3) / 1e9
    traffic, tsrc = None, None
    tpath = args.traffic_json or os.path.join(PROFILES, "r02_traffic_{}.json".format(args.config))
    if os.path.exists(tpath):
        with open(tpath) as fh:
            tj = json.load(fh)
        if tj.get("config") == args.config and tj.get("contigs") == N:
            traffic = tj.get("hbm_bytes_per_launch")
            tsrc = {k: tj.get(k) for k in ("fetch_bytes_raw", "fetch_bytes_x2", "write_bytes",
                                           "hbm_bytes_raw", "hbm_bytes_x2",
                                           "dispatches_per_pass", "source")}
    spec = synth.CONFIGS[args.config]
    result = {
        "metric": "contigs scored/sec + k2 clade-pair evals/sec at 1/2/4/8 MI355X vs CPU ref",
        "value": value, "unit": "contigs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (seeded generator, SURVEY §8(d) shapes)",
        "config": {"workload": "{}: {} contigs x {} genes x {} clades, {} hits, default flags"
                               .format(args.config, n_total, spec["genes"], spec["clades"],
                                       NH * world if world == 1 else "~{}".format(NH * world)),
                   "contigs_total": n_total, "contigs_per_gpu": N, "hits_per_gpu": NH,
                   "parallelism": "dp{} (static contig split, no collective)".format(world)},
        "k2_pair_evals_per_sec": pairs / (elapsed / args.steps),
        "k2_pair_evals_note": "reference-equivalent count: sum of P_pot(P_pot-1)/2 over "
                              "explain_two calls (orgscorer.py:606-608 score(c1,c2) calls), "
                              "not pairs the mask-class search evaluates",
        "k2_counts": k2_counts,
        "calls": {"lgt": int(n_lgt), "no_lgt": int(n_no), "unclassified": int(n_un),
                  "rolled_up": int(n_up)},
        "kernel_ms": {"wf_score_pass": pass_ms},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": "wf_score pass (every kernel of one pass: wave kernels + staged remainder; HIP events on its stream)",
                     "algorithmic_bytes_per_launch": b_alg,
                     "algorithmic_bytes_rule": "24 B/hit + 12 B/locus + 96 B/contig",
                     "traffic_detail": tsrc},
        "generate_s": t_gen,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and os.path.exists(args.k2_json):
        with open(args.k2_json) as fh:
            result["k2"] = json.load(fh)
    if rank == 0 and world == 1 and args.pcie:
        # scope (ii): host (pageable numpy) arrays in, host results out, second call timed
        s = engine.GpuScorer(local)
        s.set_taxonomy(tax)
        s.score(batch, pdict)
        t0 = time.perf_counter()
        s.score(batch, pdict)
        dt = time.perf_counter() - t0
        s.close()
        result["pcie_inclusive"] = {
            "value": N / dt, "unit": "contigs/s", "wall_s": dt,
            "h2d_bytes": int(sum(getattr(batch, f).nbytes for f in (
                "hit_off", "hit_qlo", "hit_qhi", "hit_taxon", "hit_strand", "hit_score",
                "hit_scov", "hit_sysmask", "loc_off", "loc_start", "loc_end", "loc_strand"))),
            "scope": "host arrays -> wf_score host mode (H2D, kernels, D2H of the records)"}
    so.wf_free(h)
    result["cpu_baseline"] = cpu_line
    if e2e_line is not None:
        result["cli_end_to_end"] = e2e_line
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
