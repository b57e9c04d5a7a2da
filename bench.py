"""Benchmark: contigs scored/sec + k2 clade-pair evals/sec on MI355X.

Main line (`value`): BASELINE.json configs[3], the north-star configuration -- synthetic
1,000,000 contigs x 10 genes x 2000 clades, 20 decoy hits per gene (210 M hits), default
waafle_orgscorer parameters, roll-up enabled, one wf_score pass over the whole batch with
inputs resident in HBM.  For N GPUs (torch.distributed.run, one process per GPU) the SAME
1M-contig batch is split into N contiguous contig ranges, rank r scoring contigs
[r n / N, (r + 1) n / N) (strong scaling, `value` = 1M / the slowest rank's pass time);
contigs are independent, so there is no data-path collective -- only the barrier, the
max-over-ranks timing and the sums of the call counts.  At N > 1 the line also carries
`weak`: every rank its own 1M contigs (rank r: [r n, (r + 1) n) of one N n-contig stream),
value = N n / the slowest rank's pass time.

k2 leg (`k2`, top-level `k2_pair_evals_per_sec`): BASELINE.json configs[4], the explain_two
stress set (20 genes, 5000 clades, ~12.5 M reference clade pairs per contig).  Every rank
times a 6,250-contig share of the 50,000 contigs (the per-GPU share at 8 GPUs: at N = 8
the leg is the whole config), with the per-phase HIP-event timing of the library
(wf_timing.phase_ms): the explain_two kernels' time, the B_k2 bytes they stand for, and
the whole pass.  Its HBM fraction is per GPU: the bytes of all ranks / the slowest rank's
explain_two time / (N x 8 TB/s).

Each rank generates its contig ranges before the GPU is touched (synth.generate_batch:
every chunk from its own seed, in parallel worker processes).  cfg2 / cfg3 / cfg5 stay
available as the main workload with --config.

Extra keys on the line (rank 0, N=1): `cpu_baseline` (the oracle port on 1 core, on the
job's cores in parallel processes over disjoint shards, and its explain_two pair rate on a
stress contig), `pcie_inclusive` (scope ii: host arrays -> wf_score host mode -> host
results), `cli_end_to_end` (scope iii: text files -> `python -m waafle_amd.orgscorer` ->
TSVs, cfg2 and cfg3).

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
    ap.add_argument("--cpu-parallel", type=int, default=10000,
                    help="contigs of the parallel CPU leg (split over the job's cores); 0 disables")
    ap.add_argument("--cpu-k2-clades", type=int, default=1000,
                    help="clades of the stress contig timed for the CPU pair rate; 0 disables")
    ap.add_argument("--e2e", default="cfg2,cfg3", help="CLI end-to-end configs ('' disables)")
    ap.add_argument("--pcie", type=int, default=1, help="time the host-array scope")
    ap.add_argument("--k2-contigs", type=int, default=6250,
                    help="cfg5 contigs per rank for the k2 leg; 0 disables")
    ap.add_argument("--k2-steps", type=int, default=3)
    ap.add_argument("--flags", default="",
                    help="waafle_orgscorer flags for the main workload, e.g. '--weak-loci assign-unknown'")
    ap.add_argument("--option", action="append", default=[],
                    help="wf_set_option NAME=VALUE (sparse_big, att_limit, dump_cap, triage); repeatable")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for N > 1 (nccl = RCCL over xGMI; gloo: "
                         "control traffic on the CPU, e.g. with several ranks on one device)")
    ap.add_argument("--device-map", default=None,
                    help="device of each local rank, e.g. '0,0' (two ranks on device 0: a "
                         "rehearsal of the N > 1 branch on one GPU, not a scaling number)")
    ap.add_argument("--weak", type=int, default=1,
                    help="N > 1: also time the weak-scaling workload (every rank its own n contigs)")
    ap.add_argument("--shares", default="2,4,8",
                    help="N = 1: time every rank's strong-scaling share of the workload at these "
                         "N on this one GPU (`strong_share_projection`); '' disables")
    ap.add_argument("--traffic-json", default=None)
    ap.add_argument("--valu-pmc-json", default=os.path.join(PROFILES, "r06", "cfg4_valu.json"),
                    help="PMC VALU counts of the main pass (scripts/pmc_main.py, optional)")
    ap.add_argument("--k2-traffic-json", default=os.path.join(PROFILES, "r06", "traffic_cfg5.json"),
                    help="FETCH/WRITE of the k2 leg's kernels (scripts/pmc_k2_r5.sh)")
    ap.add_argument("--k2-pmc-json", default=os.path.join(PROFILES, "r06", "k2_pmc.json"),
                    help="PMC VALU counts of the k2 leg's kernels (rocprofv3 --pmc, optional)")
    return ap.parse_args()


def algorithmic_bytes(batch):
    """24 B/hit + 12 B/locus + 16 B/contig offsets + 80 B/contig result."""
    N = batch.n_contigs
    return 24 * batch.n_hits + 12 * batch.n_loci + 16 * (N + 1) + 80 * N


def k2_algorithmic(pair_evals, batch, ppot_sum=None):
    """SURVEY §8(d) counts for the isolated explain_two kernel: B_k2 = sum over the explain_two
    calls of P_pot*G*8 (the S rows of the potential clades; ppot_sum: the library's per-contig
    sum of P_pot over its calls, one per roll-up level) and OPS_pair = sum pairs*G (this rank
    only).  Without ppot_sum, P_pot is solved from the contig's summed pairs P_pot(P_pot-1)/2,
    which undercounts contigs with explain_two at several levels."""
    sel = pair_evals > 0
    p = pair_evals[sel].astype(np.float64)
    one = np.rint((1.0 + np.sqrt(1.0 + 8.0 * p)) / 2.0)   # (one call's P_pot from its pairs)
    ppot = ppot_sum[sel].astype(np.float64) if ppot_sum is not None else one
    g = np.diff(batch.loc_off)[sel].astype(np.float64)
    return {"contigs_explain_two": int(sel.sum()), "p_pot_max": int(one.max()) if p.size else 0,
            "b_k2_bytes": float((ppot * g * 8.0).sum()), "ops_pair": float((p * g).sum()),
            "pairs": float(p.sum()),
            "b_k2_from": "ppot_sum (per call)" if ppot_sum is not None else "pairs (one call per contig)"}


OPS_PEAK = 3.93e13            # 256 CUs x 64 lanes x 2.4 GHz simple fp64 / int ops


def ops_site(batch, parent, pdict, iters, pair_budget=20_000_000):
    """OPS_site = sum over the levels a contig is evaluated at of sum over its
    (clade, locus) pairs with an attached hit of len(locus) -- the reference's site updates and
    np.mean adds (score_hit / update_gene_scores, orgscorer.py:371-406; raise_taxonomy :431-445)
    -- from the attachment rule of orgscorer.py:359-369 (calc_overlap, utils.py:487-500) in
    numpy, on the first contigs whose hit x locus pairs fit `pair_budget`, scaled by contigs.
    iters: the contigs' evaluated levels (wf_result.iterations; at least level 0).
    -> (OPS_site for the batch, contigs sampled)."""
    N = batch.n_contigs
    if N == 0:
        return 0.0, 0
    H, G = np.diff(batch.hit_off), np.diff(batch.loc_off)
    S = int(np.clip(np.searchsorted(np.cumsum(H * G), pair_budget, side="right"), 1, N))
    h1 = int(batch.hit_off[S])
    hc = np.repeat(np.arange(S), H[:S])                       # each hit's contig
    reps = G[hc]
    hi = np.repeat(np.arange(h1), reps)                       # (hit, locus of its contig) pairs
    k = np.arange(len(hi)) - np.repeat(np.cumsum(reps) - reps, reps)
    li = np.repeat(batch.loc_off[:S][hc], reps) + k
    qlo, qhi = batch.hit_qlo[hi].astype(np.int64), batch.hit_qhi[hi].astype(np.int64)
    a, b = qlo.copy(), qhi.copy()
    qlo, qhi = np.minimum(a, b), np.maximum(a, b)
    lo = np.minimum(batch.loc_start[li], batch.loc_end[li]).astype(np.int64)
    up = np.maximum(batch.loc_start[li], batch.loc_end[li]).astype(np.int64)
    llen = up - lo + 1
    disjoint = (lo > qhi) | (qlo > up)
    ov = (np.minimum(qhi, up) - np.maximum(qlo, lo) + 1).astype(np.float64)
    frac = np.where(disjoint, 0.0, ov / np.minimum(qhi - qlo + 1, llen))
    ok = (frac >= float(pdict["min_overlap"])) & (batch.hit_scov[hi] >= float(pdict["min_scov"]))
    if pdict.get("stranded"):
        ok &= batch.hit_strand[hi] == batch.loc_strand[li]
    clade = batch.hit_taxon[hi][ok].astype(np.int64)
    loc, ln, lev = li[ok], llen[ok], np.maximum(iters[:S].astype(np.int64), 1)[hc[hi][ok]]
    parent = np.asarray(parent, np.int64)
    for _ in range(max(0, int(pdict.get("jump_taxonomy") or 0))):   # orgscorer.py:955-957
        clade = parent[clade]
    T = len(parent)
    total, L = 0, 0
    while len(clade) and (lev > L).any():
        sel = lev > L
        _, first = np.unique(loc[sel] * T + clade[sel], return_index=True)
        total += int(ln[sel][first].sum())
        clade = parent[clade]
        L += 1
    return float(total) * N / S, S


def file_sha(path):
    """sha256 of a file (the library build a PMC summary was taken on), first 16 hex digits."""
    import hashlib
    with open(path, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()[:16]


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


def _oracle_pairs(clades, seed=5):
    """The oracle's explain_two on one cfg5-shaped stress contig with `clades` clades
    (P_pot ~ clades): (reference-equivalent pairs, seconds of the scoring call)."""
    from oracle import orgscorer_oracle as orc
    from oracle_bridge import oracle_hits_from_batch, oracle_loci_from_batch
    from waafle_amd import cli, synth
    data = synth.generate(n=1, genes=20, clades=clades, seed=seed, stress=True)
    batch, tax = synth.to_batch(data, with_codes=False)
    hits, loci = oracle_hits_from_batch(batch, tax), oracle_loci_from_batch(batch)
    lengths = dict(zip(batch.contig_names, batch.contig_lengths.tolist()))
    params = orc.Params(**cli.param_dict(cli.parse_flags([])))
    t0 = time.perf_counter()
    contigs = orc.score_contigs(lengths, loci, hits, orc.Taxonomy(data.tax.edges), params)
    dt = time.perf_counter() - t0
    return sum(C.pair_evals for C in contigs.values()), dt


def cpu_baseline(config, n_one, n_par, k2_clades):
    """The oracle (Python/numpy restatement of waafle_orgscorer) on chunk 0 of the same
    workload, inputs pre-parsed (same scope as the GPU value): one core; then the job's P
    cores as P processes on disjoint contig shards (fork), rate = contigs / slowest shard;
    and the explain_two pair rate on one stress contig (cfg5 shape, fewer clades)."""
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
    n_par = min(n_par, batch.n_contigs)
    if n_par > 0 and cores >= 2:
        import multiprocessing as mp
        P = cores
        cuts = np.linspace(0, n_par, P + 1).astype(int)
        shards = [(int(x), int(y)) for x, y in zip(cuts[:-1], cuts[1:])]
        t0 = time.perf_counter()
        pool = mp.get_context("fork").Pool(P)      # close + join (see synth.generate_batch)
        try:
            secs = pool.starmap(_oracle_contigs, shards)
        finally:
            pool.close()
            pool.join()
        wall = time.perf_counter() - t0
        out["parallel"] = {"value": n_par / max(secs), "unit": "contigs/s", "cores": P,
                           "kind": "port", "slowest_shard_s": max(secs), "wall_s": wall,
                           "sample": "contigs 0..{} of chunk 0 in {} processes (disjoint "
                                     "shards of ~{}), rate = contigs / slowest shard; {} = "
                                     "this job's CPU share (sched_getaffinity, "
                                     "OMP_NUM_THREADS)".format(n_par, P, n_par // P, P)}
    if k2_clades > 0:
        pairs, sec = _oracle_pairs(k2_clades)
        full = 12_497_500
        out["k2_pairs"] = {
            "value": pairs / sec, "unit": "clade-pair evals/s", "cores": 1, "kind": "port",
            "pairs": pairs, "seconds": sec,
            "extrapolated_s_per_cfg5_contig": full / (pairs / sec),
            "sample": "one cfg5-shaped stress contig with {} clades (P_pot ~ {}), oracle "
                      "explain_two on 1 core; a cfg5 contig (5000 clades, 12,497,500 pairs) "
                      "extrapolated at the same per-pair rate".format(k2_clades, k2_clades)}
    return out


# ---- scope (iii): CLI text -> TSV ---------------------------------------------------------
def cli_end_to_end(config, workers):
    """`python -m waafle_amd.orgscorer` on the text rendering of a config (native ingest,
    one GPU, TSV writer): wall clock of the whole process, and the CLI's own phase split.
    The text is written chunk-parallel (synth.write_text_chunked) before the timed run."""
    from waafle_amd import synth
    with tempfile.TemporaryDirectory() as tmp:
        t0 = time.perf_counter()
        paths, n, nh = synth.write_text_chunked(config, tmp, "e2e", workers=workers)
        t_text = time.perf_counter() - t0
        size = sum(os.path.getsize(p) for p in paths)
        cmd = [sys.executable, "-m", "waafle_amd.orgscorer"] + paths + ["--outdir", tmp]
        t0 = time.perf_counter()
        run = subprocess.run(cmd, capture_output=True, text=True, cwd=REPO, timeout=900)
        wall = time.perf_counter() - t0
    if run.returncode != 0:
        return {"config": config, "error": run.stderr.strip().splitlines()[-3:]}
    phases = [l for l in run.stderr.splitlines() if l.startswith("Finished successfully")]
    return {"config": config, "contigs": n, "hits": nh, "input_bytes": size,
            "value": n / wall, "unit": "contigs/s", "wall_s": wall, "text_write_s": t_text,
            "phases": phases[-1] if phases else None,
            "scope": "text files -> native ingest -> wf_score (1 GPU) -> 3 TSVs, one process "
                     "incl. interpreter start and GPU init"}


class DeviceBatch:
    """A batch's arrays and result records in HBM (torch tensors) with the wf_batch /
    wf_result structs pointing at them.  `min_scov`: the packed hit_key (wf_batch.hit_key,
    built on the host with the arrays, as the CLI packs it at parse time) for that value."""

    def __init__(self, batch, dev, min_scov=None, ppot=False):
        import torch
        from waafle_amd import lib as L
        N, NH, NL = batch.n_contigs, batch.n_hits, batch.n_loci
        self.d = {}
        for f in ("hit_off", "hit_qlo", "hit_qhi", "hit_taxon", "hit_strand", "hit_score",
                  "hit_scov", "hit_sysmask", "loc_off", "loc_start", "loc_end", "loc_strand"):
            arr = getattr(batch, f)
            if arr.dtype == np.uint32:
                arr = arr.view(np.int32)
            self.d[f] = torch.from_numpy(np.ascontiguousarray(arr)).to(dev)
        if min_scov is not None:
            from waafle_amd import engine
            self.d["hit_key"] = torch.from_numpy(engine.hit_keys(batch, min_scov).view(np.int32)).to(dev)
        e = lambda n, t: torch.empty(max(n, 1), dtype=t, device=dev)
        self.out = {
            "call": e(N, torch.int8), "crit": e(N, torch.float64), "rank": e(N, torch.float64),
            "clade1": e(N, torch.int32), "clade2": e(N, torch.int32),
            "direction": e(N, torch.int8), "iterations": e(N, torch.int16),
            "synteny": e(NL, torch.uint8), "n_meld1": e(N, torch.int32),
            "n_meld2": e(N, torch.int32), "meld": e(2 * NH + 2 * N, torch.int32),
            "annot_hit": e(NL, torch.int32), "pair_evals": e(N, torch.int64),
            "status": e(N, torch.int32), "need_bytes": e(N, torch.int64)}
        if ppot:                                     # wf_result.ppot_sum (the k2 leg's B_k2)
            self.out["ppot_sum"] = e(N, torch.int64)
        self.bs = L.WfBatch(n_contigs=N, n_systems=1, n_hits=NH, n_loci=NL,
                            max_hits=batch.max_hits, max_loci=batch.max_loci,
                            device_resident=1, _pad=0,
                            **{f: C.c_void_p(self.d[f].data_ptr()) for f in self.d})
        self.keys_packed = min_scov is not None
        self.rs = L.WfResult(**{f: C.c_void_p(self.out[f].data_ptr()) if f in self.out else None
                                for f, _ in L.WfResult._fields_})

    def host(self, f):
        return self.out[f].cpu().numpy()


def timed_passes(so, h, chk, db, params, steps, warmup, dist, dev, cdev=None):
    """W untimed passes, then K passes bracketed by barrier + synchronize, with the
    library's HIP-event timing on: (elapsed seconds max over ranks, wf_timing)."""
    import torch
    from waafle_amd import dist as wdist, lib as L

    def step():
        chk(so.wf_score(h, C.byref(db.bs), C.byref(params), C.byref(db.rs)))
    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    status = db.host("status")
    assert not status.any(), "contig status errors: {}".format(np.unique(status))
    if dist:
        dist.barrier()
    torch.cuda.synchronize(dev)
    chk(so.wf_timing_enable(h, 1))
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    if dist:
        dist.barrier()
    t1 = time.perf_counter()
    tm = L.WfTiming()
    chk(so.wf_timing_read(h, C.byref(tm)))
    chk(so.wf_timing_enable(h, 0))
    return wdist.max_over_ranks(t1 - t0, dist, cdev), tm


def k2_leg(so, h, chk, kbatch, params, steps, dist, dev, world, pmc_json, cdev=None, traffic_json=None):
    """The explain_two stress leg (BASELINE configs[4]) on this rank's cfg5 share."""
    import torch
    db = DeviceBatch(kbatch, dev, params.min_scov, ppot=True)
    elapsed, tm = timed_passes(so, h, chk, db, params, steps, 1, dist, dev, cdev)
    pe = db.host("pair_evals")
    calls = db.host("call")
    counts = k2_algorithmic(pe, kbatch, db.host("ppot_sum"))
    del db
    torch.cuda.empty_cache()
    ph = tm.phases()
    per = lambda k: ph[k][0] / max(1, tm.passes)
    k2_ms = per("decide") + per("big") + per("handover")
    # whole-job: pairs and B_k2 summed over ranks, times max over ranks
    v = np.array([counts["pairs"], counts["b_k2_bytes"], kbatch.n_contigs,
                  float((calls == 2).sum())], dtype=np.float64)
    if dist:
        t = torch.tensor(v, device=cdev)
        dist.all_reduce(t)
        v = t.cpu().numpy()
    k2_max = float(wdist_max(k2_ms * 1e-3, dist, cdev))
    pass_s = elapsed / steps
    # per GPU: every rank's B_k2 over the slowest rank's explain_two time, against the
    # peak of the `world` devices that moved them
    achieved = v[1] / k2_max / 1e9 / world
    own = counts["b_k2_bytes"] / max(k2_ms * 1e-3, 1e-12) / 1e9
    out = {
        "source": "this run: {} timed passes, HIP events per phase (wf_timing)".format(steps),
        "workload": "cfg5 stress: {} contigs per GPU x {} GPUs (rank r: contigs "
                    "[6250r, 6250(r+1)) of the 50,000), 20 genes, 5000 clades".format(
                        kbatch.n_contigs, world),
        "contigs": int(v[2]), "lgt_calls": int(v[3]),
        "pairs_reference_equivalent": v[0],
        "k2_pair_evals_per_sec": v[0] / pass_s,
        "contigs_per_sec": v[2] / pass_s,
        "pass_ms": pass_s * 1e3,
        "explain_two_ms_per_pass": k2_max * 1e3,
        "explain_two_phases_ms": {"decide": per("decide"), "big": per("big"),
                                  "handover": per("handover")},
        "other_phases_ms": {k: per(k) for k in ("waves", "attach", "segments")},
        "b_k2_bytes": v[1], "b_k2_rule": "sum over explain_two calls (every roll-up level) of "
                                        "P_pot * G * 8 (SURVEY 8(d): the potential clades' score "
                                        "rows; P_pot summed per contig by the library, "
                                        "wf_result.ppot_sum)",
        "b_k2_one_call_per_contig": k2_algorithmic(pe, kbatch)["b_k2_bytes"],
        "hbm": {"achieved_GBs": achieved, "peak_GBs": HBM_PEAK_GBS,
                "frac": achieved / HBM_PEAK_GBS,
                "rule": "sum of B_k2 over ranks / max explain_two time over ranks / "
                        "n_gpus: per GPU",
                "rank0": {"achieved_GBs": own, "frac": own / HBM_PEAK_GBS}},
        "p_pot_max": counts["p_pot_max"],
    }
    if pmc_json and os.path.exists(pmc_json):
        with open(pmc_json) as fh:
            pj = json.load(fh)
        from waafle_amd import lib as L
        if pj.get("contigs") == kbatch.n_contigs and pj.get("lib_sha") == file_sha(L.LIB_PATH):
            insts = pj["valu_insts_per_pass"]
            peak = pj.get("valu_peak_insts_per_s", 2.4576e12)
            out["valu"] = {"insts_per_pass": insts, "achieved_insts_per_s": insts / (k2_max),
                           "peak_insts_per_s": peak, "frac": insts / k2_max / peak,
                           "source": pj.get("source")}
            bs = {k: v for k, v in pj.get("per_kernel", {}).items() if k.startswith("k_big_sparse")}
            if bs:
                b = next(iter(bs.values()))
                out["valu"]["k_big_sparse"] = {"valu_insts_per_pass": b.get("SQ_INSTS_VALU"),
                                               "salu_insts_per_pass": b.get("SQ_INSTS_SALU"),
                                               "lds_insts_per_pass": b.get("SQ_INSTS_LDS")}
        else:
            out["valu"] = {"skipped": "k2 PMC file of another library build or shape"}
    # what the explain_two kernel actually moved (FETCH_SIZE / WRITE_SIZE of k_big_sparse, PMC
    # runs of this library build): b_k2_actual beside the notional B_k2
    if traffic_json and os.path.exists(traffic_json):
        with open(traffic_json) as fh:
            tj = json.load(fh)
        from waafle_amd import lib as L
        if tj.get("contigs") == kbatch.n_contigs and tj.get("lib_sha") == file_sha(L.LIB_PATH):
            kb = tj.get("per_kernel_kb", {}).get("k_big_sparse", {})
            f, w = kb.get("FETCH_SIZE", 0.0) * 1024.0, kb.get("WRITE_SIZE", 0.0) * 1024.0
            big_ms = per("big")
            moved = 2.0 * f + w
            out["b_k2_actual"] = {
                "kernel": "k_big_sparse", "fetch_bytes_raw": f, "fetch_bytes_x2": 2.0 * f, "write_bytes": w,
                "bytes_per_pass": moved, "achieved_GBs": moved / max(big_ms * 1e-3, 1e-12) / 1e9,
                "frac": moved / max(big_ms * 1e-3, 1e-12) / 1e9 / HBM_PEAK_GBS,
                "rule": "k_big_sparse 2 x FETCH_SIZE (gfx950 correction) + WRITE_SIZE per pass (rocprofv3 "
                        "--pmc, separate runs, this build) / this run's 'big' phase time (k_big_sparse and "
                        "the dense decisions it declines)",
                "source": tj.get("source")}
        else:
            out["b_k2_actual"] = {"skipped": "traffic file of another library build or shape"}
    return out


def share_projection(so, h, chk, batch, params, ns, steps, warmup, dev, t_full, min_scov=None):
    """The strong-scaling shares of this workload timed one at a time on this GPU: for each N,
    every rank's contig range [r n / N, (r + 1) n / N) (exactly what bench.py --gpus N gives
    rank r) as its own device-resident batch, W + K passes as the main line.  The path has no
    collective, so an N-GPU pass is the slowest share's pass (plus the barrier): projected
    value = n / that time, projected efficiency = t(n) / (N t(slowest share)).  What it leaves
    out: host-side contention of N processes, and the per-device clocks."""
    import torch
    N = batch.n_contigs
    out = {"rule": "each of the N contiguous shares timed alone on this GPU (W untimed + K "
                   "timed passes, HIP-event phases); projected N-GPU time = the slowest share; "
                   "efficiency = t(whole) / (N x t(slowest share))",
           "t_whole_ms": t_full * 1e3, "per_n": {}}
    for n in ns:
        rows = []
        for r in range(n):
            a, b = r * N // n, (r + 1) * N // n
            db = DeviceBatch(batch.slice(a, b), dev, min_scov)
            el, tm = timed_passes(so, h, chk, db, params, steps, warmup, None, dev)
            del db
            torch.cuda.empty_cache()
            ph = {k: v[0] / max(1, tm.passes) for k, v in tm.phases().items() if v[0] > 0.0}
            rows.append({"rank": r, "contigs": b - a, "ms_per_pass": el / steps * 1e3,
                         "phases_ms": {k: round(v, 4) for k, v in ph.items()},
                         "dispatch_ms": tm.pass_ms / max(1, tm.passes)})
        slow = max(rows, key=lambda x: x["ms_per_pass"])
        t = slow["ms_per_pass"] * 1e-3
        out["per_n"][str(n)] = {
            "contigs_per_gpu": slow["contigs"], "ms_slowest_share": t * 1e3,
            "ms_mean_share": float(np.mean([x["ms_per_pass"] for x in rows])),
            "projected_value": N / t, "projected_efficiency": t_full / (n * t),
            "slowest_rank": slow["rank"], "slowest_phases_ms": slow["phases_ms"],
            "shares_ms": [round(x["ms_per_pass"], 4) for x in rows]}
    return out


def wdist_max(x, dist, dev):
    from waafle_amd import dist as wdist
    return wdist.max_over_ranks(x, dist, dev)


def main():
    args = parse_args()
    # stdout carries the one JSON line alone: anything a library prints there (gloo's
    # connection notices, runtime messages) goes to stderr instead
    json_out = os.fdopen(os.dup(1), "w")
    sys.stdout.flush()
    os.dup2(2, 1)
    from waafle_amd import dist as wdist
    from waafle_amd import synth
    rank, world, local = wdist.rank_env()
    cores, _ = host_cpus()
    workers = max(1, min(16, cores // world))

    # ---- generate this rank's contigs BEFORE touching the GPU (fork-safe) ----
    # Strong scaling (the headline): the configuration's n contigs split over the ranks,
    # rank r the contigs [r n / N, (r + 1) n / N).  Weak scaling (N > 1, `weak`): every rank
    # its own n contigs, [r n, (r + 1) n) of one seeded stream of N n contigs.
    n_cfg = args.contigs or synth.CONFIGS[args.config]["n"]
    n_total = n_cfg
    a, b = rank * n_cfg // world, (rank + 1) * n_cfg // world
    t_gen = time.perf_counter()
    batch, tax = synth.generate_batch(args.config, a, b, workers=workers, n_total=n_cfg)
    wbatch = None
    if world > 1 and args.weak:
        wbatch, _ = synth.generate_batch(args.config, rank * n_cfg, (rank + 1) * n_cfg,
                                         workers=workers, n_total=world * n_cfg)
    kbatch = ktax = None
    if args.k2_contigs > 0:
        k0 = (rank * args.k2_contigs) % synth.CONFIGS["cfg5"]["n"]
        kbatch, ktax = synth.generate_batch("cfg5", k0, k0 + args.k2_contigs, workers=workers)
    t_gen = time.perf_counter() - t_gen
    # CPU legs before the GPU is initialised: the parallel leg forks worker processes, and
    # the end-to-end legs are processes that initialise the GPU themselves
    cpu_line, e2e_lines = None, []
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        cpu_line = cpu_baseline(args.config, args.cpu_sample, args.cpu_parallel,
                                args.cpu_k2_clades)
    if rank == 0 and world == 1 and args.e2e:
        e2e_lines = [cli_end_to_end(c, workers) for c in args.e2e.split(",") if c]

    import torch
    from waafle_amd import cli, engine, lib as L
    dist = None
    dmap = [int(x) for x in args.device_map.split(",")] if args.device_map else None
    ordinal = dmap[local] if dmap else local
    dev = torch.device("cuda", ordinal)
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(dev)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")
    torch.cuda.set_device(dev)
    # collectives' tensors: on the device for RCCL, on the host for gloo
    cdev = dev if args.backend == "nccl" else None

    N, NH = batch.n_contigs, batch.n_hits
    pdict = cli.param_dict(cli.parse_flags(args.flags.split()))
    params = engine.params_struct(pdict)
    k2_params = engine.params_struct(cli.param_dict(cli.parse_flags([])))
    so = L.load()
    h = C.c_void_p()
    assert so.wf_init(ordinal, C.byref(h)) == 0, "wf_init failed"

    def chk(rc):
        if rc:
            raise RuntimeError(so.wf_last_error(h).decode())
    if args.lds_bytes:
        chk(so.wf_set_lds_bytes(h, args.lds_bytes))
    if args.mode:
        chk(so.wf_set_mode(h, engine.MODES[args.mode]))
    for o in args.option:
        name, val = o.split("=")
        chk(so.wf_set_option(h, {"sparse_big": L.OPT_SPARSE_BIG, "att_limit": L.OPT_ATT_LIMIT,
                                       "wave_two": L.OPT_WAVE_TWO, "dump_cap": L.OPT_DUMP_CAP,
                                       "triage": L.OPT_TRIAGE}[name],
                             int(val)))
    tstruct = engine.taxonomy_struct(tax)
    chk(so.wf_set_taxonomy(h, C.byref(tstruct)))
    stream = torch.cuda.current_stream(dev)
    chk(so.wf_set_stream(h, C.c_void_p(stream.cuda_stream)))

    db = DeviceBatch(batch, dev, params.min_scov)
    elapsed, tm = timed_passes(so, h, chk, db, params, args.steps, args.warmup, dist, dev, cdev)
    calls, pe, iters = db.host("call"), db.host("pair_evals"), db.host("iterations")
    del db
    torch.cuda.empty_cache()
    weak = None
    if wbatch is not None:
        wdb = DeviceBatch(wbatch, dev, params.min_scov)
        w_el, _ = timed_passes(so, h, chk, wdb, params, args.steps, args.warmup, dist, dev, cdev)
        del wdb
        torch.cuda.empty_cache()
        weak = {"value": world * n_cfg / (w_el / args.steps), "unit": "contigs/s",
                "ms_per_step": w_el / args.steps * 1e3, "contigs_total": world * n_cfg,
                "contigs_per_gpu": wbatch.n_contigs, "hits_per_gpu": wbatch.n_hits,
                "scaling": "weak",
                "workload": "every rank its own {} contigs ([r n, (r + 1) n) of one {}-contig "
                            "stream), same flags, same timing".format(n_cfg, world * n_cfg)}
        del wbatch
    projection = None
    if world == 1 and args.shares:
        projection = share_projection(so, h, chk, batch, params,
                                      [int(x) for x in args.shares.split(",") if x],
                                      args.steps, args.warmup, dev, elapsed / args.steps, params.min_scov)
    pairs = float(pe.sum())
    k2_counts = k2_algorithmic(pe, batch)
    if dist:          # whole-job counts
        v = torch.tensor([pairs, float((calls == 2).sum()), float((calls == 1).sum()),
                          float((calls == 0).sum()), float((iters > 1).sum())],
                         dtype=torch.float64, device=cdev)
        dist.all_reduce(v)
        pairs, n_lgt, n_no, n_un, n_up = v.tolist()
    else:
        n_lgt, n_no, n_un, n_up = ((calls == 2).sum(), (calls == 1).sum(), (calls == 0).sum(),
                                   (iters > 1).sum())
    ms_step = elapsed / args.steps * 1e3
    value = n_total / (elapsed / args.steps)
    pass_ms = tm.pass_ms / max(1, tm.passes)
    phases = tm.phases()
    # The dominant kernel: the level-0 triage launch when it runs (wf_phase "triage" spans that
    # launch alone), else the first wave form's level-0 launch (wf_phase "waves").  Its
    # algorithmic bytes: every contig's hits, loci and offsets read once (24 B/hit, 12 B/locus,
    # 16 B/contig) and the 80 B records of the contigs explain_one decided at level 0 (call
    # no_lgt after one iteration: an upper bound on the ones this launch wrote -- the wave form
    # decides the few the triage hands on).  `pass`: the whole pass's bytes over its time.
    tri_ms = phases["triage"][0] / max(1, tm.passes)
    cap = 224 if batch.max_hits <= 224 else (256 if batch.max_hits <= 256 else 512)
    if tri_ms > 0.0:
        dom_kernel, dom_ms = "k_triage", tri_ms
        dom_label = "k_triage: the level-0 triage launch (HIP events on its stream, wf_phase triage)"
    else:
        dom_kernel, dom_ms = "k_wave<{}, false, false>".format(cap), phases["waves"][0] / max(1, tm.passes)
        dom_label = dom_kernel + ": the first wave form's level-0 launch (HIP events, wf_phase waves)"
    n_rec = int(((calls == 1) & (iters == 1)).sum())
    b_dom = 24 * batch.n_hits + 12 * batch.n_loci + 16 * (N + 1) + 80 * n_rec
    b_alg = algorithmic_bytes(batch)
    achieved = b_dom / (dom_ms * 1e-3) / 1e9
    achieved_pass = b_alg / (pass_ms * 1e-3) / 1e9
    # SURVEY 8(d)'s op roofline of the whole pass (this rank's contigs)
    ops_s, ops_n = ops_site(batch, tax.parent, pdict, iters)
    t_hbm, t_ops = b_alg / (HBM_PEAK_GBS * 1e9), (ops_s + k2_counts["ops_pair"]) / OPS_PEAK
    ops_roofline = {
        "rule": "SURVEY 8(d): roofline_time = max(B_alg / 8.0e12 B/s, OPS_alg / 3.93e13 op/s), OPS_alg "
                "= OPS_site + OPS_pair; achieved = roofline_time / the pass time",
        "b_alg": b_alg, "ops_site": ops_s, "ops_pair": k2_counts["ops_pair"],
        "ops_site_rule": "sum over evaluated levels of len(locus) per (clade, locus) with an attached hit "
                         "(the reference's site updates); numpy attachment rule on the first {} contigs, "
                         "scaled".format(ops_n),
        "t_hbm_ms": t_hbm * 1e3, "t_ops_ms": t_ops * 1e3, "roofline_time_ms": max(t_hbm, t_ops) * 1e3,
        "pass_ms": pass_ms, "bound": "ops" if t_ops > t_hbm else "hbm",
        "achieved": max(t_hbm, t_ops) * 1e3 / pass_ms,
        "note": "counts the reference's per-site work; the closed-form means and the mask-class "
                "pair search do far less of it"}
    lib_sha = file_sha(L.LIB_PATH)

    def pmc_file(path, kind):
        """A PMC summary of this config, contig count, dominant kernel and library build, or
        (None, why not)."""
        if not path or not os.path.exists(path):
            return None, "no {} file".format(kind)
        with open(path) as fh:
            j = json.load(fh)
        if j.get("config") != args.config or j.get("contigs") != N:
            return None, "{} file of another workload".format(kind)
        if j.get("dominant_kernel") != dom_kernel:
            return None, "{} file of another dominant kernel ({})".format(kind, j.get("dominant_kernel"))
        if j.get("lib_sha") != lib_sha:
            return None, "{} file of another libwaafle_hip.so build".format(kind)
        return j, None
    traffic, tsrc = None, None
    tj, why_t = pmc_file(args.traffic_json or os.path.join(PROFILES, "r06", "traffic_{}.json".format(args.config)),
                         "traffic")
    if tj:
        # per launch, corrected as MI355X_MICROARCH.md's HBM / rocprofv3 section prescribes:
        # gfx950's FETCH_SIZE counts half the bytes of a coalesced streaming read (x2)
        traffic = 2.0 * tj["dominant_fetch_bytes_raw"] + tj["dominant_write_bytes"]
        tsrc = {"rule": "2 x FETCH_SIZE + WRITE_SIZE of the dominant kernel per launch (gfx950 FETCH x2)"}
        tsrc.update({k: tj.get(k) for k in ("dominant_kernel", "dominant_fetch_bytes_raw",
                                       "dominant_write_bytes", "fetch_bytes_raw",
                                       "fetch_bytes_x2", "write_bytes", "hbm_bytes_raw",
                                       "hbm_bytes_x2", "dispatches_per_pass", "source")})
    else:
        tsrc = {"skipped": why_t}
    valu = None
    vj, why_v = pmc_file(args.valu_pmc_json, "VALU")
    if vj:
        peak = vj.get("valu_peak_insts_per_s", 1.2288e12)
        vi, vd = vj["valu_insts_per_pass"], vj["dominant_valu_insts_per_pass"]
        valu = {"unit": "wave-instructions/s", "peak": peak,
                "pass": {"insts": vi, "achieved": vi / (pass_ms * 1e-3),
                         "frac": vi / (pass_ms * 1e-3) / peak},
                "dominant": {"kernel": vj.get("dominant_kernel"), "insts": vd,
                             "achieved": vd / (dom_ms * 1e-3),
                             "frac": vd / (dom_ms * 1e-3) / peak,
                             "wait_frac": vj.get("dominant_wait_frac")},
                "source": vj.get("source")}
    else:
        valu = {"skipped": why_v}
    spec = synth.CONFIGS[args.config]
    result = {
        "metric": "contigs scored/sec + k2 clade-pair evals/sec at 1/2/4/8 MI355X vs CPU ref",
        "value": value, "unit": "contigs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True,
        "scaling": "strong", "vs_baseline": None, "dtype": "f64",
        "data": "synthetic (seeded generator, SURVEY §8(d) shapes)",
        "config": {"workload": "{}: {} contigs x {} genes x {} clades{}, {} hits{}, {}"
                               .format(args.config, n_cfg, spec["genes"], spec["clades"],
                                       "" if world == 1 else " split over {} GPUs".format(world),
                                       NH, "" if world == 1 else " on rank 0",
                                       "flags " + args.flags if args.flags else "default flags"),
                   "contigs_total": n_total, "contigs_per_gpu": N, "hits_per_gpu": NH,
                   "parallelism": "dp{} (contig ranges [r n/N, (r+1) n/N), no data-path "
                                  "collective)".format(world)},
        "weak": weak,
        "strong_share_projection": projection,
        "k2_pair_evals_per_sec": None,
        "k2_pair_evals_note": "reference-equivalent count: sum of P_pot(P_pot-1)/2 over "
                              "explain_two calls (orgscorer.py:606-608 score(c1,c2) calls), "
                              "on the cfg5 stress leg (`k2`); the mask-class search "
                              "evaluates far fewer pairs",
        "calls": {"lgt": int(n_lgt), "no_lgt": int(n_no), "unclassified": int(n_un),
                  "rolled_up": int(n_up),
                  "iterations_rank0": {int(k): int(v) for k, v in
                                       enumerate(np.bincount(iters[calls != 0].astype(np.int64)))
                                       if v}},
        "main_k2_counts": dict(k2_counts, pair_evals_per_sec=pairs / (elapsed / args.steps)),
        "ops_roofline": ops_roofline,
        "kernel_ms": dict({"wf_score_pass": pass_ms},
                          **{"phase_" + k: v[0] / max(1, tm.passes)
                             for k, v in tm.phases().items()}),
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": dom_label,
                     "kernel_ms": dom_ms,
                     "algorithmic_bytes_per_launch": b_dom,
                     "algorithmic_bytes_rule": "24 B/hit + 12 B/locus + 16 B/contig + 80 B per "
                                               "record of a contig explain_one decided at level 0 "
                                               "({} of {})".format(n_rec, N),
                     "pass": {"ms": pass_ms, "achieved": achieved_pass, "bytes": b_alg,
                              "bytes_rule": "24 B/hit + 12 B/locus + 96 B/contig",
                              "frac": achieved_pass / HBM_PEAK_GBS,
                              "note": "every kernel of one wf_score pass (level 0, hand-over, "
                                      "roll-up levels, staged remainder)"},
                     "valu": valu,
                     "traffic_detail": tsrc},
        "options": args.option or None,
        "ranks": {"backend": args.backend if world > 1 else None,
                  "devices": dmap[:world] if dmap else list(range(world)),
                  "note": (None if not dmap or len(set(dmap[:world])) == world else
                           "ranks share a device: a rehearsal of the N > 1 branch, not a "
                           "scaling number")},
        "generate_s": t_gen,
        "cpu_baseline": None,
    }
    if kbatch is not None:
        if ktax.names != tax.names:
            tk = engine.taxonomy_struct(ktax)
            chk(so.wf_set_taxonomy(h, C.byref(tk)))
        result["k2"] = k2_leg(so, h, chk, kbatch, k2_params, args.k2_steps, dist, dev, world,
                              args.k2_pmc_json, cdev, args.k2_traffic_json)
        result["k2_pair_evals_per_sec"] = result["k2"]["k2_pair_evals_per_sec"]
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
    if e2e_lines:
        result["cli_end_to_end"] = e2e_lines
    if rank == 0:
        print(json.dumps(result), file=json_out, flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
