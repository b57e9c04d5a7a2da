"""Benchmark: contigs scored/sec (+ k2 clade-pair evals/sec) on MI355X.

Workload (BASELINE.json configs[1]): synthetic 10k contigs x 8 genes x 200 clades,
20 decoy hits per gene (1.68 M hits), default waafle_orgscorer parameters, roll-up
enabled.  One step = one wf_score pass over the whole batch with inputs already
resident in HBM.  For N GPUs (torch.distributed.run, one process per GPU) every rank
scores its own 10k-contig shard (weak scaling; contigs are independent, so there is
no data-path collective -- only the barrier and the max-over-ranks timing).

    python bench.py [--gpus N --steps K --warmup W] [--config cfg2|cfg3|cfg4|cfg5]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8.0 TB/s spec
VALU_F64_PEAK = 3.93e13        # 256 CU x 64 lanes x 2.4 GHz simple fp64/int ops


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--contigs", type=int, default=None, help="override contigs per GPU")
    ap.add_argument("--lds-bytes", type=int, default=None)
    ap.add_argument("--threads", type=int, default=None, help="threads per contig (64/128/256)")
    ap.add_argument("--mode", default="staged", choices=["staged", "fused"])
    ap.add_argument("--cpu-sample", type=int, default=6000,
                    help="contigs timed on the CPU oracle (rank 0, N=1); 0 disables")
    ap.add_argument("--traffic-json", default=os.path.join(REPO, "profiles", "traffic_cfg2.json"))
    return ap.parse_args()


def algorithmic_bytes(batch):
    """24 B/hit + 12 B/locus + 16 B/contig offsets + 80 B/contig result."""
    N = batch.n_contigs
    return 24 * batch.n_hits + 12 * batch.n_loci + 16 * (N + 1) + 80 * N


def site_ops_level0(batch, min_overlap=0.1, min_scov=0.75):
    """Algorithmic site additions at the first level: sum over distinct (taxon, locus)
    pairs with an attached hit of len(locus) (vectorised attach test)."""
    total = 0
    hc = np.repeat(np.arange(batch.n_contigs), np.diff(batch.hit_off))
    lstart = np.minimum(batch.loc_start, batch.loc_end).astype(np.int64)
    lend = np.maximum(batch.loc_start, batch.loc_end).astype(np.int64)
    lcount = np.diff(batch.loc_off)
    G = int(lcount.max()) if len(lcount) else 0
    for g in range(G):
        has = lcount[hc] > g
        li = batch.loc_off[hc[has]] + g
        qlo = batch.hit_qlo[has].astype(np.int64)
        qhi = batch.hit_qhi[has].astype(np.int64)
        l1, l2 = lstart[li], lend[li]
        ov = np.minimum(qhi, l2) - np.maximum(qlo, l1) + 1
        den = np.minimum(qhi - qlo + 1, l2 - l1 + 1)
        frac = np.where(ov > 0, ov / den, 0.0)
        ok = (frac >= min_overlap) & (batch.hit_scov[has] >= min_scov)
        pairs = np.unique(np.stack([li[ok], batch.hit_taxon[has][ok].astype(np.int64)]), axis=1)
        lens = (lend - lstart + 1)[pairs[0]]
        total += int(lens.sum())
    return total


def to_device(batch, torch, dev):
    t = {}
    for f in ("hit_off", "hit_qlo", "hit_qhi", "hit_taxon", "hit_strand", "hit_score",
              "hit_scov", "hit_sysmask", "loc_off", "loc_start", "loc_end", "loc_strand"):
        a = getattr(batch, f)
        if a.dtype == np.uint32:
            a = a.view(np.int32)
        t[f] = torch.from_numpy(np.ascontiguousarray(a)).to(dev)
    return t


def cpu_baseline(data, batch, tax, n_sample, config):
    """Time the oracle (a Python/numpy port of the reference) on the first n_sample
    contigs of the same workload, inputs pre-parsed (same scope as the GPU value)."""
    from oracle import orgscorer_oracle as orc
    from waafle_amd import cli
    sys.path.insert(0, os.path.join(REPO, "tests"))
    from oracle_bridge import oracle_hits_from_batch, oracle_loci_from_batch
    sub = batch.slice(0, n_sample)
    params = orc.Params(**cli.param_dict(cli.parse_flags([])))
    otax = orc.Taxonomy(data.tax.edges)
    hits = oracle_hits_from_batch(sub, tax)
    loci = oracle_loci_from_batch(sub)
    lengths = dict(zip(sub.contig_names, sub.contig_lengths.tolist()))
    t0 = time.perf_counter()
    orc.score_contigs(lengths, loci, hits, otax, params)
    dt = time.perf_counter() - t0
    return {"value": n_sample / dt, "unit": "contigs/s", "cores": 1, "kind": "port",
            "sample": "first {} contigs of the {} workload, oracle (Python/numpy restatement "
                      "of waafle_orgscorer) on 1 host core, inputs pre-parsed; {:.1f} s".format(
                          n_sample, config, dt)}


def main():
    args = parse_args()
    import torch
    from waafle_amd import cli, engine, lib as L, synth
    from waafle_amd import dist as wdist

    rank, world, local = wdist.rank_env()
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    spec = dict(synth.CONFIGS[args.config])
    if args.contigs:
        spec["n"] = args.contigs
    seed = int(args.config[-1]) + 1000 * rank
    data = synth.generate(seed=seed, **spec)
    batch, tax = synth.to_batch(data, with_codes=False)
    N, NH, NL = batch.n_contigs, batch.n_hits, batch.n_loci
    params = engine.params_struct(cli.param_dict(cli.parse_flags([])))

    so = L.load()
    h = C.c_void_p()
    assert so.wf_init(local, C.byref(h)) == 0, "wf_init failed"
    chk = lambda rc: (_ for _ in ()).throw(RuntimeError(so.wf_last_error(h).decode())) if rc else None
    chk(so.wf_set_mode(h, engine.MODES[args.mode]))
    if args.lds_bytes:
        chk(so.wf_set_lds_bytes(h, args.lds_bytes))
    if args.threads:
        chk(so.wf_set_workgroup(h, args.threads))
    tstruct = engine.taxonomy_struct(tax)
    chk(so.wf_set_taxonomy(h, C.byref(tstruct)))
    stream = torch.cuda.current_stream(dev)
    chk(so.wf_set_stream(h, C.c_void_p(stream.cuda_stream)))

    d = to_device(batch, torch, dev)
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
    pairs = int(out["pair_evals"].cpu().numpy().sum())
    iters = out["iterations"].cpu().numpy()
    ms_step = elapsed / args.steps * 1e3
    value = world * N / (elapsed / args.steps)
    k_ms = tm.lds_kernel_ms / max(1, tm.launches)
    big_ms = tm.big_kernel_ms / max(1, tm.launches)
    if args.mode == "staged":
        # the staged form has no single kernel that consumes the path's input: the unit is
        # one whole wf_score pass (HIP events around all of its kernels, on its stream)
        kname, kernel_ms = "wf_score pass (staged: all kernels)", {"wf_score_pass": k_ms}
    else:
        kname, kernel_ms = "k_contig_lds", {"k_contig_lds": k_ms, "k_contig_big": big_ms}
    b_alg = algorithmic_bytes(batch)
    achieved = b_alg / (k_ms * 1e-3) / 1e9
    traffic = None
    if os.path.exists(args.traffic_json):
        with open(args.traffic_json) as fh:
            tj = json.load(fh)
        if (tj.get("config") == args.config and tj.get("contigs") == N
                and tj.get("mode", "fused") == args.mode):
            traffic = tj.get("hbm_bytes_per_launch")
    ops0 = site_ops_level0(batch)
    result = {
        "metric": "contigs scored/sec + k2 clade-pair evals/sec at 1/2/4/8 MI355X vs CPU ref",
        "value": value, "unit": "contigs/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms_step, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": "{}: {} contigs x {} genes x {} clades per GPU, {} hits, "
                               "default flags".format(args.config, N, spec["genes"],
                                                      spec["clades"], NH),
                   "contigs_per_gpu": N, "hits_per_gpu": NH, "parallelism": "dp{}".format(world)},
        "k2_pair_evals_per_sec": world * pairs / (elapsed / args.steps),
        "calls": {"lgt": int((calls == 2).sum()), "no_lgt": int((calls == 1).sum()),
                  "unclassified": int((calls == 0).sum()),
                  "rolled_up": int((iters > 1).sum())},
        "mode": args.mode,
        "kernel_ms": kernel_ms,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                     "kernel": kname, "algorithmic_bytes_per_launch": b_alg,
                     "valu": {"site_adds_level0": ops0,
                              "achieved_ops_per_s": ops0 / (k_ms * 1e-3),
                              "peak_ops_per_s": VALU_F64_PEAK,
                              "frac": ops0 / (k_ms * 1e-3) / VALU_F64_PEAK}},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        result["cpu_baseline"] = cpu_baseline(data, batch, tax, min(args.cpu_sample, N),
                                              args.config)
    if rank == 0:
        print(json.dumps(result))
    so.wf_free(h)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
