"""Throughput of wf_genecall (waafle_genecaller on the GPU) on a synthetic workload.

    python scripts/bench_genecaller.py [--config cfg2] [--steps 20]

Contig groups and hits of the BASELINE synthetic config, device-resident (torch buffers),
one wf_genecall per step timed between stream synchronisations; the CPU oracle
(oracle/genecaller_oracle.py, 1 core) is timed on a 1,000-group sample of the same hits.
Prints one JSON line.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--cpu-sample", type=int, default=1000)
    a = ap.parse_args()
    import numpy as np
    import torch
    from waafle_amd import lib as L, synth
    spec = dict(synth.CONFIGS[a.config])
    data = synth.generate(seed=int(a.config[-1]), **spec)
    batch, _ = synth.to_batch(data, with_codes=False)
    G, NH = batch.n_contigs, batch.n_hits
    dev = torch.device("cuda", 0)
    t = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)
    d = dict(off=t(batch.hit_off.astype(np.int64)), qlo=t(batch.hit_qlo.astype(np.int32)),
             qhi=t(batch.hit_qhi.astype(np.int32)), st=t(batch.hit_strand.astype(np.int8)),
             scov=t(batch.hit_scov.astype(np.float64)))
    ng = torch.empty(G, dtype=torch.int32, device=dev)
    gs = torch.empty(NH, dtype=torch.int32, device=dev)
    ge = torch.empty(NH, dtype=torch.int32, device=dev)
    gst = torch.empty(NH, dtype=torch.int8, device=dev)
    so = L.load()
    h = C.c_void_p()
    assert so.wf_init(0, C.byref(h)) == 0
    so.wf_set_stream(h, C.c_void_p(torch.cuda.current_stream(dev).cuda_stream))
    b = L.WfGcBatch(n_groups=G, device_resident=1, n_hits=NH,
                    **{k: C.c_void_p(v.data_ptr()) for k, v in
                       (("hit_off", d["off"]), ("hit_qlo", d["qlo"]), ("hit_qhi", d["qhi"]),
                        ("hit_strand", d["st"]), ("hit_scov", d["scov"]))})
    p = L.WfGcParams(min_overlap=0.1, min_scov=0.75, min_gene_length=200.0, stranded=0)
    r = L.WfGcResult(n_genes=C.c_void_p(ng.data_ptr()), gene_start=C.c_void_p(gs.data_ptr()),
                     gene_stop=C.c_void_p(ge.data_ptr()), gene_strand=C.c_void_p(gst.data_ptr()))

    def step():
        rc = so.wf_genecall(h, C.byref(b), C.byref(p), C.byref(r))
        assert rc == 0, so.wf_last_error(h).decode()

    for _ in range(3):
        step()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    torch.cuda.synchronize(dev)
    dt = (time.perf_counter() - t0) / a.steps
    genes = int(ng.sum().item())
    # CPU oracle on a sample of groups (same hit values, restated per group)
    from oracle import genecaller_oracle as gco
    n = min(a.cpu_sample, G)
    t1 = time.perf_counter()
    cpu_genes = 0
    for g in range(n):
        lo, hi = int(batch.hit_off[g]), int(batch.hit_off[g + 1])
        ints = [(int(batch.hit_qlo[i]), int(batch.hit_qhi[i]), "-" if batch.hit_strand[i] else "+")
                for i in range(lo, hi) if batch.hit_scov[i] >= 0.75]
        cpu_genes += sum(1 for x in gco.overlap_intervals(ints, 0.1) if x[1] - x[0] + 1 >= 200)
    cpu = n / (time.perf_counter() - t1)
    assert cpu_genes == int(ng[:n].sum().item()), "GPU and oracle gene counts differ"
    print(json.dumps({"metric": "genecaller contig groups/sec", "config": a.config,
                      "groups": G, "hits": NH, "genes": genes, "ms_per_call": dt * 1e3,
                      "value": G / dt, "hits_per_sec": NH / dt,
                      "note": "wf_genecall call incl. its one D2H of group offsets and status",
                      "cpu_baseline": {"value": cpu, "unit": "groups/s", "cores": 1,
                                       "kind": "port", "sample": "{} groups".format(n)}}))
    so.wf_free(h)


if __name__ == "__main__":
    main()
