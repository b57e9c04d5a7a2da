"""Sweep launch geometry (threads per contig x LDS budget) on one device, one process,
interleaved rounds (same data, same clock conditions).  Prints ms per cfg2 step."""
import argparse
import ctypes as C
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import torch  # noqa: E402
from waafle_amd import cli, engine, lib as L, synth  # noqa: E402
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--contigs", type=int, default=None)
    ap.add_argument("--geoms", default="256:36864,64:16384,64:20480,64:24576,64:32768")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--lib", default=None, help="library variant to load (default: product)")
    a = ap.parse_args()
    spec = dict(synth.CONFIGS[a.config])
    if a.contigs:
        spec["n"] = a.contigs
    data = synth.generate(seed=int(a.config[-1]), **spec)
    batch, tax = synth.to_batch(data, with_codes=False)
    dev = torch.device("cuda", 0)
    so = L.load(a.lib) if a.lib else L.load()
    params = engine.params_struct(cli.param_dict(cli.parse_flags([])))
    d = bench.to_device(batch, torch, dev)
    N, NH, NL = batch.n_contigs, batch.n_hits, batch.n_loci
    geoms = [tuple(int(x) for x in g.split(":")) for g in a.geoms.split(",")]
    ctxs = []
    ref = None
    for th, lds in geoms:
        h = C.c_void_p()
        assert so.wf_init(0, C.byref(h)) == 0
        assert so.wf_set_workgroup(h, th) == 0 and so.wf_set_lds_bytes(h, lds) == 0
        ts = engine.taxonomy_struct(tax)
        assert so.wf_set_taxonomy(h, C.byref(ts)) == 0
        out = {f: torch.zeros(max(n, 1), dtype=dt, device=dev) for f, n, dt in [
            ("call", N, torch.int8), ("crit", N, torch.float64), ("rank", N, torch.float64),
            ("clade1", N, torch.int32), ("clade2", N, torch.int32), ("direction", N, torch.int8),
            ("iterations", N, torch.int16), ("synteny", NL, torch.uint8),
            ("n_meld1", N, torch.int32), ("n_meld2", N, torch.int32),
            ("meld", 2 * NH + 2 * N, torch.int32), ("annot_hit", NL, torch.int32),
            ("pair_evals", N, torch.int64), ("status", N, torch.int32),
            ("need_bytes", N, torch.int64)]}
        bs = L.WfBatch(n_contigs=N, n_systems=1, n_hits=NH, n_loci=NL, max_hits=batch.max_hits,
                       max_loci=batch.max_loci, device_resident=1, _pad=0,
                       **{f: C.c_void_p(d[f].data_ptr()) for f in d})
        rs = L.WfResult(**{f: C.c_void_p(out[f].data_ptr()) for f, _ in L.WfResult._fields_})
        assert so.wf_score(h, C.byref(bs), C.byref(params), C.byref(rs)) == 0
        torch.cuda.synchronize()
        res = {k: v.cpu().numpy() for k, v in out.items()}
        assert not res["status"].any()
        if ref is None:
            ref = res
        else:
            for k in ("call", "crit", "rank", "clade1", "synteny"):
                assert np.array_equal(ref[k], res[k]), (th, lds, k)
        ctxs.append((th, lds, h, bs, rs, ts, out))
    times = {g: [] for g in geoms}
    for _ in range(a.rounds):
        for th, lds, h, bs, rs, ts, out in ctxs:
            so.wf_timing_enable(h, 1)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                so.wf_score(h, C.byref(bs), C.byref(params), C.byref(rs))
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            tm = L.WfTiming()
            so.wf_timing_read(h, C.byref(tm))
            times[(th, lds)].append(((t1 - t0) / a.steps * 1e3, tm.lds_kernel_ms / tm.launches,
                                     tm.big_kernel_ms / tm.launches))
    print("{} N={} hits={}".format(a.config, N, NH))
    for g, v in times.items():
        v = np.array(v)
        print("threads={:4d} lds={:6d}  step_ms median {:.3f} min {:.3f}  lds_kernel {:.3f} "
              "big_kernel {:.3f}".format(g[0], g[1], np.median(v[:, 0]), v[:, 0].min(),
                                          np.median(v[:, 1]), np.median(v[:, 2])))


if __name__ == "__main__":
    main()
