"""Experiment: one wf_score over n contigs vs two contexts scoring the two contiguous halves
concurrently (own HIP streams, one host thread each) on the same device."""
import ctypes as C
import os, sys, threading, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
from bench import DeviceBatch
from waafle_amd import synth, cli, engine, lib as L

def ctx(tax, stream):
    so = L.load()
    h = C.c_void_p()
    assert so.wf_init(0, C.byref(h)) == 0
    ts = engine.taxonomy_struct(tax)
    assert so.wf_set_taxonomy(h, C.byref(ts)) == 0
    so.wf_set_stream(h, C.c_void_p(stream.cuda_stream))
    return so, h, ts

def run(n, parts, steps=10):
    batch, tax = synth.generate_batch("cfg4", 0, n, workers=16, n_total=1_000_000)
    params = engine.params_struct(cli.param_dict(cli.parse_flags([])))
    dev = torch.device("cuda", 0)
    cuts = np.linspace(0, n, parts + 1).astype(int)
    dbs = [DeviceBatch(batch.slice(a, b), dev, params.min_scov) for a, b in zip(cuts[:-1], cuts[1:])]
    streams = [torch.cuda.Stream(dev) for _ in range(parts)]
    ctxs = [ctx(tax, s) for s in streams]
    def one(i):
        so, h, _ = ctxs[i]
        rc = so.wf_score(h, C.byref(dbs[i].bs), C.byref(params), C.byref(dbs[i].rs))
        assert rc == 0, so.wf_last_error(h)
    def step():
        if parts == 1:
            one(0)
        else:
            th = [threading.Thread(target=one, args=(i,)) for i in range(parts)]
            for t in th: t.start()
            for t in th: t.join()
        for s in streams: s.synchronize()
    for _ in range(2): step()
    t0 = time.perf_counter()
    for _ in range(steps): step()
    dt = (time.perf_counter() - t0) / steps
    calls = np.concatenate([d.host("call") for d in dbs])
    print("n {:8d} parts {} : {:.3f} ms/pass  lgt {}".format(n, parts, dt * 1e3, int((calls == 2).sum())), flush=True)
    for so, h, _ in ctxs: so.wf_free(h)

for n in (1_000_000, 125_000):
    for rep in range(2):
        for parts in (1, 2, 3, 4):
            run(n, parts)
