"""Per-phase shader-clock laps of the first wave form (diagnostic build only).

Build:  python -m waafle_amd.build --stamps   (waafle_amd/libwaafle_hip_stamps.so)
Run:    WAAFLE_HIP_LIB=waafle_amd/libwaafle_hip_stamps.so python scripts/wave_stamps.py [--contigs N]

k_wave<CAP, false> laps every 16th contig (wf_fast.hip WLAP): the sum of the laps is that
contig's wall time in the wave, so each phase's share is its share of the kernel's time.
"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# (laps 7, 11, 14: the closed-form one-run means; 12, 13: the multi-attachment means --
# wave per segment, lane per segment or leaf per lane; 32-35 the explain_one split)
PHASES = ["loci+lut", "hits/attach", "annotations", "sort", "segments", "prune setup",
          "pass select", "one-run means p0", "post-pass", "dump/level end", "record/end",
          "one-run means p6", "multi means p0", "multi means p1/7/6/2/4/5", "one-run means p1/7/2/4/5",
          "means prep (all passes)"]
# k_triage laps (wf_triage.hip TLAP), per contig it decided
TRIAGE_PHASES = ["offsets, hits, loci, set-up", "attachments", "candidate inserts",
                 "masks, annotation pass 1", "full-clade scan", "segments, annotation pass 2",
                 "gene scores", "mask, crit, rank", "explain_one, meld_one, record"]
# sp_level laps (k_big_sparse / k_dump_sparse<0>, wf_sparse.h BLAP), every 8th contig
SP_LEVEL_PHASES = ["pass 1 maxes", "pass 2 options, classes", "explain_one, meld, record",
                   "class pairs", "pass 3 members", "groups, dense rows", "pass 4 sisters",
                   "candidates pass 1", "candidates pass 2", "meld_two, record / raise"]
STATS = {16: "contigs", 17: "attachments", 18: "segments", 19: "pass iterations",
         20: "segments listed", 21: "dumps", 22: "handed on", 23: "hits"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg4")
    ap.add_argument("--contigs", type=int, default=None)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--flags", default="")
    args = ap.parse_args()
    import numpy as np
    from waafle_amd import synth
    n = args.contigs or synth.CONFIGS[args.config]["n"]
    batch, tax = synth.generate_batch(args.config, 0, n, workers=16, n_total=n)
    import torch
    from bench import DeviceBatch
    from waafle_amd import cli, engine, lib as L
    so = L.load()
    so.wf_stamps_read_fast.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    h = C.c_void_p()
    assert so.wf_init(0, C.byref(h)) == 0
    ts = engine.taxonomy_struct(tax)
    assert so.wf_set_taxonomy(h, C.byref(ts)) == 0
    stream = torch.cuda.current_stream()
    so.wf_set_stream(h, C.c_void_p(stream.cuda_stream))
    params = engine.params_struct(cli.param_dict(cli.parse_flags(args.flags.split())))
    db = DeviceBatch(batch, torch.device("cuda", 0))
    for i in range(args.steps):
        if i == args.steps - 1:
            torch.cuda.synchronize()
            so.wf_stamps_reset_fast()
            so.wf_stamps_reset_sparse()
            so.wf_stamps_reset_triage()
        assert so.wf_score(h, C.byref(db.bs), C.byref(params), C.byref(db.rs)) == 0
    torch.cuda.synchronize()
    st = (C.c_ulonglong * 48)()
    so.wf_stamps_read_fast(st, 48)
    v = [int(x) for x in st]
    sp = (C.c_ulonglong * 16)()
    so.wf_stamps_read_sparse.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    so.wf_stamps_read_sparse(sp, 16)
    w = [int(x) for x in sp]
    tot = sum(v[:16]) + sum(v[32:36])                # (the explain_one laps are their own)
    nc = max(1, v[16])
    out = {"config": args.config, "contigs": n, "flags": args.flags, "sampled": v[16],
           "cycles_per_contig": tot / nc,
           "phases": {p: {"cycles_per_contig": v[i] / nc, "frac": v[i] / max(1, tot)}
                      for i, p in enumerate(PHASES)},
           "stats_per_contig": {name: v[i] / nc for i, name in STATS.items()},
           "pass_entries_per_contig": {str(p): v[24 + p] / nc for p in range(8)},
           "segments_listed_per_contig_by_pass": {str(p): v[40 + p] / nc for p in range(8)},
           "explain_one": {k: v[32 + i] / nc for i, k in enumerate(
               ["sure bits/pass choice", "option scan", "reduction", "meld_one+LCA"])},
           # sp_two (k_dump_sparse<1>, every launch of the pass), every 8th contig
           "sp_two": {"sampled": w[8],
                      "cycles_per_contig": sum(w[:6]) / max(1, w[8]),
                      "phases": {k: w[i] / max(1, w[8]) for i, k in enumerate(
                          ["table + loci loads", "run heads / potentials", "candidate pairs",
                           "members' parents + sister masks", "pass 1 ranks", "pass 2, eval_two, meld, record"])},
                      "per_contig": {"segments": w[9] / max(1, w[8]), "potential clades": w[10] / max(1, w[8]),
                                     "candidate pairs": w[11] / max(1, w[8])}}}
    tr = (C.c_ulonglong * 16)()
    so.wf_stamps_read_triage.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    so.wf_stamps_read_triage(tr, 16)
    t = [int(x) for x in tr]
    nt = max(1, t[15])
    out["triage"] = {"decided_sampled": t[15], "cycles_per_contig": sum(t[:9]) / nt,
                     "phases": {k: t[i] / nt for i, k in enumerate(TRIAGE_PHASES)}}
    bg = (C.c_ulonglong * 48)()
    so.wf_stamps_read_big.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    so.wf_stamps_read_big(bg, 48)
    b = [int(x) for x in bg]
    nb = max(1, b[15])
    out["sp_level"] = {"sampled": b[15], "cycles_per_contig": sum(b[:10]) / nb,
                       "phases": {k: b[i] / nb for i, k in enumerate(SP_LEVEL_PHASES)},
                       "pass 2 split": {"row summaries": b[10] / nb, "class inserts": b[11] / nb},
                       "per_contig": {"segments": b[12] / nb, "potential clades": b[13] / nb,
                                      "members": b[14] / nb},
                       "outcomes": {"declined: class table": b[16], "declined: class pairs": b[17],
                                    "explain_one": b[18]},
                       "calls_by_level": {"0": b[19], "1": b[20], "2+": b[21]},
                       "levels_1_up": {"sampled": b[34],
                                       "cycles_per_contig": sum(b[24:34]) / max(1, b[34]),
                                       "phases": {k: b[24 + i] / max(1, b[34])
                                                  for i, k in enumerate(SP_LEVEL_PHASES)}}}
    print(json.dumps(out))
    for p, d in out["phases"].items():
        print("{:24s} {:10.0f} cyc  {:5.1f}%".format(p, d["cycles_per_contig"], 100 * d["frac"]),
              file=sys.stderr)
    print(out["stats_per_contig"], out["pass_entries_per_contig"], out["explain_one"],
          file=sys.stderr)
    so.wf_free(h)


if __name__ == "__main__":
    main()
