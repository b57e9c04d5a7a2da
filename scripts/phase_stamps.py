"""Per-phase cycle breakdown of the contig kernel (diagnostic build, -DWF_STAMPS).

    python scripts/phase_stamps.py [--config cfg2] [--contigs N]
Prints shader-clock cycles per contig per phase (thread 0, measured after barriers).
Never quote this build's run time: stamps serialise; read the shares.
"""
import argparse
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from waafle_amd import build, cli, engine, lib as L, synth  # noqa: E402

NAMES = {0: "loci+leaf counts", 1: "attach count+scan", 2: "leaf tables+attach fill",
         3: "annotations+jump", 4: "keys build", 5: "bitonic sort", 6: "segments/clades scan",
         7: "S alloc/zero (staged: decide setup)", 8: "site: serial segments", 9: "maxes+weak loci", 10: "explain_one",
         11: "meld_one+write", 12: "two: pass 2 + meld", 20: "contigs (count)", 21: "levels (count)",
         22: "site: classify segments", 23: "site: 8-lane groups", 24: "site: 16-lane groups",
         25: "site: 32-lane groups", 26: "site: 64-lane groups", 16: "two: potential scan",
         17: "two: masks", 18: "two: pass 1 (best pair)", 19: "roll-up re-key (staged)"}
PHASES = list(range(13)) + list(range(16, 20)) + list(range(22, 27))
LAPS = {13: "round: load segment+atts", 14: "round: leaf value", 15: "round: combine+store"}
COUNTS = {27: "segments in 8-lane class", 28: "segments in 16-lane class",
          29: "segments in 32-lane class", 30: "segments in 64-lane class",
          31: "segments serial"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--contigs", type=int, default=None)
    ap.add_argument("--lds-bytes", type=int, default=None)
    ap.add_argument("--threads", type=int, default=None)
    ap.add_argument("--mode", default="fused", choices=["fused", "staged"])
    a = ap.parse_args()
    path = build.build(stamps=True, verbose=False)
    L._lib = None
    so = L.load(path)
    sfx = "_staged" if a.mode == "staged" else ""
    read = getattr(so, "wf_stamps_read" + sfx)
    reset = getattr(so, "wf_stamps_reset" + sfx)
    read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    spec = dict(synth.CONFIGS[a.config])
    if a.contigs:
        spec["n"] = a.contigs
    data = synth.generate(seed=int(a.config[-1]), **spec)
    batch, tax = synth.to_batch(data, with_codes=False)
    params = cli.param_dict(cli.parse_flags([]))
    s = engine.GpuScorer(0, a.lds_bytes, a.threads, mode=a.mode)
    s.set_taxonomy(tax)
    s.score(batch, params)            # warm-up
    reset()
    s.score(batch, params)
    buf = (C.c_ulonglong * 32)()
    read(buf, 32)
    n = batch.n_contigs
    total = sum(buf[i] for i in PHASES)
    print("contigs={} (stamps: s_memtime cycles per contig, thread 0)".format(
        batch.n_contigs))
    for i in PHASES:
        print("{:>2} {:28s} {:12.0f} {:6.1f}%".format(i, NAMES[i], buf[i] / n,
                                                      100.0 * buf[i] / max(1, total)))
    for i, name in LAPS.items():
        print("   lap {:24s} {:12.0f} per contig (wave 0)".format(name, buf[i] / n))
    for i, name in COUNTS.items():
        print("   {:28s} {:12.1f} per contig".format(name, buf[i] / n))
    print("   total per contig {:12.0f}".format(total / n))


if __name__ == "__main__":
    main()
