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
         7: "S alloc/zero", 8: "site means", 9: "maxes+weak loci", 10: "explain_one",
         11: "meld_one+write", 12: "explain_two", 20: "contigs (count)", 21: "levels (count)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--contigs", type=int, default=None)
    ap.add_argument("--lds-bytes", type=int, default=None)
    ap.add_argument("--threads", type=int, default=None)
    a = ap.parse_args()
    path = build.build(stamps=True, verbose=False)
    L._lib = None
    so = L.load(path)
    so.wf_stamps_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    spec = dict(synth.CONFIGS[a.config])
    if a.contigs:
        spec["n"] = a.contigs
    data = synth.generate(seed=int(a.config[-1]), **spec)
    batch, tax = synth.to_batch(data, with_codes=False)
    params = cli.param_dict(cli.parse_flags([]))
    s = engine.GpuScorer(0, a.lds_bytes, a.threads)
    s.set_taxonomy(tax)
    s.score(batch, params)            # warm-up
    so.wf_stamps_reset()
    s.score(batch, params)
    buf = (C.c_ulonglong * 32)()
    so.wf_stamps_read(buf, 32)
    n = batch.n_contigs
    total = sum(buf[i] for i in range(13))
    print("contigs={} (stamps: s_memtime cycles per contig, thread 0)".format(
        batch.n_contigs))
    for i in range(13):
        print("{:>2} {:28s} {:12.0f} {:6.1f}%".format(i, NAMES[i], buf[i] / n,
                                                      100.0 * buf[i] / max(1, total)))
    print("   total per contig {:12.0f}".format(total / n))


if __name__ == "__main__":
    main()
