"""Per-phase cycle breakdown of the fused level-0 kernel k_fast (diagnostic build with
-DWF_STAMPS: thread 0 adds s_memtime deltas after each phase's barrier).

    python scripts/fast_stamps.py [--config cfg4] [--contigs N]
Prints cycles per evaluated contig per phase.  Stamps add barriers: read the shares, never
quote this build's run time.
"""
import argparse
import ctypes as C
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from waafle_amd import build, cli, engine, lib as L, synth  # noqa: E402

NAMES = {0: "loci + LDS init", 1: "hits -> attachments (+ann pass 1)", 2: "annotation pass 2",
         3: "bitonic sort", 4: "segments scan", 5: "segment means (thread)",
         6: "multi-run segments (wave)", 7: "explain_one + meld + write"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg4")
    ap.add_argument("--contigs", type=int, default=100000)
    a = ap.parse_args()
    path = build.STAMPS_LIB
    assert os.path.exists(path), "build it first: python -m waafle_amd.build --stamps"
    L._lib = None
    so = L.load(path)
    so.wf_stamps_read_fast.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    batch, tax = synth.generate_batch(a.config, 0, a.contigs, workers=8,
                                      n_total=synth.CONFIGS[a.config]["n"])
    params = cli.param_dict(cli.parse_flags([]))
    s = engine.GpuScorer(0, mode="level0")
    s.set_taxonomy(tax)
    s.score(batch, params)
    so.wf_stamps_reset_fast()
    s.score(batch, params)
    buf = (C.c_ulonglong * 32)()
    so.wf_stamps_read_fast(buf, 32)
    n = max(1, buf[20])
    total = sum(buf[i] for i in NAMES)
    print("evaluated contigs {} / {}; attachments/contig {:.1f}, segments/contig {:.1f}, "
          "multi-run segments/contig {:.2f}".format(buf[20], a.contigs, buf[21] / n, buf[22] / n,
                                                    buf[23] / n))
    for i, name in NAMES.items():
        print("  {:2d} {:40s} {:10.0f} cycles/contig {:5.1f}%".format(
            i, name, buf[i] / n, 100.0 * buf[i] / max(total, 1)))


if __name__ == "__main__":
    main()
