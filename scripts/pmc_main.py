"""VALU side of the main line's roofline: SQ_INSTS_VALU per cfg4 pass, over every kernel of
the pass and for the dominant kernel (the first wave form's level-0 launch), from a
rocprofv3 --pmc SQ_* run of bench.py (scripts/pmc_r4.sh).  bench.py reads the output as
--valu-pmc-json and divides by the pass / kernel times it measures itself.

    pmc_main.py PMC_DIR PASSES CONFIG CONTIGS OUT.json [DOMINANT]
"""
import collections
import csv
import glob
import json
import os
import re
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from traffic import lib_sha  # noqa: E402

# wave64 VALU issue: each SIMD-32 takes 2 cycles per wave-instruction (MI355X_MICROARCH.md):
# 256 CUs x 4 SIMDs x 2.4 GHz / 2
VALU_PEAK = 256 * 4 * 2.4e9 / 2
DOMINANT = "k_triage"


def main():
    d, passes, config, contigs, out = sys.argv[1], int(sys.argv[2]), sys.argv[3], int(sys.argv[4]), sys.argv[5]
    dominant = sys.argv[6] if len(sys.argv) > 6 else DOMINANT
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+(<[^>]*>)?|rocprim[:\w]*|__amd\w*)", r["Kernel_Name"])
        acc[m.group(1) if m else r["Kernel_Name"][:40]][r["Counter_Name"]] += float(r["Counter_Value"])
    per = {k: {c: x / passes for c, x in v.items()} for k, v in acc.items()}
    total = sum(v.get("SQ_INSTS_VALU", 0.0) for v in per.values())
    dom = collections.defaultdict(float)            # every instantiation of the dominant kernel
    for k, v in per.items():
        if k == dominant or k.startswith(dominant + "<"):
            for c, x in v.items():
                dom[c] += x
    res = {"config": config, "contigs": contigs, "passes": passes,
           "valu_insts_per_pass": total,
           "salu_insts_per_pass": sum(v.get("SQ_INSTS_SALU", 0.0) for v in per.values()),
           "dominant_kernel": dominant, "lib_sha": lib_sha(),
           "dominant_valu_insts_per_pass": dom.get("SQ_INSTS_VALU", 0.0),
           "dominant_wait_frac": (dom.get("SQ_WAIT_ANY", 0.0) / dom["SQ_WAVE_CYCLES"])
           if dom.get("SQ_WAVE_CYCLES") else None,
           "per_kernel": per, "valu_peak_insts_per_s": VALU_PEAK,
           "source": "rocprofv3 --pmc SQ_* over bench.py --config {} ({}), {} passes".format(config, d, passes)}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1, sort_keys=True)
    print(json.dumps({k: v for k, v in res.items() if k != "per_kernel"}))


if __name__ == "__main__":
    main()
