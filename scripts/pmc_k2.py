"""VALU instructions of the explain_two kernels (k_decide<3...>, k_big_sparse, k_dump_sparse, k_decide_big)
per cfg5 pass, from a rocprofv3 --pmc SQ_INSTS_VALU ... run of bench.py on the cfg5
6,250-contig share: the `valu` block of bench.py's k2 leg (--k2-pmc-json).

    pmc_k2.py PMC_DIR PASSES CONTIGS OUT.json
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

# wave64 VALU issue: each SIMD-32 takes 2 cycles per wave-instruction (MI355X_MICROARCH.md)
VALU_PEAK = 256 * 4 * 2.4e9 / 2


def main():
    d, passes, contigs, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    f = glob.glob(d + "/**/*counter_collection.csv", recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_decide_big|k_big_sparse|k_dump_sparse|k_decide<3[^>]*>)", r["Kernel_Name"])
        if m:
            acc[m.group(1)][r["Counter_Name"]] += float(r["Counter_Value"])
    insts = sum(v["SQ_INSTS_VALU"] for v in acc.values()) / passes
    res = {"contigs": contigs, "passes": passes, "valu_insts_per_pass": insts, "lib_sha": lib_sha(),
           "salu_insts_per_pass": sum(v["SQ_INSTS_SALU"] for v in acc.values()) / passes,
           "per_kernel": {k: {c: x / passes for c, x in v.items()} for k, v in acc.items()},
           "valu_peak_insts_per_s": VALU_PEAK,
           "source": "rocprofv3 --pmc SQ_* over bench.py --config cfg5 --contigs {} ({})".format(contigs, d)}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
