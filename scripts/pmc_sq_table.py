"""Per-kernel SQ counter table of a rocprofv3 --pmc run (one wf_score pass).

    python scripts/pmc_sq_table.py PMC_DIR > table.txt
"""
import collections
import csv
import glob
import re
import sys

COLS = ["SQ_WAVES", "SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES",
        "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"]


def main():
    d = sys.argv[1]
    files = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(files[0])):
        m = re.search(r"(k_\w+(<[^>]*>)?)", r["Kernel_Name"])
        acc[m.group(1) if m else r["Kernel_Name"][:30]][r["Counter_Name"]] += float(r["Counter_Value"])
    print("rocprofv3 --pmc " + " ".join(COLS) + " summed over the 4 passes (1 warmup + 3 timed) of (" + d + ")")
    print("%-24s" % "kernel" + "".join("%20s" % c for c in COLS))
    for k, v in sorted(acc.items(), key=lambda x: -x[1]["SQ_WAVE_CYCLES"])[:14]:
        print("%-24s" % k[:24] + "".join("%20.4g" % v[c] for c in COLS))


if __name__ == "__main__":
    main()
