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
    seen = sorted({c for v in acc.values() for c in v})
    cols = [c for c in COLS if c in seen] or seen        # (another counter group: its own columns)
    key = cols[0] if "SQ_WAVE_CYCLES" not in cols else "SQ_WAVE_CYCLES"
    print("rocprofv3 --pmc " + " ".join(cols) + " summed over the 4 passes (1 warmup + 3 timed) of (" + d + ")")
    print("%-30s" % "kernel" + "".join("%22s" % c for c in cols))
    for k, v in sorted(acc.items(), key=lambda x: -x[1][key])[:16]:
        print("%-30s" % k[:30] + "".join("%22.4g" % v[c] for c in cols))


if __name__ == "__main__":
    main()
