"""Per-kernel table of rocprofv3 --pmc counter_collection.csv files (summed over dispatches),
with each kernel's duration from the same run's kernel trace.

    pmc_table.py DIR [DIR ...]
"""
import collections
import csv
import glob
import re
import sys


def short(n):
    m = re.search(r"(k_[a-z_0-9]+)(<[^>(]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:30]


res = collections.defaultdict(lambda: collections.defaultdict(float))
dur = collections.defaultdict(float)
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            res[short(r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
    for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
        if d == sys.argv[1]:
            for r in csv.DictReader(open(f)):
                dur[short(r["Kernel_Name"])] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
for k, v in sorted(res.items(), key=lambda x: -dur.get(x[0], 0))[:6]:
    print("{}  {:.2f} ms".format(k, dur.get(k, 0)))
    for c, x in sorted(v.items()):
        print("    {:24s} {:.4g}".format(c, x))
