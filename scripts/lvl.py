"""Per-level kernel durations of the last complete pass in a rocprofv3 kernel trace.
    python scripts/lvl.py TRACE_CSV [kernel names...]"""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
want = set(sys.argv[2:])
idx = [i for i, r in enumerate(rows) if "k_init" in r["Kernel_Name"]]
seg = rows[idx[-2]:idx[-1]]
out = []
busy = 0.0
for r in seg:
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    busy += d
    m = re.search(r"::(k_\w+)", r["Kernel_Name"])
    name = m.group(1) if m else r["Kernel_Name"][:30]
    if not want or name in want:
        out.append("%s %.0f" % (name, d))
span = (int(seg[-1]["End_Timestamp"]) - int(seg[0]["Start_Timestamp"])) / 1000
print("busy %.0f us, span %.0f us" % (busy, span))
print(" | ".join(out))
