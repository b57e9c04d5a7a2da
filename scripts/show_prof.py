"""Summarise a rocprofv3 kernel_stats.csv: kernel, calls, average and total time."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows:
    n = r["Name"]
    m = re.search(r"(k_[a-z_0-9]+)", n)
    if "rocprim" in n:
        k = re.search(r"(radix_sort_onesweep_iteration|radix_sort_onesweep_global_offsets|"
                      r"radix_sort_block_sort|merge_sort_block_merge|merge_sort_block_sort|"
                      r"scan_impl|init_lookback_scan_state|reduce)", n)
        short = "rocprim:" + (k.group(1) if k else "?")
    elif m:
        short = m.group(1) + ("<" + re.search(r"<([^>]*)>", n).group(1) + ">" if "<" in n.split("(")[0] else "")
    else:
        short = n[:40]
    print("{:45s} calls {:>5} avg_us {:9.1f} total_ms {:8.2f} {:5.1f}%".format(
        short, r["Calls"], float(r["AverageNs"]) / 1e3, float(r["TotalDurationNs"]) / 1e6,
        100 * float(r["TotalDurationNs"]) / tot))
