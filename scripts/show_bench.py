"""Print a one-line summary of each bench JSON given on the command line."""
import json
import sys

for p in sys.argv[1:]:
    try:
        d = json.load(open(p))
    except Exception as exc:   # noqa: BLE001 -- summary tool
        print(p, "unreadable:", exc)
        continue
    print("{:40s} {:9.3f} ms  {:10.4g} contigs/s  pairs/s {:9.3g}  {}".format(
        p.split("/")[-1], d["ms_per_step"], d["value"], d["k2_pair_evals_per_sec"], d["calls"]))
