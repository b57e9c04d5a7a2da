"""Print a one-line summary of each bench JSON given on the command line."""
import json
import sys

for p in sys.argv[1:]:
    try:
        d = json.load(open(p))
    except Exception as exc:   # noqa: BLE001 -- summary tool
        print(p, "unreadable:", exc)
        continue
    k2 = d.get("k2_pair_evals_per_sec")
    print("{:40s} {:9.3f} ms  {:10.4g} contigs/s  pairs/s {}  {}".format(
        p.split("/")[-1], d["ms_per_step"], d["value"],
        "{:9.3g}".format(k2) if k2 is not None else "-", d["calls"]))
    print("    kernel_ms:", {k: round(v, 3) for k, v in (d.get("kernel_ms") or {}).items()})
