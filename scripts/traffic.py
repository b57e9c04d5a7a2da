"""Per-launch HBM traffic of the tier-1 contig kernel from two rocprofv3 --pmc passes
(FETCH_SIZE and WRITE_SIZE in KB, collected in separate runs).  On gfx950 FETCH_SIZE
reports half the bytes of wide coalesced reads (MI355X_MICROARCH.md, HBM section), so it
is doubled.  Usage: traffic.py FETCH_DIR WRITE_DIR CONFIG CONTIGS OUT.json"""
import csv
import glob
import json
import sys
from collections import defaultdict


def per_dispatch(d, counter, kernel="k_contig_lds<128"):
    files = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    assert files, "no counter_collection.csv under " + d
    acc = defaultdict(float)
    for r in csv.DictReader(open(files[0])):
        if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]:
            acc[r["Dispatch_Id"]] += float(r["Counter_Value"])
    assert acc, "no {} rows for {}".format(counter, kernel)
    return sum(acc.values()) / len(acc), len(acc)


def main():
    fdir, wdir, config, contigs, out = sys.argv[1:6]
    f_kb, nf = per_dispatch(fdir, "FETCH_SIZE")
    w_kb, nw = per_dispatch(wdir, "WRITE_SIZE")
    fetch = 2.0 * f_kb * 1024.0      # gfx950 correction: FETCH_SIZE counts 64 B per 128-B request
    write = w_kb * 1024.0
    res = {"config": config, "contigs": int(contigs), "kernel": "k_contig_lds<128,false>",
           "dispatches": [nf, nw], "fetch_size_kb_raw": f_kb, "write_size_kb": w_kb,
           "fetch_bytes_corrected": fetch, "write_bytes": write,
           "hbm_bytes_per_launch": fetch + write}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
