"""Per-launch HBM traffic from two rocprofv3 --pmc passes (FETCH_SIZE and WRITE_SIZE in
KB, collected in separate runs).  On gfx950 FETCH_SIZE reports half the bytes of wide
coalesced reads (MI355X_MICROARCH.md, HBM section), so it is doubled.

    traffic.py FETCH_DIR WRITE_DIR CONFIG CONTIGS OUT.json [--pass N]

Default: the fused tier-1 kernel, averaged per dispatch.  --pass N: the staged form, all
kernels of the run (except the one-off leaf-table build) summed and divided by N passes
(warmup + timed steps of the profiled bench run)."""
import csv
import glob
import json
import sys
from collections import defaultdict


def per_dispatch(d, counter, kernel="k_contig_lds<128", passes=None):
    files = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    assert files, "no counter_collection.csv under " + d
    acc = defaultdict(float)
    for r in csv.DictReader(open(files[0])):
        if r["Counter_Name"] != counter:
            continue
        if passes is None and kernel not in r["Kernel_Name"]:
            continue
        if passes is not None and ("k_lut_" in r["Kernel_Name"] or not (
                "wf::" in r["Kernel_Name"] or "rocprim" in r["Kernel_Name"])):
            continue     # pass = our kernels + device sorts/scans (runtime fills/copies not counted)
        acc[r["Dispatch_Id"]] += float(r["Counter_Value"])
    assert acc, "no {} rows".format(counter)
    if passes is not None:
        return sum(acc.values()) / passes, len(acc)
    return sum(acc.values()) / len(acc), len(acc)


def main():
    fdir, wdir, config, contigs, out = sys.argv[1:6]
    passes = int(sys.argv[sys.argv.index("--pass") + 1]) if "--pass" in sys.argv else None
    f_kb, nf = per_dispatch(fdir, "FETCH_SIZE", passes=passes)
    w_kb, nw = per_dispatch(wdir, "WRITE_SIZE", passes=passes)
    fetch = 2.0 * f_kb * 1024.0      # gfx950 correction: FETCH_SIZE counts 64 B per 128-B request
    write = w_kb * 1024.0
    res = {"config": config, "contigs": int(contigs),
           "mode": "staged" if passes else "fused",
           "kernel": "all kernels of one wf_score pass" if passes else "k_contig_lds<128,false>",
           "passes": passes,
           "dispatches": [nf, nw], "fetch_size_kb_raw": f_kb, "write_size_kb": w_kb,
           "fetch_bytes_corrected": fetch, "write_bytes": write,
           "hbm_bytes_per_launch": fetch + write}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
