"""Per-pass HBM traffic of the staged wf_score pass from two rocprofv3 --pmc runs
(FETCH_SIZE and WRITE_SIZE in KB, collected in separate runs, MI355X_MICROARCH.md HBM
section).  All kernels of the run except the one-off leaf-table build are summed and
divided by the number of passes (warmup + timed steps of the profiled bench run).

FETCH_SIZE is reported raw and doubled side by side: the guide's x2 correction is
calibrated for wide (16 B/lane) coalesced streaming reads; most loads of this pass are
4-8 B per lane or scattered, for which the counter is uncalibrated.  `hbm_bytes_per_launch`
(what bench.py reports as roofline.traffic) is the raw sum, the x2 figure is an upper
bound beside it.

    traffic.py FETCH_DIR WRITE_DIR CONFIG CONTIGS OUT.json --pass N [--dominant NAME]

`lib_sha` stamps the libwaafle_hip.so build the counters were taken on (bench.py ignores a
file of another build).
"""
import csv
import glob
import hashlib
import json
import os
import re
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOMINANT = "k_triage"   # the level-0 triage launch (round 5; before: k_wave<224, false, false>)


def lib_sha():
    with open(os.path.join(REPO, "waafle_amd", "libwaafle_hip.so"), "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()[:16]


def kname(full):
    m = re.search(r"(k_\w+(<[^>]*>)?|rocprim[:\w]*|__amd\w*)", full)
    return m.group(1) if m else full[:40]


def per_pass(d, counter, passes, dominant, by_kernel):
    """(KB per pass over the pass's kernels, dispatches, KB per pass of the dominant kernel);
    by_kernel[name][counter] collects KB per pass per kernel"""
    files = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
    assert files, "no counter_collection.csv under " + d
    acc = defaultdict(float)
    dom = 0.0
    for r in csv.DictReader(open(files[0])):
        if r["Counter_Name"] != counter:
            continue
        if "k_lut_" in r["Kernel_Name"] or not (
                "wf::" in r["Kernel_Name"] or "rocprim" in r["Kernel_Name"]):
            continue     # pass = our kernels + device sorts/scans (runtime fills/copies not counted)
        acc[r["Dispatch_Id"]] += float(r["Counter_Value"])
        by_kernel[kname(r["Kernel_Name"])][counter] += float(r["Counter_Value"]) / passes
        k = kname(r["Kernel_Name"])
        if k == dominant or k.startswith(dominant + "<"):     # (every instantiation of it)
            dom += float(r["Counter_Value"])
    assert acc, "no {} rows".format(counter)
    return sum(acc.values()) / passes, len(acc), dom / passes


def main():
    fdir, wdir, config, contigs, out = sys.argv[1:6]
    passes = int(sys.argv[sys.argv.index("--pass") + 1])
    dominant = sys.argv[sys.argv.index("--dominant") + 1] if "--dominant" in sys.argv else DOMINANT
    by_kernel = defaultdict(lambda: defaultdict(float))
    f_kb, nf, f_dom = per_pass(fdir, "FETCH_SIZE", passes, dominant, by_kernel)
    w_kb, nw, w_dom = per_pass(wdir, "WRITE_SIZE", passes, dominant, by_kernel)
    fetch_raw = f_kb * 1024.0
    write = w_kb * 1024.0
    res = {"config": config, "contigs": int(contigs),
           "kernel": "all kernels of one wf_score pass", "passes": passes,
           "dispatches_per_pass": [nf / passes, nw / passes],
           "fetch_size_kb_raw": f_kb, "write_size_kb": w_kb,
           "fetch_bytes_raw": fetch_raw, "fetch_bytes_x2": 2.0 * fetch_raw,
           "write_bytes": write,
           "hbm_bytes_raw": fetch_raw + write, "hbm_bytes_x2": 2.0 * fetch_raw + write,
           "hbm_bytes_per_launch": fetch_raw + write,
           "dominant_kernel": dominant, "lib_sha": lib_sha(),
           "per_kernel_kb": {k: dict(v) for k, v in by_kernel.items()},
           "dominant_fetch_bytes_raw": f_dom * 1024.0, "dominant_write_bytes": w_dom * 1024.0,
           "dominant_hbm_bytes_raw": (f_dom + w_dom) * 1024.0,
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate runs ({}, {})".format(
               fdir, wdir)}
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
