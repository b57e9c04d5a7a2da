"""The isolated explain_two (k2) kernel's roofline at cfg5, for bench.py's `k2` key.

    k2_roofline.py BENCH.json KERNEL_STATS.csv PASSES OUT.json [--pmc PMC_DIR PMC_PASSES]

BENCH.json is the bench line of the profiled run (its `k2_counts`: B_k2 = sum P_pot*G*8,
OPS_pair = sum pairs*G); KERNEL_STATS.csv is rocprofv3's kernel_stats of the
same run (PASSES = warmup + steps).  k_decide<3,...> is the launch that runs explain_two
(orgscorer.py:599-619) plus meld_two / the LGT checks for the contigs it holds.  PMC_DIR
(optional) is a --pmc SQ_INSTS_VALU SQ_WAVES run: VALU instructions per k2 launch.
"""
import csv
import glob
import json
import re
import sys

VALU_PEAK = 256 * 4 * 2.4e9          # wave-instructions/s: 256 CUs x 4 SIMDs x 2.4 GHz
FP64_OPS_PEAK = 3.93e13              # simple fp64/int lane-ops/s
HBM_PEAK = 8.0e12


def main():
    bench_p, stats_p, passes, out_p = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    pmc = pmc_passes = None
    if "--pmc" in sys.argv:
        i = sys.argv.index("--pmc")
        pmc, pmc_passes = sys.argv[i + 1], int(sys.argv[i + 2])
    bench = json.loads(open(bench_p).read().strip().splitlines()[-1])
    kc = bench["k2_counts"]
    # explain_two runs in k_decide<3> (LDS arena) and, for contigs whose arena exceeds
    # it (cfg5: P_pot ~ 5,000 rows of 20 loci), in k_decide_big (HBM slots)
    rows = [r for r in csv.DictReader(open(stats_p))
            if "k_decide<3" in r["Name"] or "k_decide_big" in r["Name"]]
    assert rows, "no k_decide<3> / k_decide_big rows in " + stats_p
    tot_ns = sum(float(r["TotalDurationNs"]) for r in rows)
    calls = sum(int(r["Calls"]) for r in rows)
    t = tot_ns * 1e-9 / passes
    res = {"config": bench["config"]["workload"], "kernel": "k_decide<3> + k_decide_big (explain_two + meld_two)",
           "per_kernel_s_per_pass": {re.search(r"k_decide\w*(<[^>]*>)?", r["Name"]).group(0):
                                     float(r["TotalDurationNs"]) * 1e-9 / passes for r in rows},
           "launches_per_pass": calls / passes, "kernel_s_per_pass": t,
           "b_k2_bytes": kc["b_k2_bytes"], "ops_pair": kc["ops_pair"],
           "pairs_reference_equivalent": kc["pairs"], "p_pot_max": kc["p_pot_max"],
           "contigs_explain_two": kc["contigs_explain_two"],
           "hbm": {"achieved_GBs": kc["b_k2_bytes"] / t / 1e9, "peak_GBs": HBM_PEAK / 1e9,
                   "frac": kc["b_k2_bytes"] / t / HBM_PEAK},
           "ops_reference_equivalent": {"achieved_per_s": kc["ops_pair"] / t,
                                        "peak_per_s": FP64_OPS_PEAK,
                                        "frac": kc["ops_pair"] / t / FP64_OPS_PEAK},
           "source": {"bench": bench_p, "kernel_stats": stats_p, "passes": passes}}
    # contigs that fit the wave kernels (<= 512 hits) run explain_two inside k_wave<CAP,true>
    # together with their level-0 evaluation; reported beside, not folded into, the k2 time
    full = [r for r in csv.DictReader(open(stats_p)) if "k_wave<" in r["Name"] and ", true>" in r["Name"]]
    if full:
        res["wave_form_s_per_pass"] = sum(float(r["TotalDurationNs"]) for r in full) * 1e-9 / passes
    if pmc:
        files = glob.glob(pmc + "/**/*counter_collection.csv", recursive=True)
        valu = waves = 0.0
        for r in csv.DictReader(open(files[0])):
            if "k_decide<3" not in r["Kernel_Name"] and "k_decide_big" not in r["Kernel_Name"]:
                continue
            if r["Counter_Name"] == "SQ_INSTS_VALU":
                valu += float(r["Counter_Value"])
            elif r["Counter_Name"] == "SQ_WAVES":
                waves += float(r["Counter_Value"])
        v = valu / pmc_passes
        res["valu"] = {"insts_per_pass": v, "waves_per_pass": waves / pmc_passes,
                       "achieved_insts_per_s": v / t, "peak_insts_per_s": VALU_PEAK,
                       "frac": v / t / VALU_PEAK, "source": pmc}
    json.dump(res, open(out_p, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
