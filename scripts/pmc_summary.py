"""Per-dispatch, per-contig averages of rocprofv3 counter_collection.csv files.
Usage: pmc_summary.py DIR [DIR...] [--contigs N] [--kernel SUBSTR]"""
import csv
import glob
import sys
from collections import defaultdict

args = sys.argv[1:]
contigs = 10000
kern = "k_contig_lds<128"
if "--contigs" in args:
    i = args.index("--contigs"); contigs = int(args[i + 1]); del args[i:i + 2]
if "--kernel" in args:
    i = args.index("--kernel"); kern = args[i + 1]; del args[i:i + 2]
for d in args:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        acc = defaultdict(float)
        disp = defaultdict(set)
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                acc[r["Counter_Name"]] += float(r["Counter_Value"])
                disp[r["Counter_Name"]].add(r["Dispatch_Id"])
        for k, v in sorted(acc.items()):
            nd = len(disp[k])
            print("{:32s} per dispatch {:16.0f}  per contig {:12.1f}".format(k, v / nd, v / nd / contigs))
