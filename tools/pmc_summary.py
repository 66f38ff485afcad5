"""Summarise PMC counters per kernel name (sum over dispatches) from tools/pmc_fused.sh output."""
import csv
import glob
import sys
from collections import defaultdict

agg = defaultdict(lambda: defaultdict(float))
n = defaultdict(set)
for f in glob.glob(f"{sys.argv[1]}/pass*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        key = ("mrf32" if "Li32ELi512" in k else "mrf64" if "Li64ELi256" in k else
               "conv_gemm" if "conv_gemm" in k else None)
        if key is None:
            continue
        agg[key][r["Counter_Name"]] += float(r["Counter_Value"])
        n[key].add(r["Dispatch_Id"])
for key, c in agg.items():
    print(f"== {key} ({len(n[key])} dispatches)")
    for name in sorted(c):
        print(f"   {name:28s} {c[name]:.4g}")
