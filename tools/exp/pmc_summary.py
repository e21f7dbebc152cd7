"""Summarise rocprofv3 --pmc CSV passes (gpurun_out/pmcf/p*/.../*counter_collection.csv):
mean counter value per dispatch, per kernel.  Usage: python tools/exp/pmc_summary.py DIR"""
import csv, glob, os, sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcf"
acc = defaultdict(lambda: defaultdict(list))
for f in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "?")
        acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in acc.items():
    print(k[:110])
    for c in sorted(cs):
        v = cs[c]
        print(f"   {c:32s} {sum(v) / len(v):.4g}   (n={len(v)})")
