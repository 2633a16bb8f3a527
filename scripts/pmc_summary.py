"""Sum rocprofv3 --pmc counter CSVs per kernel (name substring) and per dispatch.
Usage: python scripts/pmc_summary.py <dir> [kernel-substring ...]"""
import csv
import sys
from collections import defaultdict
from pathlib import Path

root = Path(sys.argv[1])
pats = sys.argv[2:] or ["frontier_lds_kernel"]
for pat in pats:
    tot = defaultdict(float)
    disp = defaultdict(set)
    for f in sorted(root.rglob("*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            if pat not in r.get("Kernel_Name", ""):
                continue
            tot[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add(r.get("Dispatch_Id"))
    print(f"== {pat}")
    for k in sorted(tot):
        n = max(len(disp[k]), 1)
        print(f"  {k:34s} total {tot[k]:16.0f}  per-dispatch {tot[k] / n:14.0f}  ({n} dispatches)")
