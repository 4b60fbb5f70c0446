#!/usr/bin/env python3
"""Per-kernel averages of the tools/pmc_multi.sh passes: python3 pmc_multi_summary.py gpurun_out"""
import csv
import sys
from collections import defaultdict
from pathlib import Path

root = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out")
acc = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for d in sorted(root.glob("pmc_*")):
    if not d.is_dir():
        continue
    for f in d.rglob("*counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].split("::")[-1]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in acc.items():
    print(k)
    for n, v in sorted(c.items()):
        print(f"    {n:36s} {sum(v) / len(v):16.1f}")
