#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc csv passes: per kernel, mean counter value per dispatch."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
acc = defaultdict(lambda: defaultdict(list))
dur = defaultdict(list)
for f in sorted(set(glob.glob(f"{root}/p*/run_counter_collection.csv") + glob.glob(f"{root}/run_counter_collection.csv") + glob.glob(f"{root}/*/run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
        acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print(f"== {k}")
    for c, v in sorted(cs.items()):
        print(f"   {c:28s} n={len(v):4d} mean={sum(v)/len(v):.4g}")
