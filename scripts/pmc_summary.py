#!/usr/bin/env python3
"""Aggregate rocprofv3 counter_collection.csv files: per kernel, mean counter value per dispatch."""
import csv
import glob
import sys
from collections import defaultdict

vals = defaultdict(lambda: defaultdict(list))
for path in sys.argv[1:]:
    for f in glob.glob(path, recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = row["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
                if k.startswith("void "):
                    k = k[5:]
                vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k, cs in vals.items():
    if "mxs" not in k:
        continue
    print(f"## {k}")
    for c, v in sorted(cs.items()):
        print(f"  {c:32s} {sum(v)/len(v):16.1f}   (n={len(v)})")
