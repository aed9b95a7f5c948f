#!/usr/bin/env python3
"""Mean of every PMC counter per kernel over rocprofv3 counter_collection.csv files:
pmc_by_kernel.py <substring filter> <csv> [<csv> ...]"""
import csv, collections, sys
pat = sys.argv[1]
vals = collections.defaultdict(list)
dur = collections.defaultdict(list)
for path in sys.argv[2:]:
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        if pat not in k:
            continue
        k = k[:90]
        vals[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
kern = sorted({k for k, _ in vals})
for k in kern:
    print(k)
    for (kk, c), v in sorted(vals.items()):
        if kk == k:
            print(f"   {c:32s} {sum(v) / len(v):16.1f}  (n={len(v)})")
