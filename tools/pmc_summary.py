#!/usr/bin/env python3
"""Average each PMC counter per dispatch for every kernel in rocprofv3 counter-collection csv files."""
import collections
import csv
import glob
import sys

pat = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_sq/**/*counter_collection.csv"
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for path in glob.glob(pat, recursive=True):
    for r in csv.DictReader(open(path)):
        acc[r["Kernel_Name"][:70]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    n = max(len(v) for v in cs.values())
    if n < 5:
        continue
    print(k)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v) / len(v):16.1f}")
