#!/usr/bin/env python3
"""Per-kernel mean SQ counters from a rocprofv3 --pmc counter_collection.csv (development tool)."""
import collections
import csv
import sys

d = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    d[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
keys = sys.argv[2:] or ["k_fit_pixels_fused", "k_raster_scatter_mesh"]
for k, v in d.items():
    if any(x in k for x in keys):
        m = {c: sum(x) / len(x) for c, x in v.items()}
        w = m.get("SQ_WAVES", 1)
        print(k[:70])
        print("   ", {c.replace("SQ_", ""): f"{x / 1e6:.2f}M ({x / w:.0f}/wave)" for c, x in m.items()})
