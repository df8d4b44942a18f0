"""Brackets the offset C between stamp ticks (x10 ns) and the rocprofv3 kernel trace (ns) from the last launch of each
stamped kernel: head_k = first_k + C - begin_k >= 0 and tail_k = end_k - last_k - C >= 0 for every k (development)."""
import csv
import json
import sys

st = json.load(open(sys.argv[1]))
rows = list(csv.DictReader(open(sys.argv[2])))
names = {"warp": "k_warp_mesh_quad", "raster": "k_raster_scatter_mesh", "fit": "k_fit_pixels_fused"}
lo, hi, rec = -1e30, 1e30, {}
for k, sub in names.items():
    ks = [r for r in rows if sub in r["Kernel_Name"]]
    r = max(ks, key=lambda r: int(r["Start_Timestamp"]))
    b, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    f, l = st[k]["first_start"] * 10, st[k]["last_end"] * 10
    rec[k] = (b, e, f, l)
    lo, hi = max(lo, b - f), min(hi, e - l)
    print(f"{k}: trace {(e - b) / 1e3:.2f} us, waves {(l - f) / 1e3:.2f} us")
print(f"offset bracket width {(hi - lo) / 1e3:.2f} us")
for C, tag in ((lo, "C = lower bound"), (hi, "C = upper bound")):
    print(tag + ": " + "; ".join(f"{k} head {(f + C - b) / 1e3:.2f} tail {(e - l - C) / 1e3:.2f} us" for k, (b, e, f, l) in rec.items()))
