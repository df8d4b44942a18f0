#!/usr/bin/env python3
"""HBM traffic per launch of the GN-iteration kernels from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; csv).

gfx950 corrections (MI355X_MICROARCH.md "HBM"): FETCH_SIZE counts KiB at half the bytes of a wide coalesced read
(128-B requests tallied at 64 B) -> doubled; WRITE_SIZE counts KiB exactly. traffic = (2 * FETCH_SIZE + WRITE_SIZE) *
1024 bytes, averaged over the kernel's dispatches."""
import argparse
import csv
import glob
import json
import os


def per_dispatch(path_glob, counter, kernel_prefix):
    vals = []
    for path in glob.glob(path_glob, recursive=True):
        for r in csv.DictReader(open(path)):
            if r["Counter_Name"] == counter and any(k in r["Kernel_Name"] for k in kernel_prefix.split("|")):
                vals.append(float(r["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", default="gpurun_out/pmc_fetch/**/*counter_collection.csv")
    ap.add_argument("--write", default="gpurun_out/pmc_write/**/*counter_collection.csv")
    ap.add_argument("--kernels", nargs="+", default=["k_fit_pixels_fused<0, 4", "k_raster_scatter_mesh",
                                                      "k_warp_mesh_quad|k_warp_mesh_vertex", "k_solve_update_lanes<0"])
    ap.add_argument("--workload", required=True, help="bench.py config.workload string the passes ran")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    kernels = {}
    for sym in a.kernels:
        f = per_dispatch(a.fetch, "FETCH_SIZE", sym)
        w = per_dispatch(a.write, "WRITE_SIZE", sym)
        if not f or not w:
            raise SystemExit(f"no dispatches of {sym}: fetch {len(f)} write {len(w)}")
        fetch_kib = sum(f) / len(f)
        write_kib = sum(w) / len(w)
        # "a|b": the kernel under either name (the warp's launch path depends on the mesh size), keyed by the first
        kernels[sym.split("|")[0].split("<")[0]] = {"kernel_symbol": sym, "dispatches": [len(f), len(w)], "fetch_size_kib": fetch_kib,
                                      "write_size_kib": write_kib, "hbm_bytes_per_launch": (2 * fetch_kib + write_kib) * 1024.0}
    out = {"workload": a.workload, "kernels": kernels,
           "formula": "(2*FETCH_SIZE + WRITE_SIZE) * 1024 (gfx950 FETCH_SIZE half-count correction)"}
    text = json.dumps(out, indent=1)
    print(text)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write(text + "\n")


if __name__ == "__main__":
    main()
