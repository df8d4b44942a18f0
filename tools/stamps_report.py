#!/usr/bin/env python3
"""Phase timing from the NNRT_FIT_VARIANT=30 build (s_memrealtime stamps, 100 MHz): per kernel, per-wave phase means,
wave lifetime and start-time spread. Development tool."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
VARIANT = os.environ.get("STAMP_VARIANT", "30")
os.environ["NNRT_LIB_PATH"] = os.path.join(ROOT, "dynamicfuion_python_amd", "csrc", "variants", f"libnnrt_v{VARIANT}.so")


def report(name, st, nwaves, phases):
    st = st[: nwaves * 8].reshape(nwaves, 8).astype(np.int64)
    used = st[:, : len(phases) + 1]
    ok = (used > 0).all(1) & (np.diff(used, axis=1) >= 0).all(1)
    if not ok.any():
        print(f"{name}: no complete stamp rows; first rows:\n{st[:3]}")
        return
    st = used[ok]
    t0 = st[:, 0].min()
    rel = (st - t0) * 10 / 1000.0   # microseconds
    span = rel[:, -1].max()
    life = rel[:, -1] - rel[:, 0]
    print(f"{name}: waves {ok.sum()}/{nwaves} kernel span {span:.1f} us, wave lifetime mean {life.mean():.1f} max {life.max():.1f} us, "
          f"start spread p50 {np.percentile(rel[:, 0], 50):.1f} p90 {np.percentile(rel[:, 0], 90):.1f} max {rel[:, 0].max():.1f} us")
    blk = np.nonzero(ok)[0] // 4
    xcd = blk % 8
    ends = [rel[xcd == x, -1].max() if (xcd == x).any() else 0 for x in range(8)]
    print("    per-XCD last wave end (us): " + " ".join(f"{e:.1f}" for e in ends))
    print("    lifetime percentiles p10/p50/p90/p99: " + " ".join(f"{np.percentile(life, q):.1f}" for q in (10, 50, 90, 99)))
    d = np.diff(rel, axis=1)
    for i, ph in enumerate(phases):
        print(f"    {ph:28s} mean {d[:, i].mean():7.2f} us  p90 {np.percentile(d[:, i], 90):7.2f}")


def main():
    import torch
    import bench
    from dynamicfuion_python_amd import _native as NV
    from dynamicfuion_python_amd import synthetic as S
    from dynamicfuion_python_amd.nnrt import alignment as A
    from dynamicfuion_python_amd.nnrt import geometry as G
    from dynamicfuion_python_amd.nnrt import rendering as Rr
    torch.cuda.set_device(0)
    sc = S.make_scene("C2")
    depth = bench.render_target(sc, G, Rr)
    wf = G.HierarchicalGraphWarpField(sc.nodes, sc.coverage, False, 4, 0, G.WarpNodeCoverageComputationMethod.FIXED_NODE_COVERAGE, 1)
    ft = A.DeformableMeshToImageFitter(1, [A.IterationMode.ALL], preconditioning_dampening_factor=0.001)
    ft.prepare(wf, G.TriangleMesh(sc.points, sc.normals, sc.faces), depth, None, sc.K)
    for _ in range(5):
        wf.reset_motion()
        ft.iterate(wf, 0, 1)
    torch.cuda.synchronize()
    lib = NV.lib()
    lib.nnrt_dev_raster_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.nnrt_dev_fit_stamps.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int]
    F = len(sc.faces)
    nr = (F + 255) // 256 * 4
    buf = np.zeros(1 << 18, np.uint64)
    assert lib.nnrt_dev_raster_stamps(buf.ctypes.data, nr * 8) == 0
    report("k_raster_scatter_mesh", buf, nr, ["project+span", "bbox barrier", "lds init barrier", "pixel loop", "flush barrier", "flush atomics"])
    tiles = ((sc.W + 15) // 16) * ((sc.H + 15) // 16)
    nw = ((tiles + 7) // 8 * 8) * 4
    buf = np.zeros(1 << 17, np.uint64)
    assert lib.nnrt_dev_fit_stamps(0, buf.ctypes.data, nw * 8) == 0
    report("k_pixel_jacobians", buf, nw, ["key/face/wpos loads+resolve", "residual+Jacobians+record"])
    assert lib.nnrt_dev_fit_stamps(1, buf.ctypes.data, nw * 8) == 0
    report("k_node_reduce_grouped", buf, nw, ["key/face/anchor loads", "grouping (+ final flush)", "Jacobians (sum)", "exact sums (sum)"])


if __name__ == "__main__":
    main()
