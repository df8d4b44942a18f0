#!/usr/bin/env python3
"""Phase timing of the dense-corner diagonal factor kernel (k_chol_diag) from the NNRT_FIT_VARIANT=30 build
(s_memrealtime stamps, 100 MHz) on one C5 ARAP iteration. Development tool."""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ["NNRT_LIB_PATH"] = os.path.join(ROOT, "dynamicfuion_python_amd", "csrc", "variants", "libnnrt_v30.so")


def main():
    import torch
    import bench
    from dynamicfuion_python_amd import _native as NV
    from dynamicfuion_python_amd import synthetic as S
    from dynamicfuion_python_amd.nnrt import alignment as A
    from dynamicfuion_python_amd.nnrt import geometry as G
    from dynamicfuion_python_amd.nnrt import rendering as Rr
    torch.cuda.set_device(0)
    sc = S.make_scene(sys.argv[1] if len(sys.argv) > 1 else "C5", hierarchy_builder=S.native_hierarchy_builder)
    depth = bench.render_target(sc, G, Rr)
    wf = G.HierarchicalGraphWarpField(sc.nodes, sc.coverage, False, 4, 0, G.WarpNodeCoverageComputationMethod.FIXED_NODE_COVERAGE, sc.layer_count)
    ft = A.DeformableMeshToImageFitter(1, [A.IterationMode.ALL], preconditioning_dampening_factor=0.001)
    ft.prepare(wf, G.TriangleMesh(sc.points, sc.normals, sc.faces), depth, None, sc.K)
    for _ in range(3):
        wf.reset_motion()
        ft.iterate(wf, 0, 1)
    torch.cuda.synchronize()
    lib = NV.lib()
    lib.nnrt_dev_chol_stamps.argtypes = [ctypes.c_void_p]
    buf = np.zeros((64, 8), np.uint64)
    assert lib.nnrt_dev_chol_stamps(buf.ctypes.data) == 0
    rows = buf[(buf[:, 3] > 0)].astype(np.int64)
    d = np.diff(rows[:, :4], axis=1) * 10 / 1000.0
    names = ["stage (update tiles)", "registers", "elimination"]
    print(f"k_chol_step diagonal workgroup: {len(rows)} blocks")
    for i, n in enumerate(names):
        print(f"    {n:16s} mean {d[:, i].mean():8.2f} us  max {d[:, i].max():8.2f}")
    clk = (rows[:, 7] - rows[:, 4]) / ((rows[:, 3] - rows[:, 0]) * 10e-9) / 1e9
    print(f"    s_memtime rate over the workgroup's span: mean {clk.mean():.3f} GHz (min {clk.min():.3f}, max {clk.max():.3f})")
    for k in (0, 1, len(rows) // 2, len(rows) - 1):
        print(f"    k={k}: " + " ".join(f"{x:7.2f}" for x in d[k]))

if __name__ == "__main__":
    main()
