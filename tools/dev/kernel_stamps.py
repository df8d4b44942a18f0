"""Per-wave timelines of k_warp_mesh_quad and k_raster_scatter_mesh (development; needs tools/dev/libnnrt_kstamps.so:
tools/dev/stamps_build.sh NNRT_KERNEL_STAMPS tools/dev/libnnrt_kstamps.so). One C2 GN iteration from the mid-motion
state (eager launches); per kernel: launch span, wave start ramp, lifetimes, SIMD placement (100 MHz clock)."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["NNRT_LIB_PATH"] = os.path.join(ROOT, "tools", "dev", "libnnrt_kstamps.so")
sys.path[:0] = [ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from dynamicfuion_python_amd import _native as NV, synthetic as S  # noqa: E402
from dynamicfuion_python_amd.nnrt import alignment as A, geometry as G, rendering as Rr  # noqa: E402
import bench  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C2"
sc = S.make_scene(name, hierarchy_builder=S.native_hierarchy_builder)
lib = NV.lib()
depth = bench.render_target(sc, G, Rr)
wf = G.HierarchicalGraphWarpField(sc.nodes, sc.coverage, False, 4, 0, G.WarpNodeCoverageComputationMethod.FIXED_NODE_COVERAGE, sc.layer_count)
R, t = sc.partial_motion(0.5)
wf.set_node_rotations(R)
wf.set_node_translations(t)
ft = A.DeformableMeshToImageFitter(1, [A.IterationMode.ALL], preconditioning_dampening_factor=0.001, use_hip_graph=0)
ft.prepare(wf, G.TriangleMesh(sc.points, sc.normals, sc.faces), depth, None, sc.K)
ft.snapshot_motion(wf)
for _ in range(5):
    ft.iterate_from_snapshot(wf, 0, 1)
torch.cuda.synchronize()
for kname, waves in (("warp", -(-4 * len(sc.points) // 256) * 4), ("raster", -(-len(sc.faces) // 32))):
    buf = np.zeros((16384, 8 if kname == "raster" else 4), np.uint64)
    fn = getattr(lib, f"nnrt_dev_{kname}_stamps")
    fn.argtypes = [ctypes.c_void_p]
    assert fn(buf.ctypes.data) == 0
    st = buf[:waves].astype(np.int64)
    t0 = st[:, 0].min()
    start, end = (st[:, 0] - t0) * 10, (st[:, 2] - t0) * 10
    life = end - start
    hw, xcc = st[:, 3] & 0xFFFFFFFF, st[:, 3] >> 32
    key = ((xcc * 4 + ((hw >> 13) & 3)) * 16 + ((hw >> 8) & 15)) * 4 + ((hw >> 4) & 3)
    us, inv, cnt = np.unique(key, return_inverse=True, return_counts=True)
    print(f"{kname}: {waves} waves, span {end.max() / 1e3:.2f} us; start: median {np.median(start) / 1e3:.2f} p90 {np.percentile(start, 90) / 1e3:.2f} "
          f"max {start.max() / 1e3:.2f}; lifetime: mean {life.mean() / 1e3:.2f} median {np.median(life) / 1e3:.2f} p90 {np.percentile(life, 90) / 1e3:.2f} "
          f"max {life.max() / 1e3:.2f}; end: median {np.median(end) / 1e3:.2f} p90 {np.percentile(end, 90) / 1e3:.2f}; waves per SIMD max {cnt.max()} "
          f"SIMDs {len(us)}")
    if kname == "raster":
        mid = (st[:, 1] - t0) * 10
        print(f"  raster setup (projection) mean {(mid - start).mean() / 1e3:.2f} us, scatter mean {(end - mid).mean() / 1e3:.2f} us")
        rows, tile, pxs, pxm = st[:, 4], st[:, 5] >> 1, st[:, 6], st[:, 7]
        staged = (st[:, 5] & 1).astype(bool)
        busy = rows > 0
        print(f"  waves with rows {busy.sum()}; rows/wave mean {rows[busy].mean():.1f} p90 {np.percentile(rows[busy], 90):.0f} max {rows.max()}; "
              f"two+ row rounds {(rows > 64).sum()}; unstaged {(busy & ~staged).sum()}; pixels/wave mean {pxs[busy].mean():.0f} max {pxs.max()}; "
              f"max pixels per lane mean {pxm[busy].mean():.1f} p90 {np.percentile(pxm[busy], 90):.0f} max {pxm.max()}")
        slow = life >= np.percentile(life, 90)
        for lab, m in (("slowest 10%", slow), ("rest", busy & ~slow)):
            print(f"  {lab}: lifetime {life[m].mean() / 1e3:.2f} us, setup {(mid - start)[m].mean() / 1e3:.2f}, rows {rows[m].mean():.1f}, "
                  f"rounds {np.ceil(rows[m] / 64).mean():.2f}, pixels {pxs[m].mean():.0f}, max px/lane {pxm[m].mean():.1f}, tile {tile[m].mean():.0f}, "
                  f"unstaged {(~staged[m]).mean():.2f}, start {start[m].mean() / 1e3:.2f}")
        cs = np.corrcoef(np.stack([life, rows, pxs, pxm, tile, start]).astype(float))[0]
        print("  corr(lifetime, [rows, pixels, max px/lane, tile, start]):", [round(float(c), 2) for c in cs[1:]])
    hist, edges = np.histogram(start / 1e3, bins=10)
    print("  start histogram (us):", [(round(float(e), 2), int(h)) for e, h in zip(edges, hist)])
