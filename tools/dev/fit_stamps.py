"""Per-wave timeline of k_fit_pixels_fused (development; needs tools/dev/libnnrt_fitstamps.so:
tools/dev/stamps_build.sh NNRT_FIT_STAMPS tools/dev/libnnrt_fitstamps.so). Runs C2 GN iterations from the mid-motion
state (eager launches) and summarises the last launch: dispatch ramp, wave lifetimes (pass 1 / pass 2), the tail, and
the load per CU / SIMD (100 MHz clock: 10 ns ticks)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["NNRT_LIB_PATH"] = os.path.join(ROOT, "tools", "dev", "libnnrt_fitstamps.so")
sys.path[:0] = [ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from dynamicfuion_python_amd import _native as NV, synthetic as S  # noqa: E402
from dynamicfuion_python_amd.nnrt import alignment as A, geometry as G, rendering as Rr  # noqa: E402
sys.path.insert(0, ROOT)
import bench  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C2"
out_json = sys.argv[2] if len(sys.argv) > 2 else None
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
buf = np.zeros((16384, 4), np.uint64)
fn = getattr(lib, "nnrt_dev_fit_stamps")
fn.argtypes = [ctypes.c_void_p]
assert fn(buf.ctypes.data) == 0
tiles = ((sc.W + 15) // 16) * ((sc.H + 15) // 16)
nw = ((tiles + 7) // 8) * 8 * 4
st = buf[:nw].astype(np.int64)
t0 = st[:, 0].min()
start, mid, end = (st[:, 0] - t0) * 10, (st[:, 1] - t0) * 10, (st[:, 2] - t0) * 10   # ns
hw = st[:, 3] & 0xFFFFFFFF
xcc = st[:, 3] >> 32
simd = (hw >> 4) & 3
cu = (hw >> 8) & 15
se = (hw >> 13) & 3
life, p1, p2 = end - start, mid - start, end - mid
span = end.max()
print(f"{name}: {nw} waves, span {span / 1e3:.2f} us; start ramp: median {np.median(start) / 1e3:.2f} us, p90 {np.percentile(start, 90) / 1e3:.2f}, max {start.max() / 1e3:.2f}")
print(f"lifetime us: mean {life.mean() / 1e3:.2f} median {np.median(life) / 1e3:.2f} p90 {np.percentile(life, 90) / 1e3:.2f} max {life.max() / 1e3:.2f}; pass1 mean {p1.mean() / 1e3:.2f} max {p1.max() / 1e3:.2f}; pass2 mean {p2.mean() / 1e3:.2f} max {p2.max() / 1e3:.2f}")
print(f"end: median {np.median(end) / 1e3:.2f} p90 {np.percentile(end, 90) / 1e3:.2f} p99 {np.percentile(end, 99) / 1e3:.2f} max {end.max() / 1e3:.2f} us")
simd_key = ((xcc * 4 + se) * 16 + cu) * 4 + simd
us, inv, cnt = np.unique(simd_key, return_inverse=True, return_counts=True)
last = np.zeros(len(us))
np.maximum.at(last, inv, end / 1e3)
for c in sorted(set(cnt)):
    m = cnt == c
    print(f"SIMDs with {c} waves: {m.sum()}, their last end: mean {last[m].mean():.1f} max {last[m].max():.1f} us")
hist, edges = np.histogram(life / 1e3, bins=12)
print("lifetime histogram (us):", [(round(float(e), 1), int(h)) for e, h in zip(edges, hist)])
if out_json:
    json.dump(dict(start=start.tolist(), mid=mid.tolist(), end=end.tolist(), hw=hw.tolist(), xcc=xcc.tolist()), open(out_json, "w"))

# pass-2 phase split (shader cycles per wave: group, gather + Jacobians, sums; chunk count)
fnp = getattr(lib, "nnrt_dev_fit_phases", None)
if fnp is not None:
    fnp.argtypes = [ctypes.c_void_p]
    ph = np.zeros((16384, 8), np.uint64)
    assert fnp(ph.ctypes.data) == 0
    ph = ph[:nw].astype(np.float64)
    busy = ph[:, 3] > 0
    tot = ph[busy, :3].sum(1)
    p2_ns = p2[busy].astype(np.float64)
    clk = (tot / np.maximum(p2_ns, 1)).mean()   # cycles per ns of wave time in pass 2 (the phases cover it)
    print(f"pass-2 phases over {busy.sum()} waves with work: chunks mean {ph[busy, 3].mean():.2f}; cycles mean group "
          f"{ph[busy, 0].mean():.0f}, gather+Jacobians {ph[busy, 1].mean():.0f}, sums {ph[busy, 2].mean():.0f} "
          f"(shares {ph[busy, 0].sum() / tot.sum():.2f} / {ph[busy, 1].sum() / tot.sum():.2f} / {ph[busy, 2].sum() / tot.sum():.2f}); "
          f"{clk:.2f} cycles per ns of pass-2 time")
    print(f"  per wave: grouping steps {ph[busy, 5].mean():.1f}, slot-serial sum batches {ph[busy, 4].mean():.2f} of "
          f"{4 * ph[busy, 3].mean():.1f} (wave-level batches: 4 per chunk)")
