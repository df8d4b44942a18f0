"""Phase timing of the Schur-corner factor launches (development; needs tools/dev/libnnrt_stamps.so:
tools/dev/stamps_build.sh NNRT_CORNER_STAMPS tools/dev/libnnrt_stamps.so).
Runs C5 GN iterations and prints, per factor launch, every workgroup's span on the constant-rate clock (100 MHz) and the
shader-clock cycles of the phases of the workgroup that ends last and of the slowest panel task: staging, first
elimination half, rank-32 update, second half, stores."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["NNRT_LIB_PATH"] = os.environ.get("STAMPS_LIB", os.path.join(ROOT, "tools", "dev", "libnnrt_stamps.so"))
sys.path[:0] = [ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from dynamicfuion_python_amd import _native as NV, synthetic as S  # noqa: E402
from dynamicfuion_python_amd.nnrt import alignment as A, geometry as G  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C5"
sc = S.make_scene(name, hierarchy_builder=S.native_hierarchy_builder)
lib = NV.lib()
wf = G.HierarchicalGraphWarpField(sc.nodes, sc.coverage, False, 4, 0, G.WarpNodeCoverageComputationMethod.FIXED_NODE_COVERAGE, sc.layer_count)
depth = np.full((sc.H, sc.W), 1.2, np.float32)
ft = A.DeformableMeshToImageFitter(1, [A.IterationMode.ALL], preconditioning_dampening_factor=0.001, use_hip_graph=0)
ft.prepare(wf, G.TriangleMesh(sc.points, sc.normals, sc.faces), depth, None, sc.K)
for _ in range(5):
    ft.iterate_from_identity(wf, 0, 1)
torch.cuda.synchronize()
buf = np.zeros((64, 512, 8), np.uint64)
fn = getattr(lib, "nnrt_dev_corner_stamps")
fn.argtypes = [ctypes.c_void_p]
assert fn(buf.ctypes.data) == 0
MASK = (1 << 62) - 1
names = ["stage", "half1", "rank32", "half2", "store"]


def phases(st):
    return "  ".join(f"{n} {int(st[i + 1]) - int(st[i]) if st[i + 1] and st[i] else -1:6d}" for i, n in enumerate(names))


for lev in range(64):
    w = buf[lev]
    live = np.nonzero(w[:, 6])[0]
    if len(live) == 0:
        break
    t0 = int(min(w[i, 6] for i in live))
    ends = [(int(w[i, 7]) & MASK, i) for i in live]
    last_end, last = max(ends)
    trailing = [i for i in live if int(w[i, 7]) >> 62 & 1]
    panels = [i for i in live if not int(w[i, 7]) >> 62 & 1]
    pspan = max(((int(w[i, 7]) & MASK) - int(w[i, 6]), i) for i in panels)
    tspan = max((((int(w[i, 7]) & MASK) - int(w[i, 6]), i) for i in trailing), default=(0, -1))
    start_spread = max(int(w[i, 6]) for i in live) - t0
    print(f"level {lev:2d}: {len(panels)} panel + {len(trailing)} trailing wgs, span {10 * (last_end - t0) / 1000:.2f} us "
          f"(last: {'trailing' if last in trailing else 'panel'} wg {last}); start spread {10 * start_spread / 1000:.2f} us; "
          f"slowest panel {10 * pspan[0] / 1000:.2f} us [{phases(w[pspan[1]])}]; slowest trailing {10 * tspan[0] / 1000:.2f} us")


# multi-wave elimination (NNRT_CORNER_ELIM_WAVES > 0): per block of the slowest panel of levels 2-5, block b's owner's
# cycles from the start of iteration b - 1 to its update by block b - 1, to publishing block b, to the barrier
fe = getattr(lib, "nnrt_dev_elim_stamps", None)
if fe is not None:
    fe.argtypes = [ctypes.c_void_p]
    eb = np.zeros((16, 128, 16, 4), np.uint64)
    assert fe(eb.ctypes.data) == 0
    for lev in range(2, 6):
        w = buf[lev]
        panels = [i for i in np.nonzero(w[:, 6])[0] if not int(w[i, 7]) >> 62 & 1 and i < 128]
        if not panels:
            continue
        slow = max(panels, key=lambda i: (int(w[i, 7]) & MASK) - int(w[i, 6]))
        rows = []
        for blk in range(1, 16):
            st = [int(x) for x in eb[lev, slow, blk]]
            if st[0] and st[3]:
                rows.append((st[1] - st[0], st[2] - st[1], st[3] - st[2]))
        if rows:
            r = np.array(rows)
            print(f"level {lev} panel wg {slow}: per block (update, factor + publish, to barrier) mean {r.mean(0).round(0)} "
                  f"over {len(rows)} blocks; first {rows[0]}, last {rows[-1]}")
