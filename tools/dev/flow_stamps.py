"""Timeline of the corner's dataflow substitution launch (k_corner_flow; development, needs tools/dev/libnnrt_stamps.so:
tools/dev/stamps_build.sh NNRT_CORNER_STAMPS tools/dev/libnnrt_stamps.so).
Runs GN iterations of a config and prints, per role of the last launch (its ticket), its start, the end of its wait and
its end on the constant-rate clock (100 MHz, us from the first ticket), and per back-chain column the time of its entry
sums, of x = M^T z and of the x store / barriers."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ["NNRT_LIB_PATH"] = os.path.join(ROOT, "tools", "dev", "libnnrt_stamps.so")
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
buf = np.zeros((128, 66, 4), np.uint64)
fn = getattr(lib, "nnrt_dev_flow_stamps")
fn.argtypes = [ctypes.c_void_p]
assert fn(buf.ctypes.data) == 0
live = [k for k in range(128) if buf[k, 64, 0]]
t0 = min(int(buf[k, 64, 0]) for k in live)


def us(v):
    return 10 * (int(v) - t0) / 1000 if v else float("nan")


chain_cols, sums, mprod, tail = [], [], [], []
for k in live:
    r = buf[k, 64]
    line = f"ticket {k:3d}: start {us(r[0]):6.2f} waited {us(r[1]):6.2f} end {us(r[2]):6.2f} us"
    cols = [q for q in range(64) if buf[k, q, 0]]
    if cols:
        parts = []
        for q in cols:
            c = [int(x) for x in buf[k, q]]
            parts.append(f"[{10 * (c[1] - c[0]) / 1000:.2f} {10 * (c[2] - c[1]) / 1000:.2f} {10 * (c[3] - c[2]) / 1000:.2f}]")
            sums.append(10 * (c[1] - c[0]) / 1000)
            mprod.append(10 * (c[2] - c[1]) / 1000)
            tail.append(10 * (c[3] - c[2]) / 1000)
        line += f"  columns {len(cols)}: " + " ".join(parts)
    print(line)
if sums:
    print(f"per column (mean over {len(sums)}): entry sums {np.mean(sums):.2f} us, z + M^T z {np.mean(mprod):.2f} us, "
          f"x store + barriers {np.mean(tail):.2f} us")
