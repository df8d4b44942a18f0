"""Phase timing of the Schur-corner factor launches (development; needs tools/dev/libnnrt_stamps.so: tools/dev/stamps_build.sh NNRT_CORNER_STAMPS tools/dev/libnnrt_stamps.so).
Runs one C5 GN iteration and prints, per factor launch, the shader-clock cycles of workgroup 0's phases: staging,
first elimination half, rank-32 update, second half, stores."""
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
for _ in range(3):
    ft.iterate_from_identity(wf, 0, 1)
torch.cuda.synchronize()
buf = np.zeros((256, 8), np.uint64)
fn = getattr(lib, "nnrt_dev_corner_stamps")
fn.argtypes = [ctypes.c_void_p]
assert fn(buf.ctypes.data) == 0
names = ["stage", "half1", "rank32", "half2", "store"]
for l in range(256):
    st = buf[l]
    if st[0] == 0:
        break
    d = [int(st[i + 1]) - int(st[i]) if st[i + 1] else -1 for i in range(5)]
    print(f"level {l:2d}: " + "  ".join(f"{n} {v:6d}" for n, v in zip(names, d)) + f"  total {int(st[5]) - int(st[0]) if st[5] else -1}")
