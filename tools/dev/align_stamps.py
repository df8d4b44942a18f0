"""Per-kernel head / tail outside wave execution (development; needs tools/dev/libnnrt_kstamps.so built with
NNRT_KERNEL_STAMPS and NNRT_FIT_STAMPS). Run under rocprofv3 --kernel-trace --output-format csv: one eager C2 GN
iteration; writes the last launch's per-wave stamps (100 MHz s_memrealtime ticks) of the warp, raster and fused pixel
kernels to argv[1] (JSON). Pair with align_report.py, which brackets the clock offset between stamps and the trace."""
import ctypes
import json
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

sc = S.make_scene("C2", hierarchy_builder=S.native_hierarchy_builder)
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
out = {}
tiles = ((sc.W + 15) // 16) * ((sc.H + 15) // 16)
for kname, waves in (("warp", -(-4 * len(sc.points) // 256) * 4), ("raster", -(-len(sc.faces) // 32)), ("fit", tiles * 4)):
    buf = np.zeros((16384, 4), np.uint64)
    fn = getattr(lib, f"nnrt_dev_{kname}_stamps")
    fn.argtypes = [ctypes.c_void_p]
    assert fn(buf.ctypes.data) == 0
    st = buf[:waves].astype(np.int64)
    end_col = 2
    out[kname] = dict(first_start=int(st[:, 0].min()), last_end=int(st[:, end_col].max()))
json.dump(out, open(sys.argv[1], "w"))
print(out)
