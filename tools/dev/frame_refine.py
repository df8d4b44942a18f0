"""Per-iteration refinement gate of a frame fit from the identity warp (development): the bench's --step frame scene
(C2_ARAP unless given), iterations run one at a time, each iteration's corner pivot / diag(S) ratio, whether the
refinement step ran, its NaN node rotations and its time (eager, median of 5 repeats from the same state).
NNRT_LIB_PATH selects the library."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bench  # noqa: E402
from dynamicfuion_python_amd import synthetic as S  # noqa: E402
from dynamicfuion_python_amd.nnrt import alignment as A, geometry as G, rendering as Rr  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C2_ARAP"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
sc = S.make_scene(name, hierarchy_builder=S.native_hierarchy_builder)
depth = bench.render_target(sc, G, Rr)
wf = G.HierarchicalGraphWarpField(sc.nodes, sc.coverage, False, 4, 0, G.WarpNodeCoverageComputationMethod.FIXED_NODE_COVERAGE, sc.layer_count)
ft = A.DeformableMeshToImageFitter(1, [A.IterationMode.ALL], preconditioning_dampening_factor=0.001, use_hip_graph=0)
ft.prepare(wf, G.TriangleMesh(sc.points, sc.normals, sc.faces), depth, None, sc.K)
for k in range(iters):
    R0, t0 = wf.get_node_rotations(True), wf.get_node_translations(True)
    times = []
    for rep in range(5):   # the same iteration from the same state
        wf.set_node_rotations(R0, True)
        wf.set_node_translations(t0, True)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        ft.iterate(wf, k, 1)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1) * 1000)
    info = ft.refine_info()
    nan = int(np.isnan(R0).reshape(len(sc.nodes), -1).any(1).sum())
    print(f"{name} iteration {k + 1}: pivot / diag(S) {info['pivot_ratio']:.3g}, refined {info['refined']}, NaN rotations "
          f"before {nan}, {np.median(times):.1f} us", flush=True)
