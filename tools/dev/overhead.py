"""Fixed cost of a short timed region (development): 2 graph launches of 10 C2 iterations, timed on the host as
bench.timed_region does (sync, launches, sync), with HIP events around the launches, and with a busy-polled event
before the final synchronize; on the default stream and on a side stream."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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
ft = A.DeformableMeshToImageFitter(1, [A.IterationMode.ALL], preconditioning_dampening_factor=0.001, use_hip_graph=A.GRAPH_ALWAYS)
ft.prepare(wf, G.TriangleMesh(sc.points, sc.normals, sc.faces), depth, None, sc.K)
ft.snapshot_motion(wf)
for name, stream in (("default stream", torch.cuda.current_stream()), ("side stream", torch.cuda.Stream())):
    sp = NV.stream_ptr(stream)
    for _ in range(20):
        lib.nnrt_fitter_iterate_from_snapshot(ft._h, wf.handle, 0, 10, sp)
    torch.cuda.synchronize()
    res = {"host": [], "events": [], "spin": [], "launch_call": []}
    for rep in range(30):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        e0.record(stream)
        for _ in range(2):
            lib.nnrt_fitter_iterate_from_snapshot(ft._h, wf.handle, 0, 10, sp)
        t1 = time.perf_counter()
        e1.record(stream)
        if rep % 2:
            while not e1.query():
                pass
            res["spin"].append(time.perf_counter() - t0)
        torch.cuda.synchronize()
        res["host"].append(time.perf_counter() - t0)
        res["events"].append(e0.elapsed_time(e1) / 1e3)
        res["launch_call"].append(t1 - t0)
    print(name + ": " + ", ".join(f"{k} median {1e6 * np.median(v) / 20:.1f} us/step" for k, v in res.items()), flush=True)
