#!/usr/bin/env python3
"""Development timing of the GN-iteration stages for the product library and the timing-variant builds
(dynamicfuion_python_amd/csrc/variants/, `make variants`). Each library runs in its own process."""
import glob
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def child(config, steps):
    sys.path.insert(0, ROOT)
    import torch
    import bench
    from dynamicfuion_python_amd import synthetic as S
    from dynamicfuion_python_amd.nnrt import alignment as A
    from dynamicfuion_python_amd.nnrt import geometry as G
    from dynamicfuion_python_amd.nnrt import rendering as Rr
    torch.cuda.set_device(0)
    sc = S.make_scene(config, hierarchy_builder=S.native_hierarchy_builder)
    depth = bench.render_target(sc, G, Rr)
    wf = G.HierarchicalGraphWarpField(sc.nodes, sc.coverage, False, 4, 0, G.WarpNodeCoverageComputationMethod.FIXED_NODE_COVERAGE,
                                      sc.layer_count)
    ft = A.DeformableMeshToImageFitter(1, [A.IterationMode.ALL], preconditioning_dampening_factor=0.001)
    ft.prepare(wf, G.TriangleMesh(sc.points, sc.normals, sc.faces), depth, None, sc.K)
    acc = {k: 0.0 for k in A.TIMED_STAGES}
    for i in range(steps + 5):
        wf.reset_motion()
        r = ft.iterate_timed(wf, 0, 1)
        if i >= 5:
            for k in acc:
                acc[k] += r[k] / steps
    for _ in range(20):
        wf.reset_motion()
        ft.iterate(wf, 0, 1)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        wf.reset_motion()
        ft.iterate(wf, 0, 1)
    torch.cuda.synchronize()
    acc["graph_step_ms"] = (time.perf_counter() - t0) * 1000 / steps
    print(json.dumps({k: round(v * 1000, 2) for k, v in acc.items()}), flush=True)   # microseconds


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(sys.argv[2], int(sys.argv[3]))
        return
    config = sys.argv[1] if len(sys.argv) > 1 else "C2"
    libs = [os.path.join(ROOT, "dynamicfuion_python_amd", "libnnrt_mi355x.so")]
    libs += sorted(glob.glob(os.path.join(ROOT, "dynamicfuion_python_amd", "csrc", "variants", "*.so")))
    for lib in libs:
        env = dict(os.environ, NNRT_LIB_PATH=lib)
        out = subprocess.run([sys.executable, __file__, "--child", config, "200"], env=env, capture_output=True, text=True, timeout=300)
        line = out.stdout.strip().splitlines()[-1] if out.stdout.strip() else out.stderr[-500:]
        print(f"{os.path.basename(lib):24s} {line}", flush=True)
        if out.returncode != 0:
            sys.exit(out.returncode)


if __name__ == "__main__":
    main()
