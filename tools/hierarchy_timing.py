"""Warp-field construction time: device path (nnrt_warp_field_create: hierarchy.hip kernels + host bookkeeping) vs the
oracle's sequential restatement (oracle/nnrt_oracle.cpp build_hierarchy + node_coverage_weights, 1 thread), on
grid-like node sets of the C2 / C5 sizes and a larger graph. Prints one JSON line per size.
    python tools/hierarchy_timing.py [N ...]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))


def grid_nodes(n, seed=1):
    rng = np.random.default_rng(seed)
    side = int(np.sqrt(n))
    i = np.arange(n)
    return np.stack([(i % side) * 0.025 + rng.uniform(-1e-3, 1e-3, n), (i // side) * 0.025, 1.5 + 0.01 * rng.uniform(-1, 1, n)], 1).astype(np.float32)


def main():
    import torch  # noqa: F401  (one HIP runtime in the process)
    import oracle as O
    from dynamicfuion_python_amd.nnrt import geometry as G
    sizes = [int(a) for a in sys.argv[1:]] or [1500, 5000, 20000]
    for n in sizes:
        nodes = grid_nodes(n)
        G.HierarchicalGraphWarpField(nodes, 0.03, False, 4, 0, G.WarpNodeCoverageComputationMethod.MINIMAL_K_NEIGHBOR_NODE_DISTANCE, 2)  # warm-up
        reps = 5
        t0 = time.perf_counter()
        for _ in range(reps):
            wf = G.HierarchicalGraphWarpField(nodes, 0.03, False, 4, 0, G.WarpNodeCoverageComputationMethod.MINIMAL_K_NEIGHBOR_NODE_DISTANCE, 2)
        gpu_ms = (time.perf_counter() - t0) / reps * 1e3
        t0 = time.perf_counter()
        vidx, counts, edges, _ = O.build_hierarchy(nodes, 0.03, 2)
        O.node_coverage_weights(nodes, 0.03)
        cpu_ms = (time.perf_counter() - t0) * 1e3
        same = bool(np.array_equal(wf.get_virtual_node_indices(), vidx) and np.array_equal(wf.get_edges(), edges))
        print(json.dumps({"nodes": n, "layers": [int(c) for c in counts], "edges": int(len(edges)), "device_create_ms": round(gpu_ms, 3),
                          "oracle_1thread_ms": round(cpu_ms, 3), "identical": same}), flush=True)


if __name__ == "__main__":
    main()
