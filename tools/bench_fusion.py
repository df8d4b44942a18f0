#!/usr/bin/env python3
"""TSDF voxel-block-grid measurement (the canonical-mesh source / sink around the fitter).

Workload: the C2 synthetic frame (640x480 float depth, 1500-node warp graph under its ground-truth motion, color),
voxel 6 mm, 8^3 blocks, truncation 4 voxels. Setup (untimed): touch + rigid integration of the frame, then sleeve
blocks twice. Timed, HIP events on the current stream:
  * integrate_non_rigid over every active block (the per-frame DynamicFusion update; no activation, async);
  * extract_triangle_mesh (marching cubes, synchronizing: counts come back to the host);
  * find_blocks_intersecting_truncation_region (synchronizing).
Prints one JSON line; algorithmic bytes for the integration: per voxel tsdf + weight + color read and written
(4 + 4 + 12 bytes each way) -- the voxel stream; depth / normals / color image reads are cache-resident.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)


def main():
    import torch
    from dynamicfuion_python_amd import synthetic as S
    from dynamicfuion_python_amd.nnrt import geometry as G
    from dynamicfuion_python_amd.nnrt import rendering as Rr
    import bench
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    torch.cuda.set_device(0)
    sc = S.make_scene("C2", hierarchy_builder=S.native_hierarchy_builder)
    depth = bench.render_target(sc, G, Rr)
    depth = torch.as_tensor(depth, device="cuda", dtype=torch.float32) if not isinstance(depth, torch.Tensor) else depth.float()
    H, W = depth.shape
    color = torch.rand((H, W, 3), device="cuda", dtype=torch.float32)
    K = np.asarray(sc.K, np.float64)
    E = np.eye(4)
    grid = G.NonRigidSurfaceVoxelBlockGrid(["tsdf", "weight", "color"], ["float32", "float32", "float32"], [1, 1, 3], 0.006, 8, 20000)
    blocks = grid.compute_unique_block_coordinates(depth, K, E, 1.0, 3.0, 4.0)
    grid.integrate(blocks, depth, color, K, K, E, 1.0, 3.0, 4.0)
    grid.activate_sleeve_blocks()
    grid.activate_sleeve_blocks()
    nb = grid.get_block_count()
    wf = G.HierarchicalGraphWarpField(sc.nodes, sc.coverage, True, 4, 1, G.WarpNodeCoverageComputationMethod.FIXED_NODE_COVERAGE, 1)
    wf.set_node_rotations(sc.gt_rotations)
    wf.set_node_translations(sc.gt_translations)
    pts, _ = G.functional.unproject_raster_depth_without_filtering(depth, K, depth_scale=1.0, depth_max=10.0)
    normals = G.functional.compute_ordered_point_cloud_normals(pts, (H, W))
    none = np.zeros((0, 3), np.int32)

    def integrate():
        return grid.integrate_non_rigid(none, wf, depth, color, normals, K, K, E, 1.0, 3.0, 4.0)

    for _ in range(5):
        integrate()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        integrate()
    e1.record()
    torch.cuda.synchronize()
    ms_int = e0.elapsed_time(e1) / steps
    mesh = grid.extract_triangle_mesh(0.0)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        mesh = grid.extract_triangle_mesh(0.0)
    torch.cuda.synchronize()
    ms_mesh = (time.perf_counter() - t0) * 100.0
    t0 = time.perf_counter()
    for _ in range(10):
        fb = grid.find_blocks_intersecting_truncation_region(depth, wf, K, E, 1.0, 3.0, 4.0)
    torch.cuda.synchronize()
    ms_find = (time.perf_counter() - t0) * 100.0
    voxels = nb * 512
    bytes_per_voxel = 2 * (4 + 4 + 12)
    gbs = voxels * bytes_per_voxel / (ms_int * 1e-3) / 1e9
    print(json.dumps({
        "metric": "TSDF non-rigid integrations/s (640x480, 1500-node warp, 6 mm voxels)", "value": 1000.0 / ms_int, "unit": "integrations/s",
        "ms_per_integration": ms_int, "voxels": voxels, "blocks": nb, "voxels_per_s": voxels / (ms_int * 1e-3),
        "roofline": {"bound": "hbm", "achieved": gbs, "peak": 8000.0, "unit": "GB/s", "frac": gbs / 8000.0,
                     "bytes_formula": "per voxel: tsdf + weight + color (f32) read and written = 40 B"},
        "mesh_ms": ms_mesh, "mesh_vertices": int(mesh.vertex_positions.shape[0]), "mesh_triangles": int(mesh.triangle_indices.shape[0]),
        "find_blocks_ms": ms_find, "found_blocks": int(fb.shape[0]), "data": "synthetic C2 frame", "dtype": "f32"}), flush=True)


if __name__ == "__main__":
    main()
