"""Real DeepDeform data through the GPU path: the committed seq017 frames 300 -> 600 and their
DeepDeformGraph nodes (tests/golden/deepdeform), stage by stage against the oracle, then the whole FusionPipeline.

Bit-exact: depth back-projection, rigid integration, marching cubes, truncation-region search, non-rigid integration.
Within the fitter's tolerances: one Gauss-Newton iteration of the canonical mesh against frame 600."""
import os
from types import SimpleNamespace

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from _util import arrowhead_fp64_solution, exact_system_solution, rel_err, rodrigues64  # noqa: E402

DD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "deepdeform")


@pytest.fixture(scope="module")
def nn():
    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible for a -m gpu test")
    from dynamicfuion_python_amd import nnrt
    return nnrt


def _np(t):
    return t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)


@pytest.fixture(scope="module")
def pair():
    from dynamicfuion_python_amd.data import frame as dfr
    return dfr.FramePairDataset(300, 600, 17, dfr.DataSplit.TEST, dfr.DatasetType.LOCAL, base_directory=DD).load()


@pytest.fixture(scope="module")
def intr(pair):
    from dynamicfuion_python_amd.data import camera as dcam
    return dcam.load_intrinsic_matrix_entries_from_text_4x4_matrix(pair.get_intrinsics_path())


def test_backproject_depth_bit_exact(nn, oracle_mod, pair, intr):
    fx, fy, cx, cy = intr
    depth = pair.source.load_depth_image_numpy()
    got = nn.backproject_depth_ushort(depth, fx, fy, cx, cy, 1000.0)            # 4-pixel vector path
    ref = oracle_mod.backproject_depth(depth, fx, fy, cx, cy, 1000.0)
    assert np.array_equal(_np(got), ref) and (ref[..., 2] > 0).sum() > 100000
    odd = np.ascontiguousarray(depth[:, :637])                                   # W % 4 != 0: scalar path
    assert np.array_equal(_np(nn.backproject_depth_ushort(odd, fx, fy, cx, cy, 1000.0)),
                          oracle_mod.backproject_depth(odd, fx, fy, cx, cy, 1000.0))
    dm = depth.astype(np.float32) / 1000.0
    assert np.array_equal(_np(nn.backproject_depth_float(dm, fx, fy, cx, cy)), oracle_mod.backproject_depth(dm, fx, fy, cx, cy))
    t = torch.from_numpy(depth.view(np.int16)).cuda().view(torch.uint16)         # device uint16 input, caller's output buffer
    out = torch.empty((480, 640, 3), dtype=torch.float32, device="cuda")
    nn.image_proc.backproject_depth_ushort(t, fx, fy, cx, cy, 1000.0, point_image_out=out)
    assert np.array_equal(_np(out), ref)
    assert nn.backproject_depth_ushort(np.zeros((0, 0), np.uint16), fx, fy, cx, cy, 1000.0).shape == (0, 0, 3)
    with pytest.raises(ValueError):
        nn.image_proc.backproject_depth_ushort(depth, fx, fy, cx, cy, 1000.0, point_image_out=out[:10])


def test_real_frame_pair_stages_vs_oracle(nn, oracle_mod, pair, intr):
    """Frame 300: rigid integration + canonical mesh; frame 600: one GN iteration, truncation-region search, non-rigid
    integration under the fitted motion, mesh -- each stage against the oracle on the same inputs."""
    G, A, O = nn.geometry, nn.alignment, oracle_mod
    fx, fy, cx, cy = intr
    K = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1]], np.float64)
    E = np.eye(4)
    src, tgt = pair.source, pair.target
    d0, c0 = src.load_depth_image_numpy(), src.load_color_image_rgb()
    d1 = tgt.load_depth_image_numpy()
    c1 = np.zeros_like(c0)
    vs, trunc = 0.005, 5.0
    grid = G.NonRigidSurfaceVoxelBlockGrid(["tsdf", "weight", "color"], ["float32", "uint16", "uint16"], [1, 1, 3], vs, 16, 1000)
    og = O.OracleGrid(vs, 16, "uint16", "uint16")
    blocks = grid.compute_unique_block_coordinates(d0, K, E, 1000.0, 3.0, trunc)
    ob = og.touch(d0, K, E, 1000.0, 3.0, trunc)
    assert np.array_equal(_np(blocks), ob) and len(ob) > 200
    grid.integrate(blocks, d0, c0, K, K, E, 1000.0, 3.0, trunc)
    og.integrate(ob, d0, c0, K, K, E, 1000.0, 3.0, trunc)
    assert np.array_equal(_np(grid.extract_voxel_values_and_coordinates()), og.values_all())
    mesh = grid.extract_triangle_mesh(0.0, -1)
    V, Nn, _, T = og.mesh(0.0)
    assert len(T) > 50000
    assert np.array_equal(_np(mesh.triangle_indices), T) and np.array_equal(_np(mesh.vertex_positions), V)
    assert np.array_equal(_np(mesh.vertex_normals), Nn)

    # one GN iteration of the canonical mesh against frame 600 (point-cloud overload), loaded graph, 2-layer ARAP
    nodes, _, _, _, _ = pair.load_graph_data(pair.graph_filename)
    wf = G.HierarchicalGraphWarpField(nodes, 0.05, False, 4, 0, G.WarpNodeCoverageComputationMethod.FIXED_NODE_COVERAGE, 2)
    vidx = wf.get_virtual_node_indices()
    vidx_o, counts, edges, elayers = O.build_hierarchy(nodes, 0.05, 2)
    assert np.array_equal(vidx, vidx_o) and np.array_equal(wf.get_edges(), edges)
    pts = O.backproject_depth(d1, fx, fy, cx, cy, 1000.0).reshape(-1, 3)
    mask = (pts[:, 2] > 0).astype(np.uint8)
    ft = A.DeformableMeshToImageFitter(1, [A.IterationMode.ALL], preconditioning_dampening_factor=0.001)
    ft.fit_to_image(wf, G.TriangleMesh(V, Nn, T), None, pts, mask, K, None, (480, 640))
    N = len(nodes)
    R_o, t_o, dg_o = O.fit(nodes=nodes[vidx], rotations=np.tile(np.eye(3, dtype=np.float32), (N, 1, 1)),
                           translations=np.zeros((N, 3), np.float32), mesh_points=V, mesh_normals=Nn, faces=T, ref_points=pts,
                           ref_mask=mask, H=480, W=640, K=K, max_iterations=1, lm_factor=0.001, coverage=0.05, edges=edges,
                           edge_layers=elayers, radii=np.array([0.05, 0.1], np.float32), first_layer_count=int(counts[0]))
    dg = ft.diagnostics()
    assert np.array_equal(dg_o["pixel_faces"].astype(np.int64), dg["pixel_faces"].astype(np.int64))
    assert np.array_equal(dg_o["residual_mask"], dg["residual_mask"]) and dg["residual_mask"].sum() > 50000
    assert np.allclose(dg_o["residuals"], dg["residuals"], rtol=0, atol=1e-6)
    assert rel_err(dg["gradient"][:N * 6], dg_o["gradient"]) < 1e-6
    u_err = rel_err(dg["updates"][:N * 6], dg_o["updates"])
    t_err = rel_err(wf.get_node_translations(True), t_o)
    r_err = rel_err(wf.get_node_rotations(True) - np.eye(3), R_o - np.eye(3))
    # the node motion is exactly the reported update applied to the identity state (t = 0 + dt, R = I . Rodrigues(w):
    # RodriguesImpl.h:66-88, A10), whichever solve path (plain or refined) wrote it
    x = np.asarray(dg["updates"][:N * 6], np.float32).reshape(N, 6)
    assert np.array_equal(wf.get_node_translations(True), np.float32(0) + x[:, 3:], equal_nan=True)
    dR = O.rodrigues(np.ascontiguousarray(x[:, :3])).reshape(N, 3, 3)
    I3f = np.eye(3, dtype=np.float32)
    R_e = np.empty_like(dR)
    for r in range(3):
        for c in range(3):
            R_e[:, r, c] = (I3f[r, 0] * dR[:, 0, c] + I3f[r, 1] * dR[:, 1, c]) + I3f[r, 2] * dR[:, 2, c]
    assert np.array_equal(wf.get_node_rotations(True).reshape(N, 3, 3), R_e, equal_nan=True)
    # the data term in the reference's own arithmetic (the product's unfused pixel-node Jacobians): H and g within the
    # fp64 summation order (measured: identical)
    h_err = rel_err(dg["hessian"][:N * 36], dg_o["hessian_diag"])
    g_err = rel_err(dg["gradient"][:N * 6], dg_o["gradient"])
    # the solve against the fp64 solution of exactly the float system the GPU factored (nnrt_fitter_get_arrowhead_system),
    # and the oracle's float32 solve (the reference's natural-order potrf) against the same solution
    x_exact, ratio_exact = exact_system_solution(ft, wf, N)
    gate = ft.refine_info()
    e_exact = rel_err(dg["updates"][:N * 6], x_exact)
    e_o_exact = rel_err(dg_o["updates"], x_exact)
    x6 = x_exact.reshape(N, 6)
    R_x = rodrigues64(x6[:, :3])   # the exact update's node motion from the identity (t = dt, R = Rodrigues(w))
    r_gpu_x = rel_err(wf.get_node_rotations(True) - np.eye(3), R_x - np.eye(3))
    r_o_x = rel_err(R_o - np.eye(3), R_x - np.eye(3))
    t_gpu_x, t_o_x = rel_err(wf.get_node_translations(True), x6[:, 3:]), rel_err(t_o, x6[:, 3:])
    print(f"real frame pair vs the oracle: H {h_err:.3g}, g {g_err:.3g}, update {u_err:.3g}, t {t_err:.3g}, R - I {r_err:.3g}")
    print(f"vs the exact solution of the GPU's float system (fp64 pivot ratio {ratio_exact:.3g}; corner pivot / diag(S) "
          f"{gate['pivot_ratio']:.3g}, refined {gate['refined']}): GPU update {e_exact:.3g}, t {t_gpu_x:.3g}, R - I {r_gpu_x:.3g}; "
          f"oracle float32 solve update {e_o_exact:.3g}, t {t_o_x:.3g}, R - I {r_o_x:.3g}")
    assert h_err < 1e-6 and g_err < 1e-6
    # the GPU's node motion -- translations and max |R - I| -- within north_star's 1e-4 of the exact solution
    assert e_exact <= 1e-4 and t_gpu_x <= 1e-4 and r_gpu_x <= 1e-4
    if not (u_err < 1e-4 and t_err < 1e-4 and r_err < 1e-4):
        # the two float32 solves differ by more than 1e-4 only where the reference-order solve is itself that far from the
        # exact solution of the same system: the difference is the oracle's own error (triangle inequality), and the GPU
        # is the closer of the two
        assert r_err <= r_gpu_x + r_o_x + 1e-6 and t_err <= t_gpu_x + t_o_x + 1e-6 and u_err <= e_exact + e_o_exact + 1e-6
        assert r_gpu_x < r_o_x and e_exact < e_o_exact, "the GPU solve must be the closer to the exact solution"
    assert np.abs(t_o).max() > 1e-4   # the frames differ: the fit moves the graph

    # fuse frame 600 under the GPU-fitted motion (both sides read the same R, t)
    nodes_v, R_v, t_v = wf.get_node_positions(True), wf.get_node_rotations(True), wf.get_node_translations(True)
    nb = grid.find_blocks_intersecting_truncation_region(d1, wf, K, E, 1000.0, 3.0, trunc)
    nb_o = og.find_blocks_intersecting_truncation_region(d1, nodes_v, R_v, t_v, 0.05, 4, 0, K, E, 1000.0, 3.0, trunc)
    assert np.array_equal(_np(nb), nb_o)   # sleeve blocks reached by the warped band (none for this small motion)
    nrm = O.ordered_point_cloud_normals(pts, 480, 640)
    assert np.array_equal(_np(G.compute_ordered_point_cloud_normals(pts, (480, 640))), nrm)
    cos = grid.integrate_non_rigid(nb, wf, d1, c1, nrm, K, K, E, 1000.0, 3.0, trunc)
    cos_o = og.integrate_non_rigid(nb_o, nodes_v, R_v, t_v, 0.05, 4, 0, d1, c1, nrm, K, K, E, 1000.0, 3.0, trunc)
    assert np.array_equal(_np(cos), cos_o) and (cos_o != 0).sum() > 10000
    assert np.array_equal(_np(grid.extract_voxel_values_and_coordinates()), og.values_all())
    mesh2 = grid.extract_triangle_mesh(1.0, -1)
    V2, _, _, T2 = og.mesh(1.0)
    assert np.array_equal(_np(mesh2.triangle_indices), T2) and np.array_equal(_np(mesh2.vertex_positions), V2)


def test_ndc_convention_on_real_frames(nn, oracle_mod, pair, intr):
    """SURVEY A11 on real data: the reference's image -> NDC mapping renders the canonical mesh y-mirrored about cy, so at
    identity the fit's residuals against the very frame the mesh was fused from are centimetres; NDC_CONSISTENT renders
    pixel (u, v) at pixel (u, v) and the residuals drop to the TSDF's own discretisation. Both conventions match the oracle."""
    G, A, O = nn.geometry, nn.alignment, oracle_mod
    fx, fy, cx, cy = intr
    K = np.array([[fx, 0, cx], [0, fy, cy], [0, 0, 1]], np.float64)
    d0 = pair.source.load_depth_image_numpy()
    grid = G.NonRigidSurfaceVoxelBlockGrid(["tsdf", "weight"], ["float32", "float32"], [1, 1], 0.005, 16, 1000)
    grid.integrate(grid.compute_unique_block_coordinates(d0, K, np.eye(4), 1000.0, 3.0, 5.0), d0, K, np.eye(4), 1000.0, 3.0, 5.0)
    mesh = grid.extract_triangle_mesh(0.0, -1)
    V, Nn, T = _np(mesh.vertex_positions), _np(mesh.vertex_normals), _np(mesh.triangle_indices)
    nodes = pair.load_graph_data(pair.graph_filename)[0]
    N = len(nodes)
    pts = O.backproject_depth(d0, fx, fy, cx, cy, 1000.0).reshape(-1, 3)
    mask = (pts[:, 2] > 0).astype(np.uint8)
    median = {}
    for conv in (A.NDC_REFERENCE, A.NDC_CONSISTENT):
        wf = G.HierarchicalGraphWarpField(nodes, 0.05, False, 4, 0, G.WarpNodeCoverageComputationMethod.FIXED_NODE_COVERAGE, 1)
        ft = A.DeformableMeshToImageFitter(1, [A.IterationMode.ALL], preconditioning_dampening_factor=0.001, ndc_convention=conv)
        ft.fit_to_image(wf, G.TriangleMesh(V, Nn, T), None, pts, mask, K, None, (480, 640))
        dg = ft.diagnostics()
        _, t_o, dg_o = O.fit(nodes=nodes, rotations=np.tile(np.eye(3, dtype=np.float32), (N, 1, 1)), translations=np.zeros((N, 3), np.float32),
                             mesh_points=V, mesh_normals=Nn, faces=T, ref_points=pts, ref_mask=mask, H=480, W=640, K=K, max_iterations=1,
                             lm_factor=0.001, coverage=0.05, ndc_consistent=conv == A.NDC_CONSISTENT)
        assert np.array_equal(dg_o["pixel_faces"].astype(np.int64), dg["pixel_faces"].astype(np.int64))
        assert np.array_equal(dg_o["residual_mask"], dg["residual_mask"])
        assert np.allclose(dg_o["residuals"], dg["residuals"], rtol=0, atol=1e-6)
        assert rel_err(wf.get_node_translations(True), t_o) < 1e-4
        median[conv] = float(np.median(np.abs(dg["residuals"][dg["residual_mask"]])))
    assert median[A.NDC_CONSISTENT] < 0.003 < 0.05 < median[A.NDC_REFERENCE], median


def test_fusion_pipeline_on_real_frames(nn, oracle_mod):
    """The whole loop with tracking method RENDERING: frame 300 fused rigidly, the DeepDeformGraph nodes as the motion
    graph, frame 600 tracked by one GPU Gauss-Newton iteration (NDC_CONSISTENT) and fused non-rigidly. The pipeline's fit
    is checked against the oracle fit of the same canonical mesh; the graph motion it produced drives the integration."""
    from dynamicfuion_python_amd.data import frame as dfr
    from dynamicfuion_python_amd import fusion as F
    O = oracle_mod
    seq = dfr.FrameSequenceDataset(17, dfr.DataSplit.TEST, base_dataset_type=dfr.DatasetType.LOCAL, base_directory=DD,
                                   frame_indices=[300, 600])
    params = F.FusionParameters()
    params.alignment.max_iteration_count = 1
    pipe = F.FusionPipeline(seq, params)
    first = pipe.process_frame(seq.get_next_frame())
    assert first.active_block_count > 200 and pipe.active_graph.node_count == 109
    canonical = pipe.canonical_mesh
    V, Nn, T = _np(canonical.vertex_positions), _np(canonical.vertex_normals), _np(canonical.triangle_indices)
    assert len(T) > 50000
    wf = pipe.active_graph
    nodes_v, weights_v = wf.get_node_positions(True), wf.get_node_coverage_weights()
    counts, edges, elayers = wf.get_layer_node_counts(), wf.get_edges(), wf.get_edge_layer_indices()
    f600 = seq.get_next_frame()
    res = pipe.process_frame(f600)
    assert res.tracked and res.canonical_triangle_count == len(T) and res.active_block_count >= first.active_block_count
    fx, fy, cx, cy = pipe.fx, pipe.fy, pipe.cx, pipe.cy
    pts = O.backproject_depth(f600.load_depth_image_numpy(), fx, fy, cx, cy, 1000.0).reshape(-1, 3)
    N = len(nodes_v)
    R_o, t_o, dg_o = O.fit(nodes=nodes_v, rotations=np.tile(np.eye(3, dtype=np.float32), (N, 1, 1)), translations=np.zeros((N, 3), np.float32),
                        mesh_points=V, mesh_normals=Nn, faces=T, ref_points=pts, ref_mask=(pts[:, 2] > 0).astype(np.uint8), H=480, W=640,
                        K=pipe.K, max_iterations=1, lm_factor=params.alignment.preconditioning_dampening_factor, coverage=0.05,
                        coverage_method=1, node_weights=weights_v, edges=edges, edge_layers=elayers,
                        radii=np.array([0.05, 0.1], np.float32), first_layer_count=int(counts[0]), ndc_consistent=True)
    t = wf.get_node_translations(True)
    assert np.isfinite(t).all() and np.abs(t).max() > 1e-3
    if rel_err(t, t_o) >= 1e-4:
        # ill-conditioned arrowhead system: both float32 solves are held against its fp64 solution (the trajectory
        # tests' rule); the translation rows of the update are the node translations (the fit starts at t = 0)
        sc = SimpleNamespace(nodes=nodes_v, hierarchy=dict(virtual_indices=np.arange(N), edges=edges, edge_layers=elayers,
                                                          radii=np.array([0.05, 0.1], np.float32), node_weights=weights_v))
        I3 = np.tile(np.eye(3, dtype=np.float32), (N, 1, 1))
        x64 = arrowhead_fp64_solution(O, sc, I3, np.zeros((N, 3), np.float32), dg_o,
                                      lm=params.alignment.preconditioning_dampening_factor).reshape(N, 6)[:, 3:]
        e_g, e_o = rel_err(t, x64), rel_err(t_o, x64)
        print(f"fp64 rule: GPU vs fp64 {e_g:.3g}, oracle vs fp64 {e_o:.3g}")
        assert e_g <= max(2.0 * e_o, 1e-4), f"translations {rel_err(t, t_o):.3g} from the oracle's; vs fp64 GPU {e_g:.3g}, oracle {e_o:.3g}"
    # the ramp asks for weight > 1 after two frames: only voxels observed in both frames under the fitted motion qualify
    assert pipe.mesh_extraction_threshold() == 1
    assert (pipe.warped_mesh is None) == (pipe.canonical_mesh.triangle_indices.shape[0] == 0)
    assert pipe.volume.extract_triangle_mesh(0.0, -1).triangle_indices.shape[0] >= len(T)
    assert not seq.has_more_frames()

    with pytest.raises(NotImplementedError):
        F.FusionPipeline(seq, F.FusionParameters(tracking_method=F.TrackingMethod.NEURAL))
