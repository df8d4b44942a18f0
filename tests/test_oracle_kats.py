"""CPU tests: pin the oracle (CPU restatement) against the reference's own known-answer tests, fixtures and the
numpy reference derivation (golden vectors from tests/golden/make_golden.py)."""
import os

import numpy as np
import pytest

from _util import (FIXTURES, GOLDEN, neighbours_valid, read_depth_png, read_ply, rel_err, render_target_oracle, sphere_open3d,
                   subdivide_midpoint, transform_mesh, xy_plane)
from golden import kat_literals as L


def test_rodrigues_kat(oracle_mod):
    # cpp/tests/test_rodrigues.cpp:31-53: AllClose(expected, actual, rtol 1e-3, atol 1e-7)
    R = oracle_mod.rodrigues(L.RODRIGUES_AXIS_ANGLE)
    assert np.allclose(R, L.RODRIGUES_EXPECTED, rtol=1e-3, atol=1e-7)


def test_rodrigues_zero_angle_is_nan(oracle_mod):
    # cpp/core/linalg/RodriguesImpl.h:80-81 divides by |w| (quirk A7)
    assert np.isnan(oracle_mod.rodrigues(np.zeros((1, 3), np.float32))).all()


def test_mesh_warping_kat(oracle_mod):
    # cpp/tests/test_mesh_warping.cpp:42-87: 9-vertex plane, every node rotated -90 deg about Y and moved rigidly
    V, Nrm, F = xy_plane(1.0, (0, 0, 0), 1)
    R = np.array([[0, 0, -1], [0, 1, 0], [1, 0, 0]], np.float32)
    nodes = V.copy()
    t = nodes @ R.T - nodes
    Rn = np.tile(R[None], (len(nodes), 1, 1))
    a, w = oracle_mod.compute_anchors(V, nodes, 4, 0.1)
    wp, wn = oracle_mod.warp_mesh(V, Nrm, nodes, Rn, t, a, w)
    assert np.allclose(wp, L.WARP_EXPECTED_POSITIONS, rtol=1e-5, atol=1e-5)
    # WarpUtilities.h:464 blends R n (unnormalized, A12); the reference KAT lists (-1, 0, 0), i.e. R^T n -- the
    # tensor-layout convention of that test is ambiguous, so the normals are checked against the formula instead.
    assert np.allclose(wn, Nrm @ R.T, atol=1e-5)


def test_extract_face_vertices_fixture(oracle_mod):
    # cpp/tests/test_extract_face_vertices.cpp:31-45 with static fixture arrays (334 of 512 faces kept)
    V, _, F = xy_plane(1.2615, (0, 0, 1), 4)
    K = np.array([[580., 0., 320.], [0., 580., 240.], [0., 0., 1.]])
    ndc, mask = oracle_mod.extract_face_ndc(V, F, K, 480, 640, 0.0, 2.0)
    gt = np.load(os.path.join(FIXTURES, "extracted_face_vertices.npy"))
    gm = np.load(os.path.join(FIXTURES, "extracted_face_mask.npy"))
    assert mask.sum() == 334
    assert np.array_equal(mask, gm)
    assert np.allclose(ndc[mask], gt[gm], atol=1e-5)


def test_hierarchy_kat(oracle_mod):
    # cpp/tests/test_graph_warp_field.cpp:30-340
    vidx, counts, edges, elayers = oracle_mod.build_hierarchy(L.HIERARCHY_NODES, 0.25, 3, 4, radii=[0.25, 0.5, 1.0])
    assert list(counts) == [19, 10, 4]
    assert sorted(vidx[:19].tolist()) == L.HIERARCHY_LAYER0
    assert sorted(vidx[19:29].tolist()) == L.HIERARCHY_LAYER1
    assert sorted(vidx[29:].tolist()) == L.HIERARCHY_LAYER2
    assert edges[:, 0].tolist() == L.HIERARCHY_EDGE_SOURCES
    pairs = sorted((int(vidx[i]), int(vidx[j])) for i, j in edges)
    assert pairs == sorted(L.HIERARCHY_EDGES_ORIGINAL)
    # targets of each source are in descending virtual order (SortTensorAlongLastDimension DESC)
    for s in range(0, len(edges), 4):
        assert list(edges[s:s + 4, 1]) == sorted(edges[s:s + 4, 1], reverse=True)
    assert set(elayers.tolist()) == {1, 2}


def test_block_diagonal_cholesky_kat(oracle_mod):
    # cpp/tests/test_linalg_cholesky.cpp:38-102 (AllClose default rtol 1e-5, atol 1e-8 -> use 1e-4 abs for float32)
    for col in range(2):
        x, rc = oracle_mod.solve_block_diagonal(L.CHOLESKY_A, L.CHOLESKY_B[:, col], 0.0)
        assert rc == 0
        assert np.allclose(x, L.CHOLESKY_X[:, col], atol=2e-5, rtol=1e-4)


def test_rasterized_jacobians_vs_reference_numpy_derivation(oracle_mod):
    # golden vectors from math_check_scripts/dense_depth_jacobians.py (float64); the C++ adds K_EPSILON = 1e-8 to the
    # parallelogram area and to its square (BarycentricCoordinateJacobians.h), hence the area-dependent tolerance.
    g = np.load(os.path.join(GOLDEN, "dense_depth_jacobians_golden.npz"))
    size = int(g["image_size"])
    K = np.array([[size, 0, size / 2], [0, size, size / 2], [0, 0, 1.]])
    faces = np.array([[0, 1, 2]], np.int64)
    for i in range(len(g["vertices"])):
        u, v = (int(x) for x in g["pixel"][i])
        pf = -np.ones((size, size, 1), np.int64)
        pf[v, u, 0] = 0
        pb = np.zeros((size, size, 1, 3), np.float32)
        pb[v, u, 0] = g["bary"][i]
        vj, nj = oracle_mod.rasterized_surface_jacobians(g["vertices"][i].astype(np.float32), g["normals"][i].astype(np.float32), faces,
                                                         pf, pb, K, True)
        tol = 5e-5 + 4e-8 / max(float(g["area"][i]) ** 2, 1e-12)
        assert rel_err(vj[v, u], g["dwl_dV"][i]) < tol, i
        dnl = nj[v, u].reshape(-1)[:27].reshape(3, 9)
        assert np.abs(dnl - g["dnl_dV"][i]).max() <= tol * max(np.abs(g["dnl_dV"][i]).max(), 1.0), i
        assert np.allclose(nj[v, u].reshape(-1)[27:], g["bary"][i], atol=1e-6)


def test_rasterizer_binned_equals_brute_force_and_fast(oracle_mod):
    from dynamicfuion_python_amd import synthetic as S
    sc = S.make_scene("S1")
    a, w = oracle_mod.compute_anchors(sc.points, sc.nodes, 4, sc.coverage)
    wp, _ = oracle_mod.warp_mesh(sc.points, sc.normals, sc.nodes, sc.gt_rotations, sc.gt_translations, a, w)
    fndc, fm = oracle_mod.extract_face_ndc(wp, sc.faces, sc.K, sc.H, sc.W, 0.0, 10.0)
    binned = oracle_mod.rasterize(fndc, fm, sc.H, sc.W, 0.5, 1, -1, -1, True, False, True)
    brute = oracle_mod.rasterize(fndc, fm, sc.H, sc.W, 0.5, 1, 0, -1, True, False, True)
    fast = oracle_mod.rasterize_k1_fast(fndc, fm, sc.H, sc.W, 0.5, True, True)
    for x, y in zip(binned, brute):
        assert np.array_equal(x, y)
    for x, y in zip(binned, fast):
        assert np.array_equal(x, y)
    # faces_per_pixel = 4: queue semantics, sorted by (depth, face)
    fi4, dep4, _, _ = oracle_mod.rasterize(fndc, fm, sc.H, sc.W, 0.5, 4, -1, -1, True, False, True)
    assert np.array_equal(fi4[..., 0], binned[0][..., 0])
    d = np.where(fi4 >= 0, dep4, np.inf)
    assert (np.diff(d, axis=-1)[np.isfinite(d[..., 1:])] >= 0).all()


def test_one_node_plane_translation_converges(oracle_mod):
    # analogue of cpp/tests/test_deformable_mesh_fitter_one_node.cpp:52-128 (100x100, fx 100, target moved +0.2 in z;
    # the reference checks AllClose(t, (0, 0, 0.2), rtol 1.0, atol 1e-5) and R = I)
    xs = np.linspace(-0.5, 0.5, 33)
    X, Y = np.meshgrid(xs, xs)
    pts = np.stack([X, Y, np.full_like(X, 1.2)], -1).reshape(-1, 3).astype(np.float32)
    idx = np.arange(33 * 33).reshape(33, 33)
    a, b, c, d = idx[:-1, :-1].ravel(), idx[1:, :-1].ravel(), idx[:-1, 1:].ravel(), idx[1:, 1:].ravel()
    faces = np.concatenate([np.stack([a, b, c], 1), np.stack([c, b, d], 1)]).astype(np.int64)
    nrm = np.tile(np.array([[0, 0, -1]], np.float32), (len(pts), 1))
    K = np.array([[100, 0, 50], [0, 100, 50], [0, 0, 1.]])
    nodes = np.array([[0, 0, 1.2]], np.float32)
    I = np.eye(3, dtype=np.float32)[None]
    depth = render_target_oracle(oracle_mod, pts, nrm, faces, nodes, I, np.array([[0, 0, 0.2]], np.float32), K, 100, 100, 0.5, 1)
    refp, refm = oracle_mod.unproject(depth, K, 1.0, 10.0)
    R, t, _ = oracle_mod.fit(nodes=nodes, rotations=I, translations=np.zeros((1, 3), np.float32), mesh_points=pts, mesh_normals=nrm,
                             faces=faces, ref_points=refp, ref_mask=refm, H=100, W=100, K=K, max_iterations=1, lm_factor=0.001,
                             anchor_count=1, coverage=0.5)
    # x/y translation is unobservable on a fronto-parallel plane; our synthetic plane (not the download-only Blender
    # mesh) leaves ~1e-5 of noise there, hence atol 5e-5 instead of the reference's 1e-5
    assert np.allclose(t, [[0, 0, 0.2]], rtol=1.0, atol=5e-5)
    assert abs(t[0, 2] - 0.2) < 1e-3
    assert np.allclose(R, I, atol=1e-4)


def test_25_node_plane_fixture_runs(oracle_mod):
    # cpp/tests/test_deformable_mesh_fitter_advanced.cpp:55-143 (asserts only REQUIRE(true); parity unpinned)
    T = np.array([[-1, 0, 0, 0], [0, 1, 0, 0], [0, 0, -1, 1.2], [0, 0, 0, 1.]])
    Ps, Ns, Fs = read_ply(os.path.join(FIXTURES, "plane_skin_25_nodes_source.ply"))
    Pt, Nt, Ft = read_ply(os.path.join(FIXTURES, "plane_skin_25_nodes_target.ply"))
    assert len(Ps) == 81 and len(Fs) == 128
    Ps, Ns = transform_mesh(Ps, Ns, T)
    Pt, Nt = transform_mesh(Pt, Nt, T)
    nodes = np.load(os.path.join(FIXTURES, "nodes_25-node_plane.npy")).astype(np.float32)
    nodes = (nodes.astype(np.float64) @ T[:3, :3].T + T[:3, 3]).astype(np.float32)
    K = np.array([[100.0, 0, 50], [0, 100.0, 50], [0, 0, 1]])
    fndc, fm = oracle_mod.extract_face_ndc(Pt, Ft, K, 100, 100, 0.0, 10.0)
    fi, dep, _, _ = oracle_mod.rasterize(fndc, fm, 100, 100, 0.0, 1, -1, -1, True, False, True)
    depth = np.where(dep[..., 0] > 0, dep[..., 0], 0).astype(np.float32)
    assert (depth > 0).sum() > 1000
    refp, refm = oracle_mod.unproject(depth, K, 1.0, 10.0)
    weights = oracle_mod.node_coverage_weights(nodes, 0.1)
    I = np.tile(np.eye(3, dtype=np.float32), (25, 1, 1))
    R, t, dg = oracle_mod.fit(nodes=nodes, rotations=I, translations=np.zeros((25, 3), np.float32), mesh_points=Ps, mesh_normals=Ns,
                              faces=Fs, ref_points=refp, ref_mask=refm, H=100, W=100, K=K, max_iterations=1, lm_factor=0.001,
                              coverage=0.1, coverage_method=1, node_weights=weights)
    assert np.isfinite(R).all() and np.isfinite(t).all()
    assert dg["residual_mask"].sum() > 500


def test_anchor_knn_matches_sorted_distances(oracle_mod):
    rng = np.random.default_rng(0)
    pts = rng.normal(size=(500, 3)).astype(np.float32)
    nodes = rng.normal(size=(40, 3)).astype(np.float32)
    a, w = oracle_mod.compute_anchors(pts, nodes, 4, 0.5)
    d = ((pts[:, None, :] - nodes[None]) ** 2).sum(-1)
    ref = np.sort(np.argsort(d, 1)[:, :4], 1)
    assert np.array_equal(np.sort(a, 1), ref)
    assert np.allclose(w.sum(1), 1, atol=1e-5)


def test_reference_float_order_noise_is_below_summation_bound(oracle_mod):
    """The reference sums the data-term products serially in float; the checker sums them in double. On S1 the two
    agree to float rounding in H and g, and the solved update moves by no more than the conditioning of the node
    blocks amplifies that rounding (DESIGN.md "Numerics": at C2 the same comparison gives ~4e-4)."""
    from _util import oracle_fit_scene, rel_err, scene_target
    from dynamicfuion_python_amd import synthetic as S
    sc = S.make_scene("S1")
    depth = scene_target(oracle_mod, sc)
    try:
        oracle_mod.set_accumulate_double(False)
        _, _, f = oracle_fit_scene(oracle_mod, sc, depth, 1, lm=0.001)
    finally:
        oracle_mod.set_accumulate_double(True)
    _, _, d = oracle_fit_scene(oracle_mod, sc, depth, 1, lm=0.001)
    assert rel_err(f["hessian_diag"], d["hessian_diag"]) < 1e-5
    assert rel_err(f["gradient"], d["gradient"]) < 1e-5
    assert rel_err(f["updates"], d["updates"]) < 1e-4
    assert np.array_equal(f["residuals"], d["residuals"])


def test_fused_jacobian_mode_is_the_same_expression(oracle_mod):
    """The checker's fused pixel-node Jacobian mode (the GPU's FMA form, NNRT_JAC_FMA) restates the same expression as
    the reference's unfused one: stored rows R (v - g), w and R n equal -(-w R (v - g)) / w to rounding, and a whole S1
    GN iteration agrees with the reference arithmetic to float rounding in H, g and the update (residuals exactly)."""
    from _util import oracle_fit_scene, rel_err, scene_target
    from dynamicfuion_python_amd import synthetic as S
    rng = np.random.default_rng(3)
    pts = rng.normal(size=(300, 3)).astype(np.float32)
    nrm = rng.normal(size=(300, 3)).astype(np.float32)
    nodes = rng.normal(size=(20, 3)).astype(np.float32)
    R = np.stack([oracle_mod.rodrigues(rng.normal(size=(1, 3)).astype(np.float32)).reshape(3, 3) for _ in range(20)])
    a, w = oracle_mod.compute_anchors(pts, nodes, 4, 2.0)
    vj, nj = oracle_mod.warped_surface_jacobians(pts, nrm, nodes, R, a, w)
    try:
        oracle_mod.set_fused_jacobians(True)
        fvj, fnj = oracle_mod.warped_surface_jacobians(pts, nrm, nodes, R, a, w)
        sc = S.make_scene("S1")
        depth = scene_target(oracle_mod, sc)
        _, _, f = oracle_fit_scene(oracle_mod, sc, depth, 1, lm=0.001)
    finally:
        oracle_mod.set_fused_jacobians(False)
    on = a >= 0
    assert np.array_equal(fvj[..., 3][on], vj[..., 3][on])
    wv = w[..., None].astype(np.float64)
    assert np.abs(-wv * fvj[..., :3] - vj[..., :3])[on].max() < 1e-5 * np.abs(vj[..., :3]).max()
    assert np.abs(-wv * fnj - nj)[on].max() < 1e-5 * np.abs(nj).max()
    assert not np.array_equal(-wv * fvj[..., :3], vj[..., :3])   # the mode is in effect
    _, _, d = oracle_fit_scene(oracle_mod, sc, depth, 1, lm=0.001)
    assert np.array_equal(f["residuals"], d["residuals"])
    assert rel_err(f["hessian_diag"], d["hessian_diag"]) < 1e-5
    assert rel_err(f["gradient"], d["gradient"]) < 1e-5
    assert rel_err(f["updates"], d["updates"]) < 1e-4


def test_normals_restatement_properties(oracle_mod):
    """Normals restatement (NormalsOperationsImpl.h): a flat z = const grid facing the camera gives (0, 0, -1) ordered
    normals inside and zeros on the border; vertex normals of a two-triangle quad are the sum of its face normals."""
    O = oracle_mod
    H, W = 6, 7
    ys, xs = np.mgrid[0:H, 0:W].astype(np.float32)
    pts = np.stack([xs * 0.01, ys * 0.01, np.full_like(xs, 1.5)], -1).reshape(-1, 3)
    n = O.ordered_point_cloud_normals(pts, H, W).reshape(H, W, 3)
    assert np.all(n[0] == 0) and np.all(n[-1] == 0) and np.all(n[:, 0] == 0) and np.all(n[:, -1] == 0)
    assert np.allclose(n[1:-1, 1:-1], (0.0, 0.0, -1.0))
    v = np.array([[0, 0, 0], [1, 0, 0], [1, 1, 0], [0, 1, 0]], np.float32)
    f = np.array([[0, 1, 2], [0, 2, 3]], np.int64)
    tn = O.triangle_normals(v, f, normalized=False)
    assert np.array_equal(tn, np.array([[0, 0, 1], [0, 0, 1]], np.float32))
    vn = O.vertex_normals(v, f, normalized=False)
    assert np.array_equal(vn, np.array([[0, 0, 2], [0, 0, 1], [0, 0, 2], [0, 0, 1]], np.float32))
    assert np.array_equal(O.vertex_normals(v, f)[:, 2], np.ones(4, np.float32))
    z = O.triangle_normals(np.zeros((3, 3), np.float32), np.array([[0, 1, 2]]), normalized=True)
    assert np.array_equal(z, np.zeros((1, 3), np.float32))   # Eigen normalize leaves zero vectors at zero


# ---------------------------------------------------------------------------------------------------------------------
# round 2: the remaining in-container reference KATs / fixtures on the nnrt.geometry.functional / rendering surface
# ---------------------------------------------------------------------------------------------------------------------
def _sorted_desc(a):
    return -np.sort(-np.asarray(a), axis=1)


def test_anchor_variable_weight_kat(oracle_mod):
    # cpp/tests/test_anchor_computation.cpp:30-83: 2 nodes for 4 anchors (empty slots -1 / weight 0)
    a, w = oracle_mod.compute_anchors(L.ANCHOR_VAR_VERTICES, L.ANCHOR_VAR_NODES, 4, node_weights=L.ANCHOR_VAR_NODE_WEIGHTS)
    assert np.array_equal(_sorted_desc(a), L.ANCHOR_VAR_ANCHORS_SORTED)
    assert np.allclose(_sorted_desc(w), L.ANCHOR_VAR_WEIGHTS_SORTED, rtol=1e-3, atol=1e-6)


def test_unproject_kat(oracle_mod):
    # cpp/tests/test_unproject_3d_points.cpp:30-78 (uint16 depth, scale 1000, max 3)
    p, m = oracle_mod.unproject_image(L.UNPROJECT_DEPTH, L.UNPROJECT_K, None, 1000.0, 3.0)
    assert np.allclose(p, L.UNPROJECT_POINTS, rtol=1e-5, atol=1e-8)
    assert np.array_equal(m, L.UNPROJECT_MASK)


def test_unproject_extrinsics_is_pose_transform(oracle_mod):
    # extrinsics E -> points in the frame of E^-1 (PerspectiveProjectionImpl.h:88-89): E applied to them gives camera points
    rng = np.random.default_rng(3)
    depth = rng.uniform(0.5, 2.5, (6, 7)).astype(np.float32)
    c, s = np.cos(0.3), np.sin(0.3)
    E = np.array([[c, -s, 0, 0.1], [s, c, 0, -0.2], [0, 0, 1, 0.3], [0, 0, 0, 1]])
    p0, m0 = oracle_mod.unproject_image(depth, L.UNPROJECT_K, None, 1.0, 3.0)
    p1, m1 = oracle_mod.unproject_image(depth, L.UNPROJECT_K, E, 1.0, 3.0)
    assert np.array_equal(m0, m1)
    back = p1.astype(np.float64) @ E[:3, :3].T + E[:3, 3]
    assert np.allclose(back, p0, atol=1e-6)


def test_multiple_meshes_ndc_fixture(oracle_mod):
    # cpp/tests/test_extract_face_vertices.cpp:72-100: faces of [plane, sphere] concatenated in mesh order
    V0, _, F0 = xy_plane(1.2615, (0, 0, 1), 4)
    V1, F1 = sphere_open3d(0.4, 32, (0.0, 0.0, 0.5))
    K = np.array([[580., 0., 320.], [0., 580., 240.], [0., 0., 1.]])
    a, ma = oracle_mod.extract_face_ndc(V0, F0, K, 480, 640, 0.0, 2.0)
    b, mb = oracle_mod.extract_face_ndc(V1, F1, K, 480, 640, 0.0, 2.0)
    mask = np.concatenate([ma, mb]).astype(bool)
    ndc = np.concatenate([a, b]).reshape(-1, 3, 3)
    ndc[~mask] = 0
    gv = np.load(os.path.join(FIXTURES, "extracted_face_vertices_multiple_meshes.npy"))
    gm = np.load(os.path.join(FIXTURES, "extracted_face_mask_multiple_meshes.npy"))
    assert mask.sum() == L.MULTI_MESH_KEPT and np.array_equal(mask, gm)
    n = L.MULTI_MESH_COMPARED_FACES
    assert np.allclose(ndc[:n], gv[:n], atol=1e-5)


def test_red_shorts_ordered_normals_fixture(oracle_mod):
    # cpp/tests/test_normals_operations.cpp:113-136: the fixture is reproduced bit for bit on every pixel whose four
    # neighbours have depth (the tensor unprojection at scale 1000, then the ordered normals); elsewhere it holds zeros
    depth = read_depth_png(os.path.join(FIXTURES, "red_shorts_200_depth.png"))
    H, W = depth.shape
    p, _ = oracle_mod.unproject_image(depth, L.RED_SHORTS_K, None, 1000.0, 1000.0)
    n = oracle_mod.ordered_point_cloud_normals(p, H, W).reshape(H, W, 3)
    gt = np.load(os.path.join(FIXTURES, "red_shorts_200_normals.npy"))
    inner = neighbours_valid(depth > 0)
    assert np.array_equal(n[inner], gt[inner])
    assert not gt[~inner].any()


def test_warp_points_threshold_semantics(oracle_mod):
    # BlendWarp_ValidAnchorCountThreshold (WarpUtilities.h:505-580): points with fewer valid anchors than the minimum
    # stay zero; with online threshold anchors the -1 slots are exactly the ones beyond 2c
    rng = np.random.default_rng(5)
    nodes = rng.uniform(-1, 1, (12, 3)).astype(np.float32)
    pts = rng.uniform(-1.2, 1.2, (300, 3)).astype(np.float32)
    R = np.tile(np.eye(3, dtype=np.float32), (12, 1, 1))
    t = rng.normal(0, 0.1, (12, 3)).astype(np.float32)
    a, w = oracle_mod.compute_anchors(pts, nodes, 4, 0.3, minimum_valid_anchor_count=0, threshold=True)
    valid = (a != -1).sum(1)
    assert 0 < (valid < 2).sum() < len(pts)
    wp, _ = oracle_mod.warp_points(pts, None, nodes, R, t, a, w, minimum_valid=2)
    assert not wp[valid < 2].any()
    ref, _ = oracle_mod.warp_points(pts, None, nodes, R, t, a, w)
    assert np.array_equal(wp[valid >= 2], ref[valid >= 2])


def test_invert_psd_blocks_kat(oracle_mod):
    # cpp/tests/test_linalg_block_routines.cpp:158-190 (potrf + potrs against the identity, InvertBlocks.cpp:82-126)
    inv, rc = oracle_mod.invert_psd_blocks(L.INVERT_PSD_BLOCKS)
    assert rc == 0
    assert np.allclose(inv, L.INVERT_PSD_BLOCKS_GT, rtol=1e-4, atol=1e-8)
    # 6x6 blocks (the arrowhead stem's D^-1): inverse times block is the identity
    rng = np.random.default_rng(3)
    a = rng.normal(size=(5, 6, 6)).astype(np.float32)
    spd = (a @ a.transpose(0, 2, 1) + 6 * np.eye(6, dtype=np.float32)).astype(np.float32)
    inv6, rc6 = oracle_mod.invert_psd_blocks(spd)
    assert rc6 == 0
    assert np.allclose(inv6.astype(np.float64) @ spd.astype(np.float64), np.eye(6), atol=1e-4)
    bad = spd.copy()
    bad[2] = -bad[2]
    assert oracle_mod.invert_psd_blocks(bad)[1] == 3


# ---- block-sparse stages of the arrowhead solve: cpp/tests/test_linalg_matmul_block_sparse.cpp,
# cpp/tests/test_linalg_block_routines.cpp (AllClose defaults rtol 1e-5 / atol 1e-8 unless the test states otherwise) ----

def _padded_rowwise_gt():
    blocks = list(L.ROWWISE_C)
    for i in L.ROWWISE_PADDED_ZERO_BLOCKS:
        blocks.insert(i, np.zeros((3, 3), np.float32))
    return np.stack(blocks)


def test_matmul_block_sparse_row_wise_kat(oracle_mod):
    # test_linalg_matmul_block_sparse.cpp:30-220
    c, mask, rc = oracle_mod.matmul_block_sparse_row_wise(L.ROWWISE_A, L.ROWWISE_B, L.ROWWISE_B_COORDS)
    assert rc == 0
    assert np.allclose(c, _padded_rowwise_gt(), rtol=1e-5, atol=1e-8)
    assert np.allclose(c[mask], L.ROWWISE_C, rtol=1e-5, atol=1e-8)
    assert np.array_equal(L.ROWWISE_B_COORDS[mask], L.ROWWISE_C_COORDS)


@pytest.mark.parametrize("case", sorted(L.MBS_CASES))
def test_matmul_block_sparse_kat(oracle_mod, case):
    # test_linalg_matmul_block_sparse.cpp:233-386
    (lhs, tl, rhs, tr), gt_blocks, gt_coords = L.MBS_CASES[case]
    ops = {"A": (L.MBS_A, L.MBS_A_BOARD), "B": (L.MBS_B, L.MBS_B_BOARD)}
    c, mask, rc = oracle_mod.matmul_block_sparse(*ops[lhs], tl, *ops[rhs], tr)
    assert rc == 0
    out_cols = (ops[rhs][1].shape[0] if tr else ops[rhs][1].shape[1])
    coords = np.stack(np.nonzero(mask.reshape(-1, out_cols)), axis=1)
    assert np.allclose(c[mask], gt_blocks, rtol=1e-5, atol=1e-8)
    assert np.array_equal(coords, gt_coords)


def test_block_sparse_and_vector_product_kat(oracle_mod):
    # test_linalg_matmul_block_sparse.cpp:398-486
    c, rc = oracle_mod.block_sparse_and_vector_product(L.MBS_A, 4, L.BSV_A_COORDS, (0, 0), False, L.BSV_V)
    assert rc == 0 and np.allclose(c, L.BSV_C, rtol=1e-5, atol=1e-8)
    d, rc = oracle_mod.block_sparse_and_vector_product(L.MBS_B, 4, L.BSV_B_COORDS, (0, 0), True, L.BSV_V)
    assert rc == 0 and np.allclose(d, L.BSV_D, rtol=1e-5, atol=1e-8)
    # a block beyond m is reported, not written
    assert oracle_mod.block_sparse_and_vector_product(L.MBS_A, 2, L.BSV_A_COORDS, (0, 0), False, L.BSV_V)[1] == 1


def test_diagonal_block_sparse_and_vector_product_kat(oracle_mod):
    # test_linalg_matmul_block_sparse.cpp:499-531
    assert np.allclose(oracle_mod.diagonal_block_sparse_and_vector_product(L.DBSV_D, L.BSV_V), L.DBSV_C, rtol=1e-5, atol=1e-8)


@pytest.mark.parametrize("upper", [False, True])
def test_invert_triangular_blocks_kat(oracle_mod, upper):
    # test_linalg_block_routines.cpp:32-110 (AllClose rtol 1e-4)
    inv, rc = oracle_mod.invert_triangular_blocks(L.TRI_UPPER if upper else L.TRI_LOWER, upper)
    assert rc == 0
    assert np.allclose(inv, L.TRI_UPPER_INV if upper else L.TRI_LOWER_INV, rtol=1e-4, atol=1e-8)
    singular = L.TRI_LOWER.copy()
    singular[1, 2, 2] = 0
    assert oracle_mod.invert_triangular_blocks(singular, False)[1] == 1


def test_fill_and_get_blocks_kat(oracle_mod):
    # test_linalg_block_routines.cpp:207-400
    diag_gt = np.zeros((12, 12), np.float32)
    for i in range(6):
        diag_gt[2 * i:2 * i + 2, 2 * i:2 * i + 2] = L.ARANGE_BLOCKS[i]
    m = np.zeros((12, 12), np.float32)
    assert oracle_mod.sparse_blocks_op(m, L.ARANGE_BLOCKS, None) == 0
    assert np.array_equal(m, diag_gt)
    assert np.array_equal(oracle_mod.get_sparse_blocks(diag_gt, 2)[0], L.ARANGE_BLOCKS)
    m = np.zeros((12, 12), np.float32)
    assert oracle_mod.sparse_blocks_op(m, L.ARANGE_BLOCKS, L.SPARSE_COORDS) == 0
    assert np.array_equal(m, L.SPARSE_FILLED)
    assert oracle_mod.sparse_blocks_op(m, L.TRANSPOSE_FILL_BLOCKS, L.TRANSPOSE_FILL_COORDS, transpose=True) == 0
    assert np.array_equal(m, L.SPARSE_FILLED_2)
    assert np.array_equal(oracle_mod.get_sparse_blocks(L.SPARSE_FILLED, 2, L.SPARSE_COORDS)[0], L.ARANGE_BLOCKS)
    # subtract undoes add; a block past the matrix edge is reported
    m2 = L.SPARSE_FILLED.copy()
    oracle_mod.sparse_blocks_op(m2, L.ARANGE_BLOCKS, L.SPARSE_COORDS, op=1)
    oracle_mod.sparse_blocks_op(m2, L.ARANGE_BLOCKS, L.SPARSE_COORDS, op=2)
    assert np.array_equal(m2, L.SPARSE_FILLED)
    assert oracle_mod.sparse_blocks_op(np.zeros((12, 12), np.float32), L.ARANGE_BLOCKS, L.SPARSE_COORDS, offset=(1, 0)) == 1


def test_block_sparse_pieces_compose_the_stem_schur_complement(oracle_mod):
    """SchurComplement.cpp:43-78 composed from the restated pieces equals the dense S = C - W^T D^-1 W (float64 check)."""
    rng = np.random.default_rng(11)
    n0, n1, s = 5, 3, 6
    a = rng.normal(size=(n0, s, s))
    D = (a @ a.transpose(0, 2, 1) + 6 * np.eye(s)).astype(np.float32)
    wing_coords = np.array([[0, 0], [1, 0], [1, 2], [3, 1], [4, 2], [2, 1]], np.int32)
    W = rng.normal(size=(len(wing_coords), s, s)).astype(np.float32)
    C = np.eye(n1 * s, dtype=np.float32) * 50
    Dinv, rc = oracle_mod.invert_psd_blocks(D)
    assert rc == 0
    DinvW, mask, rc = oracle_mod.matmul_block_sparse_row_wise(Dinv, W, wing_coords)     # SolveBlockSparseArrowheadCholesky.cpp:54
    assert rc == 0 and mask.all()
    board = np.full((n0, n1), -1, np.int16)
    board[wing_coords[:, 0], wing_coords[:, 1]] = np.arange(len(wing_coords))
    prod, pmask, rc = oracle_mod.matmul_block_sparse(W, board, 1, DinvW, board, 0)        # SchurComplement.cpp:71-73
    assert rc == 0
    S = C.copy()
    coords = np.stack(np.nonzero(pmask.reshape(n1, n1)), axis=1).astype(np.int32)
    oracle_mod.sparse_blocks_op(S, prod[pmask], coords, op=2)                              # SchurComplement.cpp:75
    Wd = np.zeros((n0 * s, n1 * s))
    for (i, j), blk in zip(wing_coords, W):
        Wd[i * s:(i + 1) * s, j * s:(j + 1) * s] = blk
    Dd = np.zeros((n0 * s, n0 * s))
    for i in range(n0):
        Dd[i * s:(i + 1) * s, i * s:(i + 1) * s] = D[i]
    S_ref = C.astype(np.float64) - Wd.T @ np.linalg.solve(Dd, Wd)
    assert np.abs(S - S_ref).max() < 1e-3 * np.abs(S_ref).max()
