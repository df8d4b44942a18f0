"""GPU parity of the nnrt mirror's drop-in surface (round 2): both overloads of warp_triangle_mesh / warp_point_cloud /
compute_point_to_plane_distances / get_mesh_ndc_face_vertices_and_clip_mask, unproject_raster_depth_without_filtering with
extrinsics, uint16 depth and preserve_pixel_layout, GraphWarpField.warp_mesh with thresholding, matmul3d and
median_grid_subsample_3d_points -- against the oracle (bit-exact: same float expression order on both sides) and against
the reference's KATs / fixtures (tests/golden/kat_literals.py, reference_fixtures/).
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from _util import FIXTURES, neighbours_valid, read_depth_png, sphere_open3d, xy_plane  # noqa: E402
from golden import kat_literals as L  # noqa: E402


@pytest.fixture(scope="module")
def nn():
    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible for a -m gpu test")
    from dynamicfuion_python_amd import _native
    _native.lib()
    from dynamicfuion_python_amd import nnrt
    return nnrt


def _np(t):
    return t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)


def _field(seed=0, n=40, v=5000):
    rng = np.random.default_rng(seed)
    nodes = rng.uniform(-1, 1, (n, 3)).astype(np.float32)
    pts = rng.uniform(-1.1, 1.1, (v, 3)).astype(np.float32)
    nrm = rng.normal(0, 1, (v, 3)).astype(np.float32)
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    w = rng.normal(0, 0.2, (n, 3))
    ang = np.linalg.norm(w, axis=1, keepdims=True)
    k = w / ang
    Kx = np.zeros((n, 3, 3))
    Kx[:, 0, 1], Kx[:, 0, 2], Kx[:, 1, 0], Kx[:, 1, 2], Kx[:, 2, 0], Kx[:, 2, 1] = -k[:, 2], k[:, 1], k[:, 2], -k[:, 0], -k[:, 1], k[:, 0]
    R = (np.eye(3) + np.sin(ang)[..., None] * Kx + (1 - np.cos(ang))[..., None] * (Kx @ Kx)).astype(np.float32)
    t = rng.normal(0, 0.05, (n, 3)).astype(np.float32)
    return nodes, pts, nrm, R, t


E_TEST = np.array([[0.9, -0.4358899, 0.0, 0.05], [0.4358899, 0.9, 0.0, -0.1], [0.0, 0.0, 1.0, 0.2], [0.0, 0.0, 0.0, 1.0]])


@pytest.mark.parametrize("threshold,min_valid", [(False, 0), (True, 0), (True, 2), (True, 4)])
@pytest.mark.parametrize("extrinsics", [None, E_TEST])
def test_warp_triangle_mesh_online_anchors(nn, oracle_mod, threshold, min_valid, extrinsics):
    """WarpTriangleMesh (Warping.cpp:169-220): online anchors (thresholded at 2c iff threshold_nodes_by_distance), points with
    fewer valid anchors than the minimum stay zero."""
    nodes, pts, nrm, R, t = _field()
    coverage = 0.25
    G = nn.geometry
    kw = {} if extrinsics is None else dict(extrinsics=extrinsics)
    out = G.functional.warp_triangle_mesh(G.TriangleMesh(pts, nrm, np.zeros((0, 3), np.int64)), nodes, R, t, 4, coverage, threshold, min_valid,
                                          **kw)
    a, w = oracle_mod.compute_anchors(pts, nodes, 4, coverage, minimum_valid_anchor_count=min_valid, threshold=threshold)
    wp, wn = oracle_mod.warp_points(pts, nrm, nodes, R, t, a, w, min_valid if threshold else -1, extrinsics)
    assert np.array_equal(_np(out.vertex_positions), wp)
    assert np.array_equal(_np(out.vertex_normals), wn)
    if threshold and min_valid > 0:
        assert (np.abs(wp).sum(1) == 0).any()   # some points really are dropped


@pytest.mark.parametrize("threshold,min_valid", [(False, 0), (True, 3)])
def test_warp_triangle_mesh_supplied_anchors_and_no_normals(nn, oracle_mod, threshold, min_valid):
    nodes, pts, nrm, R, t = _field(1)
    G = nn.geometry
    a, w = oracle_mod.compute_anchors(pts, nodes, 4, 0.3, minimum_valid_anchor_count=2)   # thresholded anchors with -1 slots
    out = G.functional.warp_triangle_mesh(G.TriangleMesh(pts, nrm, np.zeros((0, 3), np.int64)), nodes, R, t, anchors=a, anchor_weights=w,
                                          threshold_nodes_by_distance=threshold, minimum_valid_anchor_count=min_valid, extrinsics=E_TEST)
    wp, wn = oracle_mod.warp_points(pts, nrm, nodes, R, t, a, w, min_valid if threshold else -1, E_TEST)
    assert np.array_equal(_np(out.vertex_positions), wp) and np.array_equal(_np(out.vertex_normals), wn)
    bare = G.functional.warp_triangle_mesh(G.TriangleMesh(pts, None, None), nodes, R, t, a, w)   # positions only
    assert bare.vertex_normals is None
    wp0, _ = oracle_mod.warp_points(pts, None, nodes, R, t, a, w)
    assert np.array_equal(_np(bare.vertex_positions), wp0)


def test_warp_point_cloud_both_overloads(nn, oracle_mod):
    """WarpPointCloud (Warping.cpp:61-154): always the threshold variant, minimum_valid_anchor_count required."""
    nodes, pts, _, R, t = _field(2)
    G = nn.geometry
    pc = G.PointCloud(pts)
    out = G.functional.warp_point_cloud(pc, nodes, R, t, 4, 0.25, 2)
    a, w = oracle_mod.compute_anchors(pts, nodes, 4, 0.25, minimum_valid_anchor_count=2, threshold=True)
    wp, _ = oracle_mod.warp_points(pts, None, nodes, R, t, a, w, 2)
    assert np.array_equal(_np(out.point_positions), wp)
    out2 = G.functional.warp_point_cloud(pc, nodes, R, t, a, w, 3, E_TEST)
    wp2, _ = oracle_mod.warp_points(pts, None, nodes, R, t, a, w, 3, E_TEST)
    assert np.array_equal(_np(out2.point_positions), wp2)
    with pytest.raises(RuntimeError):
        G.functional.warp_point_cloud(pc, nodes, R, t, 4, 0.25, 5)   # minimum > anchor_count (Warping.cpp:76-79)


def test_graph_warp_field_warp_mesh_thresholded(nn, oracle_mod):
    """WarpField::WarpMesh (WarpField.cpp:100-143): disable_neighbor_thresholding=False applies the field's
    threshold_nodes_by_distance / minimum_valid_anchor_count."""
    nodes, pts, nrm, R, t = _field(3)
    G = nn.geometry
    wf = G.GraphWarpField(nodes, 0.25, True, 4, 2)
    wf.set_node_rotations(R)
    wf.set_node_translations(t)
    mesh = G.TriangleMesh(pts, nrm, np.zeros((0, 3), np.int64))
    out = wf.warp_mesh(mesh, False)
    a, w = oracle_mod.compute_anchors(pts, nodes, 4, 0.25, minimum_valid_anchor_count=2, threshold=True)
    wp, wn = oracle_mod.warp_points(pts, nrm, nodes, R, t, a, w, 2)
    assert np.array_equal(_np(out.vertex_positions), wp) and np.array_equal(_np(out.vertex_normals), wn)
    out_s = wf.warp_mesh(mesh, a, w, False)   # supplied-anchor overload, positional
    assert np.array_equal(_np(out_s.vertex_positions), wp)
    out_d = wf.warp_mesh(mesh)   # default: no thresholding
    a0, w0 = oracle_mod.compute_anchors(pts, nodes, 4, 0.25)
    wp0, _ = oracle_mod.warp_points(pts, nrm, nodes, R, t, a0, w0)
    assert np.array_equal(_np(out_d.vertex_positions), wp0)
    c = wf.clone()
    assert np.array_equal(c.get_node_translations(), wf.get_node_translations())
    assert np.allclose(wf.apply_transformations().nodes, nodes + t)
    assert np.array_equal(wf.get_node_extent(), np.stack([nodes.min(0), nodes.max(0)]))


def test_point_to_plane_both_overloads(nn, oracle_mod):
    nodes, pts, nrm, R, t = _field(4)
    G = nn.geometry
    other = pts + np.random.default_rng(0).normal(0, 0.01, pts.shape).astype(np.float32)
    d1 = G.functional.compute_point_to_plane_distances(G.TriangleMesh(pts, nrm, None), G.TriangleMesh(other, None, None))
    d2 = G.functional.compute_point_to_plane_distances(G.TriangleMesh(pts, nrm, None), G.PointCloud(other))
    ref = oracle_mod.point_to_plane(nrm, pts, other)
    assert np.array_equal(_np(d1), ref) and np.array_equal(_np(d2), ref)
    with pytest.raises(RuntimeError):
        G.functional.compute_point_to_plane_distances(G.TriangleMesh(pts, None, None), G.PointCloud(other))
    with pytest.raises(RuntimeError):
        G.functional.compute_point_to_plane_distances(G.TriangleMesh(pts, nrm, None), G.PointCloud(other[:-1]))


@pytest.mark.parametrize("layout", [False, True])
def test_unproject_kat(nn, layout):
    p, m = nn.geometry.functional.unproject_raster_depth_without_filtering(L.UNPROJECT_DEPTH, L.UNPROJECT_K, preserve_pixel_layout=layout)
    shape = (4, 4, 3) if layout else (16, 3)
    assert tuple(p.shape) == shape and tuple(m.shape) == shape[:-1]
    assert np.allclose(_np(p).reshape(-1, 3), L.UNPROJECT_POINTS, rtol=1e-5, atol=1e-8)
    assert np.array_equal(_np(m).reshape(-1), L.UNPROJECT_MASK)


def test_unproject_extrinsics_and_dtypes_vs_oracle(nn, oracle_mod):
    rng = np.random.default_rng(7)
    d16 = rng.integers(0, 4000, (48, 64)).astype(np.uint16)
    d32 = (d16.astype(np.float32) / 1000.0).astype(np.float32)
    K = np.array([[60.0, 0, 31.5], [0, 61.0, 23.2], [0, 0, 1]])
    for depth, scale in ((d16, 1000.0), (d32, 1.0)):
        for E in (np.eye(4), E_TEST):
            p, m = nn.geometry.functional.unproject_raster_depth_without_filtering(depth, K, E, scale, 3.0)
            po, mo = oracle_mod.unproject_image(depth, K, E, scale, 3.0)
            assert np.array_equal(_np(p), po) and np.array_equal(_np(m), mo)


def test_multiple_meshes_ndc_fixture(nn, oracle_mod):
    G, Rr = nn.geometry, nn.rendering
    V0, N0, F0 = xy_plane(1.2615, (0, 0, 1), 4)
    V1, F1 = sphere_open3d(0.4, 32, (0.0, 0.0, 0.5))
    K = np.array([[580., 0., 320.], [0., 580., 240.], [0., 0., 1.]])
    meshes = [G.TriangleMesh(V0, N0, F0), G.TriangleMesh(V1, None, F1)]
    ndc, mask, counts = Rr.functional.get_mesh_ndc_face_vertices_and_clip_mask(meshes, K, (480, 640), 0.0, 2.0)
    assert _np(counts).tolist() == [len(F0), len(F1)]
    gv = np.load(os.path.join(FIXTURES, "extracted_face_vertices_multiple_meshes.npy"))
    gm = np.load(os.path.join(FIXTURES, "extracted_face_mask_multiple_meshes.npy"))
    m = _np(mask)
    assert m.sum() == L.MULTI_MESH_KEPT and np.array_equal(m, gm)
    v = _np(ndc).copy()
    v[~m] = 0
    n = L.MULTI_MESH_COMPARED_FACES
    assert np.allclose(v[:n], gv[:n], atol=1e-5)
    for (a, fa) in ((0, F0), (1, F1)):   # = each mesh on its own, and = the oracle
        one, one_m = Rr.functional.get_mesh_ndc_face_vertices_and_clip_mask(meshes[a], K, (480, 640), 0.0, 2.0)
        off = 0 if a == 0 else len(F0)
        assert np.array_equal(_np(one), _np(ndc)[off:off + len(fa)]) and np.array_equal(_np(one_m), m[off:off + len(fa)])
        o, om = oracle_mod.extract_face_ndc((V0, V1)[a], fa, K, 480, 640, 0.0, 2.0)
        assert np.array_equal(np.where(om[:, None, None], o.reshape(-1, 3, 3), 0), np.where(om[:, None, None], _np(one), 0))


def test_red_shorts_ordered_normals_fixture(nn):
    """cpp/tests/test_normals_operations.cpp:113-136 through the GPU unprojection and ordered normals: bit-exact on every
    pixel whose four neighbours have depth (the fixture's domain; it holds zeros elsewhere)."""
    depth = read_depth_png(os.path.join(FIXTURES, "red_shorts_200_depth.png"))
    H, W = depth.shape
    G = nn.geometry
    p, _ = G.functional.unproject_raster_depth_without_filtering(depth, L.RED_SHORTS_K, depth_scale=1000.0, depth_max=1000.0)
    n = _np(G.functional.compute_ordered_point_cloud_normals(G.PointCloud(p), (H, W))).reshape(H, W, 3)
    gt = np.load(os.path.join(FIXTURES, "red_shorts_200_normals.npy"))
    inner = neighbours_valid(depth > 0)
    assert np.array_equal(n[inner], gt[inner])


def test_anchor_variable_weight_kat(nn):
    a, w = nn.geometry.functional.compute_anchors_and_weights_euclidean_variable_node_weight(
        L.ANCHOR_VAR_VERTICES, L.ANCHOR_VAR_NODES, L.ANCHOR_VAR_NODE_WEIGHTS, 4, 0)
    assert np.array_equal(-np.sort(-_np(a), axis=1), L.ANCHOR_VAR_ANCHORS_SORTED)
    assert np.allclose(-np.sort(-_np(w), axis=1), L.ANCHOR_VAR_WEIGHTS_SORTED, rtol=1e-3, atol=1e-6)


def test_invert_psd_blocks_kat(nn, oracle_mod):
    """cpp/tests/test_linalg_block_routines.cpp:158-190 through the C-ABI (the arrowhead stem's D^-1 device functions),
    bit-exact against the oracle's potrf + potrs restatement, and for 6x6 blocks; a non-PD block raises like potrf."""
    import torch
    from dynamicfuion_python_amd import _native as NV
    dev = torch.device("cuda", 0)

    def inv(blocks):
        d = torch.from_numpy(np.ascontiguousarray(blocks, np.float32)).to(dev)
        out = torch.empty_like(d)
        NV.check(NV.lib().nnrt_invert_positive_semidefinite_blocks(NV.ptr(d), d.shape[0], d.shape[1], NV.ptr(out), NV.stream_ptr()))
        return out.cpu().numpy()

    g = inv(L.INVERT_PSD_BLOCKS)
    assert np.allclose(g, L.INVERT_PSD_BLOCKS_GT, rtol=1e-4, atol=1e-8)
    assert np.array_equal(g, oracle_mod.invert_psd_blocks(L.INVERT_PSD_BLOCKS)[0])
    rng = np.random.default_rng(3)
    a = rng.normal(size=(300, 6, 6)).astype(np.float32)
    spd = (a @ a.transpose(0, 2, 1) + 6 * np.eye(6, dtype=np.float32)).astype(np.float32)
    assert np.array_equal(inv(spd), oracle_mod.invert_psd_blocks(spd)[0])
    bad = spd.copy()
    bad[7] = -bad[7]
    with pytest.raises(RuntimeError, match="potrf"):
        inv(bad)


def test_matmul3d_kat(nn):
    c = nn.core.matmul3d(L.MATMUL3D_A, L.MATMUL3D_B)
    assert np.allclose(_np(c), L.MATMUL3D_C, atol=1e-6)
    v = nn.core.matmul3d(L.MATMUL3D_A, L.MATMUL3D_B[:, :, 0])   # array of vectors -> [batch, m, 1]
    assert np.allclose(_np(v)[..., 0], L.MATMUL3D_C[..., 0], atol=1e-6)
    with pytest.raises(RuntimeError):
        nn.core.matmul3d(L.MATMUL3D_A, L.MATMUL3D_A)


def _medoids_reference(pts, cell):
    """GeometrySamplingMedian.h:264-296 restated: per grid cell (floor(p / cell)) the member with the smallest summed
    distance to the cell's members (float sums in ascending member order; first minimum wins); ascending indices."""
    keys = np.floor(pts / np.float32(cell)).astype(np.int64)
    cells = {}
    for i, k in enumerate(map(tuple, keys)):
        cells.setdefault(k, []).append(i)
    out = []
    for members in cells.values():
        best, best_i = np.float32(np.finfo(np.float32).max), members[0]
        for a in members:
            s = np.float32(0)
            for b in members:
                d = pts[b] - pts[a]
                s = np.float32(s + np.float32(np.sqrt(np.float32((d[0] * d[0] + d[1] * d[1]) + d[2] * d[2]))))
            if s < best:
                best, best_i = s, a
        out.append(best_i)
    return np.sort(np.array(out, np.int64))


def test_median_grid_subsample(nn):
    pts = np.random.default_rng(11).uniform(-1, 1, (600, 3)).astype(np.float32)
    got = _np(nn.geometry.functional.median_grid_subsample_3d_points(pts, 0.5))
    assert np.array_equal(got, _medoids_reference(pts, 0.5))


@pytest.mark.parametrize("kf", [1, 3, 8])
def test_rasterize_dense_sphere_array_vs_oracle(nn, oracle_mod, kf):
    """A dense mesh of sub-pixel triangles (the regime of the reference's 64-bunny benchmark, README.md:21-25): every
    fragment (face, depth, barycentrics, distance) identical to the oracle at K = 1, 3, 8."""
    from _util import sphere_open3d
    V1, F1 = sphere_open3d(0.06, 24)
    Vs, Fs = [], []
    for a in range(8):
        for c in range(8):
            Fs.append(F1 + len(V1) * len(Vs))
            Vs.append(V1 + np.array([(a - 3.5) * 0.11, (c - 3.5) * 0.085, 1.0 + 0.05 * ((a + c) % 3)], np.float32))
    V, F = np.concatenate(Vs), np.concatenate(Fs)
    K = np.array([[580., 0., 320.], [0., 580., 240.], [0., 0., 1.]])
    ndc, mask = oracle_mod.extract_face_ndc(V, F, K, 480, 640, 0.0, 10.0)
    ref = oracle_mod.rasterize(ndc, mask, 480, 640, 0.0, kf, -1, -1, False, False, True)
    got = nn.rendering.rasterize_ndc_triangles(ndc, mask, (480, 640), 0.0, kf, -1, -1, False, False, True)
    for r, g in zip(ref, got):
        assert np.array_equal(np.asarray(r).reshape(-1), _np(g).reshape(-1))
    assert (_np(got[0])[..., 0] >= 0).sum() > 1000
