"""GPU parity of the TSDF voxel block grid (csrc/tsdf.hip) against the oracle restatement (oracle/tsdf_oracle.cpp):
the reference KAT scene (cpp/tests/test_non_rigid_surface_voxel_block_grid.cpp) and a 640x480 synthetic frame with the
C1 / C2 warp graphs. Block order, voxel values, the cosine map, block sets and the extracted mesh (vertex and triangle
order included) are deterministic on both sides and compared exactly (float values bit-identical: same expression
order, -ffp-contract=off, correctly rounded division / square root, exp evaluated in double and rounded)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from _util import scene_target  # noqa: E402
import _tsdf_util as TU  # noqa: E402
from golden import kat_literals as L  # noqa: E402


@pytest.fixture(scope="module")
def nn():
    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible for a -m gpu test")
    from dynamicfuion_python_amd import nnrt
    return nnrt


def _np(t):
    return t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t)


def _wf(G, nodes, R, t, coverage, threshold=True, min_valid=1, K=4):
    wf = G.HierarchicalGraphWarpField(nodes, coverage, threshold, K, min_valid, G.WarpNodeCoverageComputationMethod.FIXED_NODE_COVERAGE, 1)
    wf.set_node_rotations(R)
    wf.set_node_translations(t)
    return wf


def test_boxes_and_mask_kats(nn):
    G = nn.geometry
    grid = G.NonRigidSurfaceVoxelBlockGrid(["tsdf", "weight"], ["float32", "float32"], [1, 1], L.VBG_BOX_VOXEL_SIZE, L.VBG_BOX_RESOLUTION, 16)
    R = np.tile(np.eye(3, dtype=np.float32), (4, 1, 1))
    wf = _wf(G, L.VBG_BOX_NODES, R, np.tile(L.VBG_BOX_TRANSLATION, (4, 1)), L.VBG_BOX_COVERAGE, threshold=False, min_valid=0)
    boxes = _np(grid.get_bounding_boxes_of_warped_blocks(L.VBG_BOX_KEYS, wf, np.eye(4)))
    assert np.allclose(boxes, L.VBG_BOX_EXPECTED)
    from dynamicfuion_python_amd.nnrt import voxel_grid as VG
    mask = _np(VG.get_axis_aligned_boxes_intersecting_surface_mask(L.VBG_MASK_BOXES, L.VBG_MASK_DEPTH, L.VBG_MASK_K, 1.0, 100.0,
                                                                             1, 0.5))
    assert np.array_equal(mask, L.VBG_MASK_EXPECTED)


def test_integrate_non_rigid_reference_kat_scene(nn, oracle_mod):
    """The reference KAT scene through the HIP grid equals the oracle exactly (as the reference code reads, oblique
    test included; tests/test_tsdf_oracle.py pins the oracle to the KAT's expected rows)."""
    G, O = nn.geometry, oracle_mod
    plane, color, K, deformed, nodes, R, t = TU.reference_nonrigid_kat_inputs()
    grid = G.NonRigidSurfaceVoxelBlockGrid(["tsdf", "weight", "color"], ["float32", "uint16", "uint16"], [1, 1, 3], 0.01, 8, 128)
    blocks = grid.compute_unique_block_coordinates(plane, K, np.eye(4), 1000.0, 3.0, 2.0)
    og = O.OracleGrid(0.01, 8, "uint16", "uint16")
    ob = og.touch(plane, K, np.eye(4), 1000.0, 3.0, 2.0)
    assert np.array_equal(_np(blocks), ob)
    grid.integrate(blocks, plane, color, K, K, np.eye(4), 1000.0, 3.0, 2.0)
    og.integrate(ob, plane, color, K, K, np.eye(4), 1000.0, 3.0, 2.0)
    pts = TU.unproject_points(deformed, K)
    normals = O.ordered_point_cloud_normals(pts, 100, 100)
    wf = _wf(G, nodes, R, t, 0.005)
    cos = grid.integrate_non_rigid(np.array([[0, 0, 1]], np.int32), wf, deformed, color, normals, K, K, np.eye(4), 1000.0, 3.0, 2.0)
    cos_o = og.integrate_non_rigid(np.array([[0, 0, 1]], np.int32), nodes, R, t, 0.005, 4, 1, deformed, color, normals, K, K, np.eye(4),
                                   1000.0, 3.0, 2.0)
    assert np.array_equal(_np(cos), cos_o)
    assert np.array_equal(_np(grid.get_block_coordinates()), og.block_coords())
    assert np.array_equal(_np(grid.extract_voxel_values_and_coordinates()), og.values_all())
    assert np.array_equal(_np(grid.extract_voxel_values_at(L.VBG_NR_QUERIES)), og.values_at(L.VBG_NR_QUERIES))


@pytest.mark.parametrize("name", ["C1", "C2"])
def test_fusion_frame_parity(nn, oracle_mod, name):
    """One DynamicFusion-style frame on a 640x480 synthetic depth (float32, color in [0, 1]): touch, rigid integrate,
    non-rigid integrate under the scene's ground-truth motion, truncation-region search, sleeve activation and marching
    cubes, all against the oracle."""
    from dynamicfuion_python_amd import synthetic as S
    G, O = nn.geometry, oracle_mod
    sc = S.make_scene(name, hierarchy_builder=lambda n, c, l: O.build_hierarchy(n, c, l))
    depth = scene_target(O, sc).astype(np.float32)
    color = np.random.default_rng(1).random(depth.shape + (3,), dtype=np.float32)
    E = np.eye(4)
    grid = G.NonRigidSurfaceVoxelBlockGrid(["tsdf", "weight", "color"], ["float32", "float32", "float32"], [1, 1, 3], 0.01, 8, 64)
    og = O.OracleGrid(0.01, 8, "float32", "float32")
    blocks = grid.compute_unique_block_coordinates(depth, sc.K, E, 1.0, 3.0, 4.0)
    ob = og.touch(depth, sc.K, E, 1.0, 3.0, 4.0)
    assert np.array_equal(_np(blocks), ob) and len(ob) > 100
    grid.integrate(blocks, depth, color, sc.K, sc.K, E, 1.0, 3.0, 4.0)
    og.integrate(ob, depth, color, sc.K, sc.K, E, 1.0, 3.0, 4.0)
    assert grid.get_block_count() == og.block_count() > 64   # grew past the initial capacity
    assert np.array_equal(_np(grid.extract_voxel_values_and_coordinates()), og.values_all())
    pts, _ = O.unproject(depth, sc.K, 1.0, 10.0)
    nrm = O.ordered_point_cloud_normals(pts, sc.H, sc.W)
    wf = _wf(G, sc.nodes, sc.gt_rotations, sc.gt_translations, sc.coverage)
    nodes_v = wf.get_node_positions(True)
    R_v, t_v = wf.get_node_rotations(True), wf.get_node_translations(True)
    new_blocks = grid.find_blocks_intersecting_truncation_region(depth, wf, sc.K, E, 1.0, 3.0, 4.0)
    nb_o = og.find_blocks_intersecting_truncation_region(depth, nodes_v, R_v, t_v, sc.coverage, 4, 1, sc.K, E, 1.0, 3.0, 4.0)
    assert np.array_equal(_np(new_blocks), nb_o)
    cos = grid.integrate_non_rigid(new_blocks, wf, depth, color, nrm, sc.K, sc.K, E, 1.0, 3.0, 4.0)
    cos_o = og.integrate_non_rigid(nb_o, nodes_v, R_v, t_v, sc.coverage, 4, 1, depth, color, nrm, sc.K, sc.K, E, 1.0, 3.0, 4.0)
    assert np.array_equal(_np(cos), cos_o) and (cos_o != 0).sum() > 1000
    assert np.array_equal(_np(grid.extract_voxel_values_and_coordinates()), og.values_all())
    mesh = grid.extract_triangle_mesh(0.0, -1)
    V, Nn, C, T = og.mesh(0.0)
    assert len(T) > 1000
    assert np.array_equal(_np(mesh.triangle_indices), T)
    assert np.array_equal(_np(mesh.vertex_positions), V)
    assert np.array_equal(_np(mesh.vertex_normals), Nn)
    assert np.array_equal(_np(mesh.vertex_colors), C)
    n_sleeve = grid.activate_sleeve_blocks()
    assert n_sleeve == len(og.inactive_neighbors())
    og.activate(og.inactive_neighbors())
    assert np.array_equal(_np(grid.get_block_coordinates()), og.block_coords())


def test_grid_errors_and_edge_cases(nn):
    G = nn.geometry
    with pytest.raises(RuntimeError):
        G.NonRigidSurfaceVoxelBlockGrid(["tsdf", "weight"], ["float32", "int8"], [1, 1], 0.01, 8, 16)
    grid = G.NonRigidSurfaceVoxelBlockGrid(["tsdf", "weight"], ["float32", "float32"], [1, 1], 0.01, 8, 16)
    with pytest.raises(RuntimeError):
        grid.activate(np.array([[1 << 21, 0, 0]], np.int32))
    grid.activate(np.zeros((0, 3), np.int32))
    empty = grid.extract_triangle_mesh(0.0)
    assert empty.triangle_indices.shape[0] == 0
    grid.activate(np.array([[0, 0, 0], [0, 0, 0], [1, 2, 3]], np.int32))   # duplicates collapse, first occurrence order
    assert np.array_equal(_np(grid.get_block_coordinates()), [[0, 0, 0], [1, 2, 3]])
    zero_depth = np.zeros((32, 32), np.float32)
    assert grid.compute_unique_block_coordinates(zero_depth, TU.simple_intrinsics(), np.eye(4), 1.0, 3.0, 4.0).shape[0] == 0
