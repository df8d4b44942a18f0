"""CPU: the TSDF voxel-block-grid oracle restatement (oracle/tsdf_oracle.cpp) against the reference's own known-answer
tests (cpp/tests/test_non_rigid_surface_voxel_block_grid.cpp, transcribed in tests/golden/kat_literals.py) and
structural properties of the generated marching-cubes table."""
import numpy as np
import pytest

from golden import kat_literals as L
import _tsdf_util as TU


def test_warped_block_boxes_kat(oracle_mod):
    O = oracle_mod
    t = np.tile(L.VBG_BOX_TRANSLATION, (4, 1))
    R = np.tile(np.eye(3, dtype=np.float32), (4, 1, 1))
    boxes = O.warped_block_boxes(L.VBG_BOX_KEYS, L.VBG_BOX_VOXEL_SIZE * L.VBG_BOX_RESOLUTION, L.VBG_BOX_NODES, R, t,
                                 L.VBG_BOX_COVERAGE, 4, 0, np.eye(4))
    assert np.allclose(boxes, L.VBG_BOX_EXPECTED)


def test_boxes_intercepting_surface_mask_kat(oracle_mod):
    m = oracle_mod.boxes_mask(L.VBG_MASK_BOXES, L.VBG_MASK_DEPTH, L.VBG_MASK_K, 1.0, 100.0, 1, 0.5)
    assert np.array_equal(m.astype(bool), L.VBG_MASK_EXPECTED)


def _kat_volume(O, apply_oblique_test):
    plane, color, K, deformed, nodes, R, t = TU.reference_nonrigid_kat_inputs()
    g = O.OracleGrid(0.01, 8, "uint16", "uint16")
    blocks = g.touch(plane, K, np.eye(4), 1000.0, 3.0, 2.0)
    g.integrate(blocks, plane, color, K, K, np.eye(4), 1000.0, 3.0, 2.0)
    pts = TU.unproject_points(deformed, K)
    normals = O.ordered_point_cloud_normals(pts, 100, 100)
    cos = g.integrate_non_rigid(np.array([[0, 0, 1]], np.int32), nodes, R, t, 0.005, 4, 1, deformed, color, normals, K, K, np.eye(4),
                                1000.0, 3.0, 2.0, apply_oblique_test=apply_oblique_test)
    return g, blocks, cos


def test_integrate_non_rigid_kat(oracle_mod):
    """The reference KAT's expected rows follow from its code with the oblique-view test (`cosine > 0.5`,
    NonRigidSurfaceVoxelBlockGridImpl.h:192) left out: the camera-facing normals of ComputeOrderedPointCloudNormals
    (NormalsOperationsImpl.h:208-210) give cosine ~1 on the plane, which that test rejects. With the test, as the code
    reads, the non-rigid update never applies there; both facts are checked."""
    g, blocks, _ = _kat_volume(oracle_mod, apply_oblique_test=False)
    assert {tuple(b) for b in blocks} == {(x, y, 0) for x in (-1, 0) for y in (-1, 0)}
    rows = g.values_at(L.VBG_NR_QUERIES)
    assert np.allclose(rows, L.VBG_NR_EXPECTED, rtol=1e-5, atol=5e-6)
    g2, _, cos = _kat_volume(oracle_mod, apply_oblique_test=True)
    rows2 = g2.values_at(L.VBG_NR_QUERIES)
    assert (cos[20:80, 20:80] > 0.5).any()
    # as written: every row keeps its rigid-integration value (weight 1, the non-rigid pass never reached the update)
    assert np.allclose(rows2[:, 4], 1.0) and np.allclose(rows2[:, 5:], 100.0)
    assert np.allclose(rows2[[0, 3, 4], 3], 0.0, atol=1e-6)


def test_marching_cubes_table_properties(oracle_mod):
    """Each cube state's triangles use exactly its crossing edges; closed sphere -> watertight, consistently oriented,
    Euler characteristic 2, outward normals."""
    g = oracle_mod.OracleGrid(0.1, 8)
    coords = np.array([[x, y, z] for x in (-1, 0) for y in (-1, 0) for z in (-1, 0)], np.int32)
    g.activate(coords)
    vals = g.values_all()
    # write a sphere SDF through an integration-free path: tsdf from positions (radius 0.37, truncated to [-1, 1])
    r = np.linalg.norm(vals[:, :3] + 0.05, axis=1)
    _sphere_fill(oracle_mod, g, np.clip((r - 0.37) / 0.3, -1, 1).astype(np.float32))
    V, Nn, _, T = g.mesh(0.0)
    assert len(T) > 100
    edges = {}
    for tri in T:
        for a, b in ((tri[0], tri[1]), (tri[1], tri[2]), (tri[2], tri[0])):
            edges[(a, b)] = edges.get((a, b), 0) + 1
    assert all(c == 1 for c in edges.values()), "a directed edge repeats: inconsistent orientation"
    assert all((b, a) in edges for (a, b) in edges), "open boundary: not watertight"
    assert len(V) - len(edges) // 2 + len(T) == 2
    cen = V[T].mean(1)
    fn = np.cross(V[T[:, 1]] - V[T[:, 0]], V[T[:, 2]] - V[T[:, 0]])
    assert (np.einsum("ij,ij->i", fn, cen + 0.05) > 0).mean() > 0.99, "triangles must face away from negative tsdf"
    assert (np.einsum("ij,ij->i", Nn, V + 0.05) > 0).mean() > 0.99


def _sphere_fill(O, g, tsdf):
    # weights 1 (> threshold 0) and the given tsdf, written by integrating nothing and patching through a raw pointer
    import ctypes
    lib = O.lib()
    lib.orc_grid_set_values.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    w = np.ones_like(tsdf)
    lib.orc_grid_set_values(g.h, tsdf.ctypes.data, w.ctypes.data)
