"""Generates the committed golden fixtures under tests/golden/ (run in the build container, where /root/reference exists).

1. Copies data files that the reference's own C++ tests hold (cpp/tests/test_data/...): the NDC-extraction fixture and the
   25-node plane scene. These are data (inputs/expected outputs), not source.
2. Generates per-pixel rasterized-surface Jacobian golden vectors by importing the reference's numpy derivation
   math_check_scripts/dense_depth_jacobians.py (float64) on seeded random front-facing triangles.

The reference is never needed at test time: tests read only the files written here.
"""
import contextlib
import importlib.util
import io
import os
import shutil
import sys

import numpy as np

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
FIX = os.path.join(HERE, "reference_fixtures")

COPY = [
    "cpp/tests/test_data/arrays/extracted_face_vertices.npy",
    "cpp/tests/test_data/arrays/extracted_face_mask.npy",
    "cpp/tests/test_data/arrays/nodes_25-node_plane.npy",
    "cpp/tests/test_data/arrays/edges_25-node_plane.npy",
    "cpp/tests/test_data/arrays/node_rotations_25-node_plane.npy",
    "cpp/tests/test_data/arrays/node_translations_25-node_plane.npy",
    "cpp/tests/test_data/meshes/plane_skin_25_nodes_source.ply",
    "cpp/tests/test_data/meshes/plane_skin_25_nodes_target.ply",
    "cpp/tests/test_data/arrays/extracted_face_vertices_multiple_meshes.npy",
    "cpp/tests/test_data/arrays/extracted_face_mask_multiple_meshes.npy",
    "cpp/tests/test_data/arrays/red_shorts_200_normals.npy",
    "cpp/tests/test_data/images/red_shorts_200_depth.png",
]


def copy_fixtures():
    os.makedirs(FIX, exist_ok=True)
    for rel in COPY:
        shutil.copyfile(os.path.join(REF, rel), os.path.join(FIX, os.path.basename(rel)))


def dense_depth_jacobian_goldens(count=64, seed=7):
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    spec = importlib.util.spec_from_file_location("dense_depth_jacobians", os.path.join(REF, "math_check_scripts/dense_depth_jacobians.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    rng = np.random.default_rng(seed)
    size = 100   # the script's NDC intrinsics (2, -2, 0, 0) == a 100x100 image with fx = fy = 100, cx = cy = 50
    rows = dict(vertices=[], normals=[], pixel=[], bary=[], dwl_dV=[], dnl_dV=[], area=[])
    # KAT pixel (48, 48) of the 1-node plane test (dense_depth_jacobians.py:34-49)
    tp = m.translation_case_pixel4848
    cases = [(np.stack([tp.face_vertex0, tp.face_vertex1, tp.face_vertex2]), np.stack([tp.face_normal0, tp.face_normal1, tp.face_normal2]),
              (48, 48))]
    while len(cases) < count:
        c = np.array([rng.uniform(-.2, .2), rng.uniform(-.2, .2), rng.uniform(1, 2)])
        V = c + rng.normal(0, 0.06, (3, 3))
        nd = np.array([[2 * v[0] / v[2], -2 * v[1] / v[2]] for v in V])
        area = (nd[0, 0] - nd[1, 0]) * (nd[1, 1] - nd[2, 1]) - (nd[0, 1] - nd[1, 1]) * (nd[1, 0] - nd[2, 0])
        if abs(area) < 2e-3:
            continue
        if area < 0:
            V = V[[0, 2, 1]]
        Nn = rng.normal(0, 1, (3, 3))
        Nn /= np.linalg.norm(Nn, axis=1, keepdims=True)
        cen = V.mean(0)
        u = int((2 * cen[0] / cen[2] + 1) * size / 2)
        v = int((-2 * cen[1] / cen[2] + 1) * size / 2)
        cases.append((V, Nn, (u, v)))
    for V, Nn, (u, v) in cases:
        ray = np.array([-1 + (2 * u + 1) / size, -1 + (2 * v + 1) / size])
        with contextlib.redirect_stdout(io.StringIO()):
            (d0, d1, d2), bd = m.jacobian_barycentrics_perspective_distorted_wrt_vertices(V[0], V[1], V[2], m.intrinsics_ndc, ray)
            P = [m.jacobian_percpsective_projections_wrt_vertex(V[i], m.intrinsics_ndc) for i in range(3)]
            Jd = np.hstack((d0 @ P[0], d1 @ P[1], d2 @ P[2]))
            bc = m.perspective_correct_barycentrics(bd, V[0], V[1], V[2])
            Jc = m.jacobian_barycentrics_corrected_wrt_vertices(Jd, m.compute_jacobian_perspective_correction(bd, V[0], V[1], V[2]))
        ndc = np.array([[2 * x[0] / x[2], -2 * x[1] / x[2]] for x in V])
        area = (ndc[0, 0] - ndc[1, 0]) * (ndc[1, 1] - ndc[2, 1]) - (ndc[0, 1] - ndc[1, 1]) * (ndc[1, 0] - ndc[2, 0])
        rows["vertices"].append(V)
        rows["normals"].append(Nn)
        rows["pixel"].append((u, v))
        rows["bary"].append(bc)
        rows["dwl_dV"].append(V.T @ Jc + np.kron(bc, np.eye(3)))
        rows["dnl_dV"].append(Nn.T @ Jc)
        rows["area"].append(area)
    np.savez(os.path.join(HERE, "dense_depth_jacobians_golden.npz"), **{k: np.array(v) for k, v in rows.items()}, image_size=size)


if __name__ == "__main__":
    copy_fixtures()
    if "--copy-only" not in sys.argv:
        dense_depth_jacobian_goldens()
    print("golden fixtures written to", HERE)
