"""The nnrt mirror keeps the reference bindings' argument names, order and defaults ("The build must keep
these signatures and defaults"). The reference side is tests/golden/reference_signatures.json, parsed from the
reference's pybind11 sources by tests/golden/make_signatures.py. CPU only: signatures are inspected, nothing is called.

Rule: for every reference overload of a name the mirror implements, the mirror has an overload whose leading parameters are
exactly the reference's names in order, with equal defaults where the reference has one and none where it has none;
extra mirror parameters may follow only with defaults (e.g. use_virtual_ordering, device).
"""
import inspect
import json
import math
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "reference_signatures.json")

# bindings outside SURVEY.md 8 (reason): not part of the mirror
OUT_OF_SCOPE = {
    ("nnrt.geometry.functional", "compute_anchors_and_weights_shortest_path_fixed_node_weight"): "shortest-path anchors: not on the fitter path",
    ("nnrt.geometry.functional", "compute_anchors_and_weights_shortest_path_variable_node_weight"): "shortest-path anchors: not on the fitter path",
    ("nnrt.geometry.functional", "mean_grid_downsample_3d_points"): "graph generation (apps), not on the fitter path",
    ("nnrt.geometry.functional", "closest_to_mean_grid_subsample_3d_points"): "graph generation (apps), not on the fitter path",
    ("nnrt.geometry.functional", "fast_mean_radius_downsample_3d_points"): "graph generation (apps), not on the fitter path",
    ("nnrt.geometry.functional", "fast_median_radius_subsample_3d_points"): "graph generation (apps), not on the fitter path",
    ("nnrt.core", "find_k_nearest_to_points"): "KdTree: the hierarchy's K-NN is built without one (csrc/hierarchy.hip)",
    ("nnrt.core", "__init__"): "KdTree: the hierarchy's K-NN is built without one (csrc/hierarchy.hip)",
}
VOXEL_GRID_OUT = {"voxel_indices", "voxel_coordinates", "voxel_coordinates_and_flattened_indices", "ray_cast", "extract_point_cloud", "save",
                  "attribute", "integrate"}   # integrate: one *args method dispatches the three overloads (tests/test_gpu_tsdf.py)


def _reference():
    with open(GOLDEN) as f:
        return json.load(f)


def _default(text):
    """C++ default text -> (python value, comparable)."""
    t = text.strip()
    if t in ("true", "false"):
        return t == "true"
    if t == "INFINITY":
        return math.inf
    if "Tensor::Eye(4" in t:
        return np.eye(4)
    if "Device(" in t:
        return "<device>"
    if t.rstrip("f").lstrip("-").replace(".", "", 1).isdigit():
        v = float(t.rstrip("f"))
        return int(v) if "." not in t and "f" not in t else v
    return t


def _equal(mine, ref):
    if isinstance(ref, str) and ref == "<device>":
        return True   # the mirror's device default is the current HIP device (one process per GPU)
    if isinstance(ref, np.ndarray):
        return isinstance(mine, (np.ndarray, list, tuple)) and np.array_equal(np.asarray(mine, np.float64), ref)
    if isinstance(ref, bool):
        return mine is ref or mine == ref
    if isinstance(ref, float) and math.isinf(ref):
        return isinstance(mine, float) and math.isinf(mine)
    return mine == ref


def _mirror_target(nn, row):
    mod, recv, name = row["module"], row["receiver"], row["name"]
    if mod == "nnrt.geometry" and recv == "graph_warp_field":
        cls = nn.geometry.HierarchicalGraphWarpField
        return (nn.geometry.GraphWarpField, True) if name == "__init__" else (getattr(cls, name, None), False)
    if mod == "nnrt.geometry" and recv in ("voxel_block_grid", "non_rigid_surface_voxel_block_grid"):
        cls = nn.geometry.VoxelBlockGrid if recv == "voxel_block_grid" else nn.geometry.NonRigidSurfaceVoxelBlockGrid
        return (getattr(cls, name, None), False)
    if mod == "nnrt.core.linalg":
        return getattr(nn.core.linalg, name, None), True
    if mod == "nnrt.core":
        return getattr(nn.core, name, None), True
    ns = {"nnrt.geometry.functional": nn.geometry.functional, "nnrt.rendering": nn.rendering,
          "nnrt.rendering.functional": nn.rendering.functional}[mod]
    return getattr(ns, name, None), True


def _signatures(fn, is_function):
    sigs = fn.signatures() if hasattr(fn, "signatures") else [inspect.signature(fn)]
    out = []
    for s in sigs:
        params = list(s.parameters.values())
        if not is_function and params and params[0].name == "self":
            params = params[1:]
        out.append(params)
    return out


def _matches(params, ref_args):
    if len(params) < len(ref_args):
        return False
    for p, (name, default) in zip(params, ref_args):
        if p.name != name or p.kind not in (p.POSITIONAL_OR_KEYWORD, p.POSITIONAL_ONLY):
            return False
        if default is None:
            if p.default is not inspect.Parameter.empty:
                return False
        elif p.default is inspect.Parameter.empty or not _equal(p.default, _default(default)):
            return False
    return all(p.default is not inspect.Parameter.empty or p.kind == p.VAR_KEYWORD for p in params[len(ref_args):])


def _in_scope(row):
    if (row["module"], row["name"]) in OUT_OF_SCOPE:
        return False
    if row["receiver"] == "voxel_block_grid" and row["name"] == "__init__" and not row["args"]:
        return False   # default-constructed empty grid: never used on the path
    if row["name"] == "compute_unique_block_coordinates" and row["args"] and row["args"][0][0] == "pcd":
        return False   # point-cloud overload: the fusion loop touches blocks from depth images
    if row["receiver"] in ("voxel_block_grid", "non_rigid_surface_voxel_block_grid") and row["name"] in VOXEL_GRID_OUT:
        return False
    return True


ROWS = [r for r in _reference()]


def test_fixture_covers_the_hot_path_bindings():
    names = {(r["module"], r["name"]) for r in ROWS}
    for must in [("nnrt.geometry.functional", "warp_triangle_mesh"), ("nnrt.geometry.functional", "warp_point_cloud"),
                 ("nnrt.geometry.functional", "compute_point_to_plane_distances"),
                 ("nnrt.geometry.functional", "unproject_raster_depth_without_filtering"),
                 ("nnrt.rendering", "rasterize_ndc_triangles"), ("nnrt.rendering.functional", "get_mesh_ndc_face_vertices_and_clip_mask"),
                 ("nnrt.core.linalg", "AxisAngleVectorsToMatricesRodrigues"), ("nnrt.geometry", "warp_mesh")]:
        assert must in names, must


@pytest.mark.parametrize("row", [r for r in ROWS if _in_scope(r)], ids=lambda r: f"{r['receiver']}.{r['name']}")
def test_mirror_signature_matches_reference(row):
    import dynamicfuion_python_amd.nnrt as nn
    fn, is_function = _mirror_target(nn, row)
    assert fn is not None, f"{row['module']}.{row['name']} is missing from the mirror"
    if row["args"] is None:   # positional-only binding (plain-string argument names): arity only
        return
    sigs = _signatures(fn, is_function)
    assert any(_matches(p, row["args"]) for p in sigs), (
        f"{row['module']}.{row['name']}: no mirror overload matches the reference arguments {row['args']}; mirror has "
        f"{[[(p.name, p.default) for p in ps] for ps in sigs]}")


def test_overload_dispatch_by_argument_kind():
    """pybind11 picks the first overload whose arguments convert: an int anchor_count selects the online-anchor overload,
    tensors select the supplied-anchor one; keywords of either overload bind."""
    import dynamicfuion_python_amd.nnrt as nn
    ov = nn.geometry.functional.warp_triangle_mesh
    calls = []
    saved = list(ov._overloads)
    try:
        ov._overloads = [(_rebind(f, calls, i), pred) for i, (f, pred) in enumerate(saved)]
        ov(None, 0, 0, 0, 4, 0.05)
        ov(None, 0, 0, 0, np.zeros((1, 4), np.int32), np.zeros((1, 4), np.float32))
        ov(input_mesh=None, nodes=0, node_rotations=0, node_translations=0, anchors=np.zeros((1, 4)), anchor_weights=np.zeros((1, 4)))
        ov(None, 0, 0, 0, anchor_count=2, node_coverage=0.1, minimum_valid_anchor_count=1)
    finally:
        ov._overloads = saved
    assert calls == [0, 1, 1, 0]
    assert len(saved) == 2
    with pytest.raises(TypeError):
        ov(None, 0, 0)


def _rebind(f, calls, i):
    sig = inspect.signature(f)

    def g(*a, **k):
        sig.bind(*a, **k)
        calls.append(i)
    g.__signature__ = sig
    return g
