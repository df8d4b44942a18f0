"""nnrt.geometry mirror: TriangleMesh container, WarpNodeCoverageComputationMethod, HierarchicalGraphWarpField /
GraphWarpField (cpp/geometry/HierarchicalGraphWarpField.h:37-97, cpp/pybind/geometry/geometry.cpp:278-320) and the
hot-path functions of nnrt.geometry.functional (cpp/pybind/geometry/functional/functional.cpp:52-140)."""
from __future__ import annotations

import ctypes
import enum
import types
from dataclasses import dataclass

import numpy as np
import torch

from .. import _native as N
from ._overloads import Overloaded, is_int, is_tensor
from ._tensors import to_device, to_host_f64


_EYE4 = np.eye(4)   # the bindings' default extrinsics (Tensor::Eye(4, Float64, CPU))


class WarpNodeCoverageComputationMethod(enum.IntEnum):
    FIXED_NODE_COVERAGE = 0
    MINIMAL_K_NEIGHBOR_NODE_DISTANCE = 1


@dataclass
class TriangleMesh:
    """Minimal stand-in for open3d.t.geometry.TriangleMesh on the hot path: positions [V,3] f32, normals [V,3] f32,
    triangle indices [F,3] int64 (any of numpy / torch)."""
    vertex_positions: object
    vertex_normals: object
    triangle_indices: object
    triangle_normals: object = None
    vertex_colors: object = None
    triangle_colors: object = None

    def on_device(self, device: torch.device):
        return (to_device(self.vertex_positions, torch.float32, device),
                None if self.vertex_normals is None else to_device(self.vertex_normals, torch.float32, device),
                to_device(self.triangle_indices, torch.int64, device))


@dataclass
class RGBDImage:
    """Stand-in for open3d.t.geometry.RGBDImage: colour [H,W,3] (unused by the fitter) and depth [H,W]."""
    color: object
    depth: object


class HierarchicalGraphWarpField:
    """Device-resident warp field with a regularization hierarchy (virtual node order = fine-to-coarse layers)."""

    def __init__(self, nodes, node_coverage: float = 0.05, threshold_nodes_by_distance: bool = False, anchor_count: int = 4,
                 minimum_valid_anchor_count: int = 0,
                 warp_node_coverage_computation_method=WarpNodeCoverageComputationMethod.MINIMAL_K_NEIGHBOR_NODE_DISTANCE,
                 layer_count: int = 4, max_vertex_degree: int = 4, layer_decimation_radii=None, device: int | None = None):
        device = N.current_device() if device is None else int(device)
        nodes_np = np.ascontiguousarray(nodes.detach().cpu().numpy() if isinstance(nodes, torch.Tensor) else nodes, dtype=np.float32)
        radii = None if layer_decimation_radii is None else np.ascontiguousarray(layer_decimation_radii, dtype=np.float32)
        h = ctypes.c_void_p()
        N.check(N.lib().nnrt_warp_field_create(N.ptr(nodes_np), len(nodes_np), float(node_coverage), int(threshold_nodes_by_distance),
                                               int(anchor_count), int(minimum_valid_anchor_count), int(warp_node_coverage_computation_method),
                                               int(layer_count), int(max_vertex_degree), N.ptr(radii), int(device), ctypes.byref(h)))
        self._h = h
        self._ctor = dict(nodes=nodes_np, node_coverage=node_coverage, threshold_nodes_by_distance=threshold_nodes_by_distance,
                          anchor_count=anchor_count, minimum_valid_anchor_count=minimum_valid_anchor_count,
                          warp_node_coverage_computation_method=warp_node_coverage_computation_method, layer_count=layer_count,
                          max_vertex_degree=max_vertex_degree, layer_decimation_radii=radii, device=device)
        self.device = device
        self.node_count = len(nodes_np)
        self.anchor_count = anchor_count
        self.node_coverage = node_coverage
        self.threshold_nodes_by_distance = bool(threshold_nodes_by_distance)
        self.minimum_valid_anchor_count = minimum_valid_anchor_count
        self.warp_node_coverage_computation_method = WarpNodeCoverageComputationMethod(warp_node_coverage_computation_method)

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                N.lib().nnrt_warp_field_destroy(h)
            except Exception:   # interpreter shutdown
                pass
            self._h = None

    @property
    def handle(self):
        return self._h

    def _get(self, fn, shape, virtual):
        out = np.empty(shape, np.float32)
        N.check(getattr(N.lib(), fn)(self._h, N.ptr(out), int(virtual)))
        return out

    def get_node_positions(self, use_virtual_ordering: bool = False) -> np.ndarray:
        return self._get("nnrt_warp_field_get_node_positions", (self.node_count, 3), use_virtual_ordering)

    def get_node_rotations(self, use_virtual_ordering: bool = False) -> np.ndarray:
        return self._get("nnrt_warp_field_get_node_rotations", (self.node_count, 3, 3), use_virtual_ordering)

    def get_node_translations(self, use_virtual_ordering: bool = False) -> np.ndarray:
        return self._get("nnrt_warp_field_get_node_translations", (self.node_count, 3), use_virtual_ordering)

    def set_node_rotations(self, node_rotations, use_virtual_ordering: bool = False):
        r = _host_f32(node_rotations)
        if r.shape != (self.node_count, 3, 3):
            raise RuntimeError(f"Tensor has shape {r.shape}, but is expected to have shape ({self.node_count}, 3, 3).")   # WarpField.cpp:171-176
        N.check(N.lib().nnrt_warp_field_set_node_rotations(self._h, N.ptr(r), int(use_virtual_ordering)))

    def set_node_translations(self, node_translations, use_virtual_ordering: bool = False):
        t = _host_f32(node_translations)
        if t.shape != (self.node_count, 3):
            raise RuntimeError(f"Tensor has shape {t.shape}, but is expected to have shape ({self.node_count}, 3).")
        N.check(N.lib().nnrt_warp_field_set_node_translations(self._h, N.ptr(t), int(use_virtual_ordering)))

    def translate_nodes(self, node_translation_deltas, use_virtual_ordering: bool = False):
        """t += deltas (HierarchicalGraphWarpField.cpp:261-270)"""
        self.set_node_translations(self.get_node_translations(use_virtual_ordering) + _host_f32(node_translation_deltas), use_virtual_ordering)

    def rotate_nodes(self, node_rotation_deltas, use_virtual_ordering: bool = False):
        """R <- R dR (right-multiplied, A10; HierarchicalGraphWarpField.cpp:272-282)"""
        R = self.get_node_rotations(use_virtual_ordering)
        self.set_node_rotations(np.einsum("nij,njk->nik", R, _host_f32(node_rotation_deltas)), use_virtual_ordering)

    @property
    def nodes(self) -> np.ndarray:
        """GraphWarpField.nodes (geometry.cpp:315, read-only node positions, original order)"""
        return self.get_node_positions()

    def get_node_extent(self) -> np.ndarray:
        """WarpField::GetNodeExtent (WarpField.cpp:93-98): [[min x, y, z], [max x, y, z]] of the node positions"""
        p = self.get_node_positions()
        return np.stack([p.min(0), p.max(0)])

    def clone(self) -> "HierarchicalGraphWarpField":
        """WarpField::Clone (WarpField.cpp:163-165): same nodes and parameters, copied motion"""
        c = HierarchicalGraphWarpField(**self._ctor)
        c.set_node_rotations(self.get_node_rotations())
        c.set_node_translations(self.get_node_translations())
        return c

    def apply_transformations(self) -> "HierarchicalGraphWarpField":
        """WarpField::ApplyTransformations (WarpField.cpp:158-161): a new field whose nodes are the warped nodes (motion reset)"""
        kw = dict(self._ctor)
        kw["nodes"] = self.get_warped_nodes()
        return HierarchicalGraphWarpField(**kw)

    def reset_rotations(self):
        """WarpField::ResetRotations (cpp/geometry/WarpField.cpp:151-156): identity rotations, translations kept."""
        self.set_node_rotations(np.tile(np.eye(3, dtype=np.float32), (self.node_count, 1, 1)))

    def get_warped_nodes(self) -> np.ndarray:
        """WarpField::GetWarpedNodes: node positions + translations (original order)."""
        return self.get_node_positions() + self.get_node_translations()

    warp_mesh = Overloaded("warp_mesh", "GraphWarpField.warp_mesh, both overloads (cpp/pybind/geometry/geometry.cpp:293-302 -> "
                                        "WarpField.cpp:100-143): anchors over the original-order nodes unless supplied; thresholded by the "
                                        "field's threshold_nodes_by_distance / minimum_valid_anchor_count unless disable_neighbor_thresholding.")

    @warp_mesh.overload(lambda a: not is_tensor(a["disable_neighbor_thresholding"]))
    def _warp_mesh_online(self, input_mesh, disable_neighbor_thresholding=True, extrinsics=_EYE4):
        threshold = False if disable_neighbor_thresholding else self.threshold_nodes_by_distance
        min_valid = 0 if disable_neighbor_thresholding else self.minimum_valid_anchor_count
        nodes, R, t = self.get_node_positions(), self.get_node_rotations(), self.get_node_translations()
        if self.warp_node_coverage_computation_method == WarpNodeCoverageComputationMethod.FIXED_NODE_COVERAGE:
            return warp_triangle_mesh(input_mesh, nodes, R, t, self.anchor_count, self.node_coverage, threshold, min_valid, extrinsics)
        # MINIMAL_K_NEIGHBOR_NODE_DISTANCE: the reference raises "Not implemented" (WarpField.cpp:119-121); here the anchors
        # use the field's per-node coverage weights (the fitter's own anchor rule: thresholded iff minimum > 0), then the
        # supplied-anchor warp
        weights = np.empty(self.node_count, np.float32)
        weights[self.get_virtual_node_indices()] = self.get_node_coverage_weights()
        p, _, _ = input_mesh.on_device(_dev())
        a, w = _anchors(p, nodes, self.anchor_count, 0.0, weights, min_valid if threshold else 0)
        return warp_triangle_mesh(input_mesh, nodes, R, t, a, w, threshold, min_valid, extrinsics)

    @warp_mesh.overload(lambda a: is_tensor(a["anchors"]))
    def _warp_mesh_supplied(self, input_mesh, anchors, anchor_weights, disable_neighbor_thresholding=True, extrinsics=_EYE4):
        threshold = False if disable_neighbor_thresholding else self.threshold_nodes_by_distance
        min_valid = 0 if disable_neighbor_thresholding else self.minimum_valid_anchor_count
        return warp_triangle_mesh(input_mesh, self.get_node_positions(), self.get_node_rotations(), self.get_node_translations(), anchors,
                                  anchor_weights, threshold, min_valid, extrinsics)

    def reset_motion(self, stream=None):
        """R = I, t = 0 for every node (device side, asynchronous on `stream`)."""
        N.check(N.lib().nnrt_warp_field_reset_motion(self._h, N.stream_ptr(stream)))

    def get_virtual_node_indices(self) -> np.ndarray:
        out = np.empty(self.node_count, np.int64)
        N.check(N.lib().nnrt_warp_field_get_virtual_node_indices(self._h, N.ptr(out)))
        return out

    def get_edges(self) -> np.ndarray:
        e = N.lib().nnrt_warp_field_edge_count(self._h)
        out = np.empty((e, 2), np.int32)
        N.check(N.lib().nnrt_warp_field_get_edges(self._h, N.ptr(out), None))
        return out

    def get_edge_layer_indices(self) -> np.ndarray:
        e = N.lib().nnrt_warp_field_edge_count(self._h)
        out = np.empty(e, np.int8)
        N.check(N.lib().nnrt_warp_field_get_edges(self._h, None, N.ptr(out)))
        return out

    def get_layer_node_counts(self) -> np.ndarray:
        n = N.lib().nnrt_warp_field_layer_counts(self._h, None)
        out = np.empty(n, np.int32)
        N.lib().nnrt_warp_field_layer_counts(self._h, N.ptr(out))
        return out

    def get_regularization_level_count(self) -> int:
        return int(N.lib().nnrt_warp_field_layer_counts(self._h, None))

    def get_node_coverage_weights(self) -> np.ndarray:
        out = np.empty(self.node_count, np.float32)
        N.check(N.lib().nnrt_warp_field_get_node_coverage_weights(self._h, N.ptr(out)))
        return out


def _host_f32(x) -> np.ndarray:
    if isinstance(x, torch.Tensor):
        x = x.detach().cpu().numpy()
    return np.ascontiguousarray(x, dtype=np.float32)


def GraphWarpField(nodes, node_coverage=0.05, threshold_nodes_by_distance=False, anchor_count=4, minimum_valid_anchor_count=0,
                   device: int | None = None):
    """GraphWarpField (= WarpField, cpp/pybind/geometry/geometry.cpp:278-320): a single-layer field (no edges)."""
    return HierarchicalGraphWarpField(nodes, node_coverage, threshold_nodes_by_distance, anchor_count, minimum_valid_anchor_count,
                                      WarpNodeCoverageComputationMethod.FIXED_NODE_COVERAGE, layer_count=1, device=device)


# ----------------------------------------------------------------------------------------------------------------
# nnrt.geometry.functional
# ----------------------------------------------------------------------------------------------------------------
def _dev():
    return torch.device("cuda", N.current_device())


def _anchors(points, nodes, anchor_count, coverage, node_weights, minimum_valid_anchor_count):
    dev = _dev()
    p = to_device(points, torch.float32, dev).reshape(-1, 3)
    n = to_device(nodes, torch.float32, dev).reshape(-1, 3)
    nw = None if node_weights is None else to_device(node_weights, torch.float32, dev)
    a = torch.empty((p.shape[0], anchor_count), dtype=torch.int32, device=dev)
    w = torch.empty((p.shape[0], anchor_count), dtype=torch.float32, device=dev)
    N.check(N.lib().nnrt_compute_anchors_and_weights(N.ptr(p), p.shape[0], N.ptr(n), n.shape[0], anchor_count, float(coverage), N.ptr(nw),
                                                     int(minimum_valid_anchor_count), N.ptr(a), N.ptr(w), N.stream_ptr()))
    return a, w


def compute_anchors_and_weights_euclidean_fixed_node_weight(points, nodes, anchor_count, minimum_valid_anchor_count, node_coverage_weight):
    """ComputeAnchorsAndWeights_Euclidean_FixedNodeWeight (functional.cpp:52-55 -> WarpAnchorComputationImpl.h:92-140):
    anchors [V,K] int32 (-1 = invalid), weights [V,K]; thresholded (2 c) iff minimum_valid_anchor_count > 0."""
    _check_min_valid(minimum_valid_anchor_count, anchor_count)
    return _anchors(points, nodes, anchor_count, node_coverage_weight, None, minimum_valid_anchor_count)


def compute_anchors_and_weights_euclidean_variable_node_weight(points, nodes, node_coverage_weights, anchor_count, minimum_valid_anchor_count):
    """ComputeAnchorsAndWeights_Euclidean_VariableNodeWeight (functional.cpp:57-61 -> WarpAnchorComputationImpl.h:39-90):
    per-node squared coverage weights."""
    _check_min_valid(minimum_valid_anchor_count, anchor_count)
    return _anchors(points, nodes, anchor_count, 0.0, node_coverage_weights, minimum_valid_anchor_count)


def _check_min_valid(minimum_valid_anchor_count, anchor_count):
    if minimum_valid_anchor_count > anchor_count:
        raise RuntimeError(f"minimum_valid_anchor_count (now, {minimum_valid_anchor_count}) has to be smaller than or equal to anchor_count, "
                           f"which is {anchor_count}.")   # WarpAnchorComputation.cpp:92-95


@dataclass
class PointCloud:
    """Stand-in for open3d.t.geometry.PointCloud on the hot path: positions [P,3] f32, optional normals / colors."""
    point_positions: object
    point_normals: object = None
    point_colors: object = None


def _warp(points, normals, nodes, node_rotations, node_translations, anchors, anchor_weights, anchor_count, node_coverage, threshold,
          minimum_valid_anchor_count, extrinsics):
    """One nnrt_warp_points call: online anchors when `anchors` is None, else the supplied ones."""
    dev = _dev()
    p = to_device(points, torch.float32, dev).reshape(-1, 3)
    n = None if normals is None else to_device(normals, torch.float32, dev).reshape(-1, 3)
    g = to_device(nodes, torch.float32, dev).reshape(-1, 3)
    R = to_device(node_rotations, torch.float32, dev).reshape(-1, 3, 3)
    t = to_device(node_translations, torch.float32, dev).reshape(-1, 3)
    if R.shape[0] != g.shape[0] or t.shape[0] != g.shape[0]:
        raise RuntimeError(f"Argument node_rotations needs to have shape ({g.shape[0]}, 3, 3) and node_translations ({g.shape[0]}, 3), "
                           f"but have shapes {tuple(R.shape)} and {tuple(t.shape)}")   # Warping.cpp:34-54
    a = w = None
    if anchors is not None:
        a = to_device(anchors, torch.int32, dev)
        w = to_device(anchor_weights, torch.float32, dev)
        if a.dim() != 2 or w.dim() != 2 or a.shape != w.shape or a.shape[0] != p.shape[0]:
            raise RuntimeError("Tensors `anchors` and `anchor_weights` need to both have two matching dimensions "
                               f"[point count, anchor count]. Got {tuple(a.shape)} and {tuple(w.shape)}.")   # Warping.cpp:116-125
        anchor_count = a.shape[1]
    E = None if extrinsics is None else to_host_f64(extrinsics)
    op = torch.empty_like(p)
    on = None if n is None else torch.empty_like(n)
    N.check(N.lib().nnrt_warp_points(N.ptr(p), N.ptr(n), p.shape[0], N.ptr(g), N.ptr(R), N.ptr(t), g.shape[0], N.ptr(a), N.ptr(w),
                                     int(anchor_count), float(node_coverage), int(bool(threshold)), int(minimum_valid_anchor_count), N.ptr(E),
                                     N.ptr(op), N.ptr(on), N.stream_ptr()))
    return op, on


def _warped_mesh(mesh, op, on):
    """CopyTransformIndependentTriangleMeshData (Warping.cpp:156-167): indices and colours carried over."""
    return TriangleMesh(op, on, mesh.triangle_indices, vertex_colors=mesh.vertex_colors, triangle_colors=mesh.triangle_colors)


warp_triangle_mesh = Overloaded("warp_triangle_mesh", "WarpTriangleMesh / WarpTriangleMeshUsingSuppliedAnchors (functional.cpp:77-93 -> "
                                                      "Warping.cpp:169-264): warped vertex positions (and normals, unnormalized, A12).")


@warp_triangle_mesh.overload(lambda a: is_int(a["anchor_count"]) and not is_tensor(a["threshold_nodes_by_distance"]))
def _warp_triangle_mesh_online(input_mesh, nodes, node_rotations, node_translations, anchor_count, node_coverage,
                               threshold_nodes_by_distance=False, minimum_valid_anchor_count=0, extrinsics=_EYE4):
    if anchor_count < 1:
        raise RuntimeError(f"anchor_count needs to be at least than one. Got: {anchor_count}.")   # Warping.cpp:182-184
    op, on = _warp(input_mesh.vertex_positions, input_mesh.vertex_normals, nodes, node_rotations, node_translations, None, None, anchor_count,
                   node_coverage, threshold_nodes_by_distance, minimum_valid_anchor_count, extrinsics)
    return _warped_mesh(input_mesh, op, on)


@warp_triangle_mesh.overload(lambda a: is_tensor(a["anchors"]) and not is_tensor(a["threshold_nodes_by_distance"]))
def _warp_triangle_mesh_supplied(input_mesh, nodes, node_rotations, node_translations, anchors, anchor_weights, threshold_nodes_by_distance=False,
                                 minimum_valid_anchor_count=0, extrinsics=_EYE4):
    op, on = _warp(input_mesh.vertex_positions, input_mesh.vertex_normals, nodes, node_rotations, node_translations, anchors, anchor_weights, 0,
                   0.0, threshold_nodes_by_distance, minimum_valid_anchor_count, extrinsics)
    return _warped_mesh(input_mesh, op, on)


warp_point_cloud = Overloaded("warp_point_cloud", "WarpPointCloud, both overloads (functional.cpp:95-107 -> Warping.cpp:61-154): always "
                                                  "thresholded by minimum_valid_anchor_count (Warp3dPoints threshold variants).")


@warp_point_cloud.overload(lambda a: is_int(a["anchor_count"]))
def _warp_point_cloud_online(input_point_cloud, nodes, node_rotations, node_translations, anchor_count, node_coverage, minimum_valid_anchor_count,
                             extrinsics=_EYE4):
    if anchor_count < 1 or anchor_count > 8:
        raise RuntimeError(f"`anchor_count` is {anchor_count}, but is required to satisfy 0 < anchor_count <= 8")   # Warping.cpp:70-75
    if minimum_valid_anchor_count < 0 or minimum_valid_anchor_count > anchor_count:
        raise RuntimeError(f"`minimum_valid_anchor_count` is {minimum_valid_anchor_count}, but is required to satisfy "
                           f"0 < minimum_valid_anchor_count <= {anchor_count} ")   # Warping.cpp:76-79
    op, _ = _warp(input_point_cloud.point_positions, None, nodes, node_rotations, node_translations, None, None, anchor_count, node_coverage,
                  True, minimum_valid_anchor_count, extrinsics)
    return PointCloud(op, point_colors=input_point_cloud.point_colors)


@warp_point_cloud.overload(lambda a: is_tensor(a["anchors"]))
def _warp_point_cloud_supplied(input_point_cloud, nodes, node_rotations, node_translations, anchors, anchor_weights, minimum_valid_anchor_count,
                               extrinsics=_EYE4):
    K = np.shape(anchors)[-1]
    if minimum_valid_anchor_count < 0 or minimum_valid_anchor_count > K:
        raise RuntimeError(f"`minimum_valid_anchor_count` is {minimum_valid_anchor_count}, but is required to satisfy "
                           f"0 < minimum_valid_anchor_count <= {K}, where the upper bound is the second dimension of the input "
                           "`anchors` tensor.")   # Warping.cpp:127-131
    op, _ = _warp(input_point_cloud.point_positions, None, nodes, node_rotations, node_translations, anchors, anchor_weights, K, 0.0, True,
                  minimum_valid_anchor_count, extrinsics)
    return PointCloud(op, point_colors=input_point_cloud.point_colors)


def unproject_raster_depth_without_filtering(depth, intrinsics, extrinsics=np.eye(4, dtype=np.float32), depth_scale=1000.0, depth_max=3.0,
                                             preserve_pixel_layout=False):
    """UnprojectDepthImageWithoutFiltering (functional.cpp:128-138 -> PerspectiveProjection.cpp:26-39, PerspectiveProjectionImpl.h:60-146):
    uint16 or float32 depth [H,W] (an array, tensor or an object with .as_tensor()) -> (points, mask); points are in the
    frame of extrinsics^-1, zero where depth / depth_scale is outside (0, depth_max). preserve_pixel_layout -> [H,W,3] / [H,W],
    else [H*W,3] / [H*W]."""
    dev = _dev()
    if hasattr(depth, "as_tensor"):
        depth = depth.as_tensor()
    if isinstance(depth, np.ndarray) and depth.dtype == np.uint16:
        raw = torch.from_numpy(np.ascontiguousarray(depth).view(np.int16))   # uint16 bits, carried as int16
    else:
        raw = depth if isinstance(depth, torch.Tensor) else torch.as_tensor(np.ascontiguousarray(depth))
        if raw.dtype == torch.uint16:
            raw = raw.view(torch.int16)
    if raw.dim() == 3 and raw.shape[-1] == 1:
        raw = raw[..., 0]
    u16 = raw.dtype == torch.int16
    if not (u16 or raw.is_floating_point()):
        raise RuntimeError(f"Tensor has dtype {raw.dtype}, but is expected to have dtype among {{UInt16, Float32}}.")
    d = raw.to(dev).contiguous() if u16 else to_device(raw, torch.float32, dev)
    H, W = int(d.shape[0]), int(d.shape[1])
    K = to_host_f64(intrinsics)
    E = to_host_f64(extrinsics)
    if K.shape != (3, 3) or E.shape != (4, 4):
        raise RuntimeError(f"Intrinsics must be 3x3 and extrinsics 4x4; got {K.shape} and {E.shape}.")   # CheckIntrinsic/ExtrinsicTensor
    pts = torch.empty((H * W, 3), dtype=torch.float32, device=dev)
    mask = torch.empty(H * W, dtype=torch.uint8, device=dev)
    N.check(N.lib().nnrt_unproject_depth_image(N.ptr(d), 1 if u16 else 0, H, W, N.ptr(K), N.ptr(E), float(depth_scale), float(depth_max),
                                               N.ptr(pts), N.ptr(mask), N.stream_ptr()))
    mask = mask.bool()
    if preserve_pixel_layout:
        return pts.reshape(H, W, 3), mask.reshape(H, W)
    return pts, mask


def _point_to_plane(normals1, vertices1, vertices2):
    dev = _dev()
    n = to_device(normals1, torch.float32, dev).reshape(-1, 3)
    a = to_device(vertices1, torch.float32, dev).reshape(-1, 3)
    b = to_device(vertices2, torch.float32, dev).reshape(-1, 3)
    out = torch.empty(a.shape[0], dtype=torch.float32, device=dev)
    N.check(N.lib().nnrt_compute_point_to_plane_distances(N.ptr(n), N.ptr(a), N.ptr(b), a.shape[0], N.ptr(out), N.stream_ptr()))
    return out


def _length(x) -> int:
    return int(np.shape(x)[0]) if not isinstance(x, torch.Tensor) else int(x.shape[0])


compute_point_to_plane_distances = Overloaded(
    "compute_point_to_plane_distances", "ComputePointToPlaneDistances (functional.cpp:118-125 -> PointToPlaneDistances.cpp:25-68, "
                                        "PointToPlaneDistancesImpl.h:26-50): per vertex n1 . (v1 - v2).")


@compute_point_to_plane_distances.overload(lambda a: isinstance(a["mesh2"], TriangleMesh))
def _point_to_plane_meshes(mesh1, mesh2):
    if mesh1.vertex_normals is None:
        raise RuntimeError("Mesh1 needs to have vertex normals defined.")
    if _length(mesh1.vertex_positions) != _length(mesh2.vertex_positions):
        raise RuntimeError(f"Meshes need to have matching number of vertices. Got: {_length(mesh1.vertex_positions)} and "
                           f"{_length(mesh2.vertex_positions)}.")
    return _point_to_plane(mesh1.vertex_normals, mesh1.vertex_positions, mesh2.vertex_positions)


@compute_point_to_plane_distances.overload(lambda a: isinstance(a["point_cloud"], PointCloud))
def _point_to_plane_mesh_cloud(mesh, point_cloud):
    if mesh.vertex_normals is None:
        raise RuntimeError("Mesh needs to have vertex normals defined.")
    if _length(mesh.vertex_positions) != _length(point_cloud.point_positions):
        raise RuntimeError(f"Mesh vertex count has to match the point count in the point cloud. Got: {_length(mesh.vertex_positions)} and "
                           f"{_length(point_cloud.point_positions)}.")
    return _point_to_plane(mesh.vertex_normals, mesh.vertex_positions, point_cloud.point_positions)


def median_grid_subsample_3d_points(points, grid_cell_size):
    """MedianGridSubsample3dPoints (functional.cpp:152-153 -> GeometrySamplingMedian.h:264-296): int64 indices of one medoid
    per occupied grid cell (the cell member with the smallest summed distance to the others), ascending."""
    dev = _dev()
    p = to_device(points, torch.float32, dev).reshape(-1, 3)
    out = torch.empty(max(p.shape[0], 1), dtype=torch.int64, device=dev)
    count = np.zeros(1, np.int64)
    N.check(N.lib().nnrt_median_grid_subsample_3d_points(N.ptr(p), p.shape[0], float(grid_cell_size), N.ptr(out), N.ptr(count),
                                                         N.stream_ptr()))
    return out[: int(count[0])]


def _mesh_vf(mesh: TriangleMesh, dev):
    if mesh.vertex_positions is None or mesh.triangle_indices is None:
        raise RuntimeError("Mesh needs to have both vertex positions and triangle indices to compute normals.")
    return to_device(mesh.vertex_positions, torch.float32, dev), to_device(mesh.triangle_indices, torch.int64, dev)


def compute_triangle_normals(mesh: TriangleMesh, normalized: bool = True):
    """ComputeTriangleNormals (cpp/geometry/functional/NormalsOperations.cpp:36-46): sets mesh.triangle_normals [F,3]."""
    dev = _dev()
    p, f = _mesh_vf(mesh, dev)
    out = torch.empty((f.shape[0], 3), dtype=torch.float32, device=dev)
    N.check(N.lib().nnrt_compute_triangle_normals(N.ptr(p), p.shape[0], N.ptr(f), f.shape[0], int(bool(normalized)), N.ptr(out),
                                                  N.stream_ptr()))
    mesh.triangle_normals = out
    return out


def compute_vertex_normals(mesh: TriangleMesh, normalized: bool = True):
    """ComputeVertexNormals (NormalsOperations.cpp:52-66): sum of the unnormalized incident triangle normals (ascending
    face order), optionally normalized; sets mesh.vertex_normals [V,3]."""
    dev = _dev()
    p, f = _mesh_vf(mesh, dev)
    out = torch.empty((p.shape[0], 3), dtype=torch.float32, device=dev)
    N.check(N.lib().nnrt_compute_vertex_normals(N.ptr(p), p.shape[0], N.ptr(f), f.shape[0], int(bool(normalized)), N.ptr(out),
                                                N.stream_ptr()))
    mesh.vertex_normals = out
    return out


def compute_ordered_point_cloud_normals(point_cloud, source_image_size) -> torch.Tensor:
    """ComputeOrderedPointCloudNormals (NormalsOperations.cpp:74-95): organized point cloud ([H*W,3] positions, or an
    object with `point_positions`) -> [H*W,3] normals facing the camera, zero on the image border."""
    if len(source_image_size) != 2:
        raise RuntimeError(f"Source image size must have two dimensions. Got {len(source_image_size)}.")
    dev = _dev()
    pts = getattr(point_cloud, "point_positions", point_cloud)
    q = to_device(pts, torch.float32, dev).reshape(-1, 3)
    H, W = int(source_image_size[0]), int(source_image_size[1])
    out = torch.empty_like(q)
    N.check(N.lib().nnrt_compute_ordered_point_cloud_normals(N.ptr(q), q.shape[0], H, W, N.ptr(out), N.stream_ptr()))
    return out


functional = types.SimpleNamespace(
    compute_triangle_normals=compute_triangle_normals,
    compute_vertex_normals=compute_vertex_normals,
    compute_ordered_point_cloud_normals=compute_ordered_point_cloud_normals,
    compute_anchors_and_weights_euclidean_fixed_node_weight=compute_anchors_and_weights_euclidean_fixed_node_weight,
    compute_anchors_and_weights_euclidean_variable_node_weight=compute_anchors_and_weights_euclidean_variable_node_weight,
    warp_triangle_mesh=warp_triangle_mesh,
    warp_point_cloud=warp_point_cloud,
    median_grid_subsample_3d_points=median_grid_subsample_3d_points,
    unproject_raster_depth_without_filtering=unproject_raster_depth_without_filtering,
    compute_point_to_plane_distances=compute_point_to_plane_distances,
)


from .voxel_grid import NonRigidSurfaceVoxelBlockGrid, VoxelBlockGrid  # noqa: E402,F401
