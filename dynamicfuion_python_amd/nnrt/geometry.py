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
from ._tensors import to_device, to_host_f64


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

    def on_device(self, device: torch.device):
        return (to_device(self.vertex_positions, torch.float32, device), to_device(self.vertex_normals, torch.float32, device),
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
        self.device = device
        self.node_count = len(nodes_np)
        self.anchor_count = anchor_count
        self.node_coverage = node_coverage
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

    def set_node_rotations(self, rotations, use_virtual_ordering: bool = False):
        r = np.ascontiguousarray(rotations, np.float32)
        N.check(N.lib().nnrt_warp_field_set_node_rotations(self._h, N.ptr(r), int(use_virtual_ordering)))

    def set_node_translations(self, translations, use_virtual_ordering: bool = False):
        t = np.ascontiguousarray(translations, np.float32)
        N.check(N.lib().nnrt_warp_field_set_node_translations(self._h, N.ptr(t), int(use_virtual_ordering)))

    def translate_nodes(self, deltas, use_virtual_ordering: bool = False):
        self.set_node_translations(self.get_node_translations(use_virtual_ordering) + np.asarray(deltas, np.float32), use_virtual_ordering)

    def rotate_nodes(self, deltas, use_virtual_ordering: bool = False):
        R = self.get_node_rotations(use_virtual_ordering)
        self.set_node_rotations(np.einsum("nij,njk->nik", R, np.asarray(deltas, np.float32)), use_virtual_ordering)

    def reset_rotations(self):
        """WarpField::ResetRotations (cpp/geometry/WarpField.cpp:151-156): identity rotations, translations kept."""
        self.set_node_rotations(np.tile(np.eye(3, dtype=np.float32), (self.node_count, 1, 1)))

    def get_warped_nodes(self) -> np.ndarray:
        """WarpField::GetWarpedNodes: node positions + translations (original order)."""
        return self.get_node_positions() + self.get_node_translations()

    def warp_mesh(self, input_mesh: "TriangleMesh", anchors=None, anchor_weights=None, disable_neighbor_thresholding: bool = True,
                  extrinsics=None) -> "TriangleMesh":
        """GraphWarpField.warp_mesh, both overloads (cpp/pybind/geometry/geometry.cpp:293-302 -> WarpField.cpp:129-144):
        anchors are computed over the original-order nodes unless supplied."""
        nodes = self.get_node_positions()
        if anchors is None:
            p, _, _ = input_mesh.on_device(_dev())
            min_valid = 0 if disable_neighbor_thresholding else self.minimum_valid_anchor_count
            if self.warp_node_coverage_computation_method == WarpNodeCoverageComputationMethod.FIXED_NODE_COVERAGE:
                anchors, anchor_weights = _anchors(p, nodes, self.anchor_count, self.node_coverage, None, min_valid)
            else:
                weights = np.empty(self.node_count, np.float32)
                weights[self.get_virtual_node_indices()] = self.get_node_coverage_weights()
                anchors, anchor_weights = _anchors(p, nodes, self.anchor_count, 0.0, weights, min_valid)
        return warp_triangle_mesh(input_mesh, nodes, self.get_node_rotations(), self.get_node_translations(), anchors, anchor_weights,
                                  extrinsics)

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


def compute_anchors_and_weights_euclidean_fixed_node_weight(points, nodes, anchor_count=4, minimum_valid_anchor_count=0,
                                                            node_coverage=0.05):
    return _anchors(points, nodes, anchor_count, node_coverage, None, minimum_valid_anchor_count)


def compute_anchors_and_weights_euclidean_variable_node_weight(points, nodes, node_coverage_weights, anchor_count=4,
                                                               minimum_valid_anchor_count=0):
    return _anchors(points, nodes, anchor_count, 0.0, node_coverage_weights, minimum_valid_anchor_count)


def warp_triangle_mesh(mesh: TriangleMesh, nodes, node_rotations, node_translations, anchors, anchor_weights, extrinsics=None):
    """WarpTriangleMeshUsingSuppliedAnchors (cpp/geometry/functional/Warping.cpp:222-264)."""
    dev = _dev()
    p, n, f = mesh.on_device(dev)
    g = to_device(nodes, torch.float32, dev)
    R = to_device(node_rotations, torch.float32, dev)
    t = to_device(node_translations, torch.float32, dev)
    a = to_device(anchors, torch.int32, dev)
    w = to_device(anchor_weights, torch.float32, dev)
    E = None if extrinsics is None else to_host_f64(extrinsics)
    op = torch.empty_like(p)
    on = torch.empty_like(n)
    N.check(N.lib().nnrt_warp_mesh(N.ptr(p), N.ptr(n), p.shape[0], N.ptr(g), N.ptr(R), N.ptr(t), g.shape[0], N.ptr(a), N.ptr(w), a.shape[1],
                                   N.ptr(E), N.ptr(op), N.ptr(on), N.stream_ptr()))
    return TriangleMesh(op, on, f)


def unproject_raster_depth_without_filtering(depth, intrinsics, depth_scale=1.0, depth_max=10.0):
    """UnprojectRasterWithoutDepthFiltering (cpp/geometry/functional/kernel/PerspectiveProjectionImpl.h:60-146)."""
    dev = _dev()
    d = to_device(depth, torch.float32, dev)
    H, W = d.shape[0], d.shape[1]
    K = to_host_f64(intrinsics)
    pts = torch.empty((H * W, 3), dtype=torch.float32, device=dev)
    mask = torch.empty(H * W, dtype=torch.uint8, device=dev)
    N.check(N.lib().nnrt_unproject_depth(N.ptr(d), H, W, N.ptr(K), float(depth_scale), float(depth_max), N.ptr(pts), N.ptr(mask),
                                         N.stream_ptr()))
    return pts, mask.bool()


def compute_point_to_plane_distances(normals1, vertices1, vertices2) -> torch.Tensor:
    """ComputePointToPlaneDistances (PointToPlaneDistancesImpl.h:26-50): n1 . (v1 - v2); elementwise plumbing."""
    dev = _dev()
    n = to_device(normals1, torch.float32, dev)
    d = to_device(vertices1, torch.float32, dev) - to_device(vertices2, torch.float32, dev)
    return (n[:, 0] * d[:, 0] + n[:, 1] * d[:, 1]) + n[:, 2] * d[:, 2]


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
    unproject_raster_depth_without_filtering=unproject_raster_depth_without_filtering,
    compute_point_to_plane_distances=compute_point_to_plane_distances,
)


from .voxel_grid import NonRigidSurfaceVoxelBlockGrid, VoxelBlockGrid  # noqa: E402,F401
