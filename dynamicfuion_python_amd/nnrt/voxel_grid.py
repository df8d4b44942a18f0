"""nnrt.geometry.VoxelBlockGrid / NonRigidSurfaceVoxelBlockGrid mirror over the HIP TSDF grid (csrc/tsdf.hip).

Reference: cpp/geometry/VoxelBlockGrid.{h,cpp}, cpp/geometry/NonRigidSurfaceVoxelBlockGrid.{h,cpp}, Python binding
cpp/pybind/geometry/geometry.cpp:61-275 (same method names, argument meaning and defaults). Images are [H,W] depth
(uint16 or float32) and [H,W,3] color (uint8 with uint16 depth, float32 in [0,1] with float32 depth), numpy or torch;
intrinsics 3x3 and extrinsics 4x4 (float64 on the host, as the reference). Results are torch tensors on the grid's GPU.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from .. import _native as N
from ._tensors import to_host_f64

DTYPE_NONE, DTYPE_FLOAT32, DTYPE_UINT16, DTYPE_UINT8 = -1, 0, 1, 2


def _dtype_code(dt) -> int:
    name = str(dt).lower().split(".")[-1]
    if "float32" in name:
        return DTYPE_FLOAT32
    if "uint16" in name:
        return DTYPE_UINT16
    if "uint8" in name:
        return DTYPE_UINT8
    raise RuntimeError(f"unsupported voxel attribute dtype {dt!r} (float32, uint16 or uint8)")


def _is_matrix(x, n) -> bool:
    try:
        a = np.asarray(x.detach().cpu() if isinstance(x, torch.Tensor) else x)
    except Exception:
        return False
    return a.shape == (n, n)


class _HashMap:
    def __init__(self, grid: "VoxelBlockGrid"):
        self._grid = grid

    def activate(self, block_coords):
        self._grid.activate(block_coords)

    def size(self) -> int:
        return self._grid.get_block_count()


class VoxelBlockGrid:
    """Sparse grid of res^3 voxel blocks (attributes tsdf float32 + weight + optional 3-channel color)."""

    def __init__(self, attr_names, attr_dtypes, attr_channels, voxel_size: float = 0.0058, block_resolution: int = 16,
                 block_count: int = 10000, device=None):
        names = list(attr_names)
        if "tsdf" not in names or "weight" not in names:
            raise RuntimeError("a voxel block grid needs 'tsdf' and 'weight' attributes")
        dts = dict(zip(names, attr_dtypes))
        if _dtype_code(dts["tsdf"]) != DTYPE_FLOAT32:
            raise RuntimeError("tsdf must be float32")
        wdt = _dtype_code(dts["weight"])
        cdt = _dtype_code(dts["color"]) if "color" in names else DTYPE_NONE
        if isinstance(device, torch.device):
            device = device.index or 0
        self.device = N.current_device() if device is None or not isinstance(device, int) else device
        h = ctypes.c_void_p()
        N.check(N.lib().nnrt_voxel_grid_create(float(voxel_size), int(block_resolution), int(block_count), wdt, cdt, self.device,
                                               ctypes.byref(h)))
        self._h = h
        self._has_color = cdt != DTYPE_NONE

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                N.lib().nnrt_voxel_grid_destroy(h)
            except Exception:
                pass
            self._h = None

    # ---- plumbing ----
    @property
    def _dev(self):
        return torch.device("cuda", self.device)

    def _info(self):
        a, c, v, r = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_float(), ctypes.c_int32()
        N.check(N.lib().nnrt_voxel_grid_get_info(self._h, ctypes.byref(a), ctypes.byref(c), ctypes.byref(v), ctypes.byref(r)))
        return a.value, c.value, v.value, r.value

    def _coords(self, block_coords) -> torch.Tensor:
        c = torch.as_tensor(np.asarray(block_coords) if not isinstance(block_coords, torch.Tensor) else block_coords)
        return c.to(device=self._dev, dtype=torch.int32).reshape(-1, 3).contiguous()

    def _depth(self, depth):
        d = depth if isinstance(depth, torch.Tensor) else torch.as_tensor(np.asarray(depth))
        d = d.to(self._dev)
        if d.dim() == 3 and d.shape[-1] == 1:
            d = d[..., 0]
        if d.dtype == torch.uint16:
            code = DTYPE_UINT16
        elif d.dtype in (torch.int32, torch.int64, torch.int16) and not d.is_floating_point():
            d, code = d.to(torch.int32).clamp(0, 65535).to(torch.uint16), DTYPE_UINT16
        else:
            d, code = d.to(torch.float32), DTYPE_FLOAT32
        return d.contiguous(), code

    def _color(self, color, depth_code):
        if color is None:
            return None, 0, 0
        c = color if isinstance(color, torch.Tensor) else torch.as_tensor(np.asarray(color))
        c = c.to(self._dev, dtype=torch.uint8 if depth_code == DTYPE_UINT16 else torch.float32).contiguous()
        if c.numel() == 0:
            return None, 0, 0
        return c, c.shape[0], c.shape[1]

    def _result_coords(self, count: int) -> torch.Tensor:
        out = torch.empty((count, 3), dtype=torch.int32, device=self._dev)
        N.check(N.lib().nnrt_voxel_grid_copy_result_coordinates(self._h, N.ptr(out), N.stream_ptr()))
        return out

    # ---- API ----
    def hashmap(self) -> _HashMap:
        return _HashMap(self)

    def activate(self, block_coords):
        c = self._coords(block_coords)
        N.check(N.lib().nnrt_voxel_grid_activate(self._h, N.ptr(c), c.shape[0], N.stream_ptr()))

    def get_block_resolution(self) -> int:
        return self._info()[3]

    def get_block_count(self) -> int:
        return self._info()[0]

    def get_voxel_size(self) -> float:
        return self._info()[2]

    def get_device(self):
        return self._dev

    def compute_unique_block_coordinates(self, depth, intrinsic, extrinsic, depth_scale: float = 1000.0, depth_max: float = 3.0,
                                         trunc_voxel_multiplier: float = 8.0) -> torch.Tensor:
        """GetUniqueBlockCoordinates (VoxelBlockGrid.cpp:237-270): blocks along the truncation band of every 4th pixel."""
        d, code = self._depth(depth)
        K, E = to_host_f64(intrinsic), to_host_f64(extrinsic)
        n = ctypes.c_int64()
        N.check(N.lib().nnrt_voxel_grid_unique_block_coordinates(self._h, N.ptr(d), code, d.shape[0], d.shape[1], N.ptr(K), N.ptr(E),
                                                                 float(depth_scale), float(depth_max), float(trunc_voxel_multiplier),
                                                                 ctypes.byref(n), N.stream_ptr()))
        return self._result_coords(n.value)

    def integrate(self, block_coords, depth, *args, depth_scale: float = 1000.0, depth_max: float = 3.0,
                  trunc_voxel_multiplier: float = 8.0):
        """The three Integrate overloads (VoxelBlockGrid.cpp:294-350): (block_coords, depth, intrinsic, extrinsic, ...),
        (block_coords, depth, color, intrinsic, extrinsic, ...), (block_coords, depth, color, depth_intrinsic,
        color_intrinsic, extrinsic, depth_scale, depth_max, trunc_voxel_multiplier)."""
        args = list(args)
        if args and _is_matrix(args[0], 3):
            color, Kd, Kc, E, rest = None, args[0], args[0], args[1], args[2:]
        elif len(args) >= 4 and _is_matrix(args[2], 3):
            color, Kd, Kc, E, rest = args[0], args[1], args[2], args[3], args[4:]
        else:
            color, Kd, Kc, E, rest = args[0], args[1], args[1], args[2], args[3:]
        if rest:
            depth_scale = rest[0]
        if len(rest) > 1:
            depth_max = rest[1]
        if len(rest) > 2:
            trunc_voxel_multiplier = rest[2]
        c = self._coords(block_coords)
        d, code = self._depth(depth)
        col, Hc, Wc = self._color(color, code)
        Kd, Kc, E = to_host_f64(Kd), to_host_f64(Kc), to_host_f64(E)
        N.check(N.lib().nnrt_voxel_grid_integrate(self._h, N.ptr(c), c.shape[0], N.ptr(d), code, d.shape[0], d.shape[1], N.ptr(col), Hc, Wc,
                                                  N.ptr(Kd), N.ptr(Kc), N.ptr(E), float(depth_scale), float(depth_max),
                                                  float(trunc_voxel_multiplier), N.stream_ptr()))

    def extract_triangle_mesh(self, weight_threshold: float = 3.0, estimated_vertex_number: int = -1):
        """ExtractTriangleMesh (VoxelBlockGrid.cpp:461-497): marching cubes over the active blocks."""
        from .geometry import TriangleMesh
        nv, nt = ctypes.c_int64(), ctypes.c_int64()
        N.check(N.lib().nnrt_voxel_grid_extract_triangle_mesh(self._h, float(weight_threshold), ctypes.byref(nv), ctypes.byref(nt),
                                                              N.stream_ptr()))
        V = torch.empty((nv.value, 3), dtype=torch.float32, device=self._dev)
        Nn = torch.empty_like(V)
        C = torch.empty_like(V) if self._has_color else None
        T = torch.empty((nt.value, 3), dtype=torch.int64, device=self._dev)
        N.check(N.lib().nnrt_voxel_grid_copy_mesh(self._h, N.ptr(V), N.ptr(Nn), N.ptr(C), N.ptr(T), N.stream_ptr()))
        return TriangleMesh(V, Nn, T, vertex_colors=C)


class NonRigidSurfaceVoxelBlockGrid(VoxelBlockGrid):
    """NonRigidSurfaceVoxelBlockGrid (cpp/geometry/NonRigidSurfaceVoxelBlockGrid.h:30-65)."""

    def integrate_non_rigid(self, block_coords, warp_field, depth, color, depth_normals, depth_intrinsics, color_intrinsics, extrinsics,
                            depth_scale: float, depth_max: float, truncation_voxel_multiplier: float) -> torch.Tensor:
        """IntegrateNonRigid (NonRigidSurfaceVoxelBlockGrid.cpp:33-66) -> cos(voxel ray, normal) per pixel [H,W]."""
        c = self._coords(block_coords)
        d, code = self._depth(depth)
        col, Hc, Wc = self._color(color, code)
        nrm = torch.as_tensor(depth_normals) if not isinstance(depth_normals, torch.Tensor) else depth_normals
        nrm = nrm.to(self._dev, torch.float32).reshape(-1, 3).contiguous()
        if nrm.shape[0] != d.shape[0] * d.shape[1]:
            raise RuntimeError("depth_normals must hold one normal per depth pixel")
        Kd, Kc, E = to_host_f64(depth_intrinsics), to_host_f64(color_intrinsics), to_host_f64(extrinsics)
        cos = torch.empty((d.shape[0], d.shape[1]), dtype=torch.float32, device=self._dev)
        N.check(N.lib().nnrt_voxel_grid_integrate_non_rigid(self._h, N.ptr(c), c.shape[0], warp_field.handle, N.ptr(d), code, d.shape[0],
                                                            d.shape[1], N.ptr(col), Hc, Wc, N.ptr(nrm), N.ptr(Kd), N.ptr(Kc), N.ptr(E),
                                                            float(depth_scale), float(depth_max), float(truncation_voxel_multiplier),
                                                            N.ptr(cos), N.stream_ptr()))
        return cos

    def find_blocks_intersecting_truncation_region(self, depth, warp_field, intrinsics, extrinsics, depth_scale: float, depth_max: float,
                                                   truncation_voxel_multiplier: float) -> torch.Tensor:
        """FindBlocksIntersectingTruncationRegion (NonRigidSurfaceVoxelBlockGrid.cpp:141-166)."""
        d, code = self._depth(depth)
        K, E = to_host_f64(intrinsics), to_host_f64(extrinsics)
        n = ctypes.c_int64()
        N.check(N.lib().nnrt_voxel_grid_find_blocks_intersecting_truncation_region(
            self._h, N.ptr(d), code, d.shape[0], d.shape[1], warp_field.handle, N.ptr(K), N.ptr(E), float(depth_scale), float(depth_max),
            float(truncation_voxel_multiplier), ctypes.byref(n), N.stream_ptr()))
        return self._result_coords(n.value)

    def extract_voxel_values_and_coordinates(self) -> torch.Tensor:
        active = self.get_block_count()
        res = self.get_block_resolution()
        C = 8 if self._has_color else 5
        out = torch.empty((active * res ** 3, C), dtype=torch.float32, device=self._dev)
        ch = ctypes.c_int32()
        N.check(N.lib().nnrt_voxel_grid_extract_voxel_values_and_coordinates(self._h, N.ptr(out), ctypes.byref(ch), N.stream_ptr()))
        return out

    def extract_voxel_block_coordinates(self) -> torch.Tensor:
        """ExtractVoxelBlockCoordinates (:186-191): metric block origins key * res * voxel_size."""
        keys = torch.empty((self.get_block_count(), 3), dtype=torch.int32, device=self._dev)
        N.check(N.lib().nnrt_voxel_grid_get_block_coordinates(self._h, N.ptr(keys), N.stream_ptr()))
        return keys.to(torch.float32) * self.get_block_resolution() * self.get_voxel_size()

    def get_block_coordinates(self) -> torch.Tensor:
        keys = torch.empty((self.get_block_count(), 3), dtype=torch.int32, device=self._dev)
        N.check(N.lib().nnrt_voxel_grid_get_block_coordinates(self._h, N.ptr(keys), N.stream_ptr()))
        return keys

    def extract_voxel_values_at(self, query_voxel_coordinates) -> torch.Tensor:
        """ExtractVoxelValuesAt (:193-224): rows (x, y, z, tsdf, weight[, r, g, b]) of the queries in active blocks."""
        q = self._coords(query_voxel_coordinates)
        rows, ch = ctypes.c_int64(), ctypes.c_int32()
        N.check(N.lib().nnrt_voxel_grid_extract_voxel_values_at(self._h, N.ptr(q), q.shape[0], ctypes.byref(rows), ctypes.byref(ch),
                                                                N.stream_ptr()))
        out = torch.empty((rows.value, ch.value), dtype=torch.float32, device=self._dev)
        N.check(N.lib().nnrt_voxel_grid_copy_result_rows(self._h, N.ptr(out), N.stream_ptr()))
        return out

    def activate_sleeve_blocks(self) -> int:
        n = ctypes.c_int64()
        N.check(N.lib().nnrt_voxel_grid_activate_sleeve_blocks(self._h, ctypes.byref(n), N.stream_ptr()))
        return n.value

    def get_bounding_boxes_of_warped_blocks(self, block_keys, warp_field, extrinsics) -> torch.Tensor:
        """GetBoundingBoxesOfWarpedBlocks (:113-124)."""
        k = self._coords(block_keys)
        E = to_host_f64(extrinsics)
        out = torch.empty((k.shape[0], 6), dtype=torch.float32, device=self._dev)
        N.check(N.lib().nnrt_voxel_grid_warped_block_boxes(self._h, N.ptr(k), k.shape[0], warp_field.handle, N.ptr(E), N.ptr(out),
                                                           N.stream_ptr()))
        return out

    def get_axis_aligned_boxes_intersecting_surface_mask(self, boxes, depth, intrinsics, depth_scale: float, depth_max: float,
                                                         downsampling_factor: int = 4, trunc_voxel_multiplier: float = 8.0) -> torch.Tensor:
        """GetAxisAlignedBoxesIntersectingSurfaceMask (:126-139): truncation = voxel_size * trunc_voxel_multiplier."""
        return get_axis_aligned_boxes_intersecting_surface_mask(boxes, depth, intrinsics, depth_scale, depth_max, downsampling_factor,
                                                                self.get_voxel_size() * trunc_voxel_multiplier, device=self.device)


def get_axis_aligned_boxes_intersecting_surface_mask(boxes, depth, intrinsics, depth_scale, depth_max, stride, truncation_distance,
                                                     device=None) -> torch.Tensor:
    """voxel_grid::GetAxisAlignedBoxesInterceptingSurfaceMask (NonRigidSurfaceVoxelBlockGridImpl.h:359-437)."""
    dev = torch.device("cuda", N.current_device() if device is None else device)
    b = (boxes if isinstance(boxes, torch.Tensor) else torch.as_tensor(np.asarray(boxes))).to(dev, torch.float32).reshape(-1, 6).contiguous()
    d = depth if isinstance(depth, torch.Tensor) else torch.as_tensor(np.asarray(depth))
    d = d.to(dev)
    if d.dtype == torch.uint16:
        code = DTYPE_UINT16
    else:
        d, code = d.to(torch.float32), DTYPE_FLOAT32
    d = d.contiguous()
    K = to_host_f64(intrinsics)
    mask = torch.empty(b.shape[0], dtype=torch.uint8, device=dev)
    N.check(N.lib().nnrt_boxes_intersecting_surface_mask(N.ptr(b), b.shape[0], N.ptr(d), code, d.shape[0], d.shape[1], N.ptr(K),
                                                         float(depth_scale), float(depth_max), int(stride), float(truncation_distance),
                                                         N.ptr(mask), N.stream_ptr()))
    return mask.bool()


def marching_cubes_table():
    """The marching-cubes triangle table in emission order (the published Lorensen-Cline / Bourke table Open3D indexes,
    each triangle (a, b, c) as (a, c, b)): tri [256, 31] int8 edge triples (-1 terminated), edge mask [256] uint16."""
    tri = np.zeros((256, 31), np.int8)
    mask = np.zeros(256, np.uint16)
    N.check(N.lib().nnrt_marching_cubes_table(N.ptr(tri), N.ptr(mask)))
    return tri, mask
