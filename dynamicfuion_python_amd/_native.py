"""Loader for the in-tree HIP library (libnnrt_mi355x.so) and its C-ABI (include/nnrt_mi355x.h).

torch is imported first so that the process has exactly one HIP runtime (torch's bundled libamdhip64.so.7 satisfies
the library's DT_NEEDED by SONAME). There is no CPU fallback: if the library is missing or no GPU is visible, calls
raise immediately.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import torch  # noqa: F401  (loads the HIP runtime shared with the library)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NNRT_LIB_PATH") or os.path.join(_HERE, "libnnrt_mi355x.so")   # override: development timing builds
CSRC = os.path.join(_HERE, "csrc")

_lib = None

c_int32, c_int64, c_float, c_void_p, c_double_p = ctypes.c_int32, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)


class FitterParams(ctypes.Structure):
    _fields_ = [("max_iteration_count", c_int32), ("iteration_mode_count", c_int32), ("iteration_modes", c_int32 * 16),
                ("minimal_update_threshold", c_float), ("use_perspective_correction", c_int32), ("max_depth", c_float),
                ("use_tukey_penalty_for_data_term", c_int32), ("tukey_penalty_cutoff_cm", c_float),
                ("preconditioning_dampening_factor", c_float), ("arap_term_weight", c_float),
                ("use_huber_penalty_for_arap_term", c_int32), ("huber_penalty_constant", c_float), ("use_hip_graph", c_int32),
                ("ndc_convention", c_int32)]


def build(force: bool = False) -> str:
    """Compile the HIP sources for gfx950 in-tree (hipcc; no GPU needed)."""
    if force:
        subprocess.check_call(["make", "-s", "-C", CSRC, "clean"])
    subprocess.check_call(["make", "-s", "-j8", "-C", CSRC])
    return LIB_PATH


_SIGNATURES = {
    "nnrt_last_error": (ctypes.c_char_p, []),
    "nnrt_runtime_version": (c_int32, []),
    "nnrt_device_count": (c_int32, []),
    "nnrt_build_jacobian_fma": (c_int32, []),
    "nnrt_build_refine_floor": (c_float, []),
    "nnrt_warp_field_create": (c_int32, [c_void_p, c_int32, c_float, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, c_void_p,
                                         c_int32, ctypes.POINTER(c_void_p)]),
    "nnrt_warp_field_destroy": (None, [c_void_p]),
    "nnrt_warp_field_node_count": (c_int32, [c_void_p]),
    "nnrt_warp_field_edge_count": (c_int32, [c_void_p]),
    "nnrt_warp_field_layer_counts": (c_int32, [c_void_p, c_void_p]),
    "nnrt_warp_field_get_virtual_node_indices": (c_int32, [c_void_p, c_void_p]),
    "nnrt_warp_field_get_edges": (c_int32, [c_void_p, c_void_p, c_void_p]),
    "nnrt_warp_field_get_node_positions": (c_int32, [c_void_p, c_void_p, c_int32]),
    "nnrt_warp_field_get_node_rotations": (c_int32, [c_void_p, c_void_p, c_int32]),
    "nnrt_warp_field_get_node_translations": (c_int32, [c_void_p, c_void_p, c_int32]),
    "nnrt_warp_field_set_node_rotations": (c_int32, [c_void_p, c_void_p, c_int32]),
    "nnrt_warp_field_set_node_translations": (c_int32, [c_void_p, c_void_p, c_int32]),
    "nnrt_warp_field_get_node_coverage_weights": (c_int32, [c_void_p, c_void_p]),
    "nnrt_warp_field_reset_motion": (c_int32, [c_void_p, c_void_p]),
    "nnrt_fitter_default_params": (None, [c_void_p]),
    "nnrt_fitter_create": (c_int32, [c_void_p, c_int32, ctypes.POINTER(c_void_p)]),
    "nnrt_fitter_destroy": (None, [c_void_p]),
    "nnrt_fitter_fit_to_image": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p,
                                           c_int32, c_int32, c_void_p, c_void_p, c_float, c_void_p]),
    "nnrt_fitter_prepare": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p,
                                      c_int32, c_int32, c_void_p, c_void_p, c_float, c_void_p]),
    "nnrt_fitter_prepare_point_cloud": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p,
                                                  c_int32, c_int32, c_void_p, c_void_p, c_void_p]),
    "nnrt_fitter_fit_to_point_cloud": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p,
                                                 c_int32, c_int32, c_void_p, c_void_p, c_void_p]),
    "nnrt_fitter_iterate": (c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_void_p]),
    "nnrt_fitter_iterate_from_identity": (c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_void_p]),
    "nnrt_fitter_graph_count": (c_int32, [c_void_p]),
    "nnrt_fitter_corner_info": (c_int32, [c_void_p, c_void_p]),
    "nnrt_fitter_corner_work": (c_int32, [c_void_p, c_void_p]),
    "nnrt_fitter_get_arrowhead_system": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_void_p]),
    "nnrt_fitter_get_warped_mesh": (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p]),
    "nnrt_release_arrowhead_plans": (None, []),
    "nnrt_fitter_fit_from_snapshot": (c_int32, [c_void_p, c_void_p, c_int32, c_void_p]),
    "nnrt_fitter_restore_motion": (c_int32, [c_void_p, c_void_p, c_void_p]),
    "nnrt_fitter_snapshot_motion": (c_int32, [c_void_p, c_void_p, c_void_p]),
    "nnrt_fitter_iterate_from_snapshot": (c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_void_p]),
    "nnrt_fitter_iterate_timed": (c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p]),
    "nnrt_fitter_time_kernels": (c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p]),
    "nnrt_fitter_refine_info": (c_int32, [c_void_p, c_void_p, c_void_p]),
    "nnrt_fitter_set_refine_ratio": (c_int32, [c_void_p, c_float]),
    "nnrt_fitter_check": (c_int32, [c_void_p, c_void_p]),
    "nnrt_fitter_get_diagnostics": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "nnrt_fitter_get_anchors": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "nnrt_compute_anchors_and_weights": (c_int32, [c_void_p, c_int64, c_void_p, c_int32, c_int32, c_float, c_void_p, c_int32,
                                                   c_void_p, c_void_p, c_void_p]),
    "nnrt_warp_mesh": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_int32,
                                 c_void_p, c_void_p, c_void_p, c_void_p]),
    "nnrt_warp_points": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_float,
                                   c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p]),
    "nnrt_compute_point_to_plane_distances": (c_int32, [c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_void_p]),
    "nnrt_unproject_depth_image": (c_int32, [c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_float, c_float, c_void_p, c_void_p,
                                             c_void_p]),
    "nnrt_get_meshes_ndc_face_vertices_and_clip_mask": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_int32, c_int32, c_float,
                                                                  c_float, c_void_p, c_void_p, c_void_p]),
    "nnrt_get_mesh_ndc_face_vertices_and_clip_mask": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_int32, c_int32, c_float,
                                                                c_float, c_void_p, c_void_p, c_void_p]),
    "nnrt_rasterize_ndc_triangles": (c_int32, [c_void_p, c_void_p, c_int64, c_int32, c_int32, c_float, c_int32, c_int32, c_int32,
                                               c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "nnrt_interpolate_face_attributes": (c_int32, [c_void_p, c_void_p, c_int64, c_int32, c_void_p, c_int32, c_void_p, c_void_p]),
    "nnrt_unproject_depth": (c_int32, [c_void_p, c_int32, c_int32, c_void_p, c_float, c_float, c_void_p, c_void_p, c_void_p]),
    "nnrt_backproject_depth_ushort": (c_int32, [c_void_p, c_int32, c_int32, c_float, c_float, c_float, c_float, c_float, c_void_p,
                                                c_void_p]),
    "nnrt_backproject_depth_float": (c_int32, [c_void_p, c_int32, c_int32, c_float, c_float, c_float, c_float, c_void_p, c_void_p]),
    "nnrt_matmul3d": (c_int32, [c_void_p, c_void_p, c_int64, c_int32, c_int32, c_int32, c_void_p, c_void_p]),
    "nnrt_median_grid_subsample_3d_points": (c_int32, [c_void_p, c_int64, c_float, c_void_p, c_void_p, c_void_p]),
    "nnrt_axis_angle_to_matrices_rodrigues": (c_int32, [c_void_p, c_int32, c_void_p, c_void_p]),
    "nnrt_compute_triangle_normals": (c_int32, [c_void_p, c_int64, c_void_p, c_int64, c_int32, c_void_p, c_void_p]),
    "nnrt_compute_vertex_normals": (c_int32, [c_void_p, c_int64, c_void_p, c_int64, c_int32, c_void_p, c_void_p]),
    "nnrt_compute_ordered_point_cloud_normals": (c_int32, [c_void_p, c_int64, c_int32, c_int32, c_void_p, c_void_p]),
    "nnrt_solve_block_diagonal_cholesky": (c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p]),
    "nnrt_invert_positive_semidefinite_blocks": (c_int32, [c_void_p, c_int32, c_int32, c_void_p, c_void_p]),
    "nnrt_matmul_block_sparse_row_wise": (c_int32, [c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_void_p]),
    "nnrt_matmul_block_sparse": (c_int32, [c_void_p, c_int32, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_int32, c_void_p, c_int32, c_int32,
                                           c_int32, c_int32, c_void_p, c_void_p, c_void_p]),
    "nnrt_block_sparse_and_vector_product": (c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_int32, c_int32, c_int32, c_void_p, c_int64,
                                                       c_int64, c_void_p, c_void_p]),
    "nnrt_diagonal_block_sparse_and_vector_product": (c_int32, [c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_void_p]),
    "nnrt_sparse_blocks_op": (c_int32, [c_void_p, c_int64, c_int64, c_void_p, c_void_p, c_int32, c_int32, c_int64, c_int64, c_int32, c_int32,
                                        c_void_p]),
    "nnrt_get_sparse_blocks": (c_int32, [c_void_p, c_int64, c_int64, c_int32, c_void_p, c_int32, c_void_p, c_void_p]),
    "nnrt_transpose_blocks_in_place": (c_int32, [c_void_p, c_int32, c_int32, c_void_p]),
    "nnrt_invert_triangular_blocks": (c_int32, [c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p]),
    "nnrt_solve_block_sparse_arrowhead_cholesky": (c_int32, [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p,
                                                             c_void_p, c_void_p]),
    # TSDF voxel block grid
    "nnrt_voxel_grid_create": (c_int32, [c_float, c_int32, c_int64, c_int32, c_int32, c_int32, ctypes.POINTER(c_void_p)]),
    "nnrt_voxel_grid_destroy": (None, [c_void_p]),
    "nnrt_voxel_grid_get_info": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "nnrt_voxel_grid_activate": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p]),
    "nnrt_voxel_grid_get_block_coordinates": (c_int32, [c_void_p, c_void_p, c_void_p]),
    "nnrt_voxel_grid_unique_block_coordinates": (c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_float,
                                                           c_float, c_float, c_void_p, c_void_p]),
    "nnrt_voxel_grid_copy_result_coordinates": (c_int32, [c_void_p, c_void_p, c_void_p]),
    "nnrt_voxel_grid_integrate": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_int32, c_int32,
                                            c_void_p, c_void_p, c_void_p, c_float, c_float, c_float, c_void_p]),
    "nnrt_voxel_grid_integrate_non_rigid": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p,
                                                      c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_float, c_float,
                                                      c_void_p, c_void_p]),
    "nnrt_voxel_grid_extract_voxel_values_and_coordinates": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "nnrt_voxel_grid_extract_voxel_values_at": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p]),
    "nnrt_voxel_grid_copy_result_rows": (c_int32, [c_void_p, c_void_p, c_void_p]),
    "nnrt_voxel_grid_warped_block_boxes": (c_int32, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p]),
    "nnrt_boxes_intersecting_surface_mask": (c_int32, [c_void_p, c_int64, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_float, c_float,
                                                       c_int32, c_float, c_void_p, c_void_p]),
    "nnrt_voxel_grid_find_blocks_intersecting_truncation_region": (c_int32, [c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p,
                                                                             c_void_p, c_float, c_float, c_float, c_void_p, c_void_p]),
    "nnrt_voxel_grid_activate_sleeve_blocks": (c_int32, [c_void_p, c_void_p, c_void_p]),
    "nnrt_voxel_grid_extract_triangle_mesh": (c_int32, [c_void_p, c_float, c_void_p, c_void_p, c_void_p]),
    "nnrt_voxel_grid_copy_mesh": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "nnrt_marching_cubes_table": (c_int32, [c_void_p, c_void_p]),
    # include/nnrt_dlpack.h
    "nnrt_warp_field_create_dlpack": (c_int32, [c_void_p, c_float, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, c_void_p, c_int32,
                                                c_void_p]),
    "nnrt_fitter_fit_to_image_dlpack": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                                  c_float, c_void_p]),
    "nnrt_rasterize_ndc_triangles_dlpack": (c_int32, [c_void_p, c_void_p, c_float, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p,
                                                      c_void_p, c_void_p]),
}


def dlpack(x):
    """(capsule, DLManagedTensor*) for a torch tensor or numpy array. The tensor is lent, not consumed: keep the capsule
    alive for the duration of the call; its destructor releases the tensor afterwards."""
    import torch
    cap = torch.utils.dlpack.to_dlpack(x) if isinstance(x, torch.Tensor) else x.__dlpack__()
    get = ctypes.pythonapi.PyCapsule_GetPointer
    get.restype = ctypes.c_void_p
    get.argtypes = [ctypes.py_object, ctypes.c_char_p]
    return cap, get(cap, b"dltensor")


def exported_symbols():
    return list(_SIGNATURES)


def lib():
    """Load (without requiring a GPU) and bind the library; raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"HIP extension {LIB_PATH} is missing: run __graft_entry__.build() (hipcc, gfx950)")
        l = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGNATURES.items():
            f = getattr(l, name)
            f.restype = res
            f.argtypes = args
        _lib = l
    return _lib


def jacobian_fma() -> bool:
    """Whether this build forms the pixel-node Jacobians with FMAs (csrc NNRT_JAC_FMA; the checker mirrors it)."""
    return bool(lib().nnrt_build_jacobian_fma())


def refine_floor() -> float:
    """The refinement floor this build's arrowhead solve was compiled with (csrc NNRT_REFINE_PIVOT_FLOOR)."""
    return float(lib().nnrt_build_refine_floor())


class NnrtError(RuntimeError):
    def __init__(self, message: str, status: int = -1):
        super().__init__(message)
        self.status = status


def check(status: int):
    if status != 0:
        msg = lib().nnrt_last_error()
        raise NnrtError(f"nnrt status {status}: {msg.decode() if msg else ''}", status)


def require_gpu():
    if not torch.cuda.is_available():
        raise RuntimeError("no HIP device is visible: the MI355X path has no CPU fallback")


def current_device() -> int:
    """torch's current HIP device (one process per GPU: torch.cuda.set_device(LOCAL_RANK) selects it)."""
    require_gpu()
    return torch.cuda.current_device()


def ptr(t) -> c_void_p:
    if t is None:
        return c_void_p(None)
    if isinstance(t, torch.Tensor):
        return c_void_p(t.data_ptr())
    return c_void_p(t.ctypes.data)


def stream_ptr(stream=None) -> c_void_p:
    s = stream if stream is not None else torch.cuda.current_stream()
    return c_void_p(s.cuda_stream)
