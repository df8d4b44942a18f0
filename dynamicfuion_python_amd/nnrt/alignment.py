"""nnrt.alignment: DeformableMeshToImageFitter (cpp/alignment/DeformableMeshToImageFitter.h:34-91) and IterationMode
(cpp/alignment/IterationMode.h:24-28) -- absent from the reference's bindings, added here as SURVEY 8(b) specifies."""
from __future__ import annotations

import ctypes
import enum

import numpy as np
import torch

from .. import _native as N
from ._tensors import to_device, to_host_f64
from .geometry import HierarchicalGraphWarpField, TriangleMesh

# nnrt_fitter_iterate_timed stage order (include/nnrt_mi355x.h, NNRT_TIMED_STAGES)
TIMED_STAGES = ("warp", "raster", "pixel_jacobians", "node_reduce", "arap", "solve")
# nnrt_fitter_time_kernels order (include/nnrt_mi355x.h, NNRT_KERNEL_TIMES)
KERNEL_TIMES = ("k_warp_mesh_quad", "k_raster_scatter_mesh", "k_fit_pixels_fused", "solve", "iteration")


class IterationMode(enum.IntEnum):
    ALL = 0
    TRANSLATION_ONLY = 1
    ROTATION_ONLY = 2


NDC_REFERENCE = 0     # the reference's image -> NDC mapping
NDC_CONSISTENT = 1    # raster pixel (u, v) == pixel (u, v) of the intrinsics

# use_hip_graph (include/nnrt_mi355x.h NNRT_GRAPH_*): False/0 eager launches; True/1 a sequence of iterations runs eagerly
# the first time it is requested after prepare() and is graph-captured and replayed from its second request on (the
# default: a one-off frame fit never pays capture + instantiate); 2 captures on first use
GRAPH_NEVER, GRAPH_AUTO, GRAPH_ALWAYS = 0, 1, 2


class DeformableMeshToImageFitter:
    def __init__(self, max_iteration_count: int = 100, iteration_mode_sequence=(IterationMode.ALL,), minimal_update_threshold: float = 1e-6,
                 use_perspective_correction: bool = True, max_depth: float = 10.0, use_tukey_penalty_for_data_term: bool = False,
                 tukey_penalty_cutoff_cm: float = 0.01, preconditioning_dampening_factor: float = 0.0, arap_term_weight: float = 200.0,
                 use_huber_penalty_for_arap_term: bool = False, huber_penalty_constant: float = 1e-4, device: int | None = None,
                 use_hip_graph: int = 1, ndc_convention: int = 0):
        device = N.current_device() if device is None else int(device)
        p = N.FitterParams()
        N.lib().nnrt_fitter_default_params(ctypes.byref(p))
        modes = list(iteration_mode_sequence)
        p.max_iteration_count = int(max_iteration_count)
        p.iteration_mode_count = len(modes)
        for i, m in enumerate(modes):
            p.iteration_modes[i] = int(m)
        p.minimal_update_threshold = float(minimal_update_threshold)
        p.use_perspective_correction = int(use_perspective_correction)
        p.max_depth = float(max_depth)
        p.use_tukey_penalty_for_data_term = int(use_tukey_penalty_for_data_term)
        p.tukey_penalty_cutoff_cm = float(tukey_penalty_cutoff_cm)
        p.preconditioning_dampening_factor = float(preconditioning_dampening_factor)
        p.arap_term_weight = float(arap_term_weight)
        p.use_huber_penalty_for_arap_term = int(use_huber_penalty_for_arap_term)
        p.huber_penalty_constant = float(huber_penalty_constant)
        p.use_hip_graph = int(use_hip_graph)
        p.ndc_convention = int(ndc_convention)   # NDC_REFERENCE (A11, y-mirrored renders) or NDC_CONSISTENT (real depth frames)
        h = ctypes.c_void_p()
        N.check(N.lib().nnrt_fitter_create(ctypes.byref(p), int(device), ctypes.byref(h)))
        self._h = h
        self.params = p
        self.device = torch.device("cuda", device)
        self.modes = modes
        self._frame = None

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                N.lib().nnrt_fitter_destroy(h)
            except Exception:   # interpreter shutdown
                pass
            self._h = None

    # ---- split API (once-per-frame prepare + GN iterations) ----
    def prepare(self, warp_field: HierarchicalGraphWarpField, canonical_mesh: TriangleMesh, reference_depth_image,
                reference_image_mask, intrinsic_matrix, extrinsic_matrix=None, depth_scale: float = 1.0, stream=None):
        N.require_gpu()
        dev = self.device
        p, n, f = canonical_mesh.on_device(dev)
        d = to_device(reference_depth_image, torch.float32, dev)
        if d.dim() == 3:
            d = d[..., 0].contiguous()
        H, W = d.shape
        m = None if reference_image_mask is None else to_device(reference_image_mask, torch.uint8, dev).reshape(H, W)
        K = to_host_f64(intrinsic_matrix)
        E = None if extrinsic_matrix is None else to_host_f64(extrinsic_matrix)
        self._frame = (p, n, f, d, m, K, E, H, W)   # keep device inputs alive for the duration of the frame
        self._node_count = warp_field.node_count
        N.check(N.lib().nnrt_fitter_prepare(self._h, warp_field.handle, N.ptr(p), N.ptr(n), p.shape[0], N.ptr(f), f.shape[0], N.ptr(d), N.ptr(m),
                                            H, W, N.ptr(K), N.ptr(E), float(depth_scale), N.stream_ptr(stream)))

    def prepare_point_cloud(self, warp_field: HierarchicalGraphWarpField, canonical_mesh: TriangleMesh, reference_point_cloud,
                            reference_point_mask, intrinsic_matrix, extrinsic_matrix, rendering_image_size, stream=None):
        """Once-per-frame setup of the point-cloud overload (DeformableMeshToImageFitter.cpp:85-106): organized reference
        points [H*W,3] (or [H,W,3]) and their mask, rendered at rendering_image_size = (H, W)."""
        N.require_gpu()
        dev = self.device
        p, n, f = canonical_mesh.on_device(dev)
        H, W = int(rendering_image_size[0]), int(rendering_image_size[1])
        q = to_device(reference_point_cloud, torch.float32, dev).reshape(-1, 3).contiguous()
        if q.shape[0] != H * W:
            raise ValueError(f"reference point cloud has {q.shape[0]} points, expected an organized cloud of {H}x{W}")
        m = None if reference_point_mask is None else to_device(reference_point_mask, torch.uint8, dev).reshape(-1).contiguous()
        K = to_host_f64(intrinsic_matrix)
        E = None if extrinsic_matrix is None else to_host_f64(extrinsic_matrix)
        self._frame = (p, n, f, q, m, K, E, H, W)
        self._node_count = warp_field.node_count
        N.check(N.lib().nnrt_fitter_prepare_point_cloud(self._h, warp_field.handle, N.ptr(p), N.ptr(n), p.shape[0], N.ptr(f), f.shape[0],
                                                        N.ptr(q), N.ptr(m), H, W, N.ptr(K), N.ptr(E), N.stream_ptr(stream)))

    def iterate(self, warp_field: HierarchicalGraphWarpField, first_iteration: int = 0, count: int = 1, stream=None):
        N.check(N.lib().nnrt_fitter_iterate(self._h, warp_field.handle, int(first_iteration), int(count), N.stream_ptr(stream)))

    def iterate_from_identity(self, warp_field: HierarchicalGraphWarpField, first_iteration: int = 0, count: int = 1, stream=None):
        """iterate() with the warp field's motion reset to the identity before every iteration (benchmark form: each
        iteration is the first GN iteration of the prepared frame); graph-captured like iterate()."""
        N.check(N.lib().nnrt_fitter_iterate_from_identity(self._h, warp_field.handle, int(first_iteration), int(count),
                                                           N.stream_ptr(stream)))

    def snapshot_motion(self, warp_field: HierarchicalGraphWarpField, stream=None):
        """Store the warp field's node motion (R, t) in the fitter (device copy) for iterate_from_snapshot()."""
        N.check(N.lib().nnrt_fitter_snapshot_motion(self._h, warp_field.handle, N.stream_ptr(stream)))

    def iterate_from_snapshot(self, warp_field: HierarchicalGraphWarpField, first_iteration: int = 0, count: int = 1, stream=None):
        """iterate() with the node motion restored from the snapshot before every iteration (a device copy captured
        with the iteration): each iteration is the same GN iteration k of the frame, through the general kernels."""
        N.check(N.lib().nnrt_fitter_iterate_from_snapshot(self._h, warp_field.handle, int(first_iteration), int(count),
                                                           N.stream_ptr(stream)))

    def fit_from_snapshot(self, warp_field: HierarchicalGraphWarpField, count: int, stream=None):
        """A whole frame fit of `count` iterations from the snapshot (restored once, before the first iteration)."""
        N.check(N.lib().nnrt_fitter_fit_from_snapshot(self._h, warp_field.handle, int(count), N.stream_ptr(stream)))

    def restore_motion(self, warp_field: HierarchicalGraphWarpField, stream=None):
        N.check(N.lib().nnrt_fitter_restore_motion(self._h, warp_field.handle, N.stream_ptr(stream)))

    def iterate_timed(self, warp_field: HierarchicalGraphWarpField, first_iteration: int = 0, count: int = 1, stream=None) -> dict:
        """Eager iterations with HIP events between stages; returns average device ms per iteration per stage."""
        ms = np.zeros(len(TIMED_STAGES), np.float32)
        N.check(N.lib().nnrt_fitter_iterate_timed(self._h, warp_field.handle, int(first_iteration), int(count), N.ptr(ms), N.stream_ptr(stream)))
        return {name: float(v) for name, v in zip(TIMED_STAGES, ms)}

    def refine_info(self, stream=None) -> dict:
        """The last arrowhead solve's refinement gate: the corner factorization's smallest pivot / diag(S) ratio, the
        threshold, whether the refinement step ran, its max |d| / max |x| and whether its safeguard accepted it."""
        out = np.zeros(5, np.float32)
        N.check(N.lib().nnrt_fitter_refine_info(self._h, N.ptr(out), N.stream_ptr(stream)))
        return dict(pivot_ratio=float(out[0]), threshold=float(out[1]), refined=bool(out[2]), correction=float(out[3]),
                    accepted=bool(out[4]))

    def set_refine_ratio(self, ratio: float):
        """Upper end of the arrowhead solve's refinement window: one refinement step runs when the corner
        factorization's min pivot / diag(S) lies in [floor, ratio) (floor 1e-5, _native.refine_floor(); default ratio
        1e-2; 0: never refine; inf: refine whenever the ratio is at least the floor). refine_info() reports
        the threshold the last launched iterations ran with."""
        N.check(N.lib().nnrt_fitter_set_refine_ratio(self._h, float(ratio)))

    def time_kernels(self, warp_field: HierarchicalGraphWarpField, reps: int = 20, trials: int = 5, stream=None) -> dict:
        """Per-kernel device ms of one iteration from the snapshot state, each kernel in its real context (prefix
        sequences of `reps` graph-captured iterations, median of `trials`; include/nnrt_mi355x.h)."""
        ms = np.zeros(len(KERNEL_TIMES), np.float32)
        N.check(N.lib().nnrt_fitter_time_kernels(self._h, warp_field.handle, int(reps), int(trials), N.ptr(ms), N.stream_ptr(stream)))
        return {name: float(v) for name, v in zip(KERNEL_TIMES, ms)}

    def check(self, stream=None):
        N.check(N.lib().nnrt_fitter_check(self._h, N.stream_ptr(stream)))

    def fit_to_image(self, warp_field: HierarchicalGraphWarpField, canonical_mesh: TriangleMesh, *args):
        """The three FitToImage overloads (DeformableMeshToImageFitter.h:58-90); all mutate the warp field in place:

        * (warp_field, mesh, rgbd_image, reference_image_mask, K, E, depth_scale) -- rgbd_image has .color / .depth
          (DeformableMeshToImageFitter.cpp:316-329);
        * (warp_field, mesh, color, depth, reference_image_mask, K, E, depth_scale) (:278-314);
        * (warp_field, mesh, color, reference_point_cloud, reference_point_mask, K, E, rendering_image_size) (:85-276).

        The colour image is unused, as in the reference. A14: all max_iteration_count iterations run."""
        if len(args) == 5 and hasattr(args[0], "depth"):
            rgbd, mask, K, E, scale = args
            self.prepare(warp_field, canonical_mesh, rgbd.depth, mask, K, E, scale)
        elif len(args) == 6 and isinstance(args[5], (tuple, list, torch.Size)):
            _color, points, mask, K, E, size = args
            self.prepare_point_cloud(warp_field, canonical_mesh, points, mask, K, E, size)
        elif len(args) in (5, 6):
            _color, depth, mask, K = args[:4]
            E = args[4] if len(args) > 4 else None
            scale = args[5] if len(args) > 5 else 1.0
            self.prepare(warp_field, canonical_mesh, depth, mask, K, E, scale)
        else:
            raise TypeError("fit_to_image: no overload matches the arguments (see DeformableMeshToImageFitter.h:58-90)")
        self.iterate(warp_field, 0, self.params.max_iteration_count)
        self.check()

    def diagnostics(self, stream=None) -> dict:
        """Residuals, residual mask, rasterized face per pixel, motion updates, negative gradient and data-term Hessian
        blocks of the most recent iteration (host numpy)."""
        _, _, _, _, _, _, _, H, W = self._frame
        P = H * W
        s = 6   # upper bound (3-dof modes fill the first N*3 / N*9 entries)
        nodes = self._node_count
        out = dict(residuals=np.empty(P, np.float32), residual_mask=np.empty(P, np.uint8), pixel_faces=np.empty(P, np.int32),
                   updates=np.empty(nodes * s, np.float32), gradient=np.empty(nodes * s, np.float32),
                   hessian=np.empty(nodes * s * s, np.float32))
        N.check(N.lib().nnrt_fitter_get_diagnostics(self._h, N.ptr(out["residuals"]), N.ptr(out["residual_mask"]), N.ptr(out["pixel_faces"]),
                                                    N.ptr(out["updates"]), N.ptr(out["gradient"]), N.ptr(out["hessian"]), N.stream_ptr(stream)))
        out["residual_mask"] = out["residual_mask"].astype(bool)
        return out

    def corner_info(self) -> dict:
        """Schur-corner plan of the prepared frame's arrowhead solve (csrc/corner.hip): corner nodes, tile columns,
        factorization / back-substitution launches, stored vs dense lower 64 x 64 tiles."""
        out = np.zeros(6, np.int64)
        N.check(N.lib().nnrt_fitter_corner_info(self._h, N.ptr(out)))
        keys = ("corner_nodes", "tile_columns", "factor_launches", "back_launches", "stored_tiles", "dense_lower_tiles")
        return {k: int(v) for k, v in zip(keys, out)}

    def arrowhead_system(self, node_count: int, edge_count: int, stream=None):
        """The last ARAP iteration's float arrowhead system as the fitter solved it (virtual order): diagonal blocks
        [N,6,6] with LM, wing blocks [E,6,6] (block (i, j) of edge (i, j)), right-hand side [6N]."""
        d = np.empty((node_count, 6, 6), np.float32)
        w = np.empty((edge_count, 6, 6), np.float32)
        b = np.empty(6 * node_count, np.float32)
        N.check(N.lib().nnrt_fitter_get_arrowhead_system(self._h, N.ptr(d), N.ptr(w), N.ptr(b), int(node_count), int(edge_count),
                                                          N.stream_ptr(stream)))
        return d, w, b

    def warped_mesh(self, vertex_count: int, stream=None):
        """The last iteration's warped canonical mesh (positions, normals [V,3]) as the fitter rasterized it; vertex_count
        must equal the prepared mesh's (the C-ABI refuses a mismatch instead of writing past the buffers)."""
        p = np.empty((vertex_count, 3), np.float32)
        n = np.empty((vertex_count, 3), np.float32)
        N.check(N.lib().nnrt_fitter_get_warped_mesh(self._h, N.ptr(p), N.ptr(n), int(vertex_count), N.stream_ptr(stream)))
        return p, n

    def corner_work(self) -> dict:
        """The plan's factorization work as executed (csrc/corner.hip): MFMA flops (update-term tile products + rank-32
        products), update terms, eliminated tile columns (real columns summed)."""
        out = np.zeros(3, np.int64)
        N.check(N.lib().nnrt_fitter_corner_work(self._h, N.ptr(out)))
        return {k: int(v) for k, v in zip(("mfma_flops", "update_terms", "eliminated_columns"), out)}

    def anchors(self, vertex_count: int, anchor_count: int, stream=None):
        a = np.empty((vertex_count, anchor_count), np.int32)
        w = np.empty((vertex_count, anchor_count), np.float32)
        N.check(N.lib().nnrt_fitter_get_anchors(self._h, N.ptr(a), N.ptr(w), N.stream_ptr(stream)))
        return a, w
