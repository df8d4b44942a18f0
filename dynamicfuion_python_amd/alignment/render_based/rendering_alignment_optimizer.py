"""RenderingAlignmentOptimizer.optimize_graph (alignment/render_based/rendering_alignment_optimizer.py:50-70 in the
reference, a stub there) implemented over the MI355X DeformableMeshToImageFitter, with the reference's
RenderingAlignmentParameters (settings/rendering_alignment.py:26-40) mapped onto the fitter's penalty switches.

The reference slot extracts the canonical mesh from the TSDF (`tsdf.extract_surface_mesh(-1, 0)`), renders the warped
mesh and fits the graph to the target point cloud; here the whole loop is one fit_to_image call (point-cloud overload,
DeformableMeshToImageFitter.cpp:85-276) on the GPU. The graph (a HierarchicalGraphWarpField) is updated in place.
"""
from __future__ import annotations

import enum
from dataclasses import dataclass
from typing import Tuple

import numpy as np
import torch

from ...nnrt import alignment as A
from ...nnrt import geometry as G


class PenaltyFunction(enum.Enum):
    """settings/rendering_alignment.py:20-23"""
    SQUARE = 1
    TUKEY = 2
    HUBER = 3


@dataclass
class RenderingAlignmentParameters:
    """settings/rendering_alignment.py:26-40 defaults, plus the fitter's own constructor defaults."""
    data_term_penalty_function: PenaltyFunction = PenaltyFunction.TUKEY
    data_term_penalty_constant: float = 0.01
    regularization_term_penalty_function: PenaltyFunction = PenaltyFunction.HUBER
    regularization_term_penalty_constant: float = 0.0001
    max_iteration_count: int = 100
    iteration_mode_sequence: tuple = (A.IterationMode.ALL,)
    preconditioning_dampening_factor: float = 0.001
    arap_term_weight: float = 200.0
    max_depth: float = 10.0
    use_perspective_correction: bool = True
    # A.NDC_REFERENCE reproduces the reference's y-mirrored render placement (A11); A.NDC_CONSISTENT is what real depth
    # frames need (the fusion pipeline's default)
    ndc_convention: int = A.NDC_REFERENCE


def as_triangle_mesh(mesh) -> G.TriangleMesh:
    """Accept this package's TriangleMesh or an Open3D-tensor-style mesh (vertex['positions'], vertex['normals'],
    triangle['indices'], each convertible with .numpy())."""
    if isinstance(mesh, G.TriangleMesh):
        return mesh
    try:
        def arr(t):
            return t.numpy() if hasattr(t, "numpy") else np.asarray(t)
        return G.TriangleMesh(arr(mesh.vertex["positions"]), arr(mesh.vertex["normals"]), arr(mesh.triangle["indices"]).astype(np.int64))
    except (AttributeError, KeyError, TypeError) as e:
        raise TypeError("canonical mesh must be a TriangleMesh or provide vertex['positions'/'normals'] and triangle['indices']") from e


class RenderingAlignmentOptimizer:
    def __init__(self, image_size_hw: Tuple[int, int], device=None, intrinsic_matrix=None,
                 parameters: RenderingAlignmentParameters | None = None):
        self.image_size_hw = (int(image_size_hw[0]), int(image_size_hw[1]))
        self.intrinsic_matrix = np.asarray(intrinsic_matrix, np.float64).reshape(3, 3)
        self.parameters = parameters or RenderingAlignmentParameters()
        p = self.parameters
        dev = None if device is None else (device.index if isinstance(device, torch.device) else int(device))
        self.fitter = A.DeformableMeshToImageFitter(
            max_iteration_count=p.max_iteration_count, iteration_mode_sequence=list(p.iteration_mode_sequence),
            use_perspective_correction=p.use_perspective_correction, max_depth=p.max_depth,
            use_tukey_penalty_for_data_term=p.data_term_penalty_function == PenaltyFunction.TUKEY,
            tukey_penalty_cutoff_cm=p.data_term_penalty_constant, preconditioning_dampening_factor=p.preconditioning_dampening_factor,
            arap_term_weight=p.arap_term_weight,
            use_huber_penalty_for_arap_term=p.regularization_term_penalty_function == PenaltyFunction.HUBER,
            huber_penalty_constant=p.regularization_term_penalty_constant, device=dev, ndc_convention=p.ndc_convention)

    def optimize_graph(self, graph: G.HierarchicalGraphWarpField, tsdf, target_points, target_rgb=None):
        """tsdf: an object with extract_surface_mesh(-1, 0) (NonRigidSurfaceVoxelBlockGrid) or the canonical mesh
        itself; target_points: organized [H,W,3] / [H*W,3] camera-space points (z <= 0 or non-finite = no target)."""
        mesh = tsdf.extract_surface_mesh(-1, 0) if hasattr(tsdf, "extract_surface_mesh") else tsdf
        mesh = as_triangle_mesh(mesh)
        H, W = self.image_size_hw
        pts = target_points.detach() if isinstance(target_points, torch.Tensor) else torch.as_tensor(np.asarray(target_points))
        pts = pts.to(torch.float32).reshape(H * W, 3)
        valid = torch.isfinite(pts).all(dim=1) & (pts[:, 2] > 0)
        pts = torch.where(valid[:, None], pts, torch.zeros_like(pts))
        self.fitter.fit_to_image(graph, mesh, target_rgb, pts, valid.to(torch.uint8), self.intrinsic_matrix, None, (H, W))
        return graph
