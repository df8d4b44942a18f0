"""Synthetic scenes for the BASELINE configs C1-C5.

Pure numpy input synthesis (no checkpoints or datasets exist offline). A scene holds the canonical mesh, the
deformation-graph nodes (pre-sorted so the hierarchy's virtual node order is the identity, reference quirk A5),
camera intrinsics and a ground-truth node motion. The target depth frame is produced by warping the mesh with the
ground-truth motion and rasterizing it -- on the GPU in bench.py / the product API, on the CPU oracle in tests.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

X_EXTENT = (-0.6, 0.6)
Y_EXTENT = (-0.45, 0.45)


def surface_z(x, y):
    return 1.2 + 0.05 * np.sin(2 * np.pi * x / 0.4) * np.cos(2 * np.pi * y / 0.3)


def grid_mesh(cols: int, rows: int):
    """Regular grid mesh over X_EXTENT x Y_EXTENT; two triangles per cell, front-facing under the reference's
    clockwise NDC convention (cpp/rendering/functional/kernel/BarycentricCoordinates.h:35-47, fy_ndc < 0)."""
    xs = np.linspace(X_EXTENT[0], X_EXTENT[1], cols, dtype=np.float64)
    ys = np.linspace(Y_EXTENT[0], Y_EXTENT[1], rows, dtype=np.float64)
    X, Y = np.meshgrid(xs, ys)  # [rows, cols]
    Z = surface_z(X, Y)
    points = np.stack([X, Y, Z], -1).reshape(-1, 3)
    idx = np.arange(rows * cols, dtype=np.int64).reshape(rows, cols)
    a = idx[:-1, :-1].ravel()   # (i, j)
    b = idx[1:, :-1].ravel()    # (i, j+1)  -- y up
    c = idx[:-1, 1:].ravel()    # (i+1, j)
    d = idx[1:, 1:].ravel()     # (i+1, j+1)
    faces = np.concatenate([np.stack([a, b, c], 1), np.stack([c, b, d], 1)], 0)
    # interleave per cell (two faces of a cell adjacent in memory)
    n_cells = len(a)
    faces = faces.reshape(2, n_cells, 3).transpose(1, 0, 2).reshape(-1, 3)
    normals = vertex_normals(points, faces)
    return points.astype(np.float32), normals.astype(np.float32), faces.astype(np.int64)


def vertex_normals(points, faces):
    p = np.asarray(points, np.float64)
    fn = np.cross(p[faces[:, 1]] - p[faces[:, 0]], p[faces[:, 2]] - p[faces[:, 0]])
    vn = np.zeros_like(p)
    for i in range(3):
        np.add.at(vn, faces[:, i], fn)
    vn /= np.maximum(np.linalg.norm(vn, axis=1, keepdims=True), 1e-20)
    flip = vn[:, 2] > 0          # orient toward the camera (n_z < 0)
    vn[flip] *= -1
    return vn


def node_grid(nx: int, ny: int, jitter: float = 2e-4, seed: int = 0):
    rng = np.random.default_rng(seed + 1000)
    xs = np.linspace(X_EXTENT[0], X_EXTENT[1], nx)
    ys = np.linspace(Y_EXTENT[0], Y_EXTENT[1], ny)
    X, Y = np.meshgrid(xs, ys)
    X = X + rng.uniform(-jitter, jitter, X.shape)
    Y = Y + rng.uniform(-jitter, jitter, Y.shape)
    U, Vv = np.meshgrid(np.linspace(0, 1, nx), np.linspace(0, 1, ny))
    nodes = np.stack([X, Y, surface_z(X, Y)], -1).reshape(-1, 3)
    uv = np.stack([U, Vv], -1).reshape(-1, 2)
    return nodes.astype(np.float32), uv


def ground_truth_motion(uv, seed: int = 0):
    rng = np.random.default_rng(seed)
    u, v = uv[:, 0], uv[:, 1]
    t = 0.01 * np.stack([np.sin(2 * np.pi * u), np.cos(2 * np.pi * v), 0.5 * np.sin(2 * np.pi * (u + v))], 1)
    t = t + rng.normal(0, 0.001, t.shape)
    w = 0.02 * np.stack([np.cos(2 * np.pi * v), np.sin(2 * np.pi * u), np.zeros_like(u)], 1)
    return w.astype(np.float32), t.astype(np.float32)


def rodrigues_np(w):
    w = np.asarray(w, np.float64)
    th = np.linalg.norm(w, axis=1)
    R = np.tile(np.eye(3), (len(w), 1, 1))
    nz = th > 0
    a = w[nz] / th[nz, None]
    K = np.zeros((nz.sum(), 3, 3))
    K[:, 0, 1], K[:, 0, 2] = -a[:, 2], a[:, 1]
    K[:, 1, 0], K[:, 1, 2] = a[:, 2], -a[:, 0]
    K[:, 2, 0], K[:, 2, 1] = -a[:, 1], a[:, 0]
    s, c = np.sin(th[nz])[:, None, None], np.cos(th[nz])[:, None, None]
    R[nz] = np.eye(3) + s * K + (1 - c) * (K @ K)
    return R.astype(np.float32)


CONFIGS = {
    # name: (H, W, fx, mesh cols, mesh rows, node nx, node ny, coverage, layer_count, iterations)
    "C1": (480, 640, 580.0, 321, 241, 20, 10, 0.08, 1, 1),
    "C1_ARAP": (480, 640, 580.0, 321, 241, 20, 10, 0.08, 2, 1),
    "C2": (480, 640, 580.0, 321, 241, 50, 30, 0.03, 1, 10),
    "C2_ARAP": (480, 640, 580.0, 321, 241, 50, 30, 0.03, 2, 10),
    "C3": (960, 1280, 1160.0, 1501, 1501, 75, 40, 0.022, 1, 10),
    "C5": (480, 640, 580.0, 321, 241, 100, 50, 0.018, 2, 10),
    # >= 3 layers (the binding's default is 4, HierarchicalGraphWarpField.h:44): corner off-diagonal blocks
    "C2_ARAP3": (480, 640, 580.0, 321, 241, 50, 30, 0.03, 3, 10),
    "C2_ARAP4": (480, 640, 580.0, 321, 241, 50, 30, 0.03, 4, 10),
    "C5_L4": (480, 640, 580.0, 321, 241, 100, 50, 0.018, 4, 10),
    # small configs for fast CPU-oracle parity tests
    "S1": (96, 128, 116.0, 49, 37, 6, 4, 0.25, 1, 2),
    "S1_ARAP": (96, 128, 116.0, 49, 37, 8, 6, 0.16, 2, 2),
    "S1_ARAP4": (96, 128, 116.0, 49, 37, 12, 9, 0.1, 4, 2),
}


@dataclass
class Scene:
    name: str
    H: int
    W: int
    K: np.ndarray                 # [3,3] float64 pixel intrinsics
    points: np.ndarray            # [V,3]
    normals: np.ndarray           # [V,3]
    faces: np.ndarray             # [F,3] int64
    nodes: np.ndarray             # [N,3] (original order; hierarchy["virtual_indices"] maps virtual -> original)
    coverage: float
    layer_count: int
    iterations: int
    gt_rotations: np.ndarray      # [N,3,3]
    gt_translations: np.ndarray   # [N,3]
    hierarchy: dict = field(default_factory=dict)   # edges, edge_layers, radii, layer_counts, virtual_indices (layers > 1)
    gt_axis_angles: np.ndarray = None                # [N,3] the ground-truth rotations as axis-angle vectors

    def partial_motion(self, fraction: float, seed: int = 0, noise: float = 0.0):
        """Node motion `fraction` of the way along the ground truth (R = Rodrigues(fraction * w), t = fraction * t),
        plus optional N(0, noise^2) on both (original node order). A deterministic non-identity state from which a GN
        iteration runs the general warp / update kernels on a deformed mesh."""
        rng = np.random.default_rng(seed)
        w = self.gt_axis_angles * np.float32(fraction)
        t = self.gt_translations * np.float32(fraction)
        if noise > 0:
            w = w + rng.normal(0, noise, w.shape).astype(np.float32)
            t = t + rng.normal(0, noise, t.shape).astype(np.float32)
        return rodrigues_np(w), t.astype(np.float32)


def native_hierarchy_builder(nodes, coverage, layer_count):
    """hierarchy_builder over this package's own warp field (HierarchicalGraphWarpField.cpp:74-199 semantics, built
    by the native library; needs the HIP device): (virtual_indices, layer_counts, edges, edge_layers)."""
    from .nnrt import geometry as G
    wf = G.HierarchicalGraphWarpField(nodes, coverage, False, 4, 0, G.WarpNodeCoverageComputationMethod.FIXED_NODE_COVERAGE, layer_count)
    return wf.get_virtual_node_indices(), wf.get_layer_node_counts(), wf.get_edges(), wf.get_edge_layer_indices()


def make_scene(name: str = "C2", seed: int = 0, hierarchy_builder=None) -> Scene:
    """hierarchy_builder(nodes, coverage, layer_count) -> (virtual_indices, layer_counts, edges, edge_layers) is used
    to pre-sort the nodes into virtual order (identity permutation) for multi-layer configs."""
    H, W, fx, mc, mr, nx, ny, cov, layers, iters = CONFIGS[name]
    K = np.array([[fx, 0, W / 2], [0, fx, H / 2], [0, 0, 1]], np.float64)
    points, normals, faces = grid_mesh(mc, mr)
    nodes, uv = node_grid(nx, ny, seed=seed)
    w, t = ground_truth_motion(uv, seed=seed)
    hier = {}
    if layers > 1:
        if hierarchy_builder is None:
            raise ValueError("multi-layer scenes need a hierarchy_builder (virtual order and edges)")
        # Pre-sort the nodes toward virtual order (identity permutation) where the hierarchy allows it. The median-grid
        # subsample keeps each cell's medoid with ties going to the earlier node, so a two-member cell flips its medoid
        # whenever the order changes; such scenes keep a non-identity virtual order (virtual_indices).
        for attempt in range(4):
            vidx, counts, edges, elayers = hierarchy_builder(nodes, cov, layers)
            if np.array_equal(vidx, np.arange(len(nodes))):
                break
            if attempt < 3:
                nodes, uv, w, t = nodes[vidx], uv[vidx], w[vidx], t[vidx]
        vidx, counts, edges, elayers = hierarchy_builder(nodes, cov, layers)
        radii = np.array([cov * (i + 1) for i in range(layers)], np.float32)
        hier = dict(edges=edges, edge_layers=elayers, radii=radii, layer_counts=counts, virtual_indices=np.asarray(vidx, np.int64))
    return Scene(name, H, W, K, points, normals, faces, nodes, cov, layers, iters, rodrigues_np(w), t, hier, w)
