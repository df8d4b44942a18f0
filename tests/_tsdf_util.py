"""Scene builders for the TSDF voxel-block-grid tests (inputs of the reference KAT, cpp/tests/
test_non_rigid_surface_voxel_block_grid.cpp:176-341, and a larger synthetic DynamicFusion-like frame)."""
import numpy as np


def simple_intrinsics(f=100.0, cx=50.0, cy=50.0):
    return np.array([[f, 0.0, cx], [0.0, f, cy], [0.0, 0.0, 1.0]])


def hemisphere_pinch(depth_mm: np.ndarray, radius: int, height_mm: float) -> np.ndarray:
    """HemisphereAtDepthImageCenter (:196-227): float32 tensor math as Open3D, rounded half away from zero."""
    d = int(radius) * 2
    step = 2.0 / (d - 1)
    lin = np.arange(-1.0, 1.0, step).astype(np.float32)
    lin = np.append(lin, np.float32(1.0)).astype(np.float32)
    assert lin.shape[0] == d
    y = (lin.reshape(1, d) * np.float32(radius)).astype(np.float32)
    x = (lin.reshape(d, 1) * np.float32(radius)).astype(np.float32)
    z2 = (np.float32(radius * radius) * np.ones((d, d), np.float32) - x * x - y * y).astype(np.float32)
    z2[z2 < 0] = 0
    z = np.sqrt(z2).astype(np.float32)
    delta = (np.float32(height_mm) * (z / z.max())).astype(np.float32)
    rounded = np.where(delta >= 0, np.floor(delta + 0.5), -np.floor(-delta + 0.5)).astype(np.uint16)
    out = depth_mm.copy()
    H, W = out.shape
    out[H // 2 - radius:H // 2 + radius, W // 2 - radius:W // 2 + radius] += rounded
    return out


def unproject_points(depth_mm: np.ndarray, K, scale=1000.0):
    """Open3D PointCloud::CreateFromDepthImage at stride 1 (all pixels valid here): row-major camera-space points."""
    H, W = depth_mm.shape
    fx, fy, cx, cy = np.float32(K[0, 0]), np.float32(K[1, 1]), np.float32(K[0, 2]), np.float32(K[1, 2])
    v, u = np.mgrid[0:H, 0:W].astype(np.float32)
    d = (depth_mm.astype(np.float32) / np.float32(scale)).astype(np.float32)
    x = ((u - cx) * d / fx).astype(np.float32)
    y = ((v - cy) * d / fy).astype(np.float32)
    return np.stack([x, y, d], -1).reshape(-1, 3).astype(np.float32)


def reference_nonrigid_kat_inputs():
    from golden import kat_literals as L
    plane = np.full((100, 100), 50, np.uint16)
    color = np.full((100, 100, 3), 100, np.uint8)
    K = simple_intrinsics()
    deformed = hemisphere_pinch(plane, 20, 10.0)
    nodes = L.VBG_NR_NODES
    R = np.tile(np.eye(3, dtype=np.float32), (5, 1, 1))
    t = np.zeros((5, 3), np.float32)
    t[0] = L.VBG_NR_NODE0_TRANSLATION
    return plane, color, K, deformed, nodes, R, t
