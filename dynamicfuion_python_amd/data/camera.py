"""Camera intrinsics (reference data/camera.py) and the cropping helpers the fusion app applies to them.

DeepDeform stores intrinsics as a 4x4 text matrix (`intrinsics.txt`); Open3D's PinholeCameraIntrinsic is replaced by
`PinholeCameraIntrinsic` below (width, height, 3x3 float64 matrix), which is what the fitter / TSDF entry points take.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple

import numpy as np


@dataclass
class PinholeCameraIntrinsic:
    width: int
    height: int
    intrinsic_matrix: np.ndarray   # [3, 3] float64

    @classmethod
    def from_parameters(cls, width, height, fx, fy, cx, cy) -> "PinholeCameraIntrinsic":
        return cls(int(width), int(height), np.array([[fx, 0.0, cx], [0.0, fy, cy], [0.0, 0.0, 1.0]], np.float64))


def _load_4x4(path_matrix: str) -> np.ndarray:
    m = np.loadtxt(path_matrix, dtype=np.float64)
    if m.shape != (4, 4):
        raise ValueError(f"{path_matrix}: expected a 4x4 matrix, got {m.shape}")
    return m


def load_intrinsic_3x3_matrix_from_text_4x4_matrix(path_matrix: str) -> np.ndarray:
    """data/camera.py:6-8"""
    return _load_4x4(path_matrix)[0:3, 0:3].copy()


def load_intrinsic_matrix_entries_from_text_4x4_matrix(path_matrix: str) -> Tuple[float, float, float, float]:
    """(fx, fy, cx, cy) (data/camera.py:11-17)"""
    m = _load_4x4(path_matrix)
    return float(m[0, 0]), float(m[1, 1]), float(m[0, 2]), float(m[1, 2])


def load_intrinsic_matrix_entries_as_dict_from_text_4x4_matrix(path_matrix: str) -> dict:
    """data/camera.py:20-31"""
    return dict(zip(("fx", "fy", "cx", "cy"), load_intrinsic_matrix_entries_from_text_4x4_matrix(path_matrix)))


def extract_intrinsic_projection_parameters(intrinsics: PinholeCameraIntrinsic) -> Tuple[float, float, float, float]:
    """data/camera.py:34-39"""
    k = intrinsics.intrinsic_matrix
    return float(k[0, 0]), float(k[1, 1]), float(k[0, 2]), float(k[1, 2])


def intrinsic_projection_parameters_as_dict(intrinsics: PinholeCameraIntrinsic) -> dict:
    """data/camera.py:54-65"""
    return dict(zip(("fx", "fy", "cx", "cy"), extract_intrinsic_projection_parameters(intrinsics)))


def load_open3d_intrinsics_from_text_4x4_matrix_and_image(path_matrix: str, path_image: str) \
        -> Tuple[PinholeCameraIntrinsic, np.ndarray]:
    """(intrinsics sized to the image, full 4x4 matrix) (data/camera.py:42-51)."""
    from PIL import Image
    m = _load_4x4(path_matrix)
    with Image.open(path_image) as im:
        width, height = im.size
    return PinholeCameraIntrinsic.from_parameters(width, height, m[0, 0], m[1, 1], m[0, 2], m[1, 2]), m


def print_intrinsic_projection_parameters(intrinsics: PinholeCameraIntrinsic) -> None:
    fx, fy, cx, cy = extract_intrinsic_projection_parameters(intrinsics)
    print(f"Intrinsics: \nfx={fx:f}\nfy={fy:f}\ncx={cx:f}\ncy={cy:f}")


class StaticCenterCrop:
    """Centre crop of [H, W, ...] arrays (data/cropping.py:1-10); the crop window is fixed at construction."""

    def __init__(self, image_size, crop_size):
        self.h, self.w = int(image_size[0]), int(image_size[1])
        self.th, self.tw = int(crop_size[0]), int(crop_size[1])

    def __call__(self, img):
        rows = slice((self.h - self.th) // 2, (self.h + self.th) // 2)
        cols = slice((self.w - self.tw) // 2, (self.w + self.tw) // 2)
        return img[rows, cols] if img.ndim == 2 else img[rows, cols, ...]


def modify_intrinsics_due_to_cropping(fx, fy, cx, cy, h, w, original_h=480, original_w=640):
    """image_processing/__init__.py:301-309, literally: cy += (h - original_h) / 2 but cx += (w / original_w) / 2
    (quirk D1: the x shift divides where the y shift subtracts; for the DeepDeform 640 -> 640 crop it adds 0.5 px)."""
    return fx, fy, cx + (w / original_w) / 2, cy + (h - original_h) / 2
