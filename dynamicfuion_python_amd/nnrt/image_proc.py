"""Top-level `nnrt` image functions on the fusion app's input path (cpp/pybind/nnrt_pybind.cpp:50-67): depth image ->
ordered point image, on the GPU. Inputs may be numpy or torch; outputs are device tensors [H, W, 3] float32."""
from __future__ import annotations

import numpy as np
import torch

from .. import _native as N
from ._tensors import device_of


def _depth_on_device(image_in, dtype: torch.dtype):
    """Device copy of a [H, W] depth image; uint16 depth travels as its int16 bit pattern (int32 -> int16 casts wrap)."""
    dev = device_of(N.current_device())
    if isinstance(image_in, np.ndarray):
        a = np.ascontiguousarray(image_in)
        t = torch.from_numpy(a.view(np.int16) if a.dtype == np.uint16 else a)
    else:
        t = image_in.view(torch.int16) if image_in.dtype == torch.uint16 else image_in
    if t.dim() != 2:
        raise ValueError(f"depth image must be [H, W], got {tuple(t.shape)}")
    if dtype == torch.int16 and t.dtype != torch.int16:
        t = t.to(torch.int32).to(torch.int16)
    return t.to(device=dev, dtype=dtype).contiguous()


def _out(point_image_out, H, W, dev):
    if point_image_out is None:
        return torch.empty((H, W, 3), dtype=torch.float32, device=dev)
    if not isinstance(point_image_out, torch.Tensor) or point_image_out.device != dev or point_image_out.dtype != torch.float32 \
            or tuple(point_image_out.shape) != (H, W, 3) or not point_image_out.is_contiguous():
        raise ValueError(f"point_image_out must be a contiguous float32 [{H}, {W}, 3] tensor on {dev}")
    return point_image_out


def backproject_depth_ushort(image_in, fx: float, fy: float, cx: float, cy: float, normalizer: float,
                             point_image_out: torch.Tensor | None = None) -> torch.Tensor:
    """uint16 depth (e.g. mm) -> [H, W, 3] metres (image_proc.cpp:275-309)."""
    N.require_gpu()
    d = _depth_on_device(image_in, torch.int16)
    H, W = d.shape
    out = _out(point_image_out, H, W, d.device)
    N.check(N.lib().nnrt_backproject_depth_ushort(N.ptr(d), H, W, float(fx), float(fy), float(cx), float(cy), float(normalizer),
                                                  N.ptr(out), N.stream_ptr()))
    return out


def backproject_depth_float(image_in, fx: float, fy: float, cx: float, cy: float,
                            point_image_out: torch.Tensor | None = None) -> torch.Tensor:
    """float depth in metres -> [H, W, 3] (image_proc.cpp:312-339)."""
    N.require_gpu()
    d = _depth_on_device(image_in, torch.float32)
    H, W = d.shape
    out = _out(point_image_out, H, W, d.device)
    N.check(N.lib().nnrt_backproject_depth_float(N.ptr(d), H, W, float(fx), float(fy), float(cx), float(cy), N.ptr(out), N.stream_ptr()))
    return out


def backproject_depth(depth_image, fx, fy, cx, cy, depth_scale: float = 1000.0) -> torch.Tensor:
    """image_processing/__init__.py:333-344: float32 depth is taken as metres, anything else as integer units / depth_scale."""
    is_float = (isinstance(depth_image, np.ndarray) and depth_image.dtype == np.float32) or \
               (isinstance(depth_image, torch.Tensor) and depth_image.dtype == torch.float32)
    if is_float:
        return backproject_depth_float(depth_image, fx, fy, cx, cy)
    return backproject_depth_ushort(depth_image, fx, fy, cx, cy, depth_scale)
