"""Tensor plumbing: accept numpy arrays or torch tensors, hand contiguous device tensors to the C-ABI."""
from __future__ import annotations

import numpy as np
import torch


def device_of(index: int = 0) -> torch.device:
    return torch.device("cuda", index)


def to_device(x, dtype: torch.dtype, device: torch.device) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        t = x.to(device=device, dtype=dtype)
    else:
        t = torch.as_tensor(np.asarray(x), dtype=dtype, device=device)
    return t.contiguous()


def to_host_f64(x) -> np.ndarray:
    if isinstance(x, torch.Tensor):
        x = x.detach().cpu().numpy()
    return np.ascontiguousarray(np.asarray(x, dtype=np.float64))
