"""pybind11-style overload sets for the nnrt mirror.

The reference binds several hot-path names twice (py::overload_cast, e.g. warp_triangle_mesh, warp_point_cloud,
compute_point_to_plane_distances, get_mesh_ndc_face_vertices_and_clip_mask, GraphWarpField.warp_mesh). pybind11 tries the
overloads in registration order and calls the first whose arguments bind and convert. `Overloaded` does the same: each
overload is a Python function carrying the reference's parameter names and defaults, plus a predicate standing in for
pybind11's type conversion. `signatures()` exposes them for the signature-parity test (tests/test_mirror_signatures.py).
"""
from __future__ import annotations

import inspect
import numbers

import numpy as np
import torch


def is_int(x) -> bool:
    return isinstance(x, numbers.Integral) and not isinstance(x, bool)


def is_tensor(x) -> bool:
    return isinstance(x, (torch.Tensor, np.ndarray))


class Overloaded:
    def __init__(self, name: str, doc: str = ""):
        self.__name__ = name
        self.__qualname__ = name
        self.__doc__ = doc
        self._overloads = []   # (function, predicate(bound arguments) -> bool)

    def overload(self, predicate=lambda a: True):
        def register(fn):
            self._overloads.append((fn, predicate))
            return self
        return register

    def signatures(self):
        return [inspect.signature(fn) for fn, _ in self._overloads]

    def __get__(self, obj, objtype=None):   # usable as a method (GraphWarpField.warp_mesh)
        if obj is None:
            return self
        return lambda *args, **kwargs: self(obj, *args, **kwargs)

    def __call__(self, *args, **kwargs):
        for fn, predicate in self._overloads:
            try:
                bound = inspect.signature(fn).bind(*args, **kwargs)
            except TypeError:
                continue
            bound.apply_defaults()
            if predicate(bound.arguments):
                return fn(*bound.args, **bound.kwargs)
        sigs = "\n".join(f"    {i + 1}. {self.__name__}{s}" for i, s in enumerate(self.signatures()))
        raise TypeError(f"{self.__name__}(): incompatible function arguments. The following argument types are supported:\n{sigs}")
