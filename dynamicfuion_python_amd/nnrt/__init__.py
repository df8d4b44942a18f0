"""Mirror of the reference `nnrt` module (cpp/pybind/nnrt_pybind.cpp:27-42) for the fitter hot path.

Submodules keep the reference names: nnrt.core.linalg, nnrt.geometry (+ .functional), nnrt.rendering (+ .functional),
and the new nnrt.alignment (DeformableMeshToImageFitter, IterationMode) that the reference never bound.
"""
from . import core, geometry, rendering, alignment, image_proc  # noqa: F401
from .image_proc import backproject_depth_ushort, backproject_depth_float  # noqa: F401  (nnrt_pybind.cpp:52-67)
