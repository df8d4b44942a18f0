"""Mirror of the reference `nnrt` module (cpp/pybind/nnrt_pybind.cpp:27-42) for the fitter hot path.

Submodules keep the reference names: nnrt.core.linalg, nnrt.geometry (+ .functional), nnrt.rendering (+ .functional),
and the new nnrt.alignment (DeformableMeshToImageFitter, IterationMode) that the reference never bound.
"""
from . import core, geometry, rendering, alignment  # noqa: F401
