"""MI355X-native DeformableMeshToImageFitter hot path (drop-in for henry123-boy/Dynamicfuion_python's nnrt fitter).

Layout:
  csrc/            gfx950 HIP kernels + host orchestration + C-ABI (include/nnrt_mi355x.h) -> libnnrt_mi355x.so
  _native.py       ctypes binding of the C-ABI (fails loudly when the extension or a GPU is missing)
  nnrt/            mirror of the reference's `nnrt` Python module names on the hot path
  alignment/       mirror of alignment/render_based/RenderingAlignmentOptimizer (the reference's Python API slot)
  synthetic.py     synthetic scenes for the BASELINE configs (C1-C5)
"""
__all__ = ["nnrt", "alignment", "synthetic"]
