"""CPU checks of the drop-in boundary: the HIP library loads without a GPU, exports every function that
include/nnrt_mi355x.h declares, the Python binding table matches the header, and the host-side argument checks fail
loudly (no compute is launched here)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", h) for h in ("nnrt_mi355x.h", "nnrt_dlpack.h")]


def _declared():
    names = set()
    for header in HEADERS:
        text = re.sub(r"/\*.*?\*/", "", open(header).read(), flags=re.S)
        names |= set(re.findall(r"\b(nnrt_[a-z0-9_]+)\s*\(", text))
    return sorted(names)


@pytest.fixture(scope="module")
def native():
    from dynamicfuion_python_amd import _native
    if not os.path.exists(_native.LIB_PATH):
        _native.build()
    return _native


def test_header_declares_entry_points():
    names = _declared()
    assert len(names) >= 30
    for must in ("nnrt_fitter_fit_to_image", "nnrt_fitter_prepare", "nnrt_fitter_iterate", "nnrt_warp_field_create",
                 "nnrt_rasterize_ndc_triangles", "nnrt_solve_block_sparse_arrowhead_cholesky", "nnrt_fitter_fit_to_image_dlpack",
                 "nnrt_warp_field_create_dlpack"):
        assert must in names


def test_library_exports_every_declared_symbol(native):
    out = subprocess.check_output(["nm", "-D", "--defined-only", native.LIB_PATH], text=True)
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    missing = [n for n in _declared() if n not in exported]
    assert not missing, f"declared in include/*.h but not exported: {missing}"
    # every exported nnrt_ symbol is declared (no undocumented ABI)
    extra = sorted(n for n in exported if n.startswith("nnrt_") and n not in _declared())
    assert not extra, f"exported but not declared: {extra}"


def test_binding_table_matches_header(native):
    assert sorted(native.exported_symbols()) == _declared()


def test_library_loads_without_gpu(native):
    lib = native.lib()   # dlopen + binds every signature; must not need a device
    for name in _declared():
        assert getattr(lib, name) is not None
    assert lib.nnrt_runtime_version() > 0


def test_default_params_mirror_reference_constructor(native):
    p = native.FitterParams()
    native.lib().nnrt_fitter_default_params(ctypes.byref(p))
    # DeformableMeshToImageFitter.h:34-46 defaults
    assert p.max_iteration_count == 100
    assert p.iteration_mode_count == 1 and p.iteration_modes[0] == 0
    assert p.minimal_update_threshold == pytest.approx(1e-6)
    assert p.use_perspective_correction == 1
    assert p.max_depth == pytest.approx(10.0)
    assert p.use_tukey_penalty_for_data_term == 0
    assert p.tukey_penalty_cutoff_cm == pytest.approx(0.01)
    assert p.preconditioning_dampening_factor == 0.0
    assert p.arap_term_weight == pytest.approx(200.0)
    assert p.use_huber_penalty_for_arap_term == 0
    assert p.huber_penalty_constant == pytest.approx(1e-4)
    assert p.use_hip_graph == 1


def test_struct_layout_matches_header(native):
    # 13 scalars + 16-int mode array, all 4-byte fields
    assert ctypes.sizeof(native.FitterParams) == 4 * (13 + 16)


def test_argument_errors_are_reported(native):
    lib = native.lib()
    out = ctypes.c_void_p()
    nodes = np.zeros((2, 3), np.float32)
    # anchor_count > node_count -> error (WarpField.cpp:57-61), before any device work
    st = lib.nnrt_warp_field_create(native.ptr(nodes), 2, 0.05, 0, 4, 0, 1, 1, 4, None, 0, ctypes.byref(out))
    assert st == 1
    assert b"Anchor count" in lib.nnrt_last_error()
    st = lib.nnrt_warp_field_create(None, 2, 0.05, 0, 4, 0, 1, 1, 4, None, 0, ctypes.byref(out))
    assert st == 1
    p = native.FitterParams()
    lib.nnrt_fitter_default_params(ctypes.byref(p))
    p.preconditioning_dampening_factor = 2.0   # must be in [0, 1] (DeformableMeshToImageFitter.cpp:79-82)
    st = lib.nnrt_fitter_create(ctypes.byref(p), 0, ctypes.byref(out))
    assert st == 1
    with pytest.raises(native.NnrtError):
        native.check(st)
    lib.nnrt_fitter_default_params(ctypes.byref(p))
    assert p.ndc_convention == 0   # NNRT_NDC_REFERENCE
    p.ndc_convention = 7
    assert lib.nnrt_fitter_create(ctypes.byref(p), 0, ctypes.byref(out)) == 1
    assert b"ndc_convention" in lib.nnrt_last_error()


def test_diagnostic_exports_refuse_bad_arguments(native):
    """The diagnostic copies (nnrt_fitter_get_arrowhead_system, nnrt_fitter_get_warped_mesh) check their pointers and the
    prepared frame before touching the device (a caller-sized host buffer is never written past); the build
    reports its refinement floor and Jacobian arithmetic."""
    lib = native.lib()
    buf = np.zeros(64, np.float32)
    assert lib.nnrt_fitter_get_arrowhead_system(None, native.ptr(buf), native.ptr(buf), native.ptr(buf), 1, 1, None) == 1
    assert b"null" in lib.nnrt_last_error()
    assert lib.nnrt_fitter_get_warped_mesh(None, native.ptr(buf), native.ptr(buf), 1, None) == 1
    assert native.refine_floor() == pytest.approx(1e-5)
    assert native.jacobian_fma() is False   # the product: the reference CPU path's unfused arithmetic


def test_overlapping_outputs_are_rejected(native):
    """outputs that overlap an input the kernel still reads are refused before any device work (pointer
    arithmetic only, so this runs without a GPU): InvertTriangularBlocks into its own blocks, BlockSparseAndVectorProduct
    into a range overlapping the vector."""
    lib = native.lib()
    base = 0x7f0000000000
    blocks = ctypes.c_void_p(base)
    # 3 blocks of 6x6 floats = 432 B; an output starting 4 floats in overlaps
    assert lib.nnrt_invert_triangular_blocks(blocks, 3, 6, 0, ctypes.c_void_p(base + 16), None) == 1
    assert b"overlap" in lib.nnrt_last_error()
    coords = ctypes.c_void_p(base + 0x100000)
    vec = ctypes.c_void_p(base + 0x200000)
    # vector of 12 floats at vec, output of m = 12 floats starting 8 floats into it
    assert lib.nnrt_block_sparse_and_vector_product(blocks, coords, 3, 6, 0, 0, 0, vec, 12, 12, ctypes.c_void_p(base + 0x200000 + 32), None) == 1
    assert b"overlap" in lib.nnrt_last_error()


def test_no_cpu_fallback(native, monkeypatch):
    import torch
    monkeypatch.setattr(torch.cuda, "is_available", lambda: False)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        native.require_gpu()


def test_missing_library_fails_loudly(native, monkeypatch, tmp_path):
    monkeypatch.setattr(native, "_lib", None)
    monkeypatch.setattr(native, "LIB_PATH", str(tmp_path / "absent.so"))
    with pytest.raises(RuntimeError, match="missing"):
        native.lib()


def test_dlpack_entry_points_validate_tensors(native):
    """include/nnrt_dlpack.h: dtype / shape / layout are checked on the host before any device work, and a valid tensor
    is forwarded to the pointer entry point (whose own argument check then reports)."""
    lib = native.lib()
    out = ctypes.c_void_p()

    def create(arr, anchor_count=4):
        cap, ptr = native.dlpack(arr)
        st = lib.nnrt_warp_field_create_dlpack(ptr, 0.05, 0, anchor_count, 0, 1, 1, 4, None, 0, ctypes.byref(out))
        del cap
        return st, lib.nnrt_last_error()

    st, msg = create(np.zeros((2, 3), np.float64))
    assert st == 1 and b"nodes: unsupported dtype" in msg
    st, msg = create(np.zeros((2, 4), np.float32))
    assert st == 1 and b"dimension 1 is 4, expected 3" in msg
    st, msg = create(np.zeros((2, 3, 1), np.float32))
    assert st == 1 and b"expected 2 dimensions" in msg
    st, msg = create(np.zeros((6, 2), np.float32)[:, :1].reshape(-1))   # 1-D: rank error first
    assert st == 1
    st, msg = create(np.asfortranarray(np.zeros((4, 3), np.float32)))
    assert st == 1 and b"not a compact row-major tensor" in msg
    st, msg = create(np.zeros((2, 3), np.float32))   # valid tensor -> pointer entry point: anchor_count > node_count
    assert st == 1 and b"Anchor count" in msg


def test_dlpack_rasterize_rejects_host_tensors(native):
    lib = native.lib()
    caps = [native.dlpack(np.zeros((4, 3, 3), np.float32))] + [native.dlpack(np.zeros((8, 8, 1), dt)) for dt in (np.int64, np.float32)]
    st = lib.nnrt_rasterize_ndc_triangles_dlpack(caps[0][1], None, 0.0, 1, 0, 1, caps[1][1], caps[2][1], caps[2][1], caps[2][1], None)
    assert st == 1 and b"face_ndc: must be a ROCm device tensor" in lib.nnrt_last_error()
