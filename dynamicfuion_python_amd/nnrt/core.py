"""nnrt.core / nnrt.core.linalg mirror (cpp/pybind/core/linalg/linalg.cpp)."""
from __future__ import annotations

import types

import torch

from .. import _native as N
from ._tensors import to_device


def _axis_angle_vectors_to_matrices_rodrigues(vectors) -> torch.Tensor:
    """AxisAngleVectorsToMatricesRodrigues (cpp/core/linalg/RodriguesImpl.h:66-88); |w| = 0 -> NaN as in the reference (A7)."""
    N.require_gpu()
    dev = vectors.device if isinstance(vectors, torch.Tensor) and vectors.is_cuda else torch.device("cuda", N.current_device())
    v = to_device(vectors, torch.float32, dev).reshape(-1, 3)
    out = torch.empty((v.shape[0], 3, 3), dtype=torch.float32, device=dev)
    N.check(N.lib().nnrt_axis_angle_to_matrices_rodrigues(N.ptr(v), v.shape[0], N.ptr(out), N.stream_ptr()))
    return out


def _solve_block_diagonal_cholesky(blocks, b) -> torch.Tensor:
    """SolveBlockDiagonalCholesky (cpp/core/linalg/SolveBlockDiagonalCholesky.cpp): x_i = A_i^-1 b_i."""
    N.require_gpu()
    dev = torch.device("cuda", N.current_device())
    A = to_device(blocks, torch.float32, dev)
    n, s = A.shape[0], A.shape[1]
    bb = to_device(b, torch.float32, dev).reshape(-1)
    x = torch.empty(n * s, dtype=torch.float32, device=dev)
    N.check(N.lib().nnrt_solve_block_diagonal_cholesky(N.ptr(A), N.ptr(bb), n, s, N.ptr(x), N.stream_ptr()))
    return x


def _solve_block_sparse_arrowhead_cholesky(diagonal_blocks, upper_wing_blocks, upper_wing_block_coordinates, arrow_base_block_index, b):
    """SolveBlockSparseArrowheadCholesky (cpp/core/linalg/SolveBlockSparseArrowheadCholesky.cpp:30-95), uncapped."""
    N.require_gpu()
    dev = torch.device("cuda", N.current_device())
    D = to_device(diagonal_blocks, torch.float32, dev)
    Wb = to_device(upper_wing_blocks, torch.float32, dev)
    C = to_device(upper_wing_block_coordinates, torch.int32, dev)
    bb = to_device(b, torch.float32, dev).reshape(-1)
    x = torch.empty_like(bb)
    N.check(N.lib().nnrt_solve_block_sparse_arrowhead_cholesky(N.ptr(D), N.ptr(Wb), N.ptr(C), Wb.shape[0], D.shape[0],
                                                              int(arrow_base_block_index), N.ptr(bb), N.ptr(x), N.stream_ptr()))
    return x


def matmul3d(array_of_matrices_a, array_of_matrices_b) -> torch.Tensor:
    """nnrt.core.matmul3d (cpp/pybind/core/core.cpp:32 -> cpp/core/linalg/Matmul3D.cpp:25-83): per batch entry A[b] @ B[b];
    A [batch, m, k], B [batch, k, n] or [batch, k] (array of vectors -> [batch, m, 1])."""
    N.require_gpu()
    dev = torch.device("cuda", N.current_device())
    A = to_device(array_of_matrices_a, torch.float32, dev)
    B = to_device(array_of_matrices_b, torch.float32, dev)
    if A.dim() != 3:
        raise RuntimeError(f"Tensor A must be 3D (array of matrices), but got {A.dim()}D.")
    if B.dim() not in (2, 3):
        raise RuntimeError(f"Tensor B must be 2D (array of vectors) or 3D (array of matrices), but got {B.dim()}D.")
    if A.shape[2] != B.shape[1]:
        raise RuntimeError(f"Tensor A columns {A.shape[2]} mismatch with Tensor B rows {B.shape[1]}.")
    if A.shape[0] != B.shape[0]:
        raise RuntimeError(f"Tensors A and B should have matching first dimension. Got: {A.shape[0]} vs. {B.shape[0]}")
    n = B.shape[2] if B.dim() == 3 else 1
    out = torch.empty((A.shape[0], A.shape[1], n), dtype=torch.float32, device=dev)
    N.check(N.lib().nnrt_matmul3d(N.ptr(A), N.ptr(B), A.shape[0], A.shape[1], A.shape[2], n, N.ptr(out), N.stream_ptr()))
    return out


linalg = types.SimpleNamespace(
    AxisAngleVectorsToMatricesRodrigues=_axis_angle_vectors_to_matrices_rodrigues,
    SolveBlockDiagonalCholesky=_solve_block_diagonal_cholesky,
    SolveBlockSparseArrowheadCholesky=_solve_block_sparse_arrowhead_cholesky,
)
