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


def _aligned16(t: torch.Tensor) -> torch.Tensor:
    return t if t.data_ptr() % 16 == 0 else t.clone()


def _solve_block_sparse_arrowhead_cholesky(diagonal_blocks, upper_wing_blocks, upper_wing_block_coordinates, arrow_base_block_index, b):
    """SolveBlockSparseArrowheadCholesky (cpp/core/linalg/SolveBlockSparseArrowheadCholesky.cpp:30-95), uncapped."""
    N.require_gpu()
    dev = torch.device("cuda", N.current_device())
    # the C-ABI reads 6x6 blocks as float4: a view at an offset that is not a multiple of 4 floats is copied into a fresh
    # (aligned) buffer first, as the reference accepts any contiguous tensor
    D = _aligned16(to_device(diagonal_blocks, torch.float32, dev).contiguous())
    Wb = _aligned16(to_device(upper_wing_blocks, torch.float32, dev).contiguous())
    C = to_device(upper_wing_block_coordinates, torch.int32, dev).contiguous()
    bb = to_device(b, torch.float32, dev).reshape(-1).contiguous()
    x = torch.empty_like(bb)
    N.check(N.lib().nnrt_solve_block_sparse_arrowhead_cholesky(N.ptr(D), N.ptr(Wb), N.ptr(C), Wb.shape[0], D.shape[0],
                                                              int(arrow_base_block_index), N.ptr(bb), N.ptr(x), N.stream_ptr()))
    return x


def release_arrowhead_plans() -> None:
    """Frees the per-structure plans the arrowhead solve keeps for reuse (device memory; MI355X extension, no reference
    counterpart)."""
    N.lib().nnrt_release_arrowhead_plans()


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


class MatrixPreprocessingOperation:
    """cpp/core/linalg/MatrixPreprocessingOperation.h"""
    NONE = 0
    TRANSPOSE = 1


class UpLoTriangular:
    """cpp/core/linalg/UpLoTriangular.h"""
    LOWER = 0
    UPPER = 1


def _dev():
    N.require_gpu()
    return torch.device("cuda", N.current_device())


def _blocks(x, dev):
    b = to_device(x, torch.float32, dev).contiguous()
    if b.dim() != 3 or b.shape[1] != b.shape[2]:
        raise RuntimeError(f"blocks must be [count, s, s], got {tuple(b.shape)}")
    return b


def _coords(x, dev, count):
    c = to_device(x, torch.int32, dev).contiguous()
    if tuple(c.shape) != (count, 2):
        raise RuntimeError(f"block coordinates must be [{count}, 2], got {tuple(c.shape)}")
    return c


def _matmul_block_sparse_row_wise_padded(blocks_a, blocks_b, blocks_b_coordinates, _with_mask=False):
    """MatmulBlockSparseRowWisePadded (cpp/core/linalg/MatmulBlockSparseImpl.h:39-157): a[row(b_i)] @ b_i per block of B;
    blocks whose row has no A block are zero."""
    dev = _dev()
    a, b = _blocks(blocks_a, dev), _blocks(blocks_b, dev)
    if a.shape[1] != b.shape[1]:
        raise RuntimeError("block sizes of A and B differ")
    c = _coords(blocks_b_coordinates, dev, b.shape[0])
    out = torch.empty_like(b)
    mask = torch.empty(b.shape[0], dtype=torch.uint8, device=dev)
    N.check(N.lib().nnrt_matmul_block_sparse_row_wise(N.ptr(a), a.shape[0], N.ptr(b), N.ptr(c), b.shape[0], b.shape[1], N.ptr(out), N.ptr(mask),
                                                       N.stream_ptr()))
    return (out, mask.bool(), c) if _with_mask else out


def _matmul_block_sparse_row_wise(blocks_a, blocks_b, blocks_b_coordinates):
    """MatmulBlockSparseRowWise: the padded product's blocks with an A row, and their coordinates."""
    out, mask, c = _matmul_block_sparse_row_wise_padded(blocks_a, blocks_b, blocks_b_coordinates, _with_mask=True)
    return out[mask].contiguous(), c[mask].contiguous()


def _matmul_block_sparse(blocks_a, a_block_breadboard, matrix_a_preprocessing, blocks_b, b_block_breadboard, matrix_b_preprocessing):
    """MatmulBlockSparse (cpp/core/linalg/MatmulBlockSparseImpl.h:160-439): op(A) op(B) for breadboard-indexed block matrices
    (int16 [block rows, block columns], -1 = empty) -> (blocks, coordinates) of the non-empty output blocks, row-major."""
    dev = _dev()
    a, b = _blocks(blocks_a, dev), _blocks(blocks_b, dev)
    ab = to_device(a_block_breadboard, torch.int16, dev).contiguous()
    bb = to_device(b_block_breadboard, torch.int16, dev).contiguous()
    ta, tb = int(matrix_a_preprocessing) == 1, int(matrix_b_preprocessing) == 1
    out_rows = ab.shape[1] if ta else ab.shape[0]
    out_cols = bb.shape[0] if tb else bb.shape[1]
    s = a.shape[1]
    out = torch.empty((out_rows * out_cols, s, s), dtype=torch.float32, device=dev)
    mask = torch.empty(out_rows * out_cols, dtype=torch.uint8, device=dev)
    N.check(N.lib().nnrt_matmul_block_sparse(N.ptr(a), a.shape[0], N.ptr(ab), ab.shape[0], ab.shape[1], int(ta), N.ptr(b), b.shape[0], N.ptr(bb),
                                              bb.shape[0], bb.shape[1], int(tb), s, N.ptr(out), N.ptr(mask), N.stream_ptr()))
    m = mask.bool()
    grid = torch.stack(torch.meshgrid(torch.arange(out_rows, device=dev, dtype=torch.int32),
                                      torch.arange(out_cols, device=dev, dtype=torch.int32), indexing="ij"), dim=-1).reshape(-1, 2)
    return out[m].contiguous(), grid[m].contiguous()


def _block_sparse_and_vector_product(blocks_a, m, blocks_a_coordinates, block_coordinate_offset, matrix_a_preprocessing, vector_b):
    """BlockSparseAndVectorProduct (cpp/core/linalg/MatmulBlockSparseImpl.h:441-602): op(A) v with A's blocks at
    coordinates + offset; the output keeps v's shape convention ([m] or [m, 1])."""
    dev = _dev()
    a = _blocks(blocks_a, dev)
    c = _coords(blocks_a_coordinates, dev, a.shape[0])
    v = to_device(vector_b, torch.float32, dev).contiguous()
    off = tuple(block_coordinate_offset) if block_coordinate_offset else (0, 0)
    out = torch.empty(int(m), dtype=torch.float32, device=dev)
    N.check(N.lib().nnrt_block_sparse_and_vector_product(N.ptr(a), N.ptr(c), a.shape[0], a.shape[1], int(off[0]), int(off[1]),
                                                          int(matrix_a_preprocessing), N.ptr(v), v.numel(), int(m), N.ptr(out), N.stream_ptr()))
    return out if v.dim() == 1 else out.reshape(int(m), 1)


def _diagonal_block_sparse_and_vector_product(blocks_d, vector_b):
    """DiagonalBlockSparseAndVectorProduct (cpp/core/linalg/MatmulBlockSparseImpl.h:604-690): out_i = D_i v_i."""
    dev = _dev()
    d = _blocks(blocks_d, dev)
    v = to_device(vector_b, torch.float32, dev).contiguous()
    if v.numel() != d.shape[0] * d.shape[1]:
        raise RuntimeError(f"vector length {v.numel()} does not match {d.shape[0]} blocks of size {d.shape[1]}")
    out = torch.empty_like(v)
    N.check(N.lib().nnrt_diagonal_block_sparse_and_vector_product(N.ptr(d), d.shape[0], d.shape[1], N.ptr(v), N.ptr(out), N.stream_ptr()))
    return out


def _sparse_blocks_op(op, matrix, blocks, coordinates, block_coordinate_offset=(0, 0), transpose=False):
    if not (isinstance(matrix, torch.Tensor) and matrix.is_cuda and matrix.dtype == torch.float32 and matrix.is_contiguous()):
        raise RuntimeError("matrix must be a contiguous float32 GPU tensor (modified in place)")
    dev = matrix.device
    b = _blocks(blocks, dev)
    c = None if coordinates is None else _coords(coordinates, dev, b.shape[0])
    off = tuple(block_coordinate_offset) if block_coordinate_offset else (0, 0)
    N.check(N.lib().nnrt_sparse_blocks_op(N.ptr(matrix), matrix.shape[0], matrix.shape[1], N.ptr(b), None if c is None else N.ptr(c), b.shape[0],
                                           b.shape[1], int(off[0]), int(off[1]), int(bool(transpose)), op, N.stream_ptr()))


def _fill_in_sparse_blocks(matrix, blocks, coordinates, block_coordinate_offset=(0, 0), transpose=False):
    """FillInSparseBlocks (cpp/core/linalg/SparseBlocksImpl.h:140-155), in place."""
    _sparse_blocks_op(0, matrix, blocks, coordinates, block_coordinate_offset, transpose)


def _add_sparse_blocks(matrix, blocks, coordinates, block_coordinate_offset=(0, 0), transpose=False):
    """AddSparseBlocks (cpp/core/linalg/SparseBlocksImpl.h:157-172), in place."""
    _sparse_blocks_op(1, matrix, blocks, coordinates, block_coordinate_offset, transpose)


def _subtract_sparse_blocks(matrix, blocks, coordinates, block_coordinate_offset=(0, 0), transpose=False):
    """SubtractSparseBlocks (cpp/core/linalg/SparseBlocksImpl.h:174-190), in place."""
    _sparse_blocks_op(2, matrix, blocks, coordinates, block_coordinate_offset, transpose)


def _fill_in_diagonal_blocks(matrix, blocks):
    """FillInDiagonalBlocks (cpp/core/linalg/DiagonalBlocksImpl.h), in place."""
    _sparse_blocks_op(0, matrix, blocks, None)


def _get_sparse_blocks(matrix, block_size, coordinates=None):
    dev = _dev()
    mat = to_device(matrix, torch.float32, dev).contiguous()
    if coordinates is None:
        c, n = None, mat.shape[0] // int(block_size)
    else:
        c = to_device(coordinates, torch.int32, dev).contiguous()
        n = c.shape[0]
        c = _coords(c, dev, n)
    out = torch.empty((n, int(block_size), int(block_size)), dtype=torch.float32, device=dev)
    N.check(N.lib().nnrt_get_sparse_blocks(N.ptr(mat), mat.shape[0], mat.shape[1], int(block_size), None if c is None else N.ptr(c), n,
                                            N.ptr(out), N.stream_ptr()))
    return out


def _get_sparse_blocks_public(matrix, block_size, coordinates):
    """GetSparseBlocks (cpp/core/linalg/SparseBlocksImpl.h:192-230)."""
    return _get_sparse_blocks(matrix, block_size, coordinates)


def _get_diagonal_blocks(matrix, block_size):
    """GetDiagonalBlocks (cpp/core/linalg/DiagonalBlocksImpl.h): matrix_size / block_size blocks."""
    return _get_sparse_blocks(matrix, block_size, None)


def _transpose_blocks_in_place(blocks):
    """TransposeBlocksInPlace (cpp/core/linalg/TransposeBlocks.h)."""
    if not (isinstance(blocks, torch.Tensor) and blocks.is_cuda and blocks.dtype == torch.float32 and blocks.is_contiguous()):
        raise RuntimeError("blocks must be a contiguous float32 GPU tensor (modified in place)")
    N.check(N.lib().nnrt_transpose_blocks_in_place(N.ptr(blocks), blocks.shape[0], blocks.shape[1], N.stream_ptr()))


def _invert_triangular_blocks(blocks, uplo):
    """InvertTriangularBlocks (cpp/core/linalg/InvertBlocks.cpp, trtri per block)."""
    dev = _dev()
    b = _blocks(blocks, dev)
    out = torch.empty_like(b)
    N.check(N.lib().nnrt_invert_triangular_blocks(N.ptr(b), b.shape[0], b.shape[1], int(uplo), N.ptr(out), N.stream_ptr()))
    return out


def _invert_positive_semidefinite_blocks(blocks):
    """InvertPositiveSemidefiniteBlocks (cpp/core/linalg/InvertBlocks.cpp:82-126), block size 3 or 6."""
    dev = _dev()
    b = _blocks(blocks, dev)
    out = torch.empty_like(b)
    N.check(N.lib().nnrt_invert_positive_semidefinite_blocks(N.ptr(b), b.shape[0], b.shape[1], N.ptr(out), N.stream_ptr()))
    return out


linalg = types.SimpleNamespace(
    AxisAngleVectorsToMatricesRodrigues=_axis_angle_vectors_to_matrices_rodrigues,
    SolveBlockDiagonalCholesky=_solve_block_diagonal_cholesky,
    SolveBlockSparseArrowheadCholesky=_solve_block_sparse_arrowhead_cholesky,
    # block-sparse stages of the arrowhead solve (C++ API of cpp/core/linalg; the reference binds none of them to Python)
    MatrixPreprocessingOperation=MatrixPreprocessingOperation,
    UpLoTriangular=UpLoTriangular,
    MatmulBlockSparseRowWise=_matmul_block_sparse_row_wise,
    MatmulBlockSparseRowWisePadded=_matmul_block_sparse_row_wise_padded,
    MatmulBlockSparse=_matmul_block_sparse,
    BlockSparseAndVectorProduct=_block_sparse_and_vector_product,
    DiagonalBlockSparseAndVectorProduct=_diagonal_block_sparse_and_vector_product,
    FillInSparseBlocks=_fill_in_sparse_blocks,
    AddSparseBlocks=_add_sparse_blocks,
    SubtractSparseBlocks=_subtract_sparse_blocks,
    FillInDiagonalBlocks=_fill_in_diagonal_blocks,
    GetSparseBlocks=_get_sparse_blocks_public,
    GetDiagonalBlocks=_get_diagonal_blocks,
    TransposeBlocksInPlace=_transpose_blocks_in_place,
    InvertTriangularBlocks=_invert_triangular_blocks,
    InvertPositiveSemidefiniteBlocks=_invert_positive_semidefinite_blocks,
)
