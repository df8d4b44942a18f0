"""GPU parity of the arrowhead solve's block-sparse stages as standalone nnrt.core.linalg entry points (block_sparse.hip):
the reference's KATs (cpp/tests/test_linalg_matmul_block_sparse.cpp, cpp/tests/test_linalg_block_routines.cpp) through
the C-ABI, and bit-exact agreement with the oracle's restatement on random 6x6-block operands of arrowhead shape (same
float order on both sides). BlockSparseAndVectorProduct keeps the reference's atomic row sums, so it is compared to the
oracle within 1e-5 relative.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from golden import kat_literals as L  # noqa: E402


@pytest.fixture(scope="module")
def la():
    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible for a -m gpu test")
    from dynamicfuion_python_amd import _native
    _native.lib()
    from dynamicfuion_python_amd import nnrt
    return nnrt.core.linalg


DEV = "cuda:0"


def _np(t):
    return t.detach().cpu().numpy()


def _padded_rowwise_gt():
    blocks = list(L.ROWWISE_C)
    for i in L.ROWWISE_PADDED_ZERO_BLOCKS:
        blocks.insert(i, np.zeros((3, 3), np.float32))
    return np.stack(blocks)


def test_matmul_block_sparse_row_wise_kat(la, oracle_mod):
    c, coords = la.MatmulBlockSparseRowWise(L.ROWWISE_A, L.ROWWISE_B, L.ROWWISE_B_COORDS)
    assert np.allclose(_np(c), L.ROWWISE_C, rtol=1e-5, atol=1e-8)
    assert np.array_equal(_np(coords), L.ROWWISE_C_COORDS)
    padded = la.MatmulBlockSparseRowWisePadded(L.ROWWISE_A, L.ROWWISE_B, L.ROWWISE_B_COORDS)
    assert np.allclose(_np(padded), _padded_rowwise_gt(), rtol=1e-5, atol=1e-8)
    assert np.array_equal(_np(padded), oracle_mod.matmul_block_sparse_row_wise(L.ROWWISE_A, L.ROWWISE_B, L.ROWWISE_B_COORDS)[0])


@pytest.mark.parametrize("case", sorted(L.MBS_CASES))
def test_matmul_block_sparse_kat(la, case):
    (lhs, tl, rhs, tr), gt_blocks, gt_coords = L.MBS_CASES[case]
    ops = {"A": (L.MBS_A, L.MBS_A_BOARD), "B": (L.MBS_B, L.MBS_B_BOARD)}
    c, coords = la.MatmulBlockSparse(ops[lhs][0], ops[lhs][1], tl, ops[rhs][0], ops[rhs][1], tr)
    assert np.allclose(_np(c), gt_blocks, rtol=1e-5, atol=1e-8)
    assert np.array_equal(_np(coords), gt_coords)


def test_block_sparse_and_vector_products_kat(la):
    NONE, T = la.MatrixPreprocessingOperation.NONE, la.MatrixPreprocessingOperation.TRANSPOSE
    c = la.BlockSparseAndVectorProduct(L.MBS_A, 4, L.BSV_A_COORDS, (0, 0), NONE, L.BSV_V)
    assert np.allclose(_np(c), L.BSV_C, rtol=1e-5, atol=1e-8)
    d = la.BlockSparseAndVectorProduct(L.MBS_B, 4, L.BSV_B_COORDS, (0, 0), T, L.BSV_V.reshape(-1, 1))
    assert d.shape == (4, 1) and np.allclose(_np(d).ravel(), L.BSV_D, rtol=1e-5, atol=1e-8)
    e = la.DiagonalBlockSparseAndVectorProduct(L.DBSV_D, L.BSV_V)
    assert np.allclose(_np(e), L.DBSV_C, rtol=1e-5, atol=1e-8)
    with pytest.raises(RuntimeError, match="outside"):
        la.BlockSparseAndVectorProduct(L.MBS_A, 2, L.BSV_A_COORDS, (0, 0), NONE, L.BSV_V)


@pytest.mark.parametrize("upper", [False, True])
def test_invert_triangular_blocks_kat(la, oracle_mod, upper):
    blocks = L.TRI_UPPER if upper else L.TRI_LOWER
    inv = _np(la.InvertTriangularBlocks(blocks, la.UpLoTriangular.UPPER if upper else la.UpLoTriangular.LOWER))
    assert np.allclose(inv, L.TRI_UPPER_INV if upper else L.TRI_LOWER_INV, rtol=1e-4, atol=1e-8)
    assert np.array_equal(inv, oracle_mod.invert_triangular_blocks(blocks, upper)[0])
    rng = np.random.default_rng(5)
    tri = rng.normal(size=(400, 6, 6)).astype(np.float32) + 4 * np.eye(6, dtype=np.float32)
    tri = np.triu(tri) if upper else np.tril(tri)
    assert np.array_equal(_np(la.InvertTriangularBlocks(tri, int(upper))), oracle_mod.invert_triangular_blocks(tri, upper)[0])
    singular = L.TRI_LOWER.copy()
    singular[2, 1, 1] = 0
    with pytest.raises(RuntimeError, match="trtri"):
        la.InvertTriangularBlocks(singular, la.UpLoTriangular.LOWER)


def test_transpose_and_fill_get_blocks_kat(la):
    b = torch.from_numpy(L.TRI_LOWER.copy()).to(DEV)
    la.TransposeBlocksInPlace(b)
    assert np.array_equal(_np(b), L.TRANSPOSED_TRI_LOWER)
    diag_gt = np.zeros((12, 12), np.float32)
    for i in range(6):
        diag_gt[2 * i:2 * i + 2, 2 * i:2 * i + 2] = L.ARANGE_BLOCKS[i]
    m = torch.zeros((12, 12), dtype=torch.float32, device=DEV)
    la.FillInDiagonalBlocks(m, L.ARANGE_BLOCKS)
    assert np.array_equal(_np(m), diag_gt)
    assert np.array_equal(_np(la.GetDiagonalBlocks(diag_gt, 2)), L.ARANGE_BLOCKS)
    m = torch.zeros((12, 12), dtype=torch.float32, device=DEV)
    la.FillInSparseBlocks(m, L.ARANGE_BLOCKS, L.SPARSE_COORDS, (0, 0), False)
    assert np.array_equal(_np(m), L.SPARSE_FILLED)
    la.FillInSparseBlocks(m, L.TRANSPOSE_FILL_BLOCKS, L.TRANSPOSE_FILL_COORDS, (0, 0), True)
    assert np.array_equal(_np(m), L.SPARSE_FILLED_2)
    assert np.array_equal(_np(la.GetSparseBlocks(L.SPARSE_FILLED, 2, L.SPARSE_COORDS)), L.ARANGE_BLOCKS)
    m = torch.from_numpy(L.SPARSE_FILLED.copy()).to(DEV)
    la.AddSparseBlocks(m, L.ARANGE_BLOCKS, L.SPARSE_COORDS)
    la.SubtractSparseBlocks(m, L.ARANGE_BLOCKS, L.SPARSE_COORDS)
    assert np.array_equal(_np(m), L.SPARSE_FILLED)
    with pytest.raises(RuntimeError, match="outside the matrix"):
        la.FillInSparseBlocks(torch.zeros((12, 12), dtype=torch.float32, device=DEV), L.ARANGE_BLOCKS, L.SPARSE_COORDS, (1, 0), False)


def _arrowhead_operands(seed, n0=300, n1=40, s=6, wings_per_stem=3):
    rng = np.random.default_rng(seed)
    a = rng.normal(size=(n0, s, s))
    D = (a @ a.transpose(0, 2, 1) + s * np.eye(s)).astype(np.float32)
    coords = np.array(sorted({(i, int(j)) for i in range(n0) for j in rng.choice(n1, wings_per_stem, replace=False)}), np.int32)
    W = rng.normal(size=(len(coords), s, s)).astype(np.float32)
    return D, W, coords, n0, n1


def test_stem_schur_pieces_bit_exact_vs_oracle(la, oracle_mod):
    """The arrowhead's stem pieces at arrowhead shape (300 stem blocks, 40 corner blocks, 6x6): D^-1, D^-1 W (row-wise),
    W^T (D^-1 W) (breadboards), subtract into the corner, the two vector products -- bit-exact vs the oracle except the
    atomic-summed BlockSparseAndVectorProduct (1e-5 relative)."""
    D, W, coords, n0, n1 = _arrowhead_operands(7)
    s = 6
    Dinv = _np(la.InvertPositiveSemidefiniteBlocks(D))
    Dinv_o, rc = oracle_mod.invert_psd_blocks(D)
    assert rc == 0 and np.array_equal(Dinv, Dinv_o)
    DinvW = _np(la.MatmulBlockSparseRowWisePadded(Dinv, W, coords))
    DinvW_o, mask, _ = oracle_mod.matmul_block_sparse_row_wise(Dinv_o, W, coords)
    assert mask.all() and np.array_equal(DinvW, DinvW_o)
    board = np.full((n0, n1), -1, np.int16)
    board[coords[:, 0], coords[:, 1]] = np.arange(len(coords))
    prod, pcoords = la.MatmulBlockSparse(W, board, 1, DinvW, board, 0)
    prod_o, pmask, rc = oracle_mod.matmul_block_sparse(W, board, 1, DinvW_o, board, 0)
    assert rc == 0 and np.array_equal(_np(prod), prod_o[pmask])
    assert np.array_equal(_np(pcoords), np.stack(np.nonzero(pmask.reshape(n1, n1)), axis=1))
    C = np.eye(n1 * s, dtype=np.float32) * 100
    S = torch.from_numpy(C.copy()).to(DEV)
    la.SubtractSparseBlocks(S, prod, pcoords)
    S_o = C.copy()
    oracle_mod.sparse_blocks_op(S_o, prod_o[pmask], _np(pcoords), op=2)
    assert np.array_equal(_np(S), S_o)
    rng = np.random.default_rng(8)
    b_stem = rng.normal(size=n0 * s).astype(np.float32)
    x_corner = rng.normal(size=n1 * s).astype(np.float32)
    # b_corner update (SolveBlockSparseArrowheadCholesky.cpp:66-70) and wing x corner (:81-85)
    upd = _np(la.BlockSparseAndVectorProduct(DinvW, n1 * s, coords, (0, 0), 1, b_stem))
    upd_o, _ = oracle_mod.block_sparse_and_vector_product(DinvW_o, n1 * s, coords, (0, 0), True, b_stem)
    assert np.abs(upd - upd_o).max() <= 1e-5 * np.abs(upd_o).max()
    wx = _np(la.BlockSparseAndVectorProduct(W, n0 * s, coords, (0, 0), 0, x_corner))
    wx_o, _ = oracle_mod.block_sparse_and_vector_product(W, n0 * s, coords, (0, 0), False, x_corner)
    assert np.abs(wx - wx_o).max() <= 1e-5 * np.abs(wx_o).max()
    xs = _np(la.DiagonalBlockSparseAndVectorProduct(Dinv, b_stem - wx))
    assert np.array_equal(xs, oracle_mod.diagonal_block_sparse_and_vector_product(Dinv_o, b_stem - wx))


def test_empty_operands(la):
    """Zero blocks everywhere: empty results of the right shape, no launch, no error (the reference's ParallelFor over 0)."""
    e3 = np.zeros((0, 3, 3), np.float32)
    c0 = np.zeros((0, 2), np.int32)
    assert la.MatmulBlockSparseRowWisePadded(L.ROWWISE_A, e3, c0).shape == (0, 3, 3)
    blocks, coords = la.MatmulBlockSparseRowWise(L.ROWWISE_A, e3, c0)
    assert blocks.shape == (0, 3, 3) and coords.shape == (0, 2)
    blocks, coords = la.MatmulBlockSparse(L.MBS_A, np.full((2, 3), -1, np.int16), 0, L.MBS_B, np.full((3, 2), -1, np.int16), 0)
    assert blocks.shape == (0, 2, 2) and coords.shape == (0, 2)
    out = la.BlockSparseAndVectorProduct(np.zeros((0, 2, 2), np.float32), 4, c0, (0, 0), 0, L.BSV_V)
    assert np.array_equal(_np(out), np.zeros(4, np.float32))
    assert la.DiagonalBlockSparseAndVectorProduct(np.zeros((0, 2, 2), np.float32), np.zeros(0, np.float32)).shape == (0,)
    assert la.InvertTriangularBlocks(e3, la.UpLoTriangular.LOWER).shape == (0, 3, 3)
    m = torch.zeros((4, 4), dtype=torch.float32, device=DEV)
    la.FillInSparseBlocks(m, np.zeros((0, 2, 2), np.float32), c0)
    assert not m.any()
    assert la.GetSparseBlocks(_np(m), 2, c0).shape == (0, 2, 2)
