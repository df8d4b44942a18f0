"""SolveBlockSparseArrowheadCholesky through the C-ABI (cpp/core/linalg/SolveBlockSparseArrowheadCholesky.cpp:30-95):
the tile-sparse Schur corner (csrc/corner.hip) on graph-structured systems -- a 2-D grid of corner nodes, stem nodes
attached to their four nearest corner nodes as the hierarchy's K-NN edges are, optional corner-corner blocks (>= 3
layers) -- against the oracle's dense restatement and an fp64 sparse solution; a corner beyond the old dense path's
32768-unknown co-residency limit; two solves running concurrently on two streams; argument validation.
"""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from _util import rel_err  # noqa: E402


@pytest.fixture(scope="module")
def la():
    if not torch.cuda.is_available():
        pytest.fail("no HIP device visible for a -m gpu test")
    from dynamicfuion_python_amd import _native
    _native.lib()
    from dynamicfuion_python_amd import nnrt
    return nnrt.core.linalg


def grid_arrowhead(cx, cy, stem_per_corner, corner_edges, seed):
    """Arrowhead system of a two-layer graph: corner nodes on a cx x cy grid (indices n0..), n0 = stem_per_corner * cx * cy
    stem nodes at uniform random positions, each with wing blocks to its 4 nearest corner nodes; with corner_edges, each
    corner node also couples to its right and upper neighbours. Random wing blocks, SPD diagonal blocks kept diagonally
    dominant. Returns (diag [N,6,6], wing [E,6,6], coords [E,2] int32, n0, b [6N])."""
    rng = np.random.default_rng(seed)
    n1 = cx * cy
    n0 = stem_per_corner * n1
    N = n0 + n1
    gx, gy = np.meshgrid(np.arange(cx), np.arange(cy), indexing="xy")
    cpos = np.stack([gx.ravel(), gy.ravel()], 1).astype(np.float64)
    spos = rng.uniform([0, 0], [cx - 1, cy - 1], (n0, 2))
    edges = []
    for i0 in range(0, n0, 512):
        d = ((spos[i0:i0 + 512, None, :] - cpos[None]) ** 2).sum(2)
        near = np.argpartition(d, 3, axis=1)[:, :4] if n1 > 4 else np.argsort(d, axis=1)
        edges += [np.stack([np.repeat(np.arange(i0, i0 + len(near)), near.shape[1]), n0 + near.ravel()], 1)]
    if corner_edges:
        ce = []
        for a in range(n1):
            x, y = a % cx, a // cx
            if x + 1 < cx:
                ce.append((n0 + a, n0 + a + 1))
            if y + 1 < cy:
                ce.append((n0 + a, n0 + a + cx))
        edges.append(np.array(ce, np.int64).reshape(-1, 2))
    edges = np.concatenate(edges, 0).astype(np.int32)
    wing = rng.normal(0, 0.3, (len(edges), 6, 6)).astype(np.float32)
    A = rng.normal(size=(N, 6, 6))
    diag = (A @ A.transpose(0, 2, 1) + 30.0 * np.eye(6)).astype(np.float32)
    deg = np.bincount(edges.ravel(), minlength=N)
    diag += (6.0 * deg)[:, None, None].astype(np.float32) * np.eye(6, dtype=np.float32)
    b = rng.normal(size=6 * N).astype(np.float32)
    return diag, wing, edges, n0, b


def fp64_solution(diag, wing, edges, b):
    import scipy.sparse as sp
    import scipy.sparse.linalg as spl
    N = len(diag)
    bi, bj = np.meshgrid(np.arange(6), np.arange(6), indexing="ij")
    rows = [6 * np.arange(N)[:, None] + bi.ravel()[None], 6 * edges[:, :1] + bi.ravel()[None], 6 * edges[:, 1:] + bi.ravel()[None]]
    cols = [6 * np.arange(N)[:, None] + bj.ravel()[None], 6 * edges[:, 1:] + bj.ravel()[None], 6 * edges[:, :1] + bj.ravel()[None]]
    vals = [diag.reshape(N, 36), wing.reshape(-1, 36), wing.transpose(0, 2, 1).reshape(-1, 36)]
    A = sp.csc_matrix((np.concatenate([v.ravel() for v in vals]).astype(np.float64),
                       (np.concatenate([r.ravel() for r in rows]), np.concatenate([c.ravel() for c in cols]))), shape=(6 * N, 6 * N))
    return spl.spsolve(A, b.astype(np.float64)), A


@pytest.mark.parametrize("cx,cy,corner_edges", [(12, 8, False), (12, 8, True), (3, 2, True), (1, 1, False), (30, 3, True)])
def test_grid_arrowhead_vs_oracle_and_fp64(la, oracle_mod, cx, cy, corner_edges):
    diag, wing, edges, n0, b = grid_arrowhead(cx, cy, 4, corner_edges, seed=cx * 100 + cy)
    x_g = la.SolveBlockSparseArrowheadCholesky(diag, wing, edges, n0, b).cpu().numpy()
    x_o = oracle_mod.solve_arrowhead(diag, wing, edges, n0, b)
    x64, _ = fp64_solution(diag, wing, edges, b)
    assert rel_err(x_o, x64) < 1e-5   # the oracle's dense restatement (corner off-diagonal blocks included) is right
    assert rel_err(x_g, x_o) < 1e-4
    assert rel_err(x_g, x64) < 1e-5


def test_corner_beyond_dense_limit(la):
    """A 6,400-node corner (38,400 unknowns): the dense path refused corners above 32,768 unknowns (its panel launches
    needed co-resident workgroups); the tile-sparse factorization is bounded by memory only."""
    diag, wing, edges, n0, b = grid_arrowhead(80, 80, 2, True, seed=7)
    assert 6 * (len(diag) - n0) > 32768
    x_g = la.SolveBlockSparseArrowheadCholesky(diag, wing, edges, n0, b).cpu().numpy()
    x64, A = fp64_solution(diag, wing, edges, b)
    assert np.isfinite(x_g).all()
    assert rel_err(x_g, x64) < 1e-4
    assert np.abs(A @ x_g.astype(np.float64) - b).max() < 1e-4 * np.abs(b).max()


def test_two_solves_concurrent_on_two_streams(la):
    """C5-sized systems (386 corner nodes, 4632 stem nodes) solved concurrently from two host threads, each on its own
    stream (the GIL is released inside the C-ABI call), three times each: every result equals the solve run alone, bit
    for bit -- the factorization does not depend on which workgroups share the CUs or on dispatch order."""
    systems = [grid_arrowhead(26, 15, 12, False, seed=s) for s in (1, 2)]
    alone = [la.SolveBlockSparseArrowheadCholesky(*sy).cpu().numpy() for sy in systems]
    out = [[], []]
    errors = []

    def run(k):
        try:
            st = torch.cuda.Stream()
            with torch.cuda.stream(st):
                for _ in range(3):
                    out[k].append(la.SolveBlockSparseArrowheadCholesky(*systems[k]).cpu().numpy())
        except Exception as e:   # pragma: no cover - reported below
            errors.append(e)

    threads = [threading.Thread(target=run, args=(k,)) for k in (0, 1)]
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    assert not errors, errors
    for k in (0, 1):
        assert len(out[k]) == 3
        for x in out[k]:
            assert np.array_equal(x, alone[k])


def test_arrowhead_argument_validation(la):
    from dynamicfuion_python_amd._native import NnrtError
    diag, wing, edges, n0, b = grid_arrowhead(4, 3, 2, True, seed=3)
    N = len(diag)
    bad = []
    for i, j in ((-1, n0), (0, N), (N, n0), (n0, n0), (0, 1)):   # negative row, column >= N, row >= N, diagonal, stem column
        e = edges.copy()
        e[0] = (i, j)
        bad.append(e)
    for e in bad:
        with pytest.raises(NnrtError) as ex:
            la.SolveBlockSparseArrowheadCholesky(diag, wing, e, n0, b)
        assert ex.value.status == 1, str(ex.value)   # NNRT_ERROR_ARGUMENT
    # still usable afterwards
    x = la.SolveBlockSparseArrowheadCholesky(diag, wing, edges, n0, b).cpu().numpy()
    assert np.isfinite(x).all()


def test_arrowhead_accepts_offset_views(la):
    """Blocks passed as views at an element offset that is not a multiple of 4 floats (not 16-byte aligned) give the
    same result as fresh tensors: the wrapper copies them (the C-ABI reads 6x6 blocks as float4)."""
    diag, wing, edges, n0, b = grid_arrowhead(5, 4, 3, True, seed=5)
    x_ref = la.SolveBlockSparseArrowheadCholesky(diag, wing, edges, n0, b).cpu().numpy()
    fd = torch.zeros(diag.size + 5, dtype=torch.float32, device="cuda")
    fd[5:] = torch.from_numpy(diag.ravel()).cuda()
    fw = torch.zeros(wing.size + 3, dtype=torch.float32, device="cuda")
    fw[3:] = torch.from_numpy(wing.ravel()).cuda()
    D = fd[5:].view(-1, 6, 6)
    Wb = fw[3:].view(-1, 6, 6)
    assert D.data_ptr() % 16 != 0 and Wb.data_ptr() % 16 != 0
    x = la.SolveBlockSparseArrowheadCholesky(D, Wb, edges, n0, b).cpu().numpy()
    assert np.array_equal(x, x_ref)


def test_plan_reuse_and_release(la):
    """The C-ABI keeps each wing structure's plan: solving two structures alternately (reusing both plans), new values
    on a known structure, and a solve after releasing every plan all give the fresh-plan results."""
    from dynamicfuion_python_amd.nnrt import core
    s1 = grid_arrowhead(6, 5, 3, True, seed=11)
    s2 = grid_arrowhead(7, 4, 2, False, seed=12)
    core.release_arrowhead_plans()
    ref1 = la.SolveBlockSparseArrowheadCholesky(*s1).cpu().numpy()
    ref2 = la.SolveBlockSparseArrowheadCholesky(*s2).cpu().numpy()
    for _ in range(2):
        assert np.array_equal(la.SolveBlockSparseArrowheadCholesky(*s1).cpu().numpy(), ref1)
        assert np.array_equal(la.SolveBlockSparseArrowheadCholesky(*s2).cpu().numpy(), ref2)
    diag, wing, edges, n0, b = s1
    rng = np.random.default_rng(13)
    b2 = rng.normal(size=b.shape).astype(np.float32)
    wing2 = (wing * 0.5).astype(np.float32)
    x_new = la.SolveBlockSparseArrowheadCholesky(diag, wing2, edges, n0, b2).cpu().numpy()   # same structure, new values
    core.release_arrowhead_plans()
    x_fresh = la.SolveBlockSparseArrowheadCholesky(diag, wing2, edges, n0, b2).cpu().numpy()
    assert np.array_equal(x_new, x_fresh)
    x64, _ = fp64_solution(diag, wing2, edges, b2)
    assert rel_err(x_new, x64) < 1e-5


def test_walk_plans_of_different_lds_alternate(la):
    """Two live corner plans whose single-workgroup walks need different dynamic LDS: the larger plan is
    prepared first, the smaller one after it, then the larger one is solved again from its cached plan. The walk's LDS
    cap is a per-device kernel attribute raised once to the whole LDS budget, so the last plan prepared cannot lower it
    below what an earlier plan launches with."""
    import os
    from dynamicfuion_python_amd.nnrt import core
    big = grid_arrowhead(12, 8, 3, True, seed=21)
    small = grid_arrowhead(2, 2, 2, False, seed=22)
    old = os.environ.get("NNRT_CORNER_WALK")
    os.environ["NNRT_CORNER_WALK"] = "1"   # the walk is a development option since round 5 (the dataflow launch is the default)
    try:
        core.release_arrowhead_plans()
        ref_big = la.SolveBlockSparseArrowheadCholesky(*big).cpu().numpy()
        ref_small = la.SolveBlockSparseArrowheadCholesky(*small).cpu().numpy()
        for _ in range(2):
            assert np.array_equal(la.SolveBlockSparseArrowheadCholesky(*big).cpu().numpy(), ref_big)
            assert np.array_equal(la.SolveBlockSparseArrowheadCholesky(*small).cpu().numpy(), ref_small)
    finally:
        if old is None:
            os.environ.pop("NNRT_CORNER_WALK", None)
        else:
            os.environ["NNRT_CORNER_WALK"] = old
        core.release_arrowhead_plans()
    for sy, x in ((big, ref_big), (small, ref_small)):
        x64, _ = fp64_solution(sy[0], sy[1], sy[2], sy[4])
        assert rel_err(x, x64) < 1e-5


@pytest.mark.parametrize("cx,cy,spc,corner_edges", [(26, 15, 12, False), (12, 8, 4, True), (80, 80, 2, True)])
def test_flow_matches_chain_launches(la, cx, cy, spc, corner_edges):
    """The dataflow substitution launch (k_corner_flow: every back-substitution chain and the stem pass in one launch,
    dependencies through ticket-ordered counters) against the per-depth chain launches: bit-identical solutions (the same
    float operations; with the diagonal inverses formed in the last factor launch against a k_corner_invert launch), for a
    C5-sized corner, a small one with corner-corner blocks and the 38,400-unknown corner; the flow solve repeated three
    times under two concurrent streams gives the same bits every time."""
    import os
    from dynamicfuion_python_amd.nnrt import core
    sy = grid_arrowhead(cx, cy, spc, corner_edges, seed=cx + cy)
    old = {k: os.environ.get(k) for k in ("NNRT_CORNER_FLOW", "NNRT_CORNER_WALK", "NNRT_CORNER_FOLD_INV")}
    try:
        os.environ["NNRT_CORNER_WALK"] = "0"
        xs = {}
        for flow in ("0", "1"):
            os.environ["NNRT_CORNER_FLOW"] = flow
            os.environ["NNRT_CORNER_FOLD_INV"] = flow   # the diagonal inverses in the last factor launch or their own
            core.release_arrowhead_plans()
            xs[flow] = la.SolveBlockSparseArrowheadCholesky(*sy).cpu().numpy()
        assert np.array_equal(xs["0"], xs["1"])
        other = grid_arrowhead(20, 10, 6, True, seed=99)
        out, errors = [], []

        def load():
            try:
                st = torch.cuda.Stream()
                with torch.cuda.stream(st):
                    for _ in range(3):
                        la.SolveBlockSparseArrowheadCholesky(*other)
            except Exception as e:   # pragma: no cover - reported below
                errors.append(e)

        th = threading.Thread(target=load)
        th.start()
        for _ in range(3):
            out.append(la.SolveBlockSparseArrowheadCholesky(*sy).cpu().numpy())
        th.join()
        assert not errors, errors
        for x in out:
            assert np.array_equal(x, xs["1"])
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
        core.release_arrowhead_plans()
