"""How many steps of iterative refinement an f32 Cholesky factor buys on the ARAP arrowhead systems (development, CPU
only). Runs the oracle's own trajectory of a frame (C2_ARAP unless given), builds each
iteration's normal equations in fp64 (tests/_util.arrowhead_fp64_system: data blocks + ARAP + LM), factors them densely
in float32 (LAPACK spotrf, natural order: an emulation of the GPU's f32 factor, not its nested-dissection order) and
applies 0..STEPS refinement steps with an fp64 residual, printing each step's error against the fp64 solution next to
the system's fp64 pivot ratio and its condition estimate cond ~ 1 / ratio.
   python tools/dev/refine_steps.py [scene] [iterations] [steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import scipy.linalg as sl  # noqa: E402
import scipy.sparse.linalg as spl  # noqa: E402
import oracle as O  # noqa: E402
from _util import arrowhead_fp64_system, fp64_pivot_ratio, oracle_fit_scene, rel_err, scene_target  # noqa: E402
from dynamicfuion_python_amd import synthetic as S  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C2_ARAP"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 6
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 4
O.build()
sc = S.make_scene(name, hierarchy_builder=lambda n, c, l: O.build_hierarchy(n, c, l))
depth = scene_target(O, sc)
N = len(sc.nodes)
R = np.tile(np.eye(3, dtype=np.float32), (N, 1, 1))
t = np.zeros((N, 3), np.float32)
for k in range(iters):
    R1, t1, dg = oracle_fit_scene(O, sc, depth, 1, R0=R, t0=t, raise_on_failure=False)
    A, b = arrowhead_fp64_system(O, sc, R, t, dg)
    ratio = fp64_pivot_ratio(A)
    x64 = spl.spsolve(A.tocsc(), b)
    dense = A.shape[0] <= 12000
    errs = []
    if dense:
        Ad = A.toarray()
        try:
            L = sl.cholesky(Ad.astype(np.float32), lower=True, check_finite=False)
        except np.linalg.LinAlgError:
            L = None
        if L is not None:
            def solve32(r):
                y = sl.solve_triangular(L, r.astype(np.float32), lower=True, check_finite=False)
                return sl.solve_triangular(L.T, y, lower=False, check_finite=False).astype(np.float64)

            x = solve32(b)
            errs = [rel_err(x, x64)]
            for s in range(steps):
                x = x + solve32(b - A @ x)
                errs.append(rel_err(x, x64))
    # the GPU's route: stem blocks D (layer 0, block-diagonal) inverted in f32, Schur corner S = C - B^T D^-1 B formed and
    # factored in f32, back substitution in f32; refinement residuals in fp64 (csrc/corner.hip, k_corner_flow)
    n0 = 6 * int(sc.hierarchy["layer_counts"][0])
    As = A.tocsr()
    D, Bm, C = As[:n0, :n0].toarray() if n0 <= 12000 else None, As[:n0, n0:].toarray(), As[n0:, n0:].toarray()
    Dsp = As[:n0, :n0].tocoo()
    assert np.all(Dsp.row // 6 == Dsp.col // 6), "stem not block-diagonal"
    Dinv32 = np.stack([np.linalg.inv(As[6 * i:6 * i + 6, 6 * i:6 * i + 6].toarray().astype(np.float32)) for i in range(n0 // 6)])
    B32 = Bm.astype(np.float32)
    DinvB32 = np.einsum("nij,njk->nik", Dinv32, B32.reshape(n0 // 6, 6, -1)).reshape(n0, -1).astype(np.float32)
    S32 = (C.astype(np.float32) - B32.T @ DinvB32).astype(np.float32)
    diagS = np.diag(S32).astype(np.float64)
    try:
        Ls = sl.cholesky(S32, lower=True, check_finite=False)
        piv = float((np.diag(Ls).astype(np.float64) ** 2 / diagS).min())
    except np.linalg.LinAlgError:
        Ls, piv = None, 0.0

    def schur32(r):
        r = r.astype(np.float32)
        r0, r1 = r[:n0], r[n0:]
        y0 = np.einsum("nij,nj->ni", Dinv32, r0.reshape(-1, 6)).reshape(-1).astype(np.float32)
        z = sl.solve_triangular(Ls, (r1 - B32.T @ y0).astype(np.float32), lower=True, check_finite=False)
        x1 = sl.solve_triangular(Ls.T, z, lower=False, check_finite=False).astype(np.float32)
        x0 = (y0 - DinvB32 @ x1).astype(np.float32)
        return np.concatenate([x0, x1]).astype(np.float64)

    serrs = []
    if Ls is not None:
        xs = schur32(b)
        serrs = [rel_err(xs, x64)]
        for s in range(steps):
            xs = xs + schur32(b - A @ xs)
            serrs.append(rel_err(xs, x64))
    # float-rounding-sized differences between two assemblies of the same system (e.g. the GPU's ARAP blocks against the
    # oracle's, which the GPU tests' fp64 reference uses): a symmetric relative perturbation of 2^-24 per stored entry
    rng = np.random.default_rng(k)
    Ac = A.tocoo()
    keep = Ac.row <= Ac.col
    pert = Ac.data[keep] * rng.uniform(-5.96e-8, 5.96e-8, keep.sum())
    import scipy.sparse as sp
    P = sp.coo_matrix((pert, (Ac.row[keep], Ac.col[keep])), shape=A.shape)
    P = P + sp.triu(P, 1).T
    floor = rel_err(spl.spsolve((A + P).tocsc(), b), x64)
    print(f"{name} iteration {k + 1}: fp64 pivot ratio {ratio:.2g}; a 2^-24 entry perturbation moves the fp64 solution by {floor:.2g}; err vs fp64 after 0..{steps} refinement steps -- dense f32 "
          "factor: " + (" ".join(f"{e:.2g}" for e in errs) if errs else ("breaks down" if dense else "not run")) + f"; f32 Schur route (min corner pivot / diag(S) {piv:.2g}): "
          + (" ".join(f"{e:.2g}" for e in serrs) if serrs else "f32 corner Cholesky breaks down"), flush=True)
    if dg.get("status", 0) != 0:
        break
    R, t = R1, t1
