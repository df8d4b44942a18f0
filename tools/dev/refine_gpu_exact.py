"""The GPU arrowhead solve's refinement step on EXACTLY the float system it is given (development; VERDICT r4 weak
item 7). The fitter tests judge a refined solve against the fp64 solution of a system assembled from the oracle's ARAP
blocks, which differ from the GPU's by float rounding -- and on these ill-conditioned systems a 2^-24 entry-level
difference alone moves the fp64 solution by 2e-5 .. 3e-4 (tools/dev/refine_steps.py). Here the oracle's C5 trajectory
systems (data blocks + ARAP + LM, virtual order) are rounded to float once, solved on the GPU through the standalone
C-ABI solve (nnrt_solve_block_sparse_arrowhead_cholesky: the fitter's stem + tile-sparse corner + dataflow
substitution + gated refinement) and compared with the fp64 solution of those same float values. NNRT_LIB_PATH selects
the build: the product gate window [1e-4, 1e-3), or csrc/variants refine_none (ratio 0) / refine_all (floor 0, ratio
inf). Prints one line per iteration: corner pivot / diag(S) is not exposed here, the fp64 pivot ratio is.
   python tools/dev/refine_gpu_exact.py [scene] [iterations]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402
import scipy.sparse.linalg as spl  # noqa: E402
import torch  # noqa: E402
import oracle as O  # noqa: E402
from _util import fp64_pivot_ratio, oracle_fit_scene, rel_err, scene_target  # noqa: E402
from dynamicfuion_python_amd import synthetic as S  # noqa: E402
from dynamicfuion_python_amd.nnrt import core  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "C5"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 4
lib = os.path.basename(os.environ.get("NNRT_LIB_PATH", "libnnrt_mi355x.so"))
O.build()
sc = S.make_scene(name, hierarchy_builder=lambda n, c, l: O.build_hierarchy(n, c, l))
depth = scene_target(O, sc)
N = len(sc.nodes)
h = sc.hierarchy
n0 = int(h["layer_counts"][0])
edges = np.asarray(h["edges"], np.int32)
assert (edges[:, 1] >= n0).all() and (edges[:, 0] != edges[:, 1]).all()
R = np.tile(np.eye(3, dtype=np.float32), (N, 1, 1))
t = np.zeros((N, 3), np.float32)
for k in range(iters):
    R1, t1, dg = oracle_fit_scene(O, sc, depth, 1, R0=R, t0=t, raise_on_failure=False)
    nodes = sc.nodes[h["virtual_indices"]]
    ej = O.arap_edge_jacobians(edges, h["edge_layers"], h["radii"], h.get("node_weights"), nodes, R, 200.0)
    adiag, wing = O.arap_hessian(edges, ej, N)
    D32 = (adiag.astype(np.float64) + np.asarray(dg["hessian_diag"]).reshape(N, 6, 6) + 0.001 * np.eye(6)).astype(np.float32)
    W32 = np.ascontiguousarray(wing, np.float32)
    b32 = np.asarray(dg["gradient"], np.float32)
    bi, bj = np.meshgrid(np.arange(6), np.arange(6), indexing="ij")
    rows = [6 * n + bi.ravel() for n in range(N)] + [6 * i + bi.ravel() for i, j in edges] + [6 * j + bi.ravel() for i, j in edges]
    cols = [6 * n + bj.ravel() for n in range(N)] + [6 * j + bj.ravel() for i, j in edges] + [6 * i + bj.ravel() for i, j in edges]
    vals = [D32[n].astype(np.float64).ravel() for n in range(N)] + [W32[e].astype(np.float64).ravel() for e in range(len(edges))] + \
           [W32[e].astype(np.float64).T.ravel() for e in range(len(edges))]
    A = sp.csc_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(6 * N, 6 * N))
    x64 = spl.spsolve(A, b32.astype(np.float64))
    if os.environ.get("NNRT_DRY"):   # CPU check of the assembly only
        print(f"{name} iteration {k + 1}: system {A.shape}, n0 {n0}, fp64 pivot ratio {fp64_pivot_ratio(A):.2g}", flush=True)
        R, t = R1, t1
        continue
    x = core.linalg.SolveBlockSparseArrowheadCholesky(torch.from_numpy(D32), torch.from_numpy(W32), torch.from_numpy(edges), n0,
                                                      torch.from_numpy(b32))
    torch.cuda.synchronize()
    xg = x.cpu().numpy().astype(np.float64)
    print(f"{lib} {name} iteration {k + 1}: fp64 pivot ratio {fp64_pivot_ratio(A):.2g}; GPU solve of the exact float system vs its "
          f"fp64 solution {rel_err(xg, x64):.3g}", flush=True)
    if dg.get("status", 0) != 0:
        break
    R, t = R1, t1
