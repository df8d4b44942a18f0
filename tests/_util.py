"""Shared test helpers (fixture loaders, scene rendering through the CPU oracle)."""
import os
import struct

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXTURES = os.path.join(GOLDEN, "reference_fixtures")


def rel_err(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    den = np.abs(b).max()
    return float(np.abs(a - b).max() / (den if den > 0 else 1.0))


def subdivide_midpoint(V, F, n):
    """Open3D TriangleMesh::SubdivideMidpoint face/vertex order (used by the reference's GenerateXyPlane,
    cpp/tests/test_utils/geometry.cpp:25-64)."""
    V = [tuple(v) for v in V]
    F = [tuple(f) for f in F]
    for _ in range(n):
        edge = {}

        def mid(a, b):
            k = (min(a, b), max(a, b))
            if k not in edge:
                V.append(tuple((np.array(V[a], np.float64) + np.array(V[b], np.float64)) / 2))
                edge[k] = len(V) - 1
            return edge[k]

        NF = []
        for (a, b, c) in F:
            ab, bc, ca = mid(a, b), mid(b, c), mid(c, a)
            NF += [(a, ab, ca), (ab, b, bc), (bc, c, ca), (ab, bc, ca)]
        F = NF
    return np.array(V, np.float32), np.array(F, np.int64)


def xy_plane(side, center, subdivisions):
    h = side / 2
    V = np.array([[-h, -h, 0], [-h, h, 0], [h, -h, 0], [h, h, 0]], np.float32) + np.asarray(center, np.float32)
    F = np.array([[0, 1, 2], [2, 1, 3]], np.int64)
    V, F = subdivide_midpoint(V, F, subdivisions)
    N = np.tile(np.array([[0, 0, -1]], np.float32), (len(V), 1))
    return V, N, F


def sphere_open3d(radius, resolution, center=(0.0, 0.0, 0.0)):
    """Open3D TriangleMesh::CreateSphere(radius, resolution) vertex / triangle order (Open3D 0.17 TriangleMeshFactory.cpp,
    third-party, absent here; pinned by the reference fixture extracted_face_mask_multiple_meshes.npy): poles (0, 0, +-r),
    then rings i = 1 .. res-1 of 2 res vertices (sin a cos t, sin a sin t, cos a) r with a = pi i / res, t = pi j / res;
    triangles: per j the two pole fans (0, 2+j, 2+j1) and (1, b+j1, b+j), then per ring pair (b2+j, b1+j1, b1+j),
    (b2+j, b2+j1, b1+j1). Positions computed in double, then float32 + center (the reference's FromLegacy + offset,
    cpp/tests/test_utils/geometry.cpp:76-94)."""
    V = [(0.0, 0.0, radius), (0.0, 0.0, -radius)]
    step = np.pi / resolution
    for i in range(1, resolution):
        a = step * i
        for j in range(2 * resolution):
            t = step * j
            V.append((np.sin(a) * np.cos(t) * radius, np.sin(a) * np.sin(t) * radius, np.cos(a) * radius))
    F = []
    ring = 2 * resolution
    for j in range(ring):
        j1 = (j + 1) % ring
        F.append((0, 2 + j, 2 + j1))
        b = 2 + ring * (resolution - 2)
        F.append((1, b + j1, b + j))
    for i in range(1, resolution - 1):
        b1 = 2 + ring * (i - 1)
        b2 = b1 + ring
        for j in range(ring):
            j1 = (j + 1) % ring
            F.append((b2 + j, b1 + j1, b1 + j))
            F.append((b2 + j, b2 + j1, b1 + j1))
    return np.array(V, np.float64).astype(np.float32) + np.asarray(center, np.float32), np.array(F, np.int64)


def read_depth_png(path):
    """16-bit PNG depth (PIL), as Open3D io::ReadImage gives it"""
    from PIL import Image
    return np.array(Image.open(path))


def neighbours_valid(valid):
    """pixels whose four 4-neighbours are all valid (the domain the ordered-normals fixture defines)"""
    nb = np.zeros_like(valid)
    nb[1:-1, 1:-1] = valid[:-2, 1:-1] & valid[2:, 1:-1] & valid[1:-1, :-2] & valid[1:-1, 2:]
    return nb


def read_ply(path):
    """Binary little-endian PLY (Blender export: x y z nx ny nz s t; faces as uchar count + uint indices). Quads are
    fan-triangulated (0,1,2),(0,2,3)."""
    with open(path, "rb") as f:
        data = f.read()
    head_end = data.index(b"end_header\n") + len(b"end_header\n")
    header = data[:head_end].decode().splitlines()
    nv = int([l for l in header if l.startswith("element vertex")][0].split()[-1])
    nf = int([l for l in header if l.startswith("element face")][0].split()[-1])
    props = [l.split()[-1] for l in header if l.startswith("property float")]
    body = data[head_end:]
    vert = np.frombuffer(body[: nv * 4 * len(props)], dtype="<f4").reshape(nv, len(props))
    off = nv * 4 * len(props)
    faces = []
    for _ in range(nf):
        c = body[off]
        off += 1
        idx = struct.unpack("<" + "I" * c, body[off: off + 4 * c])
        off += 4 * c
        for k in range(1, c - 1):
            faces.append((idx[0], idx[k], idx[k + 1]))
    P = vert[:, [props.index("x"), props.index("y"), props.index("z")]].astype(np.float32)
    N = vert[:, [props.index("nx"), props.index("ny"), props.index("nz")]].astype(np.float32)
    return P, N, np.array(faces, np.int64)


def transform_mesh(P, N, T):
    T = np.asarray(T, np.float64)
    P2 = (P.astype(np.float64) @ T[:3, :3].T + T[:3, 3]).astype(np.float32)
    N2 = (N.astype(np.float64) @ T[:3, :3].T).astype(np.float32)
    return P2, N2


def render_target_oracle(O, points, normals, faces, nodes, R, t, K, H, W, coverage, anchor_count=4, blur=0.5):
    """Target depth = rasterized depth of the mesh warped by (R, t), -1 -> 0 (test_deformable_mesh_fitter_one_node.cpp:94-101)."""
    a, w = O.compute_anchors(points, nodes, anchor_count, coverage)
    wp, wn = O.warp_mesh(points, normals, nodes, R, t, a, w)
    fndc, fm = O.extract_face_ndc(wp, faces, K, H, W, 0.0, 10.0)
    fi, dep, bary, dist = O.rasterize_k1_fast(fndc, fm, H, W, blur, True, True)
    return np.where(dep[..., 0] > 0, dep[..., 0], 0).astype(np.float32)


def scene_target(O, sc):
    return render_target_oracle(O, sc.points, sc.normals, sc.faces, sc.nodes, sc.gt_rotations, sc.gt_translations, sc.K, sc.H, sc.W,
                                sc.coverage)


def oracle_fit_scene(O, sc, depth, iterations=1, lm=0.001, modes=("ALL",), R0=None, t0=None, **kw):
    """FitToImage on the oracle from the node motion (R0, t0) (virtual order; default the identity warp)."""
    refp, refm = O.unproject(depth, sc.K, 1.0, 10.0)
    N = len(sc.nodes)
    R0 = np.tile(np.eye(3, dtype=np.float32), (N, 1, 1)) if R0 is None else np.ascontiguousarray(R0, np.float32).reshape(N, 3, 3)
    t0 = np.zeros((N, 3), np.float32) if t0 is None else np.ascontiguousarray(t0, np.float32).reshape(N, 3)
    h = sc.hierarchy
    hk = {}
    nodes = sc.nodes
    if h:
        # the fit runs in virtual node order (outputs are virtual-ordered too)
        nodes = sc.nodes[h["virtual_indices"]]
        hk = dict(edges=h["edges"], edge_layers=h["edge_layers"], radii=h["radii"], first_layer_count=int(h["layer_counts"][0]))
    hk.update(kw)
    return O.fit(nodes=nodes, rotations=R0, translations=t0, mesh_points=sc.points, mesh_normals=sc.normals, faces=sc.faces,
                 ref_points=refp, ref_mask=refm, H=sc.H, W=sc.W, K=sc.K, max_iterations=iterations, lm_factor=lm, modes=modes,
                 coverage=sc.coverage, **hk)


def arrowhead_fp64_solution(oracle_mod, sc, R0, t0, dg_o, lm=0.001, arap_weight=200.0, hessian_diag=None, gradient=None):
    """fp64 solution of the iteration's arrowhead system (DeformableMeshToImageFitter.cpp:222-254), solved by sparse LU
    in double (arrowhead_fp64_system)."""
    import scipy.sparse.linalg as spl
    A, b = arrowhead_fp64_system(oracle_mod, sc, R0, t0, dg_o, lm, arap_weight, hessian_diag, gradient)
    return spl.spsolve(A, b)


def fp64_system_from_blocks(diag, wing, edges, rhs):
    """fp64 matrix and right-hand side of a float arrowhead system given by its blocks -- the fitter's own system as it
    factored and refined it (nnrt_fitter_get_arrowhead_system: diagonal blocks [N,6,6] with LM, wing block (i, j) of edge
    e = (i, j) and its transpose at (j, i), rhs [6N]), every stored float taken exactly, nothing re-assembled."""
    import scipy.sparse as sp
    diag = np.asarray(diag, np.float64).reshape(-1, 6, 6)
    wing = np.asarray(wing, np.float64).reshape(-1, 6, 6)
    edges = np.asarray(edges, np.int64).reshape(-1, 2)
    N = len(diag)
    bi, bj = np.meshgrid(np.arange(6), np.arange(6), indexing="ij")
    n = np.arange(N)[:, None]
    rows = [(6 * n + bi.ravel()).ravel()]
    cols = [(6 * n + bj.ravel()).ravel()]
    vals = [diag.reshape(N, 36).ravel()]
    i, j = edges[:, :1], edges[:, 1:]
    rows += [(6 * i + bi.ravel()).ravel(), (6 * j + bi.ravel()).ravel()]
    cols += [(6 * j + bj.ravel()).ravel(), (6 * i + bj.ravel()).ravel()]
    vals += [wing.reshape(-1, 36).ravel(), np.transpose(wing, (0, 2, 1)).reshape(-1, 36).ravel()]
    A = sp.csc_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(6 * N, 6 * N))
    return A, np.asarray(rhs, np.float64)


def exact_system_solution(ft, wf, N):
    """(fp64 solution, fp64 pivot ratio) of the fitter's last arrowhead system exactly as stored on the device; (None,
    None) when it holds non-finite entries."""
    import scipy.sparse.linalg as spl
    edges = wf.get_edges()
    d, w, b = ft.arrowhead_system(N, len(edges))
    if not (np.isfinite(d).all() and np.isfinite(w).all() and np.isfinite(b).all()):
        return None, None   # A7 NaN rotations upstream: no finite system to solve
    A, b = fp64_system_from_blocks(d, w, edges, b)
    return spl.spsolve(A.tocsc(), b), fp64_pivot_ratio(A)


def rodrigues64(w):
    """fp64 Rodrigues rotations [n,3,3] of rotation vectors w [n,3] (RodriguesImpl.h:66-99; NaN at |w| = 0, quirk A7)."""
    w = np.asarray(w, np.float64).reshape(-1, 3)
    th = np.linalg.norm(w, axis=1)
    with np.errstate(invalid="ignore", divide="ignore"):
        a = w / th[:, None]
    K = np.zeros((len(w), 3, 3))
    K[:, 0, 1], K[:, 0, 2], K[:, 1, 0], K[:, 1, 2], K[:, 2, 0], K[:, 2, 1] = -a[:, 2], a[:, 1], a[:, 2], -a[:, 0], -a[:, 1], a[:, 0]
    return np.eye(3) + np.sin(th)[:, None, None] * K + (1 - np.cos(th))[:, None, None] * (K @ K)


def fp64_pivot_ratio(A):
    """min / max of the fp64 Cholesky pivots (LDLᵀ diagonal) of the symmetric sparse matrix A under a symmetric
    fill-reducing order; <= 0: not positive definite."""
    import scipy.sparse.linalg as spl
    lu = spl.splu(A.tocsc(), permc_spec="MMD_AT_PLUS_A", diag_pivot_thresh=0.0, options=dict(SymmetricMode=True))
    assert np.array_equal(lu.perm_r, lu.perm_c), "SuperLU pivoted off the diagonal"
    d = lu.U.diagonal()
    return float(d.min() / np.abs(d).max())


def arrowhead_fp64_system(oracle_mod, sc, R0, t0, dg_o=None, lm=0.001, arap_weight=200.0, hessian_diag=None, gradient=None):
    """fp64 matrix and right-hand side of the iteration's arrowhead system: data blocks (the oracle's, equal to the
    GPU's to 1e-6; or `hessian_diag`) + ARAP diagonal and wing blocks (ArapHessianImpl.h; every edge, so with >= 3 layers
    the corner off-diagonal blocks of sparse_block_cholesky_scripts.py:106-160) + LM, right-hand side = data + ARAP
    gradient (or `gradient`); assembled from the oracle's stage functions. `sc`: anything with `nodes` (original order)
    and `hierarchy` (virtual_indices, edges, edge_layers, radii, optional node_weights)."""
    import scipy.sparse as sp
    h = sc.hierarchy
    N = len(sc.nodes)
    nodes = sc.nodes[h["virtual_indices"]]
    edges = np.asarray(h["edges"], np.int32)
    # variable coverage (coverage_method 1): edge weights from the node coverage weights (virtual order)
    ej = oracle_mod.arap_edge_jacobians(edges, h["edge_layers"], h["radii"], h.get("node_weights"), nodes, R0, arap_weight)
    adiag, wing = oracle_mod.arap_hessian(edges, ej, N)
    hd = dg_o["hessian_diag"] if hessian_diag is None else hessian_diag
    D = adiag.astype(np.float64) + np.asarray(hd).reshape(N, 6, 6).astype(np.float64) + lm * np.eye(6)
    rows, cols, vals = [], [], []
    bi, bj = np.meshgrid(np.arange(6), np.arange(6), indexing="ij")
    for n in range(N):
        rows.append(6 * n + bi.ravel())
        cols.append(6 * n + bj.ravel())
        vals.append(D[n].ravel())
    for e, (i, j) in enumerate(edges):
        w = wing[e].astype(np.float64)
        rows += [6 * i + bi.ravel(), 6 * j + bi.ravel()]
        cols += [6 * j + bj.ravel(), 6 * i + bj.ravel()]
        vals += [w.ravel(), w.T.ravel()]
    A = sp.csc_matrix((np.concatenate(vals), (np.concatenate(rows), np.concatenate(cols))), shape=(6 * N, 6 * N))
    b = np.asarray(dg_o["gradient"] if gradient is None else gradient).astype(np.float64)
    return A, b
