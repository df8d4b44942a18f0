"""ctypes wrapper over oracle/libnnrt_oracle.so -- TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference hot path (see nnrt_oracle.cpp header). Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module; the product package never does.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "libnnrt_oracle.so")
_lib = None

MODE = {"ALL": 0, "TRANSLATION_ONLY": 1, "ROTATION_ONLY": 2}


def build(force: bool = False) -> str:
    srcs = [os.path.join(_HERE, f) for f in ("nnrt_oracle.cpp", "tsdf_oracle.cpp")]
    if force or not os.path.exists(_LIB_PATH) or any(os.path.getmtime(_LIB_PATH) < os.path.getmtime(f) for f in srcs):
        subprocess.check_call(["make", "-s", "-C", _HERE, "libnnrt_oracle.so"])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(_LIB_PATH)
        _lib.orc_last_error.restype = ctypes.c_char_p
    return _lib


def _p(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def _f32(a):
    return np.ascontiguousarray(a, dtype=np.float32)


def _i64(a):
    return np.ascontiguousarray(a, dtype=np.int64)


def _i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def _u8(a):
    return np.ascontiguousarray(a, dtype=np.uint8)


def _f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def _check(rc):
    if rc != 0:
        raise RuntimeError(f"oracle error {rc}: {lib().orc_last_error().decode()}")


def set_num_threads(n: int):
    lib().orc_set_num_threads(ctypes.c_int(n))


def set_accumulate_double(on: bool):
    """Data-term JtJ / Jt r summation: double (default, exact-sum checker) or the reference's float-serial order."""
    lib().orc_set_accumulate_double(ctypes.c_int(int(on)))


def set_fused_jacobians(on: bool):
    """Pixel-node Jacobian arithmetic (a10 + a12): the reference CPU path's unfused expressions (default) or the GPU
    product's FMA form (bit-identical to its terms; nnrt_oracle.cpp g_jac_fma)."""
    lib().orc_set_fused_jacobians(ctypes.c_int(int(on)))


def num_threads() -> int:
    return lib().orc_num_threads()


def compute_anchors(points, nodes, anchor_count=4, coverage=0.05, node_weights=None, minimum_valid_anchor_count=0, threshold=None):
    """threshold None: the anchor API's rule (threshold iff minimum_valid_anchor_count > 0); True / False: forced (WarpTriangleMesh
    with / without threshold_nodes_by_distance)."""
    points, nodes = _f32(points), _f32(nodes)
    V, N = len(points), len(nodes)
    anchors = np.empty((V, anchor_count), np.int32)
    weights = np.empty((V, anchor_count), np.float32)
    nw = None if node_weights is None else _f32(node_weights)
    thr = int(minimum_valid_anchor_count > 0) if threshold is None else int(bool(threshold))
    lib().orc_compute_anchors_ex(_p(points), ctypes.c_int64(V), _p(nodes), ctypes.c_int(N), ctypes.c_int(anchor_count),
                                 ctypes.c_float(coverage), _p(nw), ctypes.c_int(thr), ctypes.c_int(minimum_valid_anchor_count), _p(anchors),
                                 _p(weights))
    return anchors, weights


def node_coverage_weights(nodes, coverage):
    nodes = _f32(nodes)
    out = np.empty(len(nodes), np.float32)
    lib().orc_node_coverage_weights(_p(nodes), ctypes.c_int(len(nodes)), ctypes.c_float(coverage), _p(out))
    return out


def build_hierarchy(nodes, coverage, layer_count, max_degree=4, radii=None):
    nodes = _f32(nodes)
    N = len(nodes)
    vidx = np.empty(N, np.int64)
    counts = np.empty(layer_count, np.int32)
    cap = N * max_degree
    edges = np.empty((cap, 2), np.int32)
    elayers = np.empty(cap, np.int8)
    r = None if radii is None else _f32(radii)
    ne = lib().orc_build_hierarchy(_p(nodes), ctypes.c_int(N), ctypes.c_float(coverage), ctypes.c_int(layer_count),
                                   ctypes.c_int(max_degree), _p(r), _p(vidx), _p(counts), _p(edges), _p(elayers), ctypes.c_int(cap))
    if ne < 0:
        raise RuntimeError(lib().orc_last_error().decode())
    return vidx, counts, edges[:ne].copy(), elayers[:ne].copy()


def warp_mesh(points, normals, nodes, rotations, translations, anchors, weights, extrinsics=None):
    points, normals, nodes = _f32(points), _f32(normals), _f32(nodes)
    rotations, translations, anchors, weights = _f32(rotations), _f32(translations), _i32(anchors), _f32(weights)
    V = len(points)
    op = np.empty((V, 3), np.float32)
    on = np.empty((V, 3), np.float32)
    E = None if extrinsics is None else _f64(extrinsics)
    lib().orc_warp_mesh(_p(points), _p(normals), ctypes.c_int64(V), _p(nodes), _p(rotations), _p(translations), _p(anchors),
                        _p(weights), ctypes.c_int(anchors.shape[1]), _p(E), _p(op), _p(on))
    return op, on


def warp_points(points, normals, nodes, rotations, translations, anchors, weights, minimum_valid=-1, extrinsics=None):
    """Warp3dPoints[AndNormals] with supplied anchors; minimum_valid >= 0: BlendWarp_ValidAnchorCountThreshold. normals may be
    None (points only; the returned normals are then None)."""
    points, nodes = _f32(points), _f32(nodes)
    normals = None if normals is None else _f32(normals)
    rotations, translations, anchors, weights = _f32(rotations), _f32(translations), _i32(anchors), _f32(weights)
    V = len(points)
    op = np.empty((V, 3), np.float32)
    on = None if normals is None else np.empty((V, 3), np.float32)
    E = None if extrinsics is None else _f64(extrinsics)
    lib().orc_warp_points(_p(points), _p(normals), ctypes.c_int64(V), _p(nodes), _p(rotations), _p(translations), _p(anchors),
                          _p(weights), ctypes.c_int(anchors.shape[1]), ctypes.c_int(minimum_valid), _p(E), _p(op), _p(on))
    return op, on


def point_to_plane(normals1, vertices1, vertices2):
    n, a, b = _f32(normals1), _f32(vertices1), _f32(vertices2)
    out = np.empty(len(a), np.float32)
    lib().orc_point_to_plane(_p(n), _p(a), _p(b), ctypes.c_int64(len(a)), _p(out))
    return out


def unproject_image(depth, K, extrinsics=None, depth_scale=1000.0, depth_max=3.0):
    """uint16 or float32 depth [H,W] -> points [H*W,3] (frame of extrinsics^-1), mask [H*W] bool."""
    depth = np.ascontiguousarray(depth)
    dtype = 1 if depth.dtype == np.uint16 else 2
    if dtype == 2:
        depth = _f32(depth)
    K = _f64(K)
    E = None if extrinsics is None else _f64(extrinsics)
    H, W = depth.shape[:2]
    pts = np.empty((H * W, 3), np.float32)
    mask = np.empty(H * W, np.uint8)
    lib().orc_unproject_image(_p(depth), ctypes.c_int(dtype), ctypes.c_int(H), ctypes.c_int(W), _p(K), _p(E), ctypes.c_float(depth_scale),
                              ctypes.c_float(depth_max), _p(pts), _p(mask))
    return pts, mask.astype(bool)


def intrinsics_to_ndc(K, H, W):
    K = _f64(K)
    ndc = np.empty(9, np.float64)
    rng = np.empty(4, np.float32)
    lib().orc_intrinsics_to_ndc(_p(K), ctypes.c_int(H), ctypes.c_int(W), _p(ndc), _p(rng))
    return ndc.reshape(3, 3), rng


def extract_face_ndc(verts, faces, K, H, W, near=0.0, far=float("inf")):
    verts, faces, K = _f32(verts), _i64(faces), _f64(K)
    F = len(faces)
    out = np.empty((F, 3, 3), np.float32)
    mask = np.empty(F, np.uint8)
    lib().orc_extract_face_ndc(_p(verts), _p(faces), ctypes.c_int64(F), _p(K), ctypes.c_int(H), ctypes.c_int(W),
                               ctypes.c_float(near), ctypes.c_float(far), _p(out), _p(mask))
    return out, mask.astype(bool)


def rasterize(face_ndc, mask, H, W, blur_radius_pixels=0.0, faces_per_pixel=8, bin_size=-1, max_faces_per_bin=-1,
              perspective_correct=False, clip_barycentric=False, cull_back_faces=True):
    face_ndc = _f32(face_ndc)
    F = len(face_ndc)
    m = None if mask is None else _u8(mask)
    Kf = faces_per_pixel
    fi = np.empty((H, W, Kf), np.int64)
    dep = np.empty((H, W, Kf), np.float32)
    bary = np.empty((H, W, Kf, 3), np.float32)
    dist = np.empty((H, W, Kf), np.float32)
    _check(lib().orc_rasterize(_p(face_ndc), _p(m), ctypes.c_int64(F), ctypes.c_int(H), ctypes.c_int(W),
                               ctypes.c_float(blur_radius_pixels), ctypes.c_int(Kf), ctypes.c_int(bin_size),
                               ctypes.c_int(max_faces_per_bin), ctypes.c_int(int(perspective_correct)),
                               ctypes.c_int(int(clip_barycentric)), ctypes.c_int(int(cull_back_faces)),
                               _p(fi), _p(dep), _p(bary), _p(dist)))
    return fi, dep, bary, dist


def rasterize_k1_fast(face_ndc, mask, H, W, blur_radius_pixels=0.0, perspective_correct=False, cull_back_faces=True):
    face_ndc = _f32(face_ndc)
    F = len(face_ndc)
    m = None if mask is None else _u8(mask)
    fi = np.empty((H, W, 1), np.int64)
    dep = np.empty((H, W, 1), np.float32)
    bary = np.empty((H, W, 1, 3), np.float32)
    dist = np.empty((H, W, 1), np.float32)
    _check(lib().orc_rasterize_k1_fast(_p(face_ndc), _p(m), ctypes.c_int64(F), ctypes.c_int(H), ctypes.c_int(W),
                                       ctypes.c_float(blur_radius_pixels), ctypes.c_int(int(perspective_correct)),
                                       ctypes.c_int(int(cull_back_faces)), _p(fi), _p(dep), _p(bary), _p(dist)))
    return fi, dep, bary, dist


def interpolate_face_attributes(pixel_faces, bary, face_attrs):
    pixel_faces, bary, face_attrs = _i64(pixel_faces), _f32(bary), _f32(face_attrs)
    H, W, Kf = pixel_faces.shape
    C = face_attrs.shape[2]
    out = np.empty((H, W, Kf, C), np.float32)
    lib().orc_interpolate_face_attributes(_p(pixel_faces), _p(bary), ctypes.c_int64(H * W), ctypes.c_int(Kf), _p(face_attrs),
                                          ctypes.c_int(C), _p(out))
    return out


def unproject(depth, K, depth_scale=1.0, depth_max=10.0):
    depth, K = _f32(depth), _f64(K)
    H, W = depth.shape[:2]
    pts = np.empty((H * W, 3), np.float32)
    mask = np.empty(H * W, np.uint8)
    lib().orc_unproject(_p(depth), ctypes.c_int(H), ctypes.c_int(W), _p(K), ctypes.c_float(depth_scale), ctypes.c_float(depth_max),
                        _p(pts), _p(mask))
    return pts, mask.astype(bool)


def warped_surface_jacobians(points, normals, nodes, rotations, anchors, weights):
    points, normals, nodes, rotations, anchors, weights = _f32(points), _f32(normals), _f32(nodes), _f32(rotations), _i32(anchors), _f32(weights)
    V, K = anchors.shape
    vj = np.empty((V, K, 4), np.float32)
    nj = np.empty((V, K, 3), np.float32)
    lib().orc_warped_surface_jacobians(_p(points), _p(normals), ctypes.c_int64(V), _p(nodes), _p(rotations), _p(anchors), _p(weights),
                                       ctypes.c_int(K), _p(vj), _p(nj))
    return vj, nj


def rasterized_surface_jacobians(verts, normals, faces, pixel_faces, pixel_bary, K, perspective_correct=True):
    verts, normals, faces, pixel_faces, pixel_bary, K = _f32(verts), _f32(normals), _i64(faces), _i64(pixel_faces), _f32(pixel_bary), _f64(K)
    H, W, Kf = pixel_faces.shape
    vj = np.empty((H, W, 3, 9), np.float32)
    nj = np.empty((H, W, 3, 10), np.float32)
    lib().orc_rasterized_surface_jacobians(_p(verts), _p(normals), _p(faces), _p(pixel_faces), _p(pixel_bary), ctypes.c_int(H),
                                           ctypes.c_int(W), ctypes.c_int(Kf), _p(K), ctypes.c_int(int(perspective_correct)), _p(vj), _p(nj))
    return vj, nj


def associate_faces_with_anchors(faces, anchors):
    faces, anchors = _i64(faces), _i32(anchors)
    F, K = len(faces), anchors.shape[1]
    nodes = np.empty((F, 3 * K), np.int32)
    slots = np.empty((F, 3 * K, 3), np.int32)
    counts = np.empty(F, np.int32)
    lib().orc_associate_faces_with_anchors(_p(faces), ctypes.c_int64(F), _p(anchors), ctypes.c_int(K), _p(nodes), _p(slots), _p(counts))
    return nodes, slots, counts


def pixel_vertex_anchor_jacobians(rast_vj, rast_nj, warped_vj, warped_nj, point_map_vectors, rasterized_normals, residual_mask,
                                  pixel_faces, faces, face_nodes, face_slots, face_counts, use_tukey=False, tukey_cutoff=0.01, mode="ALL"):
    m = MODE[mode]
    rast_vj, rast_nj, warped_vj = _f32(rast_vj), _f32(rast_nj), _f32(warped_vj)
    warped_nj = _f32(warped_nj) if warped_nj is not None else np.zeros(1, np.float32)
    pmv, rn, rm = _f32(point_map_vectors), _f32(rasterized_normals), _u8(residual_mask)
    pixel_faces, faces = _i64(pixel_faces), _i64(faces)
    face_nodes, face_slots, face_counts = _i32(face_nodes), _i32(face_slots), _i32(face_counts)
    P = rm.size
    K = face_nodes.shape[1] // 3
    Kf = pixel_faces.shape[-1]
    s = 6 if m == 0 else 3
    pj = np.empty((P, 3 * K, s), np.float32)
    pc = np.empty(P, np.int32)
    lib().orc_pixel_vertex_anchor_jacobians(_p(rast_vj), _p(rast_nj), _p(warped_vj), _p(warped_nj), ctypes.c_int(K), _p(pmv), _p(rn), _p(rm),
                                            _p(pixel_faces), ctypes.c_int(Kf), _p(faces), _p(face_nodes), _p(face_slots), _p(face_counts),
                                            ctypes.c_int64(P), ctypes.c_int(int(use_tukey)), ctypes.c_float(tukey_cutoff), ctypes.c_int(m),
                                            _p(pj), _p(pc))
    return pj, pc


def data_hessian_gradient(pixel_jacobians, pixel_counts, pixel_faces, face_nodes, residuals, residual_mask, node_count, mode="ALL"):
    m = MODE[mode]
    s = 6 if m == 0 else 3
    pj, pc, pf, fn = _f32(pixel_jacobians), _i32(pixel_counts), _i64(pixel_faces), _i32(face_nodes)
    r, rm = _f32(residuals), _u8(residual_mask)
    P = rm.size
    K = fn.shape[1] // 3
    Kf = pf.shape[-1]
    H = np.empty((node_count, s, s), np.float32)
    g = np.empty(node_count * s, np.float32)
    lib().orc_data_hessian_gradient(_p(pj), _p(pc), _p(pf), ctypes.c_int(Kf), _p(fn), ctypes.c_int(K), _p(r), _p(rm), ctypes.c_int64(P),
                                    ctypes.c_int(node_count), ctypes.c_int(m), _p(H), _p(g))
    return H, g


def arap_residuals(edges, edge_layers, radii, node_weights, nodes, rotations, translations, weight, use_huber=False, huber=1e-4):
    edges = _i32(edges)
    E = len(edges)
    out = np.empty(E * 3, np.float32)
    el = None if edge_layers is None else np.ascontiguousarray(edge_layers, np.int8)
    rd = None if radii is None else _f32(radii)
    nw = None if node_weights is None else _f32(node_weights)
    nodes, rotations, translations = _f32(nodes), _f32(rotations), _f32(translations)
    _check(lib().orc_arap_residuals(_p(edges), ctypes.c_int(E), _p(el), _p(rd), _p(nw), _p(nodes), _p(rotations),
                                    _p(translations), ctypes.c_float(weight), ctypes.c_int(int(use_huber)), ctypes.c_float(huber),
                                    _p(out)))
    return out


def arap_edge_jacobians(edges, edge_layers, radii, node_weights, nodes, rotations, weight):
    edges = _i32(edges)
    E = len(edges)
    out = np.empty((E, 5), np.float32)
    el = None if edge_layers is None else np.ascontiguousarray(edge_layers, np.int8)
    rd = None if radii is None else _f32(radii)
    nw = None if node_weights is None else _f32(node_weights)
    nodes, rotations = _f32(nodes), _f32(rotations)
    lib().orc_arap_edge_jacobians(_p(edges), ctypes.c_int(E), _p(el), _p(rd), _p(nw), _p(nodes), _p(rotations),
                                  ctypes.c_float(weight), _p(out))
    return out


def arap_hessian(edges, edge_jacobians, node_count):
    edges, ej = _i32(edges), _f32(edge_jacobians)
    E = len(edges)
    diag = np.empty((node_count, 6, 6), np.float32)
    wing = np.empty((E, 6, 6), np.float32)
    lib().orc_arap_hessian(_p(edges), ctypes.c_int(E), _p(ej), ctypes.c_int(node_count), _p(diag), _p(wing))
    return diag, wing


def arap_gradient(edges, edge_jacobians, residuals, g):
    g = _f32(g).copy()
    edges, edge_jacobians, residuals = _i32(edges), _f32(edge_jacobians), _f32(residuals)
    lib().orc_arap_gradient(_p(edges), ctypes.c_int(len(edges)), _p(edge_jacobians), _p(residuals), _p(g))
    return g


def invert_psd_blocks(blocks):
    """InvertPositiveSemidefiniteBlocks (InvertBlocks.cpp:82-126) -> (inverses, rc: 0 or 1 + failing block)."""
    blocks = _f32(blocks)
    N, s = blocks.shape[0], blocks.shape[1]
    out = np.full((N, s, s), np.nan, np.float32)
    rc = lib().orc_invert_psd_blocks(_p(blocks), ctypes.c_int(N), ctypes.c_int(s), _p(out))
    return out, rc


def _i16(a):
    return np.ascontiguousarray(a, dtype=np.int16)


def matmul_block_sparse_row_wise(a_blocks, b_blocks, b_coordinates):
    """MatmulBlockSparseRowWisePadded (MatmulBlockSparseImpl.h:39-157) -> (blocks [count, s, s], mask [count] bool, rc)."""
    a, b, c = _f32(a_blocks), _f32(b_blocks), _i32(b_coordinates)
    out = np.zeros_like(b)
    mask = np.zeros(b.shape[0], np.uint8)
    rc = lib().orc_matmul_block_sparse_row_wise(_p(a), ctypes.c_int(a.shape[0]), _p(b), _p(c), ctypes.c_int(b.shape[0]),
                                                ctypes.c_int(b.shape[1]), _p(out), _p(mask))
    return out, mask.astype(bool), rc


def matmul_block_sparse(a_blocks, a_breadboard, transpose_a, b_blocks, b_breadboard, transpose_b):
    """MatmulBlockSparse (MatmulBlockSparseImpl.h:160-391) -> (dense output blocks [out_rows*out_cols, s, s], mask, rc)."""
    a, b, ab, bb = _f32(a_blocks), _f32(b_blocks), _i16(a_breadboard), _i16(b_breadboard)
    s = a.shape[1]
    out_rows = ab.shape[1] if transpose_a else ab.shape[0]
    out_cols = bb.shape[0] if transpose_b else bb.shape[1]
    out = np.zeros((out_rows * out_cols, s, s), np.float32)
    mask = np.zeros(out_rows * out_cols, np.uint8)
    rc = lib().orc_matmul_block_sparse(_p(a), ctypes.c_int(a.shape[0]), _p(ab), ctypes.c_int(ab.shape[0]), ctypes.c_int(ab.shape[1]),
                                       ctypes.c_int(int(transpose_a)), _p(b), ctypes.c_int(b.shape[0]), _p(bb), ctypes.c_int(bb.shape[0]),
                                       ctypes.c_int(bb.shape[1]), ctypes.c_int(int(transpose_b)), ctypes.c_int(s), _p(out), _p(mask))
    return out, mask.astype(bool), rc


def block_sparse_and_vector_product(blocks, m, coordinates, offset, transpose, vector):
    """BlockSparseAndVectorProduct (MatmulBlockSparseImpl.h:441-602) -> (out [m], rc)."""
    bl, c, v = _f32(blocks), _i32(coordinates), _f32(vector).reshape(-1)
    out = np.zeros(m, np.float32)
    rc = lib().orc_block_sparse_vector(_p(bl), _p(c), ctypes.c_int(bl.shape[0]), ctypes.c_int(bl.shape[1]), ctypes.c_int(offset[0]),
                                       ctypes.c_int(offset[1]), ctypes.c_int(int(transpose)), _p(v), ctypes.c_int64(v.shape[0]), _p(out),
                                       ctypes.c_int64(m))
    return out, rc


def diagonal_block_sparse_and_vector_product(blocks, vector):
    """DiagonalBlockSparseAndVectorProduct (MatmulBlockSparseImpl.h:604-690)."""
    bl, v = _f32(blocks), _f32(vector).reshape(-1)
    out = np.zeros(bl.shape[0] * bl.shape[1], np.float32)
    lib().orc_diagonal_block_vector(_p(bl), ctypes.c_int(bl.shape[0]), ctypes.c_int(bl.shape[1]), _p(v), _p(out))
    return out


def sparse_blocks_op(matrix, blocks, coordinates, offset=(0, 0), transpose=False, op=0):
    """Fill (0) / Add (1) / SubtractSparseBlocks (2) (SparseBlocksImpl.h:30-190), in place; coordinates None = diagonal."""
    bl = _f32(blocks)
    c = None if coordinates is None else _i32(coordinates)
    assert matrix.dtype == np.float32 and matrix.flags.c_contiguous
    return lib().orc_sparse_blocks_op(_p(matrix), ctypes.c_int64(matrix.shape[0]), ctypes.c_int64(matrix.shape[1]), _p(bl), _p(c),
                                      ctypes.c_int(bl.shape[0]), ctypes.c_int(bl.shape[1]), ctypes.c_int64(offset[0]),
                                      ctypes.c_int64(offset[1]), ctypes.c_int(int(transpose)), ctypes.c_int(op))


def get_sparse_blocks(matrix, block_size, coordinates=None, count=None):
    """GetSparseBlocks / GetDiagonalBlocks (SparseBlocksImpl.h:192-230) -> (blocks, rc)."""
    mat = _f32(matrix)
    c = None if coordinates is None else _i32(coordinates)
    n = c.shape[0] if c is not None else (count if count is not None else mat.shape[0] // block_size)
    out = np.zeros((n, block_size, block_size), np.float32)
    rc = lib().orc_get_sparse_blocks(_p(mat), ctypes.c_int64(mat.shape[0]), ctypes.c_int64(mat.shape[1]), ctypes.c_int(block_size), _p(c),
                                     ctypes.c_int(n), _p(out))
    return out, rc


def invert_triangular_blocks(blocks, upper):
    """InvertTriangularBlocks (InvertBlocksCPU.cpp, trtri per block) -> (inverses, rc: 1 on a zero diagonal)."""
    bl = _f32(blocks)
    out = np.zeros_like(bl)
    rc = lib().orc_invert_triangular_blocks(_p(bl), ctypes.c_int(bl.shape[0]), ctypes.c_int(bl.shape[1]), ctypes.c_int(int(upper)), _p(out))
    return out, rc


def solve_block_diagonal(H, g, lm=0.0):
    H, g = _f32(H), _f32(g)
    N, s = H.shape[0], H.shape[1]
    x = np.empty(N * s, np.float32)
    rc = lib().orc_solve_block_diagonal(_p(H), _p(g), ctypes.c_int(N), ctypes.c_int(s), ctypes.c_float(lm), _p(x))
    return x, rc


def solve_arrowhead(diag, wing, edges, n0, g):
    diag, wing, edges, g = _f32(diag), _f32(wing), _i32(edges), _f32(g)
    N = diag.shape[0]
    x = np.empty(N * 6, np.float32)
    _check(lib().orc_solve_arrowhead(_p(diag), _p(wing), _p(edges), ctypes.c_int(len(edges)), ctypes.c_int(N), ctypes.c_int(n0), _p(g), _p(x)))
    return x


# ---- normals (cpp/geometry/functional/kernel/NormalsOperationsImpl.h) : float32 numpy, one IEEE op at a time ----
def _normalize_eigen(v):
    """Eigen normalize(): divide by sqrt of the squared norm when positive (zero rows stay zero)."""
    v = np.asarray(v, np.float32)
    n2 = (v[:, 0] * v[:, 0] + v[:, 1] * v[:, 1]) + v[:, 2] * v[:, 2]
    out = v.copy()
    pos = n2 > 0
    n = np.sqrt(n2[pos])
    out[pos] = v[pos] / n[:, None]
    return out


def triangle_normals(verts, faces, normalized=True):
    """ComputeTriangleNormals (:39-68) (+ NormalizeVectors3d :75-93: NaN -> (0, 0, 1))."""
    v = np.asarray(verts, np.float32)
    f = np.asarray(faces, np.int64)
    a = v[f[:, 1]] - v[f[:, 0]]
    b = v[f[:, 2]] - v[f[:, 0]]
    n = np.stack([a[:, 1] * b[:, 2] - a[:, 2] * b[:, 1], a[:, 2] * b[:, 0] - a[:, 0] * b[:, 2], a[:, 0] * b[:, 1] - a[:, 1] * b[:, 0]], 1)
    if normalized:
        n = _normalize_eigen(n)
        n[np.isnan(n[:, 0])] = (0.0, 0.0, 1.0)
    return n.astype(np.float32)


def vertex_normals(verts, faces, normalized=True):
    """ComputeVertexNormals (:95-166): unnormalized triangle normals added per vertex in ascending face order (the
    reference's serial order), optionally normalized."""
    v = np.asarray(verts, np.float32)
    f = np.asarray(faces, np.int64)
    tn = triangle_normals(v, f, normalized=False)
    out = np.zeros((len(v), 3), np.float32)
    np.add.at(out, f.reshape(-1), np.repeat(tn, 3, axis=0))
    if normalized:
        out = _normalize_eigen(out)
        out[np.isnan(out[:, 0])] = (0.0, 0.0, 1.0)
    return out


def ordered_point_cloud_normals(points, H, W):
    """ComputeOrderedPointCloudNormals (:170-214): normalize((right - left) x (top - bottom)), flipped so n.z <= 0,
    zero on the image border."""
    p = np.asarray(points, np.float32).reshape(H, W, 3)
    out = np.zeros((H, W, 3), np.float32)
    dh = p[1:-1, 2:] - p[1:-1, :-2]
    dv = p[:-2, 1:-1] - p[2:, 1:-1]
    n = np.stack([dh[..., 1] * dv[..., 2] - dh[..., 2] * dv[..., 1], dh[..., 2] * dv[..., 0] - dh[..., 0] * dv[..., 2],
                  dh[..., 0] * dv[..., 1] - dh[..., 1] * dv[..., 0]], -1).reshape(-1, 3)
    n = _normalize_eigen(n)
    flip = n[:, 2] > 0
    n[flip] = -n[flip]
    out[1:-1, 1:-1] = n.reshape(H - 2, W - 2, 3)
    return out.reshape(-1, 3)


def rodrigues(w):
    w = _f32(w).reshape(-1, 3)
    R = np.empty((len(w), 3, 3), np.float32)
    lib().orc_rodrigues(_p(w), ctypes.c_int(len(w)), _p(R))
    return R


class _Params(ctypes.Structure):
    _fields_ = [("max_iterations", ctypes.c_int), ("mode_count", ctypes.c_int), ("modes", ctypes.c_int * 16),
                ("use_perspective_correction", ctypes.c_int), ("max_depth", ctypes.c_float), ("use_tukey", ctypes.c_int),
                ("tukey_cutoff", ctypes.c_float), ("lm_factor", ctypes.c_float), ("arap_weight", ctypes.c_float),
                ("use_huber", ctypes.c_int), ("huber_delta", ctypes.c_float), ("ndc_consistent", ctypes.c_int)]


class _WarpField(ctypes.Structure):
    _fields_ = [("N", ctypes.c_int), ("K", ctypes.c_int), ("coverage", ctypes.c_float), ("coverage_method", ctypes.c_int),
                ("min_valid_anchors", ctypes.c_int), ("nodes", ctypes.c_void_p), ("rotations", ctypes.c_void_p),
                ("translations", ctypes.c_void_p), ("node_weights", ctypes.c_void_p), ("E", ctypes.c_int), ("edges", ctypes.c_void_p),
                ("edge_layers", ctypes.c_void_p), ("radii", ctypes.c_void_p), ("first_layer_count", ctypes.c_int)]


class _Outputs(ctypes.Structure):
    _fields_ = [("residuals", ctypes.c_void_p), ("residual_mask", ctypes.c_void_p), ("pixel_faces", ctypes.c_void_p),
                ("updates", ctypes.c_void_p), ("gradient", ctypes.c_void_p), ("hessian_diag", ctypes.c_void_p),
                ("stage_seconds", ctypes.c_void_p)]


def fit(*, nodes, rotations, translations, mesh_points, mesh_normals, faces, ref_points, ref_mask, H, W, K, extrinsics=None,
        max_iterations=1, modes=("ALL",), use_perspective_correction=True, max_depth=10.0, use_tukey=False, tukey_cutoff=0.01,
        lm_factor=0.0, arap_weight=200.0, use_huber=False, huber_delta=1e-4, anchor_count=4, coverage=0.05, coverage_method=0,
        node_weights=None, min_valid_anchors=0, edges=None, edge_layers=None, radii=None, first_layer_count=None, fast_raster=True,
        ndc_consistent=False, raise_on_failure=True):
    """Full FitToImage on the CPU restatement (virtual node order). Returns (R, t, diagnostics of the last iteration).
    raise_on_failure=False: a block-diagonal potrf failure (the reference's NNRT_LAPACK_CHECK exception) returns the
    failing iteration's diagnostics (NaN updates on the failed blocks) with diag["status"] = the oracle error code."""
    nodes = _f32(nodes)
    R = _f32(rotations).copy()
    t = _f32(translations).copy()
    N = len(nodes)
    prm = _Params()
    prm.max_iterations = max_iterations
    prm.mode_count = len(modes)
    for i, m in enumerate(modes):
        prm.modes[i] = MODE[m]
    prm.use_perspective_correction = int(use_perspective_correction)
    prm.max_depth = max_depth
    prm.use_tukey = int(use_tukey)
    prm.tukey_cutoff = tukey_cutoff
    prm.lm_factor = lm_factor
    prm.arap_weight = arap_weight
    prm.use_huber = int(use_huber)
    prm.huber_delta = huber_delta
    prm.ndc_consistent = int(ndc_consistent)
    keep = []

    def ptr(a):
        keep.append(a)
        return a.ctypes.data

    wf = _WarpField()
    wf.N, wf.K, wf.coverage, wf.coverage_method, wf.min_valid_anchors = N, anchor_count, coverage, coverage_method, min_valid_anchors
    wf.nodes, wf.rotations, wf.translations = ptr(nodes), ptr(R), ptr(t)
    wf.node_weights = ptr(_f32(node_weights)) if node_weights is not None else None
    if edges is not None and len(edges) > 0:
        wf.E = len(edges)
        wf.edges = ptr(_i32(edges))
        wf.edge_layers = ptr(np.ascontiguousarray(edge_layers, np.int8))
        wf.radii = ptr(_f32(radii))
        wf.first_layer_count = first_layer_count
    else:
        wf.E = 0
    P = H * W
    s = 6 if modes[(max_iterations - 1) % len(modes)] == "ALL" else 3
    diag = dict(residuals=np.zeros(P, np.float32), residual_mask=np.zeros(P, np.uint8), pixel_faces=np.zeros(P, np.int64),
                updates=np.zeros(N * s, np.float32), gradient=np.zeros(N * s, np.float32), hessian_diag=np.zeros(N * s * s, np.float32),
                stage_seconds=np.zeros(8, np.float64))
    outs = _Outputs(*[ptr(diag[k]) for k in ("residuals", "residual_mask", "pixel_faces", "updates", "gradient", "hessian_diag",
                                               "stage_seconds")])
    E = None if extrinsics is None else ptr(_f64(extrinsics))
    rc = lib().orc_fit(ctypes.byref(prm), ctypes.byref(wf), ctypes.c_void_p(ptr(_f32(mesh_points))),
                       ctypes.c_void_p(ptr(_f32(mesh_normals))), ctypes.c_int64(len(mesh_points)),
                       ctypes.c_void_p(ptr(_i64(faces))), ctypes.c_int64(len(faces)), ctypes.c_void_p(ptr(_f32(ref_points))),
                       ctypes.c_void_p(ptr(_u8(ref_mask))), ctypes.c_int(H), ctypes.c_int(W),
                       ctypes.c_void_p(ptr(_f64(K))), ctypes.c_void_p(E), ctypes.c_int(int(fast_raster)), ctypes.byref(outs))
    if raise_on_failure or rc != 30:
        _check(rc)
    diag["status"] = rc
    diag["residual_mask"] = diag["residual_mask"].astype(bool)
    return R, t, diag


# ---------------------------------------------------------------------------------------------------------------------
# TSDF voxel block grid restatement (tsdf_oracle.cpp)
# ---------------------------------------------------------------------------------------------------------------------
DT = {"none": -1, "float32": 0, "uint16": 1, "uint8": 2}


def _depth_arg(depth):
    d = np.ascontiguousarray(depth)
    if d.dtype == np.uint16:
        return d, 1
    return np.ascontiguousarray(d, dtype=np.float32), 0


class OracleGrid:
    """CPU restatement of NonRigidSurfaceVoxelBlockGrid (test infrastructure only)."""

    def __init__(self, voxel_size, block_resolution, weight_dtype="float32", color_dtype="none"):
        L = lib()
        L.orc_grid_create.restype = ctypes.c_void_p
        L.orc_grid_create.argtypes = [ctypes.c_float, ctypes.c_int, ctypes.c_int, ctypes.c_int]
        for name in ("orc_grid_block_count", "orc_grid_touch", "orc_grid_values_at", "orc_grid_inactive_neighbors"):
            getattr(L, name).restype = ctypes.c_int64
        self.h = ctypes.c_void_p(L.orc_grid_create(float(voxel_size), int(block_resolution), DT[weight_dtype], DT[color_dtype]))
        self.res = int(block_resolution)
        self.voxel = float(voxel_size)
        self.color = color_dtype != "none"

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_grid_destroy(self.h)

    def block_count(self):
        return lib().orc_grid_block_count(self.h)

    def block_coords(self):
        out = np.zeros((self.block_count(), 3), np.int32)
        lib().orc_grid_block_coords(self.h, _p(out))
        return out

    def activate(self, coords):
        c = _i32(coords).reshape(-1, 3)
        lib().orc_grid_activate(self.h, _p(c), ctypes.c_int64(len(c)))

    def touch(self, depth, K, E, scale, dmax, trunc_mult):
        d, dt = _depth_arg(depth)
        cap = (d.shape[0] // 4) * (d.shape[1] // 4) * 4 + 1
        out = np.zeros((cap, 3), np.int32)
        n = lib().orc_grid_touch(self.h, _p(d), dt, d.shape[0], d.shape[1], _p(_f64(K)), _p(None if E is None else _f64(E)),
                                 ctypes.c_float(scale), ctypes.c_float(dmax), ctypes.c_float(trunc_mult), _p(out), ctypes.c_int64(cap))
        return out[:n]

    def integrate(self, coords, depth, color, Kd, Kc, E, scale, dmax, trunc_mult):
        c = _i32(coords).reshape(-1, 3)
        d, dt = _depth_arg(depth)
        col = None if color is None else np.ascontiguousarray(color, dtype=np.uint8 if dt == 1 else np.float32)
        Hc, Wc = (0, 0) if col is None else col.shape[:2]
        lib().orc_grid_integrate(self.h, _p(c), ctypes.c_int64(len(c)), _p(d), dt, d.shape[0], d.shape[1], _p(col), Hc, Wc, _p(_f64(Kd)),
                                 _p(_f64(Kc)), _p(None if E is None else _f64(E)), ctypes.c_float(scale), ctypes.c_float(dmax),
                                 ctypes.c_float(trunc_mult))

    def integrate_non_rigid(self, coords, nodes, R, t, coverage, K, min_valid, depth, color, normals, Kd, Kc, E, scale, dmax, trunc_mult,
                            node_coverage_sq=None, apply_oblique_test=True):
        c = _i32(coords).reshape(-1, 3)
        d, dt = _depth_arg(depth)
        col = None if color is None else np.ascontiguousarray(color, dtype=np.uint8 if dt == 1 else np.float32)
        Hc, Wc = (0, 0) if col is None else col.shape[:2]
        cos = np.zeros(d.shape[:2], np.float32)
        nodes, R, t, nrm = _f32(nodes), _f32(R), _f32(t), _f32(normals)
        c2 = None if node_coverage_sq is None else _f32(node_coverage_sq)
        lib().orc_grid_integrate_non_rigid(self.h, _p(c), ctypes.c_int64(len(c)), _p(nodes), _p(R), _p(t), _p(c2), len(nodes),
                                           ctypes.c_float(coverage), int(K), int(min_valid), _p(d), dt, d.shape[0], d.shape[1], _p(col), Hc,
                                           Wc, _p(nrm), _p(_f64(Kd)), _p(_f64(Kc)), _p(None if E is None else _f64(E)), ctypes.c_float(scale),
                                           ctypes.c_float(dmax), ctypes.c_float(trunc_mult), _p(cos), int(bool(apply_oblique_test)))
        return cos

    def channels(self):
        return 8 if self.color else 5

    def values_at(self, query):
        q = _i32(query).reshape(-1, 3)
        out = np.zeros((len(q), self.channels()), np.float32)
        n = lib().orc_grid_values_at(self.h, _p(q), ctypes.c_int64(len(q)), _p(out))
        return out[:n]

    def values_all(self):
        out = np.zeros((self.block_count() * self.res ** 3, self.channels()), np.float32)
        lib().orc_grid_values_all(self.h, _p(out))
        return out

    def inactive_neighbors(self):
        cap = 27 * self.block_count() + 1
        out = np.zeros((cap, 3), np.int32)
        n = lib().orc_grid_inactive_neighbors(self.h, _p(out), ctypes.c_int64(cap))
        return out[:n]

    def mesh(self, weight_threshold):
        nv, nt = ctypes.c_int64(), ctypes.c_int64()
        z = np.zeros((1, 3), np.float32)
        lib().orc_grid_mesh(self.h, ctypes.c_float(weight_threshold), _p(z), _p(z), _p(z), _p(np.zeros((1, 3), np.int64)), ctypes.c_int64(0),
                            ctypes.c_int64(0), ctypes.byref(nv), ctypes.byref(nt))
        V = np.zeros((max(nv.value, 1), 3), np.float32)
        Nn = np.zeros_like(V)
        C = np.zeros_like(V)
        T = np.zeros((max(nt.value, 1), 3), np.int64)
        lib().orc_grid_mesh(self.h, ctypes.c_float(weight_threshold), _p(V), _p(Nn), _p(C), _p(T), ctypes.c_int64(nv.value),
                            ctypes.c_int64(nt.value), ctypes.byref(nv), ctypes.byref(nt))
        return V[:nv.value], Nn[:nv.value], C[:nv.value], T[:nt.value]

    def find_blocks_intersecting_truncation_region(self, depth, nodes, R, t, coverage, K, min_valid, Kd, E, scale, dmax, trunc_mult):
        cand = self.inactive_neighbors()
        boxes = warped_block_boxes(cand, self.res * self.voxel, nodes, R, t, coverage, K, min_valid, E)
        mask = boxes_mask(boxes, depth, Kd, scale, dmax, 4, self.voxel * trunc_mult)
        return cand[mask.astype(bool)]


def warped_block_boxes(keys, side, nodes, R, t, coverage, K, min_valid, E):
    k = _i32(keys).reshape(-1, 3)
    nodes, R, t = _f32(nodes), _f32(R), _f32(t)
    out = np.zeros((len(k), 6), np.float32)
    lib().orc_warped_block_boxes(_p(k), ctypes.c_int64(len(k)), ctypes.c_float(side), _p(nodes), _p(R), _p(t), len(nodes),
                                 ctypes.c_float(coverage), int(K), int(min_valid), _p(None if E is None else _f64(E)), _p(out))
    return out


def boxes_mask(boxes, depth, K, scale, dmax, stride, trunc):
    b = _f32(boxes).reshape(-1, 6)
    d, dt = _depth_arg(depth)
    out = np.zeros(len(b), np.uint8)
    lib().orc_boxes_mask(_p(b), ctypes.c_int64(len(b)), _p(d), dt, d.shape[0], d.shape[1], _p(_f64(K)), ctypes.c_float(scale),
                         ctypes.c_float(dmax), int(stride), ctypes.c_float(trunc), _p(out))
    return out


def marching_cubes_table():
    """The oracle's marching-cubes table in emission order: tri [256, 16] int8 edge triples, -1 terminated."""
    tri = np.full((256, 16), -1, np.int8)
    _check(lib().orc_marching_cubes_table(_p(tri)))
    return tri


def backproject_depth(depth, fx, fy, cx, cy, normalizer=1.0):
    """image_proc.cpp:275-302 (uint16, depth = d / normalizer) and :312-339 (float32, normalizer 1) in float32 numpy: each
    operation is one correctly rounded IEEE op, in the reference's order ((depth * (x - cx)) / fx), so the GPU kernel is
    compared bit for bit. Pixels with depth <= 0 are (0, 0, 0)."""
    d = np.asarray(depth)
    H, W = d.shape
    f32 = np.float32
    dm = d.astype(f32) / f32(normalizer) if d.dtype == np.uint16 else d.astype(f32)
    xs = np.arange(W, dtype=f32)[None, :] - f32(cx)
    ys = np.arange(H, dtype=f32)[:, None] - f32(cy)
    out = np.zeros((H, W, 3), f32)
    valid = dm > 0
    out[..., 0] = np.where(valid, (dm * xs) / f32(fx), f32(0))
    out[..., 1] = np.where(valid, (dm * ys) / f32(fy), f32(0))
    out[..., 2] = np.where(valid, dm, f32(0))
    return out
