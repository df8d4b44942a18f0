"""nnrt.rendering mirror (cpp/pybind/rendering/rendering.cpp:36-43, functional/functional.cpp:36-62)."""
from __future__ import annotations

import ctypes
import types

import numpy as np
import torch

from .. import _native as N
from ._overloads import Overloaded
from ._tensors import to_device, to_host_f64


def _dev():
    return torch.device("cuda", N.current_device())


def rasterize_ndc_triangles(ndc_face_vertices, clipped_faces_mask, image_size, blur_radius_pixels=0.0, faces_per_pixel=8, bin_size=-1,
                            max_faces_per_bin=-1, perspective_correct_barycentric_coordinates=False, clip_barycentric_coordinates=False,
                            cull_back_faces=True):
    """Returns (pixel_face_indices [H,W,K] int64, depths [H,W,K], barycentrics [H,W,K,3], signed distances [H,W,K])."""
    dev = _dev()
    H, W = int(image_size[0]), int(image_size[1])
    f = to_device(ndc_face_vertices, torch.float32, dev).reshape(-1, 3, 3)
    m = None if clipped_faces_mask is None else to_device(clipped_faces_mask, torch.uint8, dev)
    K = int(faces_per_pixel)
    fi = torch.empty((H, W, K), dtype=torch.int64, device=dev)
    dep = torch.empty((H, W, K), dtype=torch.float32, device=dev)
    bary = torch.empty((H, W, K, 3), dtype=torch.float32, device=dev)
    dist = torch.empty((H, W, K), dtype=torch.float32, device=dev)
    N.check(N.lib().nnrt_rasterize_ndc_triangles(N.ptr(f), N.ptr(m), f.shape[0], H, W, float(blur_radius_pixels), K, int(bin_size),
                                                 int(max_faces_per_bin), int(perspective_correct_barycentric_coordinates),
                                                 int(clip_barycentric_coordinates), int(cull_back_faces), N.ptr(fi), N.ptr(dep), N.ptr(bary),
                                                 N.ptr(dist), N.stream_ptr()))
    return fi, dep, bary, dist


def _check_clipping(image_size, near_clipping_distance, far_clipping_distance):
    """CheckClippingRangeAndImageSize (cpp/rendering/functional/ExtractFaceVertices.cpp:41-54)."""
    if near_clipping_distance < 0.0:
        raise RuntimeError(f"near_clipping_distance cannot be less than 0.0. Got {near_clipping_distance}.")
    if near_clipping_distance > far_clipping_distance:
        raise RuntimeError("near_clipping_distance cannot be greater than far_clipping_distance. Got "
                           f"{near_clipping_distance} and {far_clipping_distance}, respectively.")
    if len(image_size) != 2:
        raise RuntimeError(f"image_size should be a SizeVector of size 2. Got size {len(image_size)}.")


def _mesh_arrays(mesh, dev):
    if mesh.triangle_indices is None or mesh.vertex_positions is None:
        raise RuntimeError("Argument mesh needs to have both triangle vertex indices and vertex positions.")
    return to_device(mesh.vertex_positions, torch.float32, dev).reshape(-1, 3), to_device(mesh.triangle_indices, torch.int64, dev).reshape(-1, 3)


get_mesh_ndc_face_vertices_and_clip_mask = Overloaded(
    "get_mesh_ndc_face_vertices_and_clip_mask",
    "GetMeshNdcFaceVerticesAndClipMask, both overloads (cpp/pybind/rendering/functional/functional.cpp:36-54 -> ExtractFaceVertices.cpp:56-126): "
    "face vertices in NDC x, y + camera z [F,3,3] and the clip mask [F] (True = keep); a list of meshes is concatenated in mesh order and "
    "also returns the per-mesh face counts.")


@get_mesh_ndc_face_vertices_and_clip_mask.overload(lambda a: isinstance(a["camera_space_meshes"], (list, tuple)))
def _ndc_meshes(camera_space_meshes, intrinsic_matrix, image_size, near_clipping_distance=0.0, far_clipping_distance=float("inf")):
    _check_clipping(image_size, near_clipping_distance, far_clipping_distance)
    dev = _dev()
    arrays = [_mesh_arrays(m, dev) for m in camera_space_meshes]
    counts = np.array([f.shape[0] for _, f in arrays], np.int64)
    total = int(counts.sum())
    K = to_host_f64(intrinsic_matrix)
    H, W = int(image_size[0]), int(image_size[1])
    out = torch.empty((total, 3, 3), dtype=torch.float32, device=dev)
    mask = torch.empty(total, dtype=torch.uint8, device=dev)
    vptr = (ctypes.c_void_p * max(len(arrays), 1))(*[v.data_ptr() for v, _ in arrays])
    fptr = (ctypes.c_void_p * max(len(arrays), 1))(*[f.data_ptr() for _, f in arrays])
    N.check(N.lib().nnrt_get_meshes_ndc_face_vertices_and_clip_mask(vptr, fptr, N.ptr(counts), len(arrays), N.ptr(K), H, W,
                                                                    float(near_clipping_distance), float(far_clipping_distance), N.ptr(out),
                                                                    N.ptr(mask), N.stream_ptr()))
    return out, mask.bool(), torch.from_numpy(counts)


@get_mesh_ndc_face_vertices_and_clip_mask.overload()
def _ndc_mesh(camera_space_mesh, intrinsic_matrix, image_size, near_clipping_distance=0.0, far_clipping_distance=float("inf")):
    _check_clipping(image_size, near_clipping_distance, far_clipping_distance)
    dev = _dev()
    p, f = _mesh_arrays(camera_space_mesh, dev)
    K = to_host_f64(intrinsic_matrix)
    H, W = int(image_size[0]), int(image_size[1])
    out = torch.empty((f.shape[0], 3, 3), dtype=torch.float32, device=dev)
    mask = torch.empty(f.shape[0], dtype=torch.uint8, device=dev)
    N.check(N.lib().nnrt_get_mesh_ndc_face_vertices_and_clip_mask(N.ptr(p), N.ptr(f), f.shape[0], N.ptr(K), H, W, float(near_clipping_distance),
                                                                  float(far_clipping_distance), N.ptr(out), N.ptr(mask), N.stream_ptr()))
    return out, mask.bool()


def interpolate_vertex_attributes(pixel_face_indices, barycentric_coordinates, face_vertex_attributes):
    dev = _dev()
    pf = to_device(pixel_face_indices, torch.int64, dev)
    b = to_device(barycentric_coordinates, torch.float32, dev)
    a = to_device(face_vertex_attributes, torch.float32, dev)
    H, W, K = pf.shape
    C = a.shape[2]
    out = torch.empty((H, W, K, C), dtype=torch.float32, device=dev)
    N.check(N.lib().nnrt_interpolate_face_attributes(N.ptr(pf), N.ptr(b), H * W, K, N.ptr(a), C, N.ptr(out), N.stream_ptr()))
    return out


functional = types.SimpleNamespace(get_mesh_ndc_face_vertices_and_clip_mask=get_mesh_ndc_face_vertices_and_clip_mask,
                                   interpolate_vertex_attributes=interpolate_vertex_attributes)
