"""nnrt.rendering mirror (cpp/pybind/rendering/rendering.cpp:36-43, functional/functional.cpp:36-62)."""
from __future__ import annotations

import types

import torch

from .. import _native as N
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


def get_mesh_ndc_face_vertices_and_clip_mask(mesh, intrinsic_matrix, image_size, near_clipping_distance=0.0,
                                             far_clipping_distance=float("inf")):
    dev = _dev()
    p, _, f = mesh.on_device(dev)
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
