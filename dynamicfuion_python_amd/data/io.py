"""DeepDeform / DeepDeformGraph on-disk formats (reference data/io.py).

Every binary format here is a little-endian header of uint32 dimensions followed by a C-order payload; the readers
decode the payload in one `np.frombuffer` call (the reference unpacks element by element with `struct`) and raise
`ValueError` on a truncated file where the reference's `struct.unpack` raises `struct.error`.

| reference (data/io.py)                     | header                                | payload                         |
|--------------------------------------------|---------------------------------------|---------------------------------|
| load/save_graph_nodes_or_deformations :200 | u32 N                                 | f32 [N, 3]                      |
| load/save_graph_edges :224, :239           | u32 N, u32 K                          | i32 [N, K]                      |
| load/save_graph_edges_weights :249, :264   | u32 N, u32 K                          | f32 [N, K]                      |
| load/save_graph_node_translations :284     | u32 N                                 | f32 [N, 3]                      |
| load/save_graph_node_rotations :308        | u32 N                                 | f32 [N, 3, 3]                   |
| load/save_graph_clusters :332, :347        | u32 N, u32 (ignored on read)          | i32 [N] -> [N, 1]               |
| load/save_float_image, int_image :357-415  | u32 dim2, u32 dim1, u32 dim0          | f32 / i32 [dim0, dim1, dim2]    |
| load/save_flow_binary (.oflow/.sflow) :121 | u32 W, u32 H, u32 C                   | f32 [C, H, W]                   |
| load/save_flow_middlebury (.flo) :149      | b"PIEH", i32 W, i32 H                 | f32 [H, W, 2]                   |
| load/save_PFM :53, :91                     | "PF"/"Pf", "W H", scale (<0: little)  | f32 rows bottom-up              |

Images (depth PNG uint16 in mm, colour JPEG/PNG) are read with PIL (OpenCV / Open3D are not part of this build).
"""
from __future__ import annotations

import os
import re
import sys

import numpy as np

_U32 = np.dtype("<u4")
_I32 = np.dtype("<i4")
_F32 = np.dtype("<f4")


# ----------------------------------------------------------------------------------------------------------------
# header + payload helpers
# ----------------------------------------------------------------------------------------------------------------
def _read_file(filename) -> bytes:
    if not os.path.isfile(filename):
        raise FileNotFoundError(f"File not found: {filename}")
    with open(filename, "rb") as f:
        return f.read()


def _payload(buf: bytes, offset: int, dtype: np.dtype, shape, filename) -> np.ndarray:
    count = int(np.prod(shape, dtype=np.int64))
    need = offset + count * dtype.itemsize
    if len(buf) < need:
        raise ValueError(f"{filename}: truncated file ({len(buf)} bytes, header asks for {need})")
    return np.frombuffer(buf, dtype, count, offset).reshape(shape).astype(dtype.newbyteorder("="), copy=True)


def _header(buf: bytes, count: int, filename) -> list:
    if len(buf) < 4 * count:
        raise ValueError(f"{filename}: truncated header")
    return [int(v) for v in np.frombuffer(buf, _U32, count, 0)]


def _write(filename, header, payload: np.ndarray, dtype: np.dtype):
    with open(filename, "wb") as f:
        f.write(np.asarray(header, _U32).tobytes())
        f.write(np.ascontiguousarray(payload, dtype=dtype).tobytes())


# ----------------------------------------------------------------------------------------------------------------
# graph files
# ----------------------------------------------------------------------------------------------------------------
def load_graph_nodes_or_deformations(filename) -> np.ndarray:
    """[N, 3] float32 node positions (or per-node deformations) (data/io.py:200-211)."""
    buf = _read_file(filename)
    (n,) = _header(buf, 1, filename)
    return _payload(buf, 4, _F32, (n, 3), filename)


def _check_rows3(a: np.ndarray, cols=(3,)):
    a = np.asarray(a)
    if a.ndim != 1 + len(cols) or tuple(a.shape[1:]) != tuple(cols):
        raise ValueError(f"expected an array of shape [N, {', '.join(map(str, cols))}], got {a.shape}")
    return a


def save_graph_nodes(filename, nodes):
    """data/io.py:214-221"""
    nodes = _check_rows3(nodes)
    _write(filename, [nodes.shape[0]], nodes, _F32)


def save_graph_node_deformations(filename, node_deformations):
    """data/io.py:274-281"""
    d = _check_rows3(node_deformations)
    _write(filename, [d.shape[0]], d, _F32)


def _load_n_by_k(filename, dtype) -> np.ndarray:
    buf = _read_file(filename)
    n, k = _header(buf, 2, filename)
    return _payload(buf, 8, dtype, (n, k), filename)


def _save_n_by_k(filename, a, dtype):
    a = np.asarray(a)
    if a.ndim != 2:
        raise ValueError(f"expected a 2-D array, got shape {a.shape}")
    _write(filename, [a.shape[0], a.shape[1]], a, dtype)


def load_graph_edges(filename) -> np.ndarray:
    """[N, K] int32 neighbour indices, -1 = no edge (data/io.py:224-236)."""
    return _load_n_by_k(filename, _I32)


def save_graph_edges(filename, edges):
    """data/io.py:239-246"""
    _save_n_by_k(filename, edges, _I32)


def load_graph_edges_weights(filename) -> np.ndarray:
    """[N, K] float32 edge weights (data/io.py:249-261)."""
    return _load_n_by_k(filename, _F32)


def save_graph_edges_weights(filename, edges_weights):
    """data/io.py:264-271"""
    _save_n_by_k(filename, edges_weights, _F32)


def load_graph_node_translations(filename) -> np.ndarray:
    """[N, 3] float32 (data/io.py:284-295)."""
    return load_graph_nodes_or_deformations(filename)


def save_graph_node_translations(filename, translations_vec):
    """data/io.py:298-305"""
    t = _check_rows3(translations_vec)
    _write(filename, [t.shape[0]], t, _F32)


def load_graph_node_rotations(filename) -> np.ndarray:
    """[N, 3, 3] float32 (data/io.py:308-319)."""
    buf = _read_file(filename)
    (n,) = _header(buf, 1, filename)
    return _payload(buf, 4, _F32, (n, 3, 3), filename)


def save_graph_node_rotations(filename, rotations_mat):
    """data/io.py:322-329"""
    r = _check_rows3(rotations_mat, (3, 3))
    _write(filename, [r.shape[0]], r, _F32)


def load_graph_clusters(filename) -> np.ndarray:
    """[N, 1] int32 cluster ids; the second header word is skipped, as in the reference (data/io.py:332-344)."""
    buf = _read_file(filename)
    n, _ = _header(buf, 2, filename)
    return _payload(buf, 8, _I32, (n,), filename).reshape(n, 1)


def save_graph_clusters(filename, clusters):
    """data/io.py:347-354"""
    _save_n_by_k(filename, clusters, _I32)


# ----------------------------------------------------------------------------------------------------------------
# float / int images (pixel anchors, pixel weights)
# ----------------------------------------------------------------------------------------------------------------
def _load_image3(filename, dtype) -> np.ndarray:
    buf = _read_file(filename)
    d2, d1, d0 = _header(buf, 3, filename)
    return _payload(buf, 12, dtype, (d0, d1, d2), filename)


def _save_image3(filename, image, dtype):
    image = np.asarray(image)
    if image.ndim != 3:
        raise ValueError(f"expected a 3-D image, got shape {image.shape}")
    _write(filename, [image.shape[2], image.shape[1], image.shape[0]], image, dtype)


def load_float_image(filename) -> np.ndarray:
    """float32 [d0, d1, d2] (data/io.py:357-371), e.g. pixel weights [H, W, 4]."""
    return _load_image3(filename, _F32)


def save_float_image(filename, image_input):
    """data/io.py:374-384"""
    _save_image3(filename, image_input, _F32)


def load_int_image(filename) -> np.ndarray:
    """int32 [d0, d1, d2] (data/io.py:400-414), e.g. pixel anchors [H, W, 4]."""
    return _load_image3(filename, _I32)


def save_int_image(filename, image_input):
    """data/io.py:387-397"""
    _save_image3(filename, image_input, _I32)


# ----------------------------------------------------------------------------------------------------------------
# flow / PFM
# ----------------------------------------------------------------------------------------------------------------
def load_flow_binary(filename) -> np.ndarray:
    """.oflow / .sflow: float32 [C, H, W] (data/io.py:121-135)."""
    buf = _read_file(filename)
    w, h, c = _header(buf, 3, filename)
    return _payload(buf, 12, _F32, (c, h, w), filename)


def save_flow_binary(filename, flow):
    """data/io.py:138-146"""
    flow = np.asarray(flow)
    if flow.ndim != 3:
        raise ValueError(f"flow must be [C, H, W], got {flow.shape}")
    _write(filename, [flow.shape[2], flow.shape[1], flow.shape[0]], flow, _F32)


def load_flow_middlebury(filename) -> np.ndarray:
    """.flo: float32 [H, W, 2] (data/io.py:149-161)."""
    buf = _read_file(filename)
    if buf[:4] != b"PIEH":
        raise ValueError("Flow file header does not contain PIEH")
    w, h = (int(v) for v in np.frombuffer(buf, _I32, 2, 4))
    return _payload(buf, 12, _F32, (h, w, 2), filename)


def save_flow_middlebury(name, flow):
    """data/io.py:164-169"""
    flow = np.asarray(flow, np.float32)
    with open(name, "wb") as f:
        f.write(b"PIEH")
        f.write(np.asarray([flow.shape[1], flow.shape[0]], _I32).tobytes())
        f.write(np.ascontiguousarray(flow, _F32).tobytes())


def load_PFM(file):
    """(data, scale) with rows flipped to top-down (data/io.py:53-88)."""
    with open(file, "rb") as f:
        header = f.readline().rstrip()
        if header == b"PF":
            color = True
        elif header == b"Pf":
            color = False
        else:
            raise ValueError("Not a PFM file.")
        m = re.match(r"^(\d+)\s(\d+)\s$", f.readline().decode("ascii"))
        if not m:
            raise ValueError("Malformed PFM header.")
        width, height = int(m.group(1)), int(m.group(2))
        scale = float(f.readline().decode("ascii").rstrip())
        endian = "<" if scale < 0 else ">"
        data = np.frombuffer(f.read(), np.dtype(endian + "f4"))
    shape = (height, width, 3) if color else (height, width)
    return np.flipud(data.reshape(shape)), abs(scale)


def save_PFM(file, image, scale=1):
    """data/io.py:91-118 (the reference writes the colour header as str to a binary file; here both are bytes)."""
    image = np.asarray(image)
    if image.dtype.name != "float32":
        raise ValueError("Image dtype must be float32.")
    if image.ndim == 3 and image.shape[2] == 3:
        color = True
    elif image.ndim == 2 or (image.ndim == 3 and image.shape[2] == 1):
        color = False
    else:
        raise ValueError("Image must have H x W x 3, H x W x 1 or H x W dimensions.")
    image = np.flipud(image)
    endian = image.dtype.byteorder
    if endian == "<" or (endian == "=" and sys.byteorder == "little"):
        scale = -scale
    with open(file, "wb") as f:
        f.write(b"PF\n" if color else b"Pf\n")
        f.write(b"%d %d\n" % (image.shape[1], image.shape[0]))
        f.write(b"%f\n" % scale)
        f.write(np.ascontiguousarray(image).tobytes())


_FLOW_LOADERS = {".pfm": lambda p: load_PFM(p)[0][:, :, 0:2], ".oflow": load_flow_binary, ".sflow": load_flow_binary,
                 ".flo": load_flow_middlebury}


def load_flow(filename):
    """Dispatch on extension (data/io.py:172-183); an unknown extension raises (the reference prints and exits)."""
    ext = os.path.splitext(filename)[1].lower()
    if ext not in _FLOW_LOADERS:
        raise ValueError(f"Wrong flow extension: {filename}")
    return _FLOW_LOADERS[ext](filename)


def save_flow(filename, flow):
    """data/io.py:186-197"""
    ext = os.path.splitext(filename)[1].lower()
    if ext == ".pfm":
        save_PFM(filename, flow)
    elif ext in (".oflow", ".sflow"):
        save_flow_binary(filename, flow)
    elif ext == ".flo":
        save_flow_middlebury(filename, flow)
    else:
        raise ValueError(f"Wrong flow extension: {filename}")


# ----------------------------------------------------------------------------------------------------------------
# PNG / JPEG frames
# ----------------------------------------------------------------------------------------------------------------
def load_depth_image(path) -> np.ndarray:
    """uint16 [H, W] depth in the sensor's unit (mm for DeepDeform), as o3d.io.read_image / cv2 IMREAD_UNCHANGED give."""
    from PIL import Image
    with Image.open(path) as im:
        a = np.array(im)
    if a.ndim != 2:
        raise ValueError(f"{path}: a depth image must be single-channel, got shape {a.shape}")
    return a.astype(np.uint16, copy=False)


def load_color_image(path) -> np.ndarray:
    """uint8 [H, W, 3] in RGB order (o3d.io.read_image). FrameDataset.load_color_image_numpy (cv2) is BGR."""
    from PIL import Image
    with Image.open(path) as im:
        return np.array(im.convert("RGB"))


def load_mask_image(path) -> np.ndarray:
    from PIL import Image
    with Image.open(path) as im:
        return np.array(im)


def save_rgb_image(filename, image_numpy):
    """data/io.py:11-27: [H, W, 3] uint8 or [3, H, W] float in [0, 1]."""
    from PIL import Image
    a = np.asarray(image_numpy)
    if a.ndim == 3 and a.shape[0] == 3 and a.shape[2] != 3:
        a = np.moveaxis(a, 0, -1)
    if a.shape[-1] != 3:
        raise ValueError(f"image has {a.shape[-1]} channels, expected 3")
    if a.dtype == np.float32:
        if a.max() > 1.0:
            raise ValueError("float32 images must lie in [0, 1]")
        a = (a * 255.0).astype(np.uint8)
    Image.fromarray(np.ascontiguousarray(a, np.uint8), "RGB").save(filename)


def save_grayscale_image(filename, image_numpy):
    """data/io.py:30-40: values in [0, 1] scaled by 255 (any dtype, as in the reference); [H, W], [1, H, W] or [H, W, 1]."""
    from PIL import Image
    a = (np.asarray(image_numpy) * 255).astype(np.uint8)
    Image.fromarray(a.reshape(a.shape[-2:]) if a.ndim == 3 else a, "L").save(filename)
