"""Builds tests/golden/deepdeform/ from the reference's example_data (run in the build container, where /root/reference
exists; tests only read what this writes).

* Copies the DeepDeform test sequence seq017 as shipped: depth 000300/000600 (uint16 PNG, mm), colour 000300/000600 (JPEG),
  intrinsics.txt and the DeepDeformGraph files of graph 300 -> 600 (nodes, edges, edge weights, clusters). These are data
  files the reference holds, unchanged.
* Crops the train-sequence optical / scene flow (.oflow / .sflow, [C, H, W] float32) to 8 image rows so the committed
  fixture stays small; the crop is re-encoded here with `struct`, independently of the package's writers.
* Writes expected.json: every binary file decoded element by element with `struct` (the reference's decoding method,
  data/io.py:121-415), reduced to shape, float64 sum, sum of squares and the first / last rows, for the loader tests.
"""
import json
import os
import shutil
import struct

import numpy as np

EX = "/root/reference/example_data"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "deepdeform")
GRAPH = "5dbd7c9104df0300f329f294_shirt_000300_000600_geodesic_0.05"
ROWS = (232, 240)   # flow crop (image rows)


def struct_decode(path, header_words, elem):
    with open(path, "rb") as f:
        hdr = struct.unpack("I" * header_words, f.read(4 * header_words))
        body = f.read()
    n = len(body) // 4
    return hdr, np.asarray(struct.unpack(elem * n, body), dtype=np.float64)


def stats(values: np.ndarray, row: int):
    finite = values[np.isfinite(values)]
    return {"count": int(values.size), "finite": int(finite.size), "sum": float(finite.sum()), "sumsq": float((finite ** 2).sum()),
            "first_row": [float(v) for v in values[:min(row, 8)]], "last_row": [float(v) for v in values[-min(row, 8):]]}


def crop_flow(src, dst):
    with open(src, "rb") as f:
        w, h, c = struct.unpack("III", f.read(12))
        data = struct.unpack("f" * (w * h * c), f.read(4 * w * h * c))
    rows = ROWS[1] - ROWS[0]
    out = []
    for ch in range(c):
        base = ch * h * w
        out.extend(data[base + ROWS[0] * w: base + ROWS[1] * w])
    with open(dst, "wb") as f:
        f.write(struct.pack("III", w, rows, c))
        f.write(struct.pack("=%df" % len(out), *out))


def main():
    seq = os.path.join(OUT, "test", "seq017")
    for sub in ("depth", "color", "graph_nodes", "graph_edges", "graph_edges_weights", "graph_clusters"):
        os.makedirs(os.path.join(seq, sub), exist_ok=True)
    src = os.path.join(EX, "test", "seq017")
    for rel in ("depth/000300.png", "depth/000600.png", "color/000300.jpg", "color/000600.jpg", "intrinsics.txt"):
        shutil.copyfile(os.path.join(src, rel), os.path.join(seq, rel))
    for sub in ("graph_nodes", "graph_edges", "graph_edges_weights", "graph_clusters"):
        shutil.copyfile(os.path.join(src, sub, GRAPH + ".bin"), os.path.join(seq, sub, GRAPH + ".bin"))

    flow_dir = os.path.join(OUT, "flow")
    os.makedirs(flow_dir, exist_ok=True)
    tr = os.path.join(EX, "train", "seq258")
    crop_flow(os.path.join(tr, "optical_flow", "shirt_000000_000110.oflow"), os.path.join(flow_dir, "shirt_000000_000110_rows.oflow"))
    crop_flow(os.path.join(tr, "scene_flow", "shirt_000000_000110.sflow"), os.path.join(flow_dir, "shirt_000000_000110_rows.sflow"))

    expected = {"graph": GRAPH, "flow_rows": list(ROWS)}
    h, v = struct_decode(os.path.join(seq, "graph_nodes", GRAPH + ".bin"), 1, "f")
    expected["graph_nodes"] = {"header": list(h), **stats(v, 3)}
    h, v = struct_decode(os.path.join(seq, "graph_edges", GRAPH + ".bin"), 2, "i")
    expected["graph_edges"] = {"header": list(h), **stats(v, h[1])}
    h, v = struct_decode(os.path.join(seq, "graph_edges_weights", GRAPH + ".bin"), 2, "f")
    expected["graph_edges_weights"] = {"header": list(h), **stats(v, h[1])}
    h, v = struct_decode(os.path.join(seq, "graph_clusters", GRAPH + ".bin"), 2, "i")
    expected["graph_clusters"] = {"header": list(h), **stats(v, 1)}
    for ext in ("oflow", "sflow"):
        h, v = struct_decode(os.path.join(flow_dir, f"shirt_000000_000110_rows.{ext}"), 3, "f")
        expected[ext] = {"header": list(h), **stats(v, h[0])}
    with open(os.path.join(OUT, "expected.json"), "w") as f:
        json.dump(expected, f, indent=1)


if __name__ == "__main__":
    main()
