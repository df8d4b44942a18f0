"""Write the arrowhead structure of a synthetic config's hierarchy (CPU oracle hierarchy builder) for
tools/dev/corner_plan_stats.hip: python tools/dev/corner_plan_stats.py C5 /tmp/c5.bin"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
from dynamicfuion_python_amd import synthetic as S  # noqa: E402


def builder(nodes, cov, layers):
    return O.build_hierarchy(nodes, cov, layers)


sc = S.make_scene(sys.argv[1], seed=0, hierarchy_builder=builder)
h = sc.hierarchy
n0, N = int(h["layer_counts"][0]), len(sc.nodes)
edges = np.asarray(h["edges"], np.int32)
pos = sc.nodes[np.asarray(h["virtual_indices"])][n0:].astype(np.float32)
with open(sys.argv[2], "wb") as f:
    np.array([len(edges), n0, N], np.int32).tofile(f)
    edges.tofile(f)
    pos.tofile(f)
print("E", len(edges), "n0", n0, "N", N)
