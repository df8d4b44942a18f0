"""The Schur-corner plan (csrc/corner.hip plan_corner: nested dissection, tile symbolic factorisation, launch levels,
back-substitution chains) checked on the host, without a GPU: tests/native/corner_plan_check.hip compiles the product
plan code for the host and emulates every factor launch task by task in double precision -- fill completeness,
race freedom within each launch (no task writes what another task of the launch reads or writes), back-substitution
order, and the residual of a random SPD system with the structure (< 1e-9). Structures: 2-D grid hierarchies as the
fitter builds them (stem nodes attached to their 4 nearest corner nodes), with and without corner-corner edges (>= 3
layers), with positions (coordinate bisection, the fitter path) and without (BFS separators, the C-ABI path), random
point clouds, disconnected corners and the degenerate sizes."""
import os
import shutil
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "dynamicfuion_python_amd", "csrc")
SRC = os.path.join(ROOT, "tests", "native", "corner_plan_check.hip")
BUILD = os.path.join(ROOT, "tests", "native", "build")
HIPCC = shutil.which("hipcc") or ("/opt/rocm/bin/hipcc" if os.path.exists("/opt/rocm/bin/hipcc") else None)


@pytest.fixture(scope="module")
def checker():
    if HIPCC is None:
        pytest.skip("hipcc not available")
    os.makedirs(BUILD, exist_ok=True)
    exe = os.path.join(BUILD, "corner_plan_check")
    deps = [SRC] + [os.path.join(CSRC, f) for f in ("corner.hip", "fitter_kernels.hpp", "arrow_device.hpp", "kernels.hpp", "common.hpp")]
    if not os.path.exists(exe) or os.path.getmtime(exe) < max(os.path.getmtime(d) for d in deps):
        tmp = f"{exe}.{os.getpid()}.tmp"   # concurrent workers (pytest -n) each build their own copy, then swap it in
        subprocess.check_call([HIPCC, "-O2", "-std=c++17", "--offload-arch=gfx950", "-I", os.path.join(ROOT, "include"), "-I", CSRC,
                               "-x", "hip", SRC, "-o", tmp], stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        os.replace(tmp, exe)
    return exe


def _nearest(points, centres, k):
    d = ((points[:, None, :] - centres[None]) ** 2).sum(2)
    k = min(k, len(centres))
    return np.argsort(d, axis=1, kind="stable")[:, :k]


def structure(corner_pos, stem_per_corner, corner_knn, seed):
    """Arrowhead edges of a two-layer hierarchy: corner nodes at corner_pos [n1, 3], n0 = stem_per_corner * n1 stem
    nodes scattered among them, each with edges to its 4 nearest corner nodes; corner_knn > 0 adds edges from every
    corner node to its corner_knn nearest corner nodes (the corner-corner blocks of >= 3 layers)."""
    rng = np.random.default_rng(seed)
    n1 = len(corner_pos)
    n0 = stem_per_corner * n1
    lo, hi = corner_pos.min(0), corner_pos.max(0)
    stem = rng.uniform(lo, np.maximum(hi, lo + 1e-3), (n0, 3))
    edges = []
    if n0:
        near = _nearest(stem, corner_pos, 4)
        edges.append(np.stack([np.repeat(np.arange(n0), near.shape[1]), n0 + near.ravel()], 1))
    if corner_knn and n1 > 1:
        near = _nearest(corner_pos, corner_pos, corner_knn + 1)[:, 1:]
        pairs = {(max(a, b), min(a, b)) for a in range(n1) for b in near[a] if a != b}
        edges.append(np.array([(n0 + a, n0 + b) for a, b in sorted(pairs)], np.int64).reshape(-1, 2))
    e = np.concatenate(edges, 0).astype(np.int32) if edges else np.zeros((0, 2), np.int32)
    return e, n0, n0 + n1


def grid(cx, cy, jitter, seed):
    rng = np.random.default_rng(seed)
    gx, gy = np.meshgrid(np.arange(cx, dtype=np.float32), np.arange(cy, dtype=np.float32), indexing="xy")
    p = np.stack([gx.ravel(), gy.ravel(), np.zeros(cx * cy, np.float32)], 1)
    return (p + rng.normal(0, jitter, p.shape)).astype(np.float32)


def run(checker, tmp_path, edges, n0, N, pos):
    f = tmp_path / "structure.bin"
    with open(f, "wb") as fh:
        np.array([len(edges), n0, N], np.int32).tofile(fh)
        edges.astype(np.int32).tofile(fh)
        if pos is not None:
            pos.astype(np.float32).tofile(fh)
    r = subprocess.run([checker, str(f)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    return r.stdout


CASES = {
    # name: (corner positions, stem nodes per corner node, corner-corner K-NN, seed)
    "grid_12x8": (lambda: grid(12, 8, 0.0, 0), 4, 0, 1),
    "grid_12x8_corner_edges": (lambda: grid(12, 8, 0.0, 0), 4, 2, 2),
    "grid_26x15_c5_like": (lambda: grid(26, 15, 0.1, 3), 12, 0, 3),
    "grid_30x3_strip": (lambda: grid(30, 3, 0.05, 4), 4, 2, 4),
    "random_cloud_300": (lambda: np.random.default_rng(5).uniform(0, 10, (300, 3)).astype(np.float32), 6, 0, 5),
    "random_cloud_150_knn3": (lambda: np.random.default_rng(6).uniform(0, 5, (150, 3)).astype(np.float32), 3, 3, 6),
    "two_clusters": (lambda: np.concatenate([grid(8, 8, 0.0, 7), grid(8, 8, 0.0, 8) + np.float32([100, 0, 0])]), 3, 0, 7),
    "leaf_sized_42": (lambda: grid(7, 6, 0.0, 9), 3, 1, 9),
    "just_above_leaf_43": (lambda: grid(43, 1, 0.0, 10), 2, 1, 10),
    "single_corner_node": (lambda: grid(1, 1, 0.0, 11), 5, 0, 11),
    "two_corner_nodes_no_stem": (lambda: grid(2, 1, 0.0, 12), 0, 1, 12),
}


@pytest.mark.parametrize("with_positions", [True, False], ids=["coordinate_bisection", "bfs_separators"])
@pytest.mark.parametrize("name", list(CASES))
def test_corner_plan_emulated(checker, tmp_path, name, with_positions):
    make_pos, spc, knn, seed = CASES[name]
    pos = make_pos()
    edges, n0, N = structure(pos, spc, knn, seed)
    out = run(checker, tmp_path, edges, n0, N, pos if with_positions else None)
    assert "residual" in out
