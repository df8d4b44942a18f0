"""Sweep FusionPipeline settings on the committed DeepDeform frames (seq017 300 -> 600): per configuration, whether the
GN fit stays positive-definite and how far the warped canonical surface sits from frame 600 (median |dz|, metres)."""
import itertools
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dynamicfuion_python_amd import fusion as F  # noqa: E402
from dynamicfuion_python_amd.data import frame as dfr  # noqa: E402
from dynamicfuion_python_amd.nnrt import geometry as G  # noqa: E402

DD = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden", "deepdeform")


def gap(V, depth, K):
    v = V[V[:, 2] > 0]
    u = np.round(v[:, 0] * K[0, 0] / v[:, 2] + K[0, 2]).astype(int)
    w = np.round(v[:, 1] * K[1, 1] / v[:, 2] + K[1, 2]).astype(int)
    ok = (u >= 0) & (u < depth.shape[1]) & (w >= 0) & (w < depth.shape[0])
    d = depth[w[ok], u[ok]].astype(np.float64) / 1000.0
    good = d > 0
    return float(np.median(np.abs(v[ok, 2][good] - d[good])))


for ndc, min_valid, method, iters, lm, layers in itertools.product([1, 0], [0, 3], [0, 1], [1, 3, 10], [0.001, 0.1], [1, 2]):
    seq = dfr.FrameSequenceDataset(17, dfr.DataSplit.TEST, base_dataset_type=dfr.DatasetType.LOCAL, base_directory=DD,
                                   frame_indices=[300, 600])
    p = F.FusionParameters(fusion_minimum_valid_anchor_count=min_valid, graph_layer_count=layers)
    p.alignment.max_iteration_count = iters
    p.alignment.preconditioning_dampening_factor = lm
    p.alignment.ndc_convention = ndc
    pipe = F.FusionPipeline(seq, p)
    if method == 0:   # fixed coverage
        orig = pipe.make_warp_field
        def mk(nodes, _orig=orig, _p=p):
            return G.HierarchicalGraphWarpField(np.ascontiguousarray(nodes, np.float32), _p.node_coverage, False, _p.anchor_node_count,
                                                _p.fusion_minimum_valid_anchor_count, G.WarpNodeCoverageComputationMethod.FIXED_NODE_COVERAGE,
                                                _p.graph_layer_count)
        pipe.make_warp_field = mk
    pipe.process_frame(seq.get_next_frame())
    canonical = pipe.canonical_mesh
    f = seq.get_next_frame()
    depth = f.load_depth_image_numpy()
    try:
        pipe.process_frame(f)
        after = gap(pipe.active_graph.warp_mesh(canonical).vertex_positions.cpu().numpy(), depth, pipe.K)
        status = "ok"
    except Exception as e:   # noqa: BLE001
        after, status = float("nan"), type(e).__name__ + ": " + str(e)[:60]
    before = gap(canonical.vertex_positions.cpu().numpy(), depth, pipe.K)
    print(f"ndc={ndc} min_valid={min_valid} fixed={method == 0} iters={iters:2d} lm={lm} layers={layers}: before {before:.4f} after {after:.4f} {status}",
          flush=True)
