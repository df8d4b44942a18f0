# developer smoke (not collected by pytest): stage parity GPU vs oracle on a small scene + C2 timing
import os, sys, time, numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import torch
from dynamicfuion_python_amd import _native as NV
from dynamicfuion_python_amd import synthetic as S
from dynamicfuion_python_amd.nnrt import geometry as G, rendering as Rr, alignment as A
import oracle as O
print("device count", NV.lib().nnrt_device_count(), "runtime", NV.lib().nnrt_runtime_version(), torch.cuda.is_available(), flush=True)
sc = S.make_scene("S1")
a_o, w_o = O.compute_anchors(sc.points, sc.nodes, 4, sc.coverage)
a_g, w_g = G.compute_anchors_and_weights_euclidean_fixed_node_weight(sc.points, sc.nodes, 4, 0, sc.coverage)
a_g, w_g = a_g.cpu().numpy(), w_g.cpu().numpy()
print("anchors equal", np.array_equal(a_o, a_g), "weights maxdiff", np.abs(w_o - w_g).max(), flush=True)
wp_o, wn_o = O.warp_mesh(sc.points, sc.normals, sc.nodes, sc.gt_rotations, sc.gt_translations, a_o, w_o)
m = G.warp_triangle_mesh(G.TriangleMesh(sc.points, sc.normals, sc.faces), sc.nodes, sc.gt_rotations, sc.gt_translations, a_o, w_o)
print("warp maxdiff", np.abs(m.vertex_positions.cpu().numpy() - wp_o).max(), np.abs(m.vertex_normals.cpu().numpy() - wn_o).max(), flush=True)
fndc_o, fm_o = O.extract_face_ndc(wp_o, sc.faces, sc.K, sc.H, sc.W, 0, 10)
fndc_g, fm_g = Rr.get_mesh_ndc_face_vertices_and_clip_mask(G.TriangleMesh(wp_o, wn_o, sc.faces), sc.K, (sc.H, sc.W), 0, 10)
print("ndc equal", np.array_equal(fndc_o, fndc_g.cpu().numpy()), np.array_equal(fm_o, fm_g.cpu().numpy()), flush=True)
fi_o, dep_o, b_o, d_o = O.rasterize(fndc_o, fm_o, sc.H, sc.W, 0.5, 1, -1, -1, True, False, True)
fi_g, dep_g, b_g, d_g = Rr.rasterize_ndc_triangles(fndc_o, fm_o, (sc.H, sc.W), 0.5, 1, -1, -1, True, False, True)
print("raster faces equal", np.array_equal(fi_o, fi_g.cpu().numpy()), "depth eq", np.array_equal(dep_o, dep_g.cpu().numpy()),
      "bary eq", np.array_equal(b_o, b_g.cpu().numpy()), "dist eq", np.array_equal(d_o, d_g.cpu().numpy()), flush=True)
fi4_o, dep4_o, _, _ = O.rasterize(fndc_o, fm_o, sc.H, sc.W, 0.5, 4, -1, -1, True, False, True)
fi4_g, dep4_g, _, _ = Rr.rasterize_ndc_triangles(fndc_o, fm_o, (sc.H, sc.W), 0.5, 4, -1, -1, True, False, True)
print("raster K=4 faces equal", np.array_equal(fi4_o, fi4_g.cpu().numpy()), np.array_equal(dep4_o, dep4_g.cpu().numpy()), flush=True)
# fit one iteration
depth = np.where(dep_o[..., 0] > 0, dep_o[..., 0], 0).astype(np.float32)
refp, refm = O.unproject(depth, sc.K, 1.0, 10.0)
N = len(sc.nodes)
R0 = np.tile(np.eye(3, dtype=np.float32), (N, 1, 1)); t0 = np.zeros((N, 3), np.float32)
Ro, to, dg = O.fit(nodes=sc.nodes, rotations=R0, translations=t0, mesh_points=sc.points, mesh_normals=sc.normals, faces=sc.faces,
                   ref_points=refp, ref_mask=refm, H=sc.H, W=sc.W, K=sc.K, max_iterations=1, lm_factor=0.001, coverage=sc.coverage)
wf = G.HierarchicalGraphWarpField(sc.nodes, sc.coverage, False, 4, 0, G.WarpNodeCoverageComputationMethod.FIXED_NODE_COVERAGE, 1)
ft = A.DeformableMeshToImageFitter(1, [A.IterationMode.ALL], preconditioning_dampening_factor=0.001)
ft.fit_to_image(wf, G.TriangleMesh(sc.points, sc.normals, sc.faces), None, depth, None, sc.K, None, 1.0)
dgg = ft.diagnostics()
Rg, tg = wf.get_node_rotations(), wf.get_node_translations()
print("faces eq frac", (dgg["pixel_faces"] == dg["pixel_faces"]).mean(), "mask eq", np.array_equal(dgg["residual_mask"], dg["residual_mask"]),
      "resid maxdiff", np.abs(dgg["residuals"] - dg["residuals"]).max(), flush=True)
H_o = dg["hessian_diag"]; H_g = dgg["hessian"][:H_o.size]
print("H rel", np.abs(H_o - H_g).max() / np.abs(H_o).max(), "g rel", np.abs(dg["gradient"] - dgg["gradient"]).max() / np.abs(dg["gradient"]).max(),
      "x rel", np.abs(dg["updates"] - dgg["updates"]).max() / np.abs(dg["updates"]).max(), flush=True)
print("R maxdiff", np.abs(Ro - Rg).max(), "t maxdiff", np.abs(to - tg).max(), flush=True)
# C2 timing
sc = S.make_scene("C2")
wf = G.HierarchicalGraphWarpField(sc.nodes, sc.coverage, False, 4, 0, G.WarpNodeCoverageComputationMethod.FIXED_NODE_COVERAGE, 1)
wf.set_node_rotations(sc.gt_rotations); wf.set_node_translations(sc.gt_translations)
ft = A.DeformableMeshToImageFitter(1, [A.IterationMode.ALL], preconditioning_dampening_factor=0.001)
mesh = G.TriangleMesh(sc.points, sc.normals, sc.faces)
for graph in [0, 1]:
    ft = A.DeformableMeshToImageFitter(1, [A.IterationMode.ALL], preconditioning_dampening_factor=0.001, use_hip_graph=bool(graph))
    ft.prepare(wf, mesh, np.full((sc.H, sc.W), 1.2, np.float32), None, sc.K)
    ft.iterate(wf, 0, 3); torch.cuda.synchronize()
    t0 = time.perf_counter(); n = 200
    ft.iterate(wf, 0, n); torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    print(f"C2 graph={graph}: {dt*1e6:.1f} us/iter -> {1/dt:.0f} it/s", flush=True)
