/*
 * nnrt_mi355x.h -- C-ABI of the MI355X-native DeformableMeshToImageFitter hot path.
 *
 * Drop-in boundary for henry123-boy/Dynamicfuion_python's dense non-rigid tracker. Every entry point replaces a
 * reference interface, cited per function (paths relative to the reference repository root). Plain pointers and
 * sizes only: arrays marked d_ are DEVICE pointers (hipMalloc'd or torch.cuda tensors on the same device), h_ arrays
 * are HOST pointers. All functions return 0 on success and a non-zero nnrt_status otherwise, with a message retrievable
 * through nnrt_last_error() (thread-local). No exceptions cross the ABI. A `stream` argument is a hipStream_t (NULL =
 * the legacy default stream). Handles are not thread-safe: use one handle per host thread.
 *
 * Layout conventions follow the reference tensors: float32 row-major, vertex/face/node-major; rotations [N,3,3]
 * row-major; triangle indices int64 [F,3]; intrinsics/extrinsics float64 [3,3]/[4,4] on the host.
 */
#ifndef NNRT_MI355X_H
#define NNRT_MI355X_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef int32_t nnrt_status;
enum {
	NNRT_OK = 0,
	NNRT_ERROR_ARGUMENT = 1,
	NNRT_ERROR_HIP = 2,
	NNRT_ERROR_NOT_POSITIVE_DEFINITE = 3,   /* reference: NNRT_LAPACK_CHECK potrf failure -> RuntimeError */
	NNRT_ERROR_UNSUPPORTED = 4,
	NNRT_ERROR_CAPACITY = 5
};

/* iteration modes: cpp/alignment/IterationMode.h:24-28 */
enum { NNRT_ITERATION_ALL = 0, NNRT_ITERATION_TRANSLATION_ONLY = 1, NNRT_ITERATION_ROTATION_ONLY = 2 };
/* warp-node coverage: cpp/geometry/WarpNodeCoverageComputationMethod.h */
enum { NNRT_FIXED_NODE_COVERAGE = 0, NNRT_MINIMAL_K_NEIGHBOR_NODE_DISTANCE = 1 };

typedef struct nnrt_warp_field nnrt_warp_field;
typedef struct nnrt_fitter nnrt_fitter;

const char* nnrt_last_error(void);
/* HIP runtime version the library was built against and the number of visible devices (-1 on error). */
int32_t nnrt_runtime_version(void);
int32_t nnrt_device_count(void);
/* Pixel-node Jacobian arithmetic of this build: 0 = the reference CPU path's unfused expressions (the product), 1 = FMA
 * form (a development build, -DNNRT_JAC_FMA=1). Both are the reference's expression (PixelVertexAnchorJacobiansImpl.h
 * :179-363, WarpedSurfaceJacobiansImpl.h:117-156); the test checker selects its matching mode from this. */
int32_t nnrt_build_jacobian_fma(void);
/* The arrowhead solve's refinement floor of this build (NNRT_REFINE_PIVOT_FLOOR): no refinement step below this corner
 * pivot / diag(S) ratio. */
float nnrt_build_refine_floor(void);

/* ---------------------------------------------------------------------------------------------------------------
 * Warp field -- replaces nnrt::geometry::HierarchicalGraphWarpField (cpp/geometry/HierarchicalGraphWarpField.h:37-97,
 * cpp/geometry/HierarchicalGraphWarpField.cpp:37-313) and the exported GraphWarpField accessors
 * (cpp/pybind/geometry/geometry.cpp:278-320). Node state lives on the device in virtual (hierarchy) order.
 * h_layer_radii may be NULL (default radius (i+1) * node_coverage, HierarchicalGraphWarpField.h:46-47).
 * ------------------------------------------------------------------------------------------------------------- */
nnrt_status nnrt_warp_field_create(const float* h_nodes, int32_t node_count, float node_coverage, int32_t threshold_nodes_by_distance,
                                   int32_t anchor_count, int32_t minimum_valid_anchor_count, int32_t coverage_method,
                                   int32_t layer_count, int32_t max_vertex_degree, const float* h_layer_radii, int32_t device,
                                   nnrt_warp_field** out);
void nnrt_warp_field_destroy(nnrt_warp_field* warp_field);
int32_t nnrt_warp_field_node_count(const nnrt_warp_field* warp_field);
int32_t nnrt_warp_field_edge_count(const nnrt_warp_field* warp_field);
/* layer sizes (fine -> coarse) into h_counts[layer_count]; returns layer_count */
int32_t nnrt_warp_field_layer_counts(const nnrt_warp_field* warp_field, int32_t* h_counts);
/* HierarchicalGraphWarpField::GetVirtualNodeIndices (:206-208): h_out[N] int64 (virtual -> original) */
nnrt_status nnrt_warp_field_get_virtual_node_indices(const nnrt_warp_field* warp_field, int64_t* h_out);
/* GetEdges / GetEdgeLayerIndices (:201-228): h_edges[E,2] int32 virtual indices, h_edge_layers[E] int8 (either may be NULL) */
nnrt_status nnrt_warp_field_get_edges(const nnrt_warp_field* warp_field, int32_t* h_edges, int8_t* h_edge_layers);
/* GetNodePositions/Rotations/Translations(use_virtual_ordering) (:210-224) and Set/Translate/Rotate counterparts. */
nnrt_status nnrt_warp_field_get_node_positions(const nnrt_warp_field* warp_field, float* h_out, int32_t virtual_order);
nnrt_status nnrt_warp_field_get_node_rotations(const nnrt_warp_field* warp_field, float* h_out, int32_t virtual_order);
nnrt_status nnrt_warp_field_get_node_translations(const nnrt_warp_field* warp_field, float* h_out, int32_t virtual_order);
nnrt_status nnrt_warp_field_set_node_rotations(nnrt_warp_field* warp_field, const float* h_in, int32_t virtual_order);
nnrt_status nnrt_warp_field_set_node_translations(nnrt_warp_field* warp_field, const float* h_in, int32_t virtual_order);
/* Resets every node to the identity motion on `stream`: R = I (as WarpField::ResetRotations, WarpField.cpp:151-156) and t = 0. */
nnrt_status nnrt_warp_field_reset_motion(nnrt_warp_field* warp_field, void* stream);
/* node coverage weights (MINIMAL_K_NEIGHBOR_NODE_DISTANCE, WarpField.cpp:249-263), virtual order */
nnrt_status nnrt_warp_field_get_node_coverage_weights(const nnrt_warp_field* warp_field, float* h_out);

/* ---------------------------------------------------------------------------------------------------------------
 * Fitter -- replaces nnrt::alignment::DeformableMeshToImageFitter (cpp/alignment/DeformableMeshToImageFitter.h:34-91,
 * .cpp:56-448). Parameters mirror the constructor (.h:34-46).
 * ------------------------------------------------------------------------------------------------------------- */
typedef struct nnrt_fitter_params {
	int32_t max_iteration_count;            /* 100 */
	int32_t iteration_mode_count;           /* 1 */
	int32_t iteration_modes[16];            /* {NNRT_ITERATION_ALL} */
	float minimal_update_threshold;         /* 1e-6 (never effective in the reference: A14) */
	int32_t use_perspective_correction;     /* 1 */
	float max_depth;                        /* 10 */
	int32_t use_tukey_penalty_for_data_term;/* 0 */
	float tukey_penalty_cutoff_cm;          /* 0.01 */
	float preconditioning_dampening_factor; /* 0 ; must be in [0, 1] */
	float arap_term_weight;                 /* 200 */
	int32_t use_huber_penalty_for_arap_term;/* 0 */
	float huber_penalty_constant;           /* 1e-4 */
	int32_t use_hip_graph;                  /* NNRT_GRAPH_AUTO (1, default): an iteration sequence runs eagerly the first
	                                           time it is requested after (re)preparation and is captured into a hipGraph
	                                           and replayed from its second request on; NNRT_GRAPH_ALWAYS (2): captured on
	                                           first use; NNRT_GRAPH_NEVER (0): always eager launches */
	int32_t ndc_convention;                 /* NNRT_NDC_REFERENCE (0): the reference's image-space -> NDC mapping, whose
	                                           rendered points are y-mirrored about cy (CoordinateSystemConversions.h:
	                                           130-136); NNRT_NDC_CONSISTENT (1): raster pixel (u, v) is pixel (u, v) of K, for
	                                           fitting real depth frames (a deliberate divergence) */
} nnrt_fitter_params;
#define NNRT_NDC_REFERENCE 0
#define NNRT_NDC_CONSISTENT 1
#define NNRT_GRAPH_NEVER 0
#define NNRT_GRAPH_AUTO 1
#define NNRT_GRAPH_ALWAYS 2

void nnrt_fitter_default_params(nnrt_fitter_params* params);
nnrt_status nnrt_fitter_create(const nnrt_fitter_params* params, int32_t device, nnrt_fitter** out);
void nnrt_fitter_destroy(nnrt_fitter* fitter);

/* FitToImage(warp_field, canonical_mesh, color, depth, mask, K, E, depth_scale) (DeformableMeshToImageFitter.cpp:278-314).
 * d_depth: float32 [H,W] metric depth * depth_scale; d_mask: uint8 [H,W] or NULL; h_K: float64[9]; h_E: float64[16] or
 * NULL (identity). Mutates the warp field's rotations/translations in place. */
nnrt_status nnrt_fitter_fit_to_image(nnrt_fitter* fitter, nnrt_warp_field* warp_field, const float* d_vertices, const float* d_normals,
                                     int64_t vertex_count, const int64_t* d_faces, int64_t face_count, const float* d_depth,
                                     const uint8_t* d_mask, int32_t height, int32_t width, const double* h_K, const double* h_E,
                                     float depth_scale, void* stream);
/* The same call split in two for benchmarking / streaming use: prepare() runs the once-per-frame setup of
 * FitToImage (:96-106: anchors, NDC intrinsics, face<->anchor association, reference point cloud); iterate() runs
 * `count` GN iterations (loop body :111-275) starting at iteration index `first_iteration` (selects the mode). */
nnrt_status nnrt_fitter_prepare(nnrt_fitter* fitter, nnrt_warp_field* warp_field, const float* d_vertices, const float* d_normals,
                                int64_t vertex_count, const int64_t* d_faces, int64_t face_count, const float* d_depth,
                                const uint8_t* d_mask, int32_t height, int32_t width, const double* h_K, const double* h_E,
                                float depth_scale, void* stream);
/* FitToImage(warp_field, canonical_mesh, color, reference_point_cloud, reference_point_mask, K, E, rendering_image_size)
 * (DeformableMeshToImageFitter.cpp:85-276, the overload the depth variant forwards to): d_points float32 [H*W,3]
 * organized reference points, d_point_mask uint8 [H*W] or NULL (all valid), (height, width) = rendering image size. */
nnrt_status nnrt_fitter_prepare_point_cloud(nnrt_fitter* fitter, nnrt_warp_field* warp_field, const float* d_vertices,
                                            const float* d_normals, int64_t vertex_count, const int64_t* d_faces, int64_t face_count,
                                            const float* d_points, const uint8_t* d_point_mask, int32_t height, int32_t width,
                                            const double* h_K, const double* h_E, void* stream);
nnrt_status nnrt_fitter_fit_to_point_cloud(nnrt_fitter* fitter, nnrt_warp_field* warp_field, const float* d_vertices,
                                           const float* d_normals, int64_t vertex_count, const int64_t* d_faces, int64_t face_count,
                                           const float* d_points, const uint8_t* d_point_mask, int32_t height, int32_t width,
                                           const double* h_K, const double* h_E, void* stream);
/* Iterations are enqueued on `stream` itself. With use_hip_graph the `count` iterations (up to 64 per launch) are
 * captured once as one graph per mode sequence and replayed on `stream` as a single launch. */
nnrt_status nnrt_fitter_iterate(nnrt_fitter* fitter, nnrt_warp_field* warp_field, int32_t first_iteration, int32_t count, void* stream);
/* Benchmark / diagnostic form of iterate(): every iteration first resets the warp field's motion to the identity
 * (R = I, t = 0, as nnrt_warp_field_reset_motion), so each is the first GN iteration of the prepared frame. Same
 * graph behaviour as iterate() (the resets are captured with the iterations). */
nnrt_status nnrt_fitter_iterate_from_identity(nnrt_fitter* fitter, nnrt_warp_field* warp_field, int32_t first_iteration, int32_t count,
                                              void* stream);
/* Number of instantiated iteration-sequence graphs the fitter holds (diagnostic for the use_hip_graph policy). */
int32_t nnrt_fitter_graph_count(const nnrt_fitter* fitter);
/* Schur-corner plan of the prepared frame's arrowhead solve (diagnostic; zeros without ARAP): h_out[6] = corner nodes,
 * 64-unknown tile columns, factorization launches (elimination-tree levels), back-substitution launches, stored
 * (structurally non-zero) tiles, lower tiles of the dense corner. */
nnrt_status nnrt_fitter_corner_info(const nnrt_fitter* fitter, int64_t* h_out);
/* Work of that plan's factorization as executed (diagnostic; zeros without ARAP): h_out[3] = MFMA flops per
 * factorization (every update term's 64 x 64 x 64 tile product + the rank-32 products of the split eliminations),
 * update terms, tile-column eliminations (real columns summed). The reference's dense count is (6 n1)^3 / 3 + ... */
nnrt_status nnrt_fitter_corner_work(const nnrt_fitter* fitter, int64_t* h_out);
/* The last iteration's warped canonical mesh (diagnostic; synchronizes `stream`): h_positions / h_normals [V,3] as the
 * fitter rasterized them (Warping.cpp:222-264 of the motion the iteration started from). */
nnrt_status nnrt_fitter_get_warped_mesh(nnrt_fitter* fitter, float* h_positions, float* h_normals, int64_t vertex_count, void* stream);
/* The last ARAP iteration's float arrowhead system exactly as the fitter factored and refined it (diagnostic; synchronizes
 * `stream`; virtual node order): h_diag [N,36] diagonal blocks (data + ARAP + LM), h_wing [E,36] wing blocks (block (i, j)
 * of edge e = (i, j), its transpose at (j, i)), h_rhs [6N] right-hand side (negative gradient). The reference holds the
 * same system between ComputeArapHessian and SolveBlockSparseArrowheadCholesky (DeformableMeshToImageFitter.cpp:223-247). */
nnrt_status nnrt_fitter_get_arrowhead_system(nnrt_fitter* fitter, float* h_diag, float* h_wing, float* h_rhs, int64_t node_count,
                                             int64_t edge_count, void* stream);
/* The last arrowhead solve's refinement gate (diagnostic; synchronizes `stream`): h_out[5] = the corner factorization's
 * smallest pivot / diag(S) ratio (1 without ARAP), the threshold below which one step of iterative refinement runs (it
 * does not below the build's floor, 1e-5, where one step is not relied on), 1 if it ran, the step's max |d| / max |x|
 * and 1 if its safeguard accepted it (max |d| <= 1e-2 max |x|; else the plain solve stands). */
nnrt_status nnrt_fitter_refine_info(nnrt_fitter* fitter, float* h_out, void* stream);
/* Threshold of the refinement gate (default 1e-2): the arrowhead solve refines when the corner's smallest pivot /
 * diag(S) ratio falls below it (and is at least 1e-5); 0 never refines. Drops the fitter's cached graphs (a launch
 * argument). */
nnrt_status nnrt_fitter_set_refine_ratio(nnrt_fitter* fitter, float ratio);
/* Store the warp field's current node motion (R, t) in the fitter (a device copy on `stream`). */
nnrt_status nnrt_fitter_snapshot_motion(nnrt_fitter* fitter, nnrt_warp_field* warp_field, void* stream);
/* Benchmark form of iterate() that runs the general (non-identity) kernels: before every iteration the warp field's
 * node motion is restored from the snapshot by a device copy (captured into the graph with the iteration), so each
 * iteration is the same GN iteration k of the frame (the state it was taken at). Requires nnrt_fitter_snapshot_motion
 * after the last prepare(). */
nnrt_status nnrt_fitter_iterate_from_snapshot(nnrt_fitter* fitter, nnrt_warp_field* warp_field, int32_t first_iteration, int32_t count,
                                              void* stream);
/* A whole frame fit (the FitToImage loop, :111-275) from the stored snapshot: the node motion is restored once, then
 * iterations 0 .. count-1 run (graph-captured as one sequence under the use_hip_graph policy). */
nnrt_status nnrt_fitter_fit_from_snapshot(nnrt_fitter* fitter, nnrt_warp_field* warp_field, int32_t count, void* stream);
/* Restore the warp field's node motion from the snapshot (a device copy on `stream`). */
nnrt_status nnrt_fitter_restore_motion(nnrt_fitter* fitter, nnrt_warp_field* warp_field, void* stream);
/* iterate() without graphs, with HIP events between the stages of every iteration; h_stage_ms[NNRT_TIMED_STAGES]
 * receives the average per-iteration device time of: 0 warp (+warped Jacobians), 1 raster scatter, 2 pixel pass
 * (0: fused into 3), 3 pixel + node pass (residuals, rasterized Jacobians, node Jacobians, JtJ / Jt r: one launch,
 * k_fit_pixels_fused), 4 ARAP edges, 5 linear solve + update ("ms/solve"). Synchronizes `stream`. */
#define NNRT_TIMED_STAGES 6
nnrt_status nnrt_fitter_iterate_timed(nnrt_fitter* fitter, nnrt_warp_field* warp_field, int32_t first_iteration, int32_t count,
                                      float* h_stage_ms, void* stream);
/* Per-kernel device time of one GN iteration in its real context (measurement; loop body
 * DeformableMeshToImageFitter.cpp:111-275). Four prefix sequences of `reps` iterations from the snapshot state are each
 * captured as one graph -- [warp, raster, pixel, solve], [raster, pixel, solve], [raster, pixel], [raster] -- and
 * replayed `trials` times, interleaved, between HIP events on the fitter's stream; the median per-iteration times give
 * h_kernel_ms[NNRT_KERNEL_TIMES] = 0 warp (k_warp_mesh_quad), 1 raster (k_raster_scatter_mesh), 2 fused pixel launch
 * (k_fit_pixels_fused), 3 solve + update (k_solve_update; ARAP: the whole arrowhead chain), 4 whole iteration, by
 * differences. Leaves raster keys empty, the accumulators zero and the node motion at the snapshot's one-iteration
 * result. Requires nnrt_fitter_snapshot_motion after the last prepare(). Synchronizes `stream`. */
#define NNRT_KERNEL_TIMES 5
nnrt_status nnrt_fitter_time_kernels(nnrt_fitter* fitter, nnrt_warp_field* warp_field, int32_t reps, int32_t trials, float* h_kernel_ms,
                                     void* stream);
/* Reports (and clears) a failure recorded on the device by earlier iterate() calls (e.g. a non-positive-definite block,
 * which the reference raises from potrf). Synchronizes `stream`. */
nnrt_status nnrt_fitter_check(nnrt_fitter* fitter, void* stream);
/* Diagnostics of the most recent iteration, copied to the host (any pointer may be NULL): residuals [H*W] float32,
 * residual mask [H*W] uint8, rasterized face per pixel [H*W] int32 (-1 = none), motion updates [N*s] (s = 6 for ALL,
 * 3 otherwise), negative gradient [N*s], data-term Hessian blocks [N*s*s]. Synchronizes `stream`. */
nnrt_status nnrt_fitter_get_diagnostics(nnrt_fitter* fitter, float* h_residuals, uint8_t* h_residual_mask, int32_t* h_pixel_faces,
                                        float* h_updates, float* h_negative_gradient, float* h_hessian_blocks, void* stream);
/* Once-per-frame outputs of prepare(): anchors [V,K] int32 and weights [V,K] float32 (device -> host). */
nnrt_status nnrt_fitter_get_anchors(nnrt_fitter* fitter, int32_t* h_anchors, float* h_weights, void* stream);

/* ---------------------------------------------------------------------------------------------------------------
 * Stage entry points (parity surface; all device pointers, all asynchronous on `stream`)
 * ------------------------------------------------------------------------------------------------------------- */
/* nnrt.geometry.functional.compute_anchors_and_weights_euclidean_{fixed,variable}_node_weight
 * (cpp/pybind/geometry/functional/functional.cpp:52-90 -> WarpAnchorComputationImpl.h:42-140).
 * d_node_coverage_weights == NULL -> fixed coverage. */
nnrt_status nnrt_compute_anchors_and_weights(const float* d_points, int64_t point_count, const float* d_nodes, int32_t node_count,
                                             int32_t anchor_count, float node_coverage, const float* d_node_coverage_weights,
                                             int32_t minimum_valid_anchor_count, int32_t* d_anchors, float* d_weights, void* stream);
/* WarpTriangleMeshUsingSuppliedAnchors (cpp/geometry/functional/Warping.cpp:222-264). h_E may be NULL. */
nnrt_status nnrt_warp_mesh(const float* d_vertices, const float* d_normals, int64_t vertex_count, const float* d_nodes,
                           const float* d_rotations, const float* d_translations, int32_t node_count, const int32_t* d_anchors,
                           const float* d_weights, int32_t anchor_count, const double* h_E, float* d_out_vertices,
                           float* d_out_normals, void* stream);
/* nnrt.geometry.functional.warp_triangle_mesh (both overloads, threshold_nodes_by_distance / minimum_valid_anchor_count /
 * extrinsics) and warp_point_cloud (both overloads) (cpp/pybind/geometry/functional/functional.cpp:77-111 ->
 * cpp/geometry/functional/Warping.cpp:61-264 -> Warp3dPointsAndNormalsImpl.h:33-438, WarpUtilities.h:34-580).
 * d_normals / d_out_normals may be NULL (points only). d_anchors == NULL: anchors computed over d_nodes with the fixed
 * node_coverage (the online-anchor overloads); otherwise d_anchors int32 / d_weights float32 [count, anchor_count].
 * threshold_nodes_by_distance = 0: BlendWarp over the valid slots; 1: online anchors farther than 2 * node_coverage are
 * dropped and a point with fewer than minimum_valid_anchor_count valid anchors stays (0, 0, 0) (warp_point_cloud always
 * thresholds). h_E: float64[16] or NULL (identity). Outputs [count,3]. */
nnrt_status nnrt_warp_points(const float* d_points, const float* d_normals, int64_t count, const float* d_nodes, const float* d_rotations,
                             const float* d_translations, int32_t node_count, const int32_t* d_anchors, const float* d_weights,
                             int32_t anchor_count, float node_coverage, int32_t threshold_nodes_by_distance,
                             int32_t minimum_valid_anchor_count, const double* h_E, float* d_out_points, float* d_out_normals, void* stream);
/* nnrt.geometry.functional.compute_point_to_plane_distances(mesh1, mesh2 | point_cloud) (functional.cpp:118-125 ->
 * PointToPlaneDistances.cpp:25-90, kernel PointToPlaneDistancesImpl.h:26-50): d_out [count] = n1 . (v1 - v2). */
nnrt_status nnrt_compute_point_to_plane_distances(const float* d_normals1, const float* d_vertices1, const float* d_vertices2, int64_t count,
                                                  float* d_out, void* stream);
/* nnrt.geometry.functional.unproject_raster_depth_without_filtering(depth, intrinsics, extrinsics, depth_scale, depth_max,
 * preserve_pixel_layout) (functional.cpp:128-140 -> PerspectiveProjection.cpp:26-39, PerspectiveProjectionImpl.h:60-146):
 * depth uint16 (NNRT_DTYPE_UINT16) or float32 (NNRT_DTYPE_FLOAT32) [H,W]; points [H*W,3] in the frame of
 * extrinsics^-1 (h_E float64[16] or NULL = identity), zero where rejected; d_mask uint8 [H*W]. The pixel layout of the
 * outputs is the same either way (preserve_pixel_layout is a shape, [H,W,3] vs [H*W,3]). */
nnrt_status nnrt_unproject_depth_image(const void* d_depth, int32_t depth_dtype, int32_t height, int32_t width, const double* h_K,
                                       const double* h_E, float depth_scale, float depth_max, float* d_points, uint8_t* d_mask, void* stream);
/* nnrt.rendering.functional.get_mesh_ndc_face_vertices_and_clip_mask([meshes], ...) (cpp/pybind/rendering/functional/
 * functional.cpp:36-44 -> ExtractFaceVertices.cpp:87-126): the meshes' faces concatenated in mesh order; h_vertex_sets /
 * h_face_sets are HOST arrays of mesh_count DEVICE pointers, h_face_counts the per-mesh face counts (the reference's
 * face_counts output). d_face_ndc [sum F,3,3], d_clip_mask [sum F]. */
nnrt_status nnrt_get_meshes_ndc_face_vertices_and_clip_mask(const float* const* h_vertex_sets, const int64_t* const* h_face_sets,
                                                            const int64_t* h_face_counts, int32_t mesh_count, const double* h_K,
                                                            int32_t height, int32_t width, float near_clip, float far_clip,
                                                            float* d_face_ndc, uint8_t* d_clip_mask, void* stream);
/* nnrt.rendering.functional.get_mesh_ndc_face_vertices_and_clip_mask (cpp/rendering/functional/ExtractFaceVertices.cpp:56-85).
 * d_face_ndc [F,3,3], d_clip_mask [F] uint8 (1 = keep). */
nnrt_status nnrt_get_mesh_ndc_face_vertices_and_clip_mask(const float* d_vertices, const int64_t* d_faces, int64_t face_count,
                                                          const double* h_K, int32_t height, int32_t width, float near_clip,
                                                          float far_clip, float* d_face_ndc, uint8_t* d_clip_mask, void* stream);
/* nnrt.rendering.rasterize_ndc_triangles (cpp/pybind/rendering/rendering.cpp:36-43 -> RasterizeNdcTriangles.cpp:33-129).
 * Outputs fragments: face [H,W,Kf] int64 (-1), depth [H,W,Kf], barycentrics [H,W,Kf,3], signed distance [H,W,Kf]
 * (-1 fill). d_clip_mask may be NULL. bin_size / max_faces_per_bin are accepted for signature parity; the MI355X
 * rasterizer does not need coarse bins (faces_per_pixel == 1: per-face scatter with a (depth, face) 64-bit atomic
 * minimum; faces_per_pixel > 1: per-pixel lists of the faces covering the pixel centre, replayed in ascending face
 * order through the reference's bounded queue). */
nnrt_status nnrt_rasterize_ndc_triangles(const float* d_face_ndc, const uint8_t* d_clip_mask, int64_t face_count, int32_t height,
                                         int32_t width, float blur_radius_pixels, int32_t faces_per_pixel, int32_t bin_size,
                                         int32_t max_faces_per_bin, int32_t perspective_correct_barycentric_coordinates,
                                         int32_t clip_barycentric_coordinates, int32_t cull_back_faces, int64_t* d_pixel_faces,
                                         float* d_pixel_depths, float* d_pixel_barycentrics, float* d_pixel_face_distances,
                                         void* stream);
/* nnrt.rendering.functional.interpolate_vertex_attributes (InterpolateFaceAttributesImpl.h:30-75): [H,W,Kf,C] */
nnrt_status nnrt_interpolate_face_attributes(const int64_t* d_pixel_faces, const float* d_barycentrics, int64_t pixel_count,
                                             int32_t faces_per_pixel, const float* d_face_attributes, int32_t channels,
                                             float* d_out, void* stream);
/* nnrt.geometry.functional.unproject_raster_depth_without_filtering (PerspectiveProjectionImpl.h:60-146), float32 depth */
nnrt_status nnrt_unproject_depth(const float* d_depth, int32_t height, int32_t width, const double* h_K, float depth_scale,
                                 float depth_max, float* d_points, uint8_t* d_mask, void* stream);
/* nnrt.backproject_depth_ushort(image_in, point_image_out, fx, fy, cx, cy, normalizer) (cpp/pybind/nnrt_pybind.cpp:52-57,
 * cpp/cpu/image_proc.cpp:275-302): uint16 depth [H,W] -> ordered point image d_points [H,W,3]; depth = d / normalizer,
 * (depth*(x-cx)/fx, depth*(y-cy)/fy, depth), zeros where depth <= 0 (the reference leaves those entries as allocated). */
nnrt_status nnrt_backproject_depth_ushort(const uint16_t* d_depth, int32_t height, int32_t width, float fx, float fy, float cx, float cy,
                                          float normalizer, float* d_points, void* stream);
/* nnrt.backproject_depth_float(image_in, point_image_out, fx, fy, cx, cy) (nnrt_pybind.cpp:66-67, image_proc.cpp:312-339): float
 * depth in metres [H,W] -> [H,W,3], as above with normalizer 1. */
nnrt_status nnrt_backproject_depth_float(const float* d_depth, int32_t height, int32_t width, float fx, float fy, float cx, float cy,
                                         float* d_points, void* stream);
/* nnrt.geometry.functional.compute_triangle_normals(mesh, normalized=True) (cpp/geometry/functional/NormalsOperations.cpp:36-46,
 * kernel NormalsOperationsImpl.h:39-68): d_out [F,3] = (v1 - v0) x (v2 - v0), optionally normalized (zero stays zero,
 * NaN -> (0,0,1)) */
nnrt_status nnrt_compute_triangle_normals(const float* d_vertices, int64_t vertex_count, const int64_t* d_faces, int64_t face_count,
                                          int32_t normalized, float* d_out, void* stream);
/* nnrt.geometry.functional.compute_vertex_normals(mesh, normalized=True) (NormalsOperations.cpp:52-66, kernel :95-166): sum of the
 * unnormalized incident triangle normals, in ascending face order (the reference's serial order; its CUDA path uses
 * unordered atomics), optionally normalized. Synchronizes `stream`. */
nnrt_status nnrt_compute_vertex_normals(const float* d_vertices, int64_t vertex_count, const int64_t* d_faces, int64_t face_count,
                                        int32_t normalized, float* d_out, void* stream);
/* nnrt.geometry.functional.compute_ordered_point_cloud_normals(point_cloud, source_image_size) (NormalsOperations.cpp:74-95,
 * kernel NormalsOperationsImpl.h:170-214): organized [H*W,3] points -> [H*W,3] normals facing the camera, 0 on the border */
nnrt_status nnrt_compute_ordered_point_cloud_normals(const float* d_points, int64_t point_count, int32_t height, int32_t width, float* d_out,
                                                     void* stream);
/* nnrt.core.matmul3d(array_of_matrices_a, array_of_matrices_b) (cpp/pybind/core/core.cpp:32 -> cpp/core/linalg/Matmul3D.cpp:25-83):
 * d_c [batch, m, n] = d_a [batch, m, k] x d_b [batch, k, n] per batch entry, float32 row-major (n = 1: array of vectors). */
nnrt_status nnrt_matmul3d(const float* d_a, const float* d_b, int64_t batch, int32_t m, int32_t k, int32_t n, float* d_c, void* stream);
/* nnrt.geometry.functional.median_grid_subsample_3d_points(points, grid_cell_size) (functional.cpp:152-153 ->
 * GeometrySampling.cpp:62-68, GeometrySamplingMedian.h:264-296): indices of one medoid per occupied grid cell, in ascending
 * index order (the reference's order is its hash map's bin order). d_out_indices needs room for point_count int64;
 * *h_sample_count receives the number written. Synchronizes `stream`. */
nnrt_status nnrt_median_grid_subsample_3d_points(const float* d_points, int64_t point_count, float grid_cell_size, int64_t* d_out_indices,
                                                 int64_t* h_sample_count, void* stream);
/* nnrt.core.linalg AxisAngleVectorsToMatricesRodrigues (cpp/core/linalg/RodriguesImpl.h:66-88) */
nnrt_status nnrt_axis_angle_to_matrices_rodrigues(const float* d_vectors, int32_t count, float* d_matrices, void* stream);
/* SolveBlockDiagonalCholesky (cpp/core/linalg/SolveBlockDiagonalCholesky.cpp): x_i = A_i^-1 b_i, block size 3 or 6 */
nnrt_status nnrt_solve_block_diagonal_cholesky(const float* d_blocks, const float* d_b, int32_t block_count, int32_t block_size,
                                               float* d_x, void* stream);
/* InvertPositiveSemidefiniteBlocks (cpp/core/linalg/InvertBlocks.cpp:82-126: potrf + potrs against the identity per
 * block), block size 3 or 6, row-major [count, s, s] -> [count, s, s]; the arrowhead stem's D^-1 runs the same device
 * functions. NNRT_ERROR_NOT_POSITIVE_DEFINITE if a block's potrf fails (its output is NaN). */
nnrt_status nnrt_invert_positive_semidefinite_blocks(const float* d_blocks, int32_t block_count, int32_t block_size, float* d_out,
                                                     void* stream);
/* ---- block-sparse stages of the arrowhead solve (SolveBlockSparseArrowheadCholesky.cpp:30-95, SchurComplement.cpp:43-78),
 * standalone; row-major [count, s, s] float blocks, int32 [count, 2] block coordinates (row, column). Coordinates outside
 * the matrix / vector give NNRT_ERROR_ARGUMENT (the reference does not check them). ---- */
/* MatmulBlockSparseRowWisePadded (cpp/core/linalg/MatmulBlockSparse.h; MatmulBlockSparseImpl.h:39-157): c_i = a[row_i] b_i;
 * blocks whose row has no A block (row >= a_block_count) are zero with mask 0. MatmulBlockSparseRowWise = the mask-1 blocks
 * and their coordinates. */
nnrt_status nnrt_matmul_block_sparse_row_wise(const float* d_a_blocks, int32_t a_block_count, const float* d_b_blocks,
                                              const int32_t* d_b_coordinates, int32_t b_block_count, int32_t block_size, float* d_c_blocks,
                                              uint8_t* d_c_mask, void* stream);
/* MatmulBlockSparse (MatmulBlockSparseImpl.h:160-439): op(A) op(B) with int16 breadboards [block rows, block columns]
 * holding block indices (-1 = empty); op = transpose when transpose_x != 0. Output: d_c_blocks [out_rows * out_cols, s, s]
 * in row-major block order and d_c_mask (1 = some block pair contributes); the reference returns the mask-1 blocks and
 * their (row, column) coordinates. */
nnrt_status nnrt_matmul_block_sparse(const float* d_a_blocks, int32_t a_block_count, const int16_t* d_a_breadboard, int32_t a_block_rows,
                                     int32_t a_block_columns, int32_t transpose_a, const float* d_b_blocks, int32_t b_block_count,
                                     const int16_t* d_b_breadboard, int32_t b_block_rows, int32_t b_block_columns, int32_t transpose_b,
                                     int32_t block_size, float* d_c_blocks, uint8_t* d_c_mask, void* stream);
/* BlockSparseAndVectorProduct (MatmulBlockSparseImpl.h:441-602): out [m] = op(A) v, A given by blocks at coordinates + the
 * (row, column) block offset; transpose places block (i, j) at (j, i) transposed. d_out must not overlap d_vector
 * (NNRT_ERROR_ARGUMENT). */
nnrt_status nnrt_block_sparse_and_vector_product(const float* d_blocks, const int32_t* d_coordinates, int32_t block_count, int32_t block_size,
                                                 int32_t block_row_offset, int32_t block_column_offset, int32_t transpose,
                                                 const float* d_vector, int64_t vector_length, int64_t m, float* d_out, void* stream);
/* DiagonalBlockSparseAndVectorProduct (MatmulBlockSparseImpl.h:604-690): out_i = D_i v_i, [count * s] */
nnrt_status nnrt_diagonal_block_sparse_and_vector_product(const float* d_blocks, int32_t block_count, int32_t block_size, const float* d_vector,
                                                          float* d_out, void* stream);
/* FillInSparseBlocks / AddSparseBlocks / SubtractSparseBlocks (SparseBlocksImpl.h:30-190), op 0 / 1 / 2, into a row-major
 * [rows, columns] matrix; d_coordinates == NULL: block i at (i, i) (FillInDiagonalBlocks, DiagonalBlocksImpl.h). Add and
 * subtract are atomic; a fill with repeated coordinates keeps one of the blocks, unspecified which (the reference's
 * ParallelFor races the same way). */
nnrt_status nnrt_sparse_blocks_op(float* d_matrix, int64_t rows, int64_t columns, const float* d_blocks, const int32_t* d_coordinates,
                                  int32_t block_count, int32_t block_size, int64_t block_row_offset, int64_t block_column_offset,
                                  int32_t transpose, int32_t op, void* stream);
/* GetSparseBlocks (SparseBlocksImpl.h:192-230); d_coordinates == NULL: GetDiagonalBlocks */
nnrt_status nnrt_get_sparse_blocks(const float* d_matrix, int64_t rows, int64_t columns, int32_t block_size, const int32_t* d_coordinates,
                                   int32_t block_count, float* d_blocks, void* stream);
/* TransposeBlocksInPlace (TransposeBlocks.h) */
nnrt_status nnrt_transpose_blocks_in_place(float* d_blocks, int32_t block_count, int32_t block_size, void* stream);
/* InvertTriangularBlocks (InvertBlocks.cpp, trtri per block), upper != 0: UpLoTriangular::UPPER; a zero diagonal entry
 * gives NNRT_ERROR_NOT_POSITIVE_DEFINITE (trtri info > 0). d_out must not overlap d_blocks (NNRT_ERROR_ARGUMENT). */
nnrt_status nnrt_invert_triangular_blocks(const float* d_blocks, int32_t block_count, int32_t block_size, int32_t upper, float* d_out,
                                          void* stream);
/* SolveBlockSparseArrowheadCholesky (cpp/core/linalg/SolveBlockSparseArrowheadCholesky.cpp:30-95), 6x6 blocks:
 * d_diagonal_blocks [N,6,6], d_wing_blocks [E,6,6] at block coordinates d_wing_coordinates [E,2] (row < arrow_base
 * <= column for stem-to-corner blocks; row >= arrow_base for corner off-diagonal blocks), b [6N]. Coordinates outside
 * [0, N), a diagonal coordinate (row == column) or a column inside the stem (column < arrow_base) give
 * NNRT_ERROR_ARGUMENT, checked before any allocation. The Schur corner is factored tile-sparse (nested-dissection order
 * of the corner blocks); its size is bounded by device memory only. The structure-derived plan (stem lists, corner plan,
 * scratch) of the 4 most recently solved wing structures is kept per process and reused by a later call with the same
 * device, block count, arrow base and coordinates (one call owns a plan at a time; calls synchronise their stream
 * before returning it); nnrt_release_arrowhead_plans frees them. */
nnrt_status nnrt_solve_block_sparse_arrowhead_cholesky(const float* d_diagonal_blocks, const float* d_wing_blocks,
                                                       const int32_t* d_wing_coordinates, int32_t wing_block_count,
                                                       int32_t diagonal_block_count, int32_t arrow_base_block_index,
                                                       const float* d_b, float* d_x, void* stream);
/* Frees the arrowhead plans kept by nnrt_solve_block_sparse_arrowhead_cholesky (device memory; none is in use by a
 * concurrent call: plans being solved with are not in the pool). */
void nnrt_release_arrowhead_plans(void);

/* ---- TSDF voxel block grid (NonRigidSurfaceVoxelBlockGrid, cpp/geometry/NonRigidSurfaceVoxelBlockGrid.h:30-65 over
 * VoxelBlockGrid, cpp/geometry/VoxelBlockGrid.h; Python: nnrt.geometry.NonRigidSurfaceVoxelBlockGrid, pybind
 * cpp/pybind/geometry/geometry.cpp:61-275). Attributes tsdf (float32), weight (float32 | uint16), color (none |
 * float32 | uint16 | uint8, 3 channels). Block coordinates are int32 [n,3]; images are device arrays: depth [H,W]
 * uint16 or float32, color [Hc,Wc,3] uint8 (uint16 depth) or float32 (float32 depth, [0,1]); intrinsics double[9],
 * extrinsics double[16] (NULL: identity). Functions producing a variable-size result return its size and keep it in
 * the grid until the matching copy_* call (the grid owns the workspace). ---- */
typedef struct nnrt_voxel_grid nnrt_voxel_grid;
#define NNRT_DTYPE_NONE -1
#define NNRT_DTYPE_FLOAT32 0
#define NNRT_DTYPE_UINT16 1
#define NNRT_DTYPE_UINT8 2
/* VoxelBlockGrid(attr_names, attr_dtypes, attr_channels, voxel_size, block_resolution, block_count, device)
 * (VoxelBlockGrid.h:52-58); storage grows (x2) past block_count as Open3D's hash map does. */
nnrt_status nnrt_voxel_grid_create(float voxel_size, int32_t block_resolution, int64_t block_count, int32_t weight_dtype,
                                   int32_t color_dtype, int32_t device, nnrt_voxel_grid** out);
void nnrt_voxel_grid_destroy(nnrt_voxel_grid* grid);
nnrt_status nnrt_voxel_grid_get_info(const nnrt_voxel_grid* grid, int64_t* h_active_blocks, int64_t* h_capacity, float* h_voxel_size,
                                     int32_t* h_block_resolution);
/* hashmap().activate(block_coords) (Open3D HashMap::Activate); new blocks start at zero */
nnrt_status nnrt_voxel_grid_activate(nnrt_voxel_grid* grid, const int32_t* d_block_coords, int64_t count, void* stream);
/* active block coordinates [active,3] in buffer order (ExtractVoxelBlockCoordinates before its metric scaling,
 * NonRigidSurfaceVoxelBlockGrid.cpp:186-191) */
nnrt_status nnrt_voxel_grid_get_block_coordinates(const nnrt_voxel_grid* grid, int32_t* d_out, void* stream);
/* GetUniqueBlockCoordinates(depth, intrinsic, extrinsic, depth_scale, depth_max, trunc_voxel_multiplier)
 * (VoxelBlockGrid.cpp:237-270, Open3D DepthTouch); result -> nnrt_voxel_grid_copy_result_coordinates */
nnrt_status nnrt_voxel_grid_unique_block_coordinates(nnrt_voxel_grid* grid, const void* d_depth, int32_t depth_dtype, int32_t height,
                                                     int32_t width, const double* h_K, const double* h_E, float depth_scale,
                                                     float depth_max, float trunc_voxel_multiplier, int64_t* h_count, void* stream);
nnrt_status nnrt_voxel_grid_copy_result_coordinates(const nnrt_voxel_grid* grid, int32_t* d_out, void* stream);
/* Integrate(block_coords, depth, color, depth_intrinsic, color_intrinsic, extrinsic, depth_scale, depth_max,
 * trunc_voxel_multiplier) (VoxelBlockGrid.cpp:317-350, Open3D voxel_grid::Integrate); d_color may be NULL */
nnrt_status nnrt_voxel_grid_integrate(nnrt_voxel_grid* grid, const int32_t* d_block_coords, int64_t count, const void* d_depth,
                                      int32_t depth_dtype, int32_t height, int32_t width, const void* d_color, int32_t color_height,
                                      int32_t color_width, const double* h_depth_K, const double* h_color_K, const double* h_E,
                                      float depth_scale, float depth_max, float trunc_voxel_multiplier, void* stream);
/* IntegrateNonRigid(block_coords, warp_field, depth, color, depth_normals, depth_intrinsics, color_intrinsics,
 * extrinsics, depth_scale, depth_max, truncation_voxel_multiplier) -> cos_voxel_ray_to_normal [H,W]
 * (NonRigidSurfaceVoxelBlockGrid.cpp:33-66, NonRigidSurfaceVoxelBlockGridImpl.h:52-229); d_depth_normals [H,W,3] */
nnrt_status nnrt_voxel_grid_integrate_non_rigid(nnrt_voxel_grid* grid, const int32_t* d_block_coords, int64_t count,
                                                const nnrt_warp_field* warp_field, const void* d_depth, int32_t depth_dtype,
                                                int32_t height, int32_t width, const void* d_color, int32_t color_height,
                                                int32_t color_width, const float* d_depth_normals, const double* h_depth_K,
                                                const double* h_color_K, const double* h_E, float depth_scale, float depth_max,
                                                float trunc_voxel_multiplier, float* d_cos_out, void* stream);
/* ExtractVoxelValuesAndCoordinates (NonRigidSurfaceVoxelBlockGrid.cpp:168-184): d_out [active * res^3, C], rows
 * (x, y, z, tsdf, weight[, r, g, b]), C = 5 or 8 (h_channels) */
nnrt_status nnrt_voxel_grid_extract_voxel_values_and_coordinates(const nnrt_voxel_grid* grid, float* d_out, int32_t* h_channels,
                                                                 void* stream);
/* ExtractVoxelValuesAt(query_voxel_coordinates) (NonRigidSurfaceVoxelBlockGrid.cpp:193-224): rows of the queries whose
 * block is active -> nnrt_voxel_grid_copy_result_rows */
nnrt_status nnrt_voxel_grid_extract_voxel_values_at(nnrt_voxel_grid* grid, const int32_t* d_query, int64_t count, int64_t* h_rows,
                                                    int32_t* h_channels, void* stream);
nnrt_status nnrt_voxel_grid_copy_result_rows(const nnrt_voxel_grid* grid, float* d_out, void* stream);
/* GetBoundingBoxesOfWarpedBlocks(block_keys, warp_field, extrinsics) (NonRigidSurfaceVoxelBlockGrid.cpp:113-124):
 * d_boxes [n,6] (min xyz, max xyz) */
nnrt_status nnrt_voxel_grid_warped_block_boxes(const nnrt_voxel_grid* grid, const int32_t* d_block_keys, int64_t count,
                                               const nnrt_warp_field* warp_field, const double* h_E, float* d_boxes, void* stream);
/* GetAxisAlignedBoxesInterceptingSurfaceMask (NonRigidSurfaceVoxelBlockGridImpl.h:359-437): d_mask [n] uint8 */
nnrt_status nnrt_boxes_intersecting_surface_mask(const float* d_boxes, int64_t count, const void* d_depth, int32_t depth_dtype,
                                                 int32_t height, int32_t width, const double* h_K, float depth_scale, float depth_max,
                                                 int32_t stride, float truncation_distance, uint8_t* d_mask, void* stream);
/* FindBlocksIntersectingTruncationRegion(depth, warp_field, intrinsics, extrinsics, depth_scale, depth_max,
 * truncation_voxel_multiplier) (NonRigidSurfaceVoxelBlockGrid.cpp:141-166) -> nnrt_voxel_grid_copy_result_coordinates */
nnrt_status nnrt_voxel_grid_find_blocks_intersecting_truncation_region(nnrt_voxel_grid* grid, const void* d_depth, int32_t depth_dtype,
                                                                       int32_t height, int32_t width, const nnrt_warp_field* warp_field,
                                                                       const double* h_K, const double* h_E, float depth_scale,
                                                                       float depth_max, float trunc_voxel_multiplier, int64_t* h_count,
                                                                       void* stream);
/* ActivateSleeveBlocks() (NonRigidSurfaceVoxelBlockGrid.cpp:98-109): returns the inactive-neighbour count */
nnrt_status nnrt_voxel_grid_activate_sleeve_blocks(nnrt_voxel_grid* grid, int64_t* h_count, void* stream);
/* ExtractTriangleMesh(weight_threshold, estimated_vertex_number) (VoxelBlockGrid.cpp:461-497, Open3D marching cubes)
 * -> counts; then nnrt_voxel_grid_copy_mesh: vertices [V,3], normals [V,3], colors [V,3] in [0,1] (may be NULL),
 * triangles int64 [T,3] */
nnrt_status nnrt_voxel_grid_extract_triangle_mesh(nnrt_voxel_grid* grid, float weight_threshold, int64_t* h_vertex_count,
                                                  int64_t* h_triangle_count, void* stream);
nnrt_status nnrt_voxel_grid_copy_mesh(const nnrt_voxel_grid* grid, float* d_vertices, float* d_normals, float* d_colors,
                                      int64_t* d_triangles, void* stream);
/* the marching-cubes tables (host): tri [256][31] int8 edge triples in emission order (-1 terminated; the published
 * Lorensen-Cline / Bourke table Open3D indexes, each triangle (a, b, c) emitted as (c, b, a), Open3D's slot 2 - v), edge mask [256] */
nnrt_status nnrt_marching_cubes_table(int8_t* h_tri, uint16_t* h_edge_mask);

#ifdef __cplusplus
}
#endif

#endif /* NNRT_MI355X_H */
