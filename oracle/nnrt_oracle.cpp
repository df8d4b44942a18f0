// =====================================================================================================================
// nnrt_oracle.cpp -- TEST INFRASTRUCTURE ONLY (parity oracle + CPU baseline). NOT PART OF THE PRODUCT PATH.
//
// A plain C++17 / OpenMP restatement of the reference's DeformableMeshToImageFitter hot path
// (henry123-boy/Dynamicfuion_python, cpp/alignment/DeformableMeshToImageFitter.cpp:85-448) and of every kernel it calls.
// Each function cites the reference file:line whose semantics it follows. Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg may load this library; the HIP product path never links or calls it.
//
// Parity pinning: see oracle/README.md and DESIGN.md section "Oracle". The reference C++ cannot be compiled here
// (needs Open3D 0.17, Eigen master, MKL), so this restatement is pinned by the reference's own known-answer tests and
// fixtures (tests/golden/*) and by golden vectors generated from the importable numpy reference script
// math_check_scripts/dense_depth_jacobians.py (tests/golden/make_golden.py).
//
// Deterministic policies where the reference is order-nondeterministic (atomics, hash maps), all documented in DESIGN.md:
//   * rasterizer ties: lexicographic (depth, face index) -- the reference's own operator< (RayFaceIntersection.h:42-45);
//   * node->pixel Jacobian lists: ascending (pixel, face-anchor slot) order, no 4000 cap (A4);
//   * median-grid subsample: points of a bin visited in ascending index; coarse-layer sample in ascending node index.
// Floating-point expression order follows the Eigen expressions in the reference; build with -ffp-contract=off.
// =====================================================================================================================
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <numeric>
#include <string>
#include <tuple>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

#define ORC_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr float K_EPSILON = 1e-8f;            // cpp/rendering/kernel/RasterizationConstants.h:24
constexpr int MAX_POINTS_PER_PIXEL = 8;       // RasterizationConstants.h:20
constexpr int MAX_BINS_ALONG_IMAGE_DIMENSION = 22;  // RasterizationConstants.h:26
constexpr int MAX_ANCHOR_COUNT = 8;           // cpp/geometry/functional/kernel/Defines.h

thread_local std::string g_error;

inline float dot3(const float* a, const float* b) { return (a[0] * b[0] + a[1] * b[1]) + a[2] * b[2]; }
inline void matvec3(const float* R, const float* v, float* o) {
	float r0 = (R[0] * v[0] + R[1] * v[1]) + R[2] * v[2];
	float r1 = (R[3] * v[0] + R[4] * v[1]) + R[5] * v[2];
	float r2 = (R[6] * v[0] + R[7] * v[1]) + R[8] * v[2];
	o[0] = r0; o[1] = r1; o[2] = r2;
}
// row-vector r times skew(a) == r x a  (Eigen::SkewSymmetricMatrix3 convention [a]_x b = a x b)
inline void row_times_skew(const float* r, const float* a, float* o) {
	o[0] = r[1] * a[2] - r[2] * a[1];
	o[1] = r[2] * a[0] - r[0] * a[2];
	o[2] = r[0] * a[1] - r[1] * a[0];
}
inline float fmin3f(float a, float b, float c) { return fminf(fminf(a, b), c); }
inline float fmax3f(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }
inline float saturatef(float x) { return fminf(fmaxf(x, 0.f), 1.f); }
// float transcendentals evaluated in double and rounded once (correctly rounded except for double-rounding ties), so
// the host restatement and the gfx950 kernels agree bit-for-bit; within 1 ulp of the reference's expf/sinf/cosf.
inline float exp_cr(float x) { return static_cast<float>(std::exp(static_cast<double>(x))); }
inline float sin_cr(float x) { return static_cast<float>(std::sin(static_cast<double>(x))); }
inline float cos_cr(float x) { return static_cast<float>(std::cos(static_cast<double>(x))); }

// ---- cpp/rendering/kernel/CoordinateSystemConversions.h:45-73 ----
inline float GetNdcRange(int d1, int d2) {
	float range = 2.0f;
	if (d1 > d2) range = (static_cast<float>(d1) * range) / static_cast<float>(d2);
	return range;
}
inline float PixelToNdc(int i, int d1, int d2) {
	float range = GetNdcRange(d1, d2);
	const float offset = (range / 2.0f);
	return -offset + (range * static_cast<float>(i) + offset) / static_cast<float>(d1);
}

struct NdcCamera {   // TransformIndexer with float intrinsics (Open3D t/geometry/kernel/GeometryIndexer.h)
	float fx, fy, cx, cy;
	void Project(float x, float y, float z, float* u, float* v) const {
		float inv_z = 1.0f / z;
		*u = fx * x * inv_z + cx;
		*v = fy * y * inv_z + cy;
	}
};
struct Box2 { float min_x, max_x, min_y, max_y;   // cpp/geometry/kernel/AxisAlignedBoundingBox.h:24-33
	bool Contains(float x, float y) const { return y >= min_y && x >= min_x && y <= max_y && x <= max_x; } };

// ---- CoordinateSystemConversions.h:109-146 ImageSpaceIntrinsicsToNdc ----
// g_ndc_consistent (set by orc_fit for the fitter's NNRT_NDC_CONSISTENT option, a deliberate divergence from the reference):
// pixel (u, v) of K lands on the centre of raster pixel (u, v) instead of the reference's y-mirrored placement (A11), and
// the clip window is the image itself.
static bool g_ndc_consistent = false;   // orc_fit is not re-entrant; read inside its OpenMP regions
void IntrinsicsToNdc(const double* K, int H, int W, double* ndcK, Box2* range) {
	double fx = K[0], fy = K[4], cx = K[2], cy = K[5];
	double height = H, width = W;
	double s = std::min(width, height);
	float range_x = GetNdcRange(W, H);
	float range_y = GetNdcRange(H, W);
	double fx_ndc = 2.0 * fx / s;
	double fy_ndc = (g_ndc_consistent ? 2.0 : -2.0) * fy / s;
	double cx_ndc = g_ndc_consistent ? (2.0 * cx + 1.0 - width) / s : -(2.0 * cx - width) / s;
	double cy_ndc = g_ndc_consistent ? (2.0 * cy + 1.0 - height) / s : (2.0 * cy - height) / s;
	double m[9] = {fx_ndc, 0.0, cx_ndc, 0.0, fy_ndc, cy_ndc, 0.0, 0.0, 1.0};
	std::memcpy(ndcK, m, sizeof(m));
	double wx = g_ndc_consistent ? 0.0 : cx_ndc, wy = g_ndc_consistent ? 0.0 : cy_ndc;
	range->min_x = static_cast<float>(wx - range_x / 2.f);
	range->max_x = static_cast<float>(wx + range_x / 2.f);
	range->min_y = static_cast<float>(wy - range_y / 2.f);
	range->max_y = static_cast<float>(wy + range_y / 2.f);
}

inline float SPA_CW(float px, float py, float v0x, float v0y, float v1x, float v1y) {
	// cpp/rendering/functional/kernel/BarycentricCoordinates.h:35-47 (ClockWise)
	return (px - v0x) * (v0y - v1y) - (py - v0y) * (v0x - v1x);
}

} // namespace

ORC_API const char* orc_last_error() { return g_error.c_str(); }

ORC_API int orc_num_threads() {
#ifdef _OPENMP
	return omp_get_max_threads();
#else
	return 1;
#endif
}

ORC_API void orc_set_num_threads(int n) {
#ifdef _OPENMP
	omp_set_num_threads(n);
#else
	(void) n;
#endif
}

// =====================================================================================================================
// Anchors: cpp/geometry/functional/kernel/WarpAnchorComputationImpl.h:42-140, WarpUtilities.h:34-247,
//          cpp/core/kernel/KnnUtilities.h:64-117 (brute-force replace-max K-NN in ascending node order)
// =====================================================================================================================
namespace {
void KnnBruteForce(const float* p, const float* nodes, int N, int K, int32_t* idx, float* d2) {
	for (int k = 0; k < K; k++) d2[k] = INFINITY;
	int max_at = 0;
	float maxd = INFINITY;
	for (int i = 0; i < N; i++) {
		const float* q = nodes + 3 * i;
		float dx = q[0] - p[0], dy = q[1] - p[1], dz = q[2] - p[2];
		float sq = (dx * dx + dy * dy) + dz * dz;
		if (sq < maxd) {
			d2[max_at] = sq;
			idx[max_at] = i;
			max_at = 0;
			maxd = d2[0];
			for (int j = 1; j < K; j++) {
				if (d2[j] > maxd) { max_at = j; maxd = d2[j]; }
			}
		}
	}
}
void NormalizeAnchorWeights(float* w, float sum, int K, int valid) {
	if (sum > 0.0f) {
		for (int k = 0; k < K; k++) w[k] /= sum;
	} else if (valid > 0) {
		for (int k = 0; k < K; k++) w[k] = 1.0f / static_cast<float>(valid);
	}
}
} // namespace

// node_weights == nullptr -> FIXED_NODE_COVERAGE (c^2 = coverage^2), else MINIMAL_K_NEIGHBOR_NODE_DISTANCE (c^2 = node_weights[n])
// threshold: FindAnchorsAndWeightsForPoint_Euclidean_Threshold_* (the anchor API thresholds iff minimum_valid_anchor_count > 0,
// kernel/WarpAnchorComputation.cpp; WarpTriangleMesh with threshold_nodes_by_distance thresholds at any minimum, Warping.cpp:198-213)
ORC_API void orc_compute_anchors_ex(const float* points, int64_t V, const float* nodes, int N, int K, float coverage,
                                    const float* node_weights, int threshold, int minimum_valid_anchor_count, int32_t* anchors,
                                    float* weights);
ORC_API void orc_compute_anchors(const float* points, int64_t V, const float* nodes, int N, int K, float coverage,
                                 const float* node_weights, int minimum_valid_anchor_count, int32_t* anchors, float* weights) {
	orc_compute_anchors_ex(points, V, nodes, N, K, coverage, node_weights, minimum_valid_anchor_count > 0, minimum_valid_anchor_count, anchors,
	                       weights);
}

ORC_API void orc_compute_anchors_ex(const float* points, int64_t V, const float* nodes, int N, int K, float coverage,
                                    const float* node_weights, int threshold, int minimum_valid_anchor_count, int32_t* anchors,
                                    float* weights) {
	float c2_fixed = coverage * coverage;
#pragma omp parallel for schedule(static)
	for (int64_t v = 0; v < V; v++) {
		int32_t* a = anchors + v * K;
		float* w = weights + v * K;
		for (int k = 0; k < K; k++) a[k] = -1;
		KnnBruteForce(points + 3 * v, nodes, N, K, a, w);   // weights array holds squared distances first
		float sum = 0.f;
		int valid = 0;
		if (threshold) {
			for (int k = 0; k < K; k++) {
				float sq = w[k];
				float c2 = node_weights ? (a[k] >= 0 ? node_weights[a[k]] : 1.f) : c2_fixed;   // empty slot (N < K): fails the test
				if (sq > 4 * c2) { a[k] = -1; continue; }
				float wt = exp_cr(-sq / (2 * c2));
				sum += wt;
				w[k] = wt;
				valid++;
			}
			if (valid < minimum_valid_anchor_count) continue;   // WarpUtilities.h:242-244 (weights left un-normalized)
			NormalizeAnchorWeights(w, sum, K, valid);
		} else {
			for (int k = 0; k < K; k++) {
				float sq = w[k];
				float c2 = node_weights ? (a[k] >= 0 ? node_weights[a[k]] : 1.f) : c2_fixed;   // empty slot: exp(-inf) = 0
				float wt = exp_cr(-sq / (2 * c2));
				sum += wt;
				w[k] = wt;
			}
			NormalizeAnchorWeights(w, sum, K, K);
		}
	}
}

// cpp/geometry/WarpField.cpp:249-263 : squared distance to the nearest *other* node (2-NN incl. self)
ORC_API void orc_node_coverage_weights(const float* nodes, int N, float coverage, float* out) {
	if (N == 1) { out[0] = coverage; return; }
	for (int i = 0; i < N; i++) {
		int32_t idx[2] = {-1, -1};
		float d2[2];
		KnnBruteForce(nodes + 3 * i, nodes, N, 2, idx, d2);
		// sorted K-NN: second-smallest distance
		float second = std::max(d2[0], d2[1]);
		float d = sqrtf(second);
		out[i] = d * d;
	}
}

// =====================================================================================================================
// Hierarchy: cpp/geometry/HierarchicalGraphWarpField.cpp:74-199; median grid subsample
// cpp/geometry/functional/kernel/GeometrySamplingMedian.h:260-290 + GeometrySamplingGridBinning.h:27-46;
// edges cpp/geometry/kernel/HierarchicalGraphWarpFieldImpl.h:218-297 (flip_source_order = true).
// Outputs: virtual_node_indices[N] (virtual -> original), layer_counts[layer_count], edges[E,2] (virtual indices),
// edge_layer_indices[E]. Returns edge count or -1 on error.
// =====================================================================================================================
namespace {
std::vector<int> MedianGridSubsample(const std::vector<float>& pts, float cell) {
	int n = static_cast<int>(pts.size() / 3);
	std::map<std::tuple<int, int, int>, std::vector<int>> bins;   // bin contents in ascending point order
	std::vector<std::tuple<int, int, int>> order;
	for (int i = 0; i < n; i++) {
		auto key = std::make_tuple(static_cast<int>(floorf(pts[3 * i] / cell)), static_cast<int>(floorf(pts[3 * i + 1] / cell)),
		                           static_cast<int>(floorf(pts[3 * i + 2] / cell)));
		auto it = bins.find(key);
		if (it == bins.end()) { bins[key] = {i}; order.push_back(key); }
		else it->second.push_back(i);
	}
	std::vector<int> sample;
	for (auto& key : order) {
		const auto& members = bins[key];
		float best = 3.402823466e+38f;
		int best_i = members[0];
		for (int a : members) {
			float sum = 0.f;
			for (int b : members) {
				float dx = pts[3 * b] - pts[3 * a], dy = pts[3 * b + 1] - pts[3 * a + 1], dz = pts[3 * b + 2] - pts[3 * a + 2];
				sum += sqrtf((dx * dx + dy * dy) + dz * dz);
			}
			if (sum < best) { best = sum; best_i = a; }
		}
		sample.push_back(best_i);
	}
	std::sort(sample.begin(), sample.end());
	return sample;
}
// sorted K nearest (ties -> lower index), -1 padded
void KnnSorted(const float* q, const std::vector<float>& ref, int k, int32_t* out) {
	int n = static_cast<int>(ref.size() / 3);
	std::vector<std::pair<float, int>> d(n);
	for (int i = 0; i < n; i++) {
		float dx = ref[3 * i] - q[0], dy = ref[3 * i + 1] - q[1], dz = ref[3 * i + 2] - q[2];
		d[i] = {(dx * dx + dy * dy) + dz * dz, i};
	}
	std::sort(d.begin(), d.end());
	for (int j = 0; j < k; j++) out[j] = j < n ? d[j].second : -1;
}
} // namespace

ORC_API int orc_build_hierarchy(const float* nodes, int N, float coverage, int layer_count, int max_degree, const float* radii,
                                int64_t* virtual_node_indices, int* layer_counts, int32_t* edges, int8_t* edge_layer_indices,
                                int edge_capacity) {
	struct Layer { std::vector<int64_t> idx; std::vector<float> pos; std::vector<int32_t> edges; float radius; };
	std::vector<Layer> layers(layer_count);
	layers[0].radius = coverage;
	for (int i = 0; i < N; i++) { layers[0].idx.push_back(i); for (int c = 0; c < 3; c++) layers[0].pos.push_back(nodes[3 * i + c]); }
	for (int l = 1; l < layer_count; l++) {
		Layer& finer = layers[l - 1];
		Layer& cur = layers[l];
		cur.radius = radii ? radii[l] : static_cast<float>(l + 1) * coverage;
		std::vector<int> sample = MedianGridSubsample(finer.pos, cur.radius * 2);
		if (sample.size() == finer.idx.size()) {
			g_error = "Attempting to generate a coarser layer of the same size as the finer layer";
			return -1;
		}
		std::vector<char> keep(finer.idx.size(), 1);
		for (int s : sample) {
			keep[s] = 0;
			cur.idx.push_back(finer.idx[s]);
			for (int c = 0; c < 3; c++) cur.pos.push_back(finer.pos[3 * s + c]);
		}
		Layer filtered;
		for (size_t i = 0; i < finer.idx.size(); i++) {
			if (!keep[i]) continue;
			filtered.idx.push_back(finer.idx[i]);
			for (int c = 0; c < 3; c++) filtered.pos.push_back(finer.pos[3 * i + c]);
		}
		finer.idx = filtered.idx;
		finer.pos = filtered.pos;
	}
	std::vector<int> first_virtual(layer_count);
	int vc = 0;
	for (int l = 0; l < layer_count; l++) { first_virtual[l] = vc; layer_counts[l] = static_cast<int>(layers[l].idx.size()); vc += layer_counts[l]; }
	for (int l = layer_count - 1; l >= 1; l--) {
		Layer& cur = layers[l];
		Layer& finer = layers[l - 1];
		int ns = static_cast<int>(finer.idx.size());
		std::vector<int32_t> adj(static_cast<size_t>(ns) * max_degree);
		for (int s = 0; s < ns; s++) {
			KnnSorted(&finer.pos[3 * s], cur.pos, max_degree, &adj[static_cast<size_t>(s) * max_degree]);
			std::sort(&adj[static_cast<size_t>(s) * max_degree], &adj[static_cast<size_t>(s) * max_degree] + max_degree, std::greater<int32_t>());
		}
		std::vector<int32_t> raw(static_cast<size_t>(ns) * max_degree * 2);
		for (int s = 0; s < ns; s++) {
			for (int k = 0; k < max_degree; k++) {
				int32_t t = adj[static_cast<size_t>(s) * max_degree + k];
				int32_t* out = &raw[(static_cast<size_t>(ns - 1 - s) * max_degree + k) * 2];
				if (t != -1) { out[0] = first_virtual[l - 1] + s; out[1] = first_virtual[l] + t; }
				else { out[0] = -1; out[1] = -1; }
			}
		}
		for (size_t e = 0; e < raw.size() / 2; e++) {
			if (raw[2 * e] == -1) continue;
			finer.edges.push_back(raw[2 * e]);
			finer.edges.push_back(raw[2 * e + 1]);
		}
	}
	int ne = 0;
	for (int l = layer_count - 1; l >= 0; l--) {
		if (l < layer_count - 1) {
			for (size_t e = 0; e < layers[l].edges.size() / 2; e++) {
				if (ne >= edge_capacity) { g_error = "edge capacity exceeded"; return -1; }
				edges[2 * ne] = layers[l].edges[2 * e];
				edges[2 * ne + 1] = layers[l].edges[2 * e + 1];
				edge_layer_indices[ne] = static_cast<int8_t>(l + 1);
				ne++;
			}
		}
	}
	int o = 0;
	for (int l = 0; l < layer_count; l++) for (int64_t i : layers[l].idx) virtual_node_indices[o++] = i;
	return ne;
}

// =====================================================================================================================
// Warp: cpp/geometry/functional/kernel/Warp3dPointsAndNormalsImpl.h:334-390 + WarpUtilities.h:448-467 (BlendWarp).
// extrinsics: double[16] row-major or nullptr (identity); applied as Open3D TransformIndexer::RigidTransform in float.
// =====================================================================================================================
// minimum_valid >= 0: BlendWarp_ValidAnchorCountThreshold (WarpUtilities.h:505-580): fewer valid (!= -1) slots than
// minimum_valid -> the point / normal keep the zero they were initialised with (Warp3dPointsAndNormalsImpl.h:237-238)
ORC_API void orc_warp_points(const float* points, const float* normals, int64_t V, const float* nodes, const float* rotations,
                             const float* translations, const int32_t* anchors, const float* weights, int K, int minimum_valid,
                             const double* extrinsics, float* out_points, float* out_normals);
ORC_API void orc_warp_mesh(const float* points, const float* normals, int64_t V, const float* nodes, const float* rotations,
                           const float* translations, const int32_t* anchors, const float* weights, int K, const double* extrinsics,
                           float* out_points, float* out_normals) {
	orc_warp_points(points, normals, V, nodes, rotations, translations, anchors, weights, K, -1, extrinsics, out_points, out_normals);
}

ORC_API void orc_warp_points(const float* points, const float* normals, int64_t V, const float* nodes, const float* rotations,
                             const float* translations, const int32_t* anchors, const float* weights, int K, int minimum_valid,
                             const double* extrinsics, float* out_points, float* out_normals) {
	float E[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
	if (extrinsics) for (int i = 0; i < 12; i++) E[i] = static_cast<float>(extrinsics[i]);
#pragma omp parallel for schedule(static)
	for (int64_t v = 0; v < V; v++) {
		int valid = 0;
		for (int k = 0; k < K; k++) valid += anchors[v * K + k] != -1;
		if (minimum_valid >= 0 && valid < minimum_valid) {
			for (int c = 0; c < 3; c++) out_points[3 * v + c] = 0.f;
			if (normals) for (int c = 0; c < 3; c++) out_normals[3 * v + c] = 0.f;
			continue;
		}
		const float* p = points + 3 * v;
		float pc[3], nc[3];
		for (int r = 0; r < 3; r++) pc[r] = ((p[0] * E[4 * r] + p[1] * E[4 * r + 1]) + p[2] * E[4 * r + 2]) + E[4 * r + 3];
		const float* n = normals ? normals + 3 * v : nullptr;
		if (n) for (int r = 0; r < 3; r++) nc[r] = (n[0] * E[4 * r] + n[1] * E[4 * r + 1]) + n[2] * E[4 * r + 2];
		float wp[3] = {0, 0, 0}, wn[3] = {0, 0, 0};
		for (int k = 0; k < K; k++) {
			int32_t a = anchors[v * K + k];
			if (a == -1) continue;
			float w = weights[v * K + k];
			const float* g = nodes + 3 * a;
			const float* R = rotations + 9 * a;
			const float* t = translations + 3 * a;
			float d[3] = {pc[0] - g[0], pc[1] - g[1], pc[2] - g[2]};
			float Rd[3];
			matvec3(R, d, Rd);
			for (int c = 0; c < 3; c++) wp[c] += w * ((g[c] + Rd[c]) + t[c]);
			if (n) {
				float Rn[3];
				matvec3(R, nc, Rn);
				for (int c = 0; c < 3; c++) wn[c] += w * Rn[c];
			}
		}
		for (int c = 0; c < 3; c++) out_points[3 * v + c] = wp[c];
		if (n) for (int c = 0; c < 3; c++) out_normals[3 * v + c] = wn[c];
	}
}

ORC_API void orc_intrinsics_to_ndc(const double* K, int H, int W, double* ndcK, float* range4) {
	Box2 r;
	IntrinsicsToNdc(K, H, W, ndcK, &r);
	range4[0] = r.min_x; range4[1] = r.max_x; range4[2] = r.min_y; range4[3] = r.max_y;
}

// =====================================================================================================================
// NDC face extraction: cpp/rendering/functional/ExtractFaceVertices.cpp:56-85 ->
// ExtractClippedFaceVerticesImpl.h:108-179 (near/far test OR-accumulated: A6). Clipped faces are zero-filled.
// =====================================================================================================================
ORC_API void orc_extract_face_ndc(const float* verts, const int64_t* faces, int64_t F, const double* K, int H, int W, float near_clip,
                                  float far_clip, float* face_ndc, uint8_t* mask) {
	double ndcK[9];
	Box2 range;
	IntrinsicsToNdc(K, H, W, ndcK, &range);
	NdcCamera cam{static_cast<float>(ndcK[0]), static_cast<float>(ndcK[4]), static_cast<float>(ndcK[2]), static_cast<float>(ndcK[5])};
#pragma omp parallel for schedule(static)
	for (int64_t f = 0; f < F; f++) {
		const float* v[3] = {verts + 3 * faces[3 * f], verts + 3 * faces[3 * f + 1], verts + 3 * faces[3 * f + 2]};
		float* out = face_ndc + 9 * f;
		bool in_range = false;
		for (int i = 0; i < 3; i++) { in_range |= v[i][2] >= near_clip; in_range |= v[i][2] <= far_clip; }
		bool inlier = false;
		float xy[3][2];
		if (in_range) {
			for (int i = 0; i < 3; i++) {
				cam.Project(v[i][0], v[i][1], v[i][2], &xy[i][0], &xy[i][1]);
				inlier |= range.Contains(xy[i][0], xy[i][1]);
			}
		}
		if (!in_range || !inlier) {
			mask[f] = 0;
			for (int i = 0; i < 9; i++) out[i] = 0.f;
			continue;
		}
		mask[f] = 1;
		for (int i = 0; i < 3; i++) { out[3 * i] = xy[i][0]; out[3 * i + 1] = xy[i][1]; out[3 * i + 2] = v[i][2]; }
	}
}

// =====================================================================================================================
// Rasterizer: cpp/rendering/RasterizeNdcTriangles.cpp:33-129, kernel/RasterizeNdcTrianglesImpl.h:41-391,
// RasterizeNdcTrianglesImplCPU.h (bins filled in ascending face order), RayFaceIntersection.h:32-255.
// =====================================================================================================================
namespace {
struct Hit { float depth; int32_t face; float dist; float b[3]; };
inline bool HitLess(const Hit& a, const Hit& b) { return a.depth < b.depth || (a.depth == b.depth && a.face < b.face); }

struct RasterOpts { float blur; int faces_per_pixel; bool persp; bool clip; bool cull; };

inline void FaceBox(const float* f, float blur, float& xmin, float& xmax, float& ymin, float& ymax, bool& zinv) {
	xmin = fmin3f(f[0], f[3], f[6]) - blur;
	xmax = fmax3f(f[0], f[3], f[6]) + blur;
	ymin = fmin3f(f[1], f[4], f[7]) - blur;
	ymax = fmax3f(f[1], f[4], f[7]) + blur;
	const float zmax = fmax3f(f[2], f[5], f[8]);
	zinv = zmax < K_EPSILON;
}

inline float PointSegmentSq(float px, float py, float ax, float ay, float bx, float by) {
	float sx = bx - ax, sy = by - ay;
	float l2 = sx * sx + sy * sy;
	float t = (sx * (px - ax) + sy * (py - ay)) / l2;
	if (l2 <= K_EPSILON) {
		float dx = px - bx, dy = py - by;
		return dx * dx + dy * dy;
	}
	t = saturatef(t);
	float cx = ax + t * sx, cy = ay + t * sy;
	float dx = cx - px, dy = cy - py;
	return dx * dx + dy * dy;
}

// Faces with a non-finite vertex coordinate (A7 NaN rotations warp vertices to NaN) are rejected: the reference's queue
// would depend on its face order there, since NaN fails every comparison (RayFaceIntersection.h:162-255).
inline bool FaceFinite(const float* f) {
	for (int i = 0; i < 9; i++)
		if (!std::isfinite(f[i])) return false;
	return true;
}

// returns true and fills hit if the face is accepted for the pixel (UpdateQueueIfPixelInsideFace minus queue logic)
inline bool TestFace(const float* f, int32_t face, float px, float py, const RasterOpts& o, Hit& hit) {
	if (!FaceFinite(f)) return false;
	const float area = SPA_CW(f[0], f[1], f[3], f[4], f[6], f[7]);
	const bool back = area < 0.f;
	const bool zero_area = (area <= K_EPSILON && area >= -1.f * K_EPSILON);
	float xmin, xmax, ymin, ymax;
	bool zinv;
	FaceBox(f, o.blur, xmin, xmax, ymin, ymax, zinv);
	if ((px > xmax || px < xmin || py > ymax || py < ymin || zinv) || (o.cull && back) || zero_area) return false;
	const float A = SPA_CW(f[0], f[1], f[3], f[4], f[6], f[7]) + K_EPSILON;
	float b0 = SPA_CW(px, py, f[3], f[4], f[6], f[7]) / A;
	float b1 = SPA_CW(px, py, f[6], f[7], f[0], f[1]) / A;
	float b2 = SPA_CW(px, py, f[0], f[1], f[3], f[4]) / A;
	if (o.persp) {
		const float z0 = f[2], z1 = f[5], z2 = f[8];
		const float n0 = b0 * z1 * z2, n1 = z0 * b1 * z2, n2 = z0 * z1 * b2;
		const float den = fmaxf(n0 + n1 + n2, K_EPSILON);
		b0 = n0 / den; b1 = n1 / den; b2 = n2 / den;
	}
	float c0 = b0, c1 = b1, c2 = b2;
	if (o.clip) {
		c0 = fmaxf(b0, 0.f); c1 = fmaxf(b1, 0.f); c2 = fmaxf(b2, 0.f);
		float z = (c0 * c0 + c1 * c1) + c2 * c2;
		if (z > 0.f) { float s = sqrtf(z); c0 /= s; c1 /= s; c2 /= s; }
	}
	const float depth = c0 * f[2] + c1 * f[5] + c2 * f[8];
	if (depth < 0.f) return false;
	const float d = fmin3f(PointSegmentSq(px, py, f[0], f[1], f[3], f[4]), PointSegmentSq(px, py, f[0], f[1], f[6], f[7]),
	                       PointSegmentSq(px, py, f[3], f[4], f[6], f[7]));
	const bool inside = b0 > 0.f && b1 > 0.f && b2 > 0.f;
	if (!inside && d >= o.blur) return false;
	hit.depth = depth; hit.face = face; hit.dist = inside ? -d : d; hit.b[0] = c0; hit.b[1] = c1; hit.b[2] = c2;
	return true;
}

inline void QueueInsert(Hit* q, int& qs, float& qmax, int& qmax_at, const Hit& h, int K) {
	if (qs < K) {
		q[qs] = h;
		if (h.depth > qmax) { qmax = h.depth; qmax_at = qs; }
		qs++;
	} else if (h.depth < qmax) {
		q[qmax_at] = h;
		qmax = h.depth;
		for (int i = 0; i < K; i++) if (q[i].depth > qmax) { qmax = q[i].depth; qmax_at = i; }
	}
}

void WritePixel(int64_t pix, Hit* q, int qs, int K, int64_t* fi, float* dep, float* bary, float* dist) {
	std::sort(q, q + qs, HitLess);
	for (int i = 0; i < qs; i++) {
		int64_t o = pix * K + i;
		fi[o] = q[i].face; dep[o] = q[i].depth; dist[o] = q[i].dist;
		bary[3 * o] = q[i].b[0]; bary[3 * o + 1] = q[i].b[1]; bary[3 * o + 2] = q[i].b[2];
	}
}
} // namespace

// Literal restatement: coarse-to-fine (bin_size>0) or brute force (bin_size==0). Returns 0 on success.
ORC_API int orc_rasterize(const float* face_ndc, const uint8_t* mask, int64_t F, int H, int W, float blur_radius_pixels, int faces_per_pixel,
                          int bin_size, int max_faces_per_bin, int perspective_correct, int clip_barycentric, int cull_back_faces,
                          int64_t* out_face, float* out_depth, float* out_bary, float* out_dist) {
	if (faces_per_pixel > MAX_POINTS_PER_PIXEL) { g_error = "Need faces_per_pixel <= 8"; return 1; }
	const int K = faces_per_pixel;
	const int64_t P = static_cast<int64_t>(H) * W;
	for (int64_t i = 0; i < P * K; i++) { out_face[i] = -1; out_depth[i] = -1.f; out_dist[i] = -1.f; }
	for (int64_t i = 0; i < P * K * 3; i++) out_bary[i] = -1.f;
	int max_dim = std::max(H, W);
	if (bin_size == -1) {
		if (max_dim <= 64) bin_size = 8;
		else bin_size = static_cast<int>(std::pow(2, std::max(static_cast<int>(std::ceil(std::log2(static_cast<double>(max_dim)))) - 4, 4)));
	}
	if (bin_size != 0 && 1 + (max_dim - 1) / bin_size >= MAX_BINS_ALONG_IMAGE_DIMENSION) { g_error = "bin_size too small"; return 2; }
	if (max_faces_per_bin == -1) {
		int64_t unclipped = 0;
		if (mask) for (int64_t f = 0; f < F; f++) unclipped += mask[f] ? 1 : 0; else unclipped = F;
		max_faces_per_bin = std::max(10000, static_cast<int>(unclipped) / 5);
	}
	RasterOpts o{blur_radius_pixels / (static_cast<float>(fminf(H, W)) / 2.0f), K, perspective_correct != 0, clip_barycentric != 0,
	             cull_back_faces != 0};
	if (F == 0) return 0;
	if (bin_size > 0 && max_faces_per_bin > 0) {
		const int by = 1 + (H - 1) / bin_size, bx = 1 + (W - 1) / bin_size;
		std::vector<int32_t> bins(static_cast<size_t>(by) * bx * max_faces_per_bin, -1);
		std::vector<int> counts(static_cast<size_t>(by) * bx, 0);
		const float hpy = GetNdcRange(W, H) / 2.f / static_cast<float>(H);   // RasterizeNdcTrianglesImpl.h:380-384 (as written)
		const float hpx = GetNdcRange(H, W) / 2.f / static_cast<float>(W);
		for (int64_t f = 0; f < F; f++) {
			if (mask && !mask[f]) continue;
			float xmin, xmax, ymin, ymax;
			bool zinv;
			FaceBox(face_ndc + 9 * f, o.blur, xmin, xmax, ymin, ymax, zinv);
			if (zinv) continue;
			for (int iy = 0; iy < by; iy++) {
				const float bymin = PixelToNdc(iy * bin_size, H, W) - hpy;
				const float bymax = PixelToNdc((iy + 1) * bin_size - 1, H, W) + hpy;
				if (!((ymin <= bymax) && (bymin < ymax))) continue;
				for (int ix = 0; ix < bx; ix++) {
					const float bxmin = PixelToNdc(ix * bin_size, W, H) - hpx;
					const float bxmax = PixelToNdc((ix + 1) * bin_size - 1, W, H) + hpx;
					if (!((xmin <= bxmax) && (bxmin < xmax))) continue;
					int b = iy * bx + ix;
					if (counts[b] >= max_faces_per_bin) { g_error = "bin capacity exceeded"; return 3; }
					bins[static_cast<size_t>(b) * max_faces_per_bin + counts[b]++] = static_cast<int32_t>(f);
				}
			}
		}
#pragma omp parallel for schedule(dynamic, 64)
		for (int64_t pix = 0; pix < P; pix++) {
			int v = static_cast<int>(pix / W), u = static_cast<int>(pix % W);
			float py = PixelToNdc(v, H, W), px = PixelToNdc(u, W, H);
			const int32_t* list = &bins[static_cast<size_t>((v / bin_size) * bx + (u / bin_size)) * max_faces_per_bin];
			Hit q[MAX_POINTS_PER_PIXEL];
			int qs = 0, qat = -1;
			float qmax = -1000.f;
			for (int i = 0; i < max_faces_per_bin; i++) {
				int32_t f = list[i];
				if (f == -1) break;
				Hit h;
				if (TestFace(face_ndc + 9 * static_cast<int64_t>(f), f, px, py, o, h)) QueueInsert(q, qs, qmax, qat, h, K);
			}
			WritePixel(pix, q, qs, K, out_face, out_depth, out_bary, out_dist);
		}
	} else {
#pragma omp parallel for schedule(dynamic, 64)
		for (int64_t pix = 0; pix < P; pix++) {
			int v = static_cast<int>(pix / W), u = static_cast<int>(pix % W);
			float py = PixelToNdc(v, H, W), px = PixelToNdc(u, W, H);
			Hit q[MAX_POINTS_PER_PIXEL];
			int qs = 0, qat = -1;
			float qmax = -1000.f;
			for (int64_t f = 0; f < F; f++) {
				if (mask && !mask[f]) continue;
				Hit h;
				if (TestFace(face_ndc + 9 * f, static_cast<int32_t>(f), px, py, o, h)) QueueInsert(q, qs, qmax, qat, h, K);
			}
			WritePixel(pix, q, qs, K, out_face, out_depth, out_bary, out_dist);
		}
	}
	return 0;
}

// Same semantics for faces_per_pixel == 1, visiting each face's bounding box instead of per-pixel bin lists
// (the winner is the lexicographic (depth, face) minimum either way). Used for large parity configs.
ORC_API int orc_rasterize_k1_fast(const float* face_ndc, const uint8_t* mask, int64_t F, int H, int W, float blur_radius_pixels,
                                  int perspective_correct, int cull_back_faces, int64_t* out_face, float* out_depth, float* out_bary,
                                  float* out_dist) {
	const int64_t P = static_cast<int64_t>(H) * W;
	RasterOpts o{blur_radius_pixels / (static_cast<float>(fminf(H, W)) / 2.0f), 1, perspective_correct != 0, false, cull_back_faces != 0};
	std::vector<Hit> best(P);
	for (int64_t i = 0; i < P; i++) { best[i].face = -1; best[i].depth = 0.f; }
	const float rx = GetNdcRange(W, H), ry = GetNdcRange(H, W);
	// row bands per thread: every thread scans all faces but only writes its own rows (the winner per pixel is the
	// strict minimum under HitLess, so the result does not depend on the partition)
#pragma omp parallel
	{
	const int nt = omp_get_num_threads(), tid = omp_get_thread_num();
	const int band_lo = static_cast<int>(static_cast<int64_t>(H) * tid / nt), band_hi = static_cast<int>(static_cast<int64_t>(H) * (tid + 1) / nt) - 1;
	for (int64_t f = 0; f < F; f++) {
		if (mask && !mask[f]) continue;
		const float* fv = face_ndc + 9 * f;
		float xmin, xmax, ymin, ymax;
		bool zinv;
		FaceBox(fv, o.blur, xmin, xmax, ymin, ymax, zinv);
		if (zinv || !(xmax >= xmin) || !(ymax >= ymin)) continue;
		// invert x = -r/2 + (r*u + r/2)/W  ->  u = (x + r/2) * W / r - 1/2 ; widen by one pixel each side, exact test below
		double ulo = std::floor((static_cast<double>(xmin) + rx / 2.0) * W / rx - 0.5) - 1;
		double uhi = std::ceil((static_cast<double>(xmax) + rx / 2.0) * W / rx - 0.5) + 1;
		double vlo = std::floor((static_cast<double>(ymin) + ry / 2.0) * H / ry - 0.5) - 1;
		double vhi = std::ceil((static_cast<double>(ymax) + ry / 2.0) * H / ry - 0.5) + 1;
		int u0 = static_cast<int>(std::max(0.0, ulo)), u1 = static_cast<int>(std::min<double>(W - 1, uhi));
		int v0 = static_cast<int>(std::max<double>(band_lo, vlo)), v1 = static_cast<int>(std::min<double>(band_hi, vhi));
		if (v0 > v1) continue;
		for (int v = v0; v <= v1; v++) {
			float py = PixelToNdc(v, H, W);
			for (int u = u0; u <= u1; u++) {
				float px = PixelToNdc(u, W, H);
				Hit h;
				if (!TestFace(fv, static_cast<int32_t>(f), px, py, o, h)) continue;
				Hit& b = best[static_cast<int64_t>(v) * W + u];
				if (b.face == -1 || HitLess(h, b)) b = h;
			}
		}
	}
	}
	for (int64_t i = 0; i < P; i++) {
		if (best[i].face == -1) { out_face[i] = -1; out_depth[i] = -1.f; out_dist[i] = -1.f; out_bary[3 * i] = out_bary[3 * i + 1] = out_bary[3 * i + 2] = -1.f; continue; }
		out_face[i] = best[i].face; out_depth[i] = best[i].depth; out_dist[i] = best[i].dist;
		for (int c = 0; c < 3; c++) out_bary[3 * i + c] = best[i].b[c];
	}
	return 0;
}

// cpp/rendering/functional/kernel/InterpolateFaceAttributesImpl.h:30-75 ; face_attrs [F,3,C]
ORC_API void orc_interpolate_face_attributes(const int64_t* pixel_faces, const float* bary, int64_t P, int K, const float* face_attrs,
                                             int C, float* out) {
	for (int64_t i = 0; i < P * K * C; i++) out[i] = 0.f;
#pragma omp parallel for schedule(static)
	for (int64_t p = 0; p < P; p++) {
		for (int k = 0; k < K; k++) {
			int64_t f = pixel_faces[p * K + k];
			if (f < 0) break;
			for (int c = 0; c < C; c++) {
				float acc = 0.0f;
				for (int i = 0; i < 3; i++) acc += bary[(p * K + k) * 3 + i] * face_attrs[f * 3 * C + i * C + c];
				out[(p * K + k) * C + c] = acc;
			}
		}
	}
}

// cpp/geometry/functional/kernel/PerspectiveProjectionImpl.h:60-146 (identity extrinsics). depth is float32 [H,W]
ORC_API void orc_unproject(const float* depth, int H, int W, const double* K, float depth_scale, float depth_max, float* points, uint8_t* mask) {
	const float fx = static_cast<float>(K[0]), fy = static_cast<float>(K[4]), cx = static_cast<float>(K[2]), cy = static_cast<float>(K[5]);
#pragma omp parallel for schedule(static)
	for (int64_t i = 0; i < static_cast<int64_t>(H) * W; i++) {
		int64_t y = i / W, x = i % W;
		float d = depth[i] / depth_scale;
		float* o = points + 3 * i;
		if (d > 0 && d < depth_max) {
			o[0] = (static_cast<float>(x) - cx) * d / fx;
			o[1] = (static_cast<float>(y) - cy) * d / fy;
			o[2] = d;
			mask[i] = 1;
		} else {
			o[0] = o[1] = o[2] = 0.f;
			mask[i] = 0;
		}
	}
}

// UnprojectRasterWithoutDepthFiltering with extrinsics (PerspectiveProjectionImpl.h:60-146): depth uint16 (dtype 1) or float32
// (any other dtype code) [H,W]; camera point by TransformIndexer::Unproject, then RigidTransform by pose = extrinsics^-1 (Open3D
// InverseTransformation [R^T | -R^T t], here in double, rounded once to the indexer's floats; extrinsics nullptr = identity).
ORC_API void orc_unproject_image(const void* depth, int dtype, int H, int W, const double* K, const double* extrinsics, float depth_scale,
                                 float depth_max, float* points, uint8_t* mask) {
	const float fx = static_cast<float>(K[0]), fy = static_cast<float>(K[4]), cx = static_cast<float>(K[2]), cy = static_cast<float>(K[5]);
	float P[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
	bool identity = true;
	if (extrinsics) {
		for (int r = 0; r < 3; r++) {
			double tr = 0.0;
			for (int c = 0; c < 3; c++) {
				P[4 * r + c] = static_cast<float>(extrinsics[4 * c + r]);
				tr += extrinsics[4 * c + r] * extrinsics[4 * c + 3];
			}
			P[4 * r + 3] = static_cast<float>(-tr);
		}
		const float I[12] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0};
		for (int i = 0; i < 12; i++) identity &= P[i] == I[i];
	}
#pragma omp parallel for schedule(static)
	for (int64_t i = 0; i < static_cast<int64_t>(H) * W; i++) {
		int64_t y = i / W, x = i % W;
		const float raw = dtype == 1 ? static_cast<float>(static_cast<const uint16_t*>(depth)[i]) : static_cast<const float*>(depth)[i];
		float d = raw / depth_scale;
		float* o = points + 3 * i;
		if (d > 0 && d < depth_max) {
			const float c[3] = {(static_cast<float>(x) - cx) * d / fx, (static_cast<float>(y) - cy) * d / fy, d};
			for (int r = 0; r < 3; r++)
				o[r] = identity ? c[r] : ((c[0] * P[4 * r] + c[1] * P[4 * r + 1]) + c[2] * P[4 * r + 2]) + P[4 * r + 3];
			mask[i] = 1;
		} else {
			o[0] = o[1] = o[2] = 0.f;
			mask[i] = 0;
		}
	}
}

// ComputePointToPlaneDistances (PointToPlaneDistancesImpl.h:26-50): n1 . (v1 - v2), summed left to right
ORC_API void orc_point_to_plane(const float* n1, const float* v1, const float* v2, int64_t count, float* out) {
#pragma omp parallel for schedule(static)
	for (int64_t i = 0; i < count; i++) {
		const float d[3] = {v1[3 * i] - v2[3 * i], v1[3 * i + 1] - v2[3 * i + 1], v1[3 * i + 2] - v2[3 * i + 2]};
		out[i] = dot3(n1 + 3 * i, d);
	}
}

// =====================================================================================================================
// Jacobians
// =====================================================================================================================
// Arithmetic of the pixel-node Jacobians (a10 + a12). 0 (default): the reference's CPU-path expressions as written
// (-w R (v - g) and -w R n stored per (vertex, anchor), then dv [.]_x + dn [.]_x; no contraction, as the reference's
// gcc build on x86-64 runs them). 1: the GPU product's fused form (csrc/fitter_kernels.hip, NNRT_JAC_FMA): R (v - g)
// and R n as FMA chains, jr += -w (dv x R (v - g) + dn x R n) and jt += w dv as FMAs -- the same real-number expression,
// within a few float ulps of form 0 per term, and bit-identical to the GPU's terms (fmaf is correctly rounded here and
// on gfx950). In mode 1 orc_warped_surface_jacobians stores (R (v - g), w) and R n (without -w).
static int g_jac_fma = 0;
ORC_API void orc_set_fused_jacobians(int on) { g_jac_fma = on; }
namespace {
inline void matvec3_fma(const float* R, const float* v, float* o) {
	o[0] = std::fmaf(R[0], v[0], std::fmaf(R[1], v[1], R[2] * v[2]));
	o[1] = std::fmaf(R[3], v[0], std::fmaf(R[4], v[1], R[5] * v[2]));
	o[2] = std::fmaf(R[6], v[0], std::fmaf(R[7], v[1], R[8] * v[2]));
}
}  // namespace

// cpp/alignment/functional/kernel/WarpedSurfaceJacobiansImpl.h:117-156 ; out_vj [V,K,4], out_nj [V,K,3]
ORC_API void orc_warped_surface_jacobians(const float* points, const float* normals, int64_t V, const float* nodes, const float* rotations,
                                          const int32_t* anchors, const float* weights, int K, float* out_vj, float* out_nj) {
	std::memset(out_vj, 0, sizeof(float) * V * K * 4);
	std::memset(out_nj, 0, sizeof(float) * V * K * 3);
#pragma omp parallel for schedule(static)
	for (int64_t v = 0; v < V; v++) {
		for (int k = 0; k < K; k++) {
			int32_t n = anchors[v * K + k];
			if (n == -1) continue;
			float w = weights[v * K + k];
			const float* R = rotations + 9 * n;
			const float* g = nodes + 3 * n;
			const float* p = points + 3 * v;
			float d[3] = {p[0] - g[0], p[1] - g[1], p[2] - g[2]}, Rd[3];
			if (g_jac_fma) {   // fused mode: R (v - g), w and R n, unscaled (see g_jac_fma)
				float* vj = out_vj + (v * K + k) * 4;
				matvec3_fma(R, d, vj);
				vj[3] = w;
				matvec3_fma(R, normals + 3 * v, out_nj + (v * K + k) * 3);
				continue;
			}
			matvec3(R, d, Rd);
			float* vj = out_vj + (v * K + k) * 4;
			for (int c = 0; c < 3; c++) vj[c] = -w * Rd[c];
			vj[3] = w;
			float Rn[3];
			matvec3(R, normals + 3 * v, Rn);
			float* nj = out_nj + (v * K + k) * 3;
			for (int c = 0; c < 3; c++) nj[c] = -w * Rn[c];
		}
	}
}

namespace {
// cpp/alignment/functional/kernel/BarycentricCoordinateJacobians.h:85-181 ; D[i] is the 3x2 d(rho)/d(ndc vertex i)
void BaryWrtNdc(const float* p, const float ndc[3][2], float A, const float a[3], float D[3][3][2]) {
	const float A2 = A * A;
	const float den = A2 + K_EPSILON;
	float dA[3][2] = {{ndc[1][1] - ndc[2][1], ndc[2][0] - ndc[1][0]},
	                  {ndc[2][1] - ndc[0][1], ndc[0][0] - ndc[2][0]},
	                  {ndc[0][1] - ndc[1][1], ndc[1][0] - ndc[0][0]}};
	auto sub = [&](int ia, int ib, float out[2][2]) {   // d(sub-area(p, va, vb)) / d(va, vb)
		out[0][0] = ndc[ib][1] - p[1]; out[0][1] = p[0] - ndc[ib][0];
		out[1][0] = p[1] - ndc[ia][1]; out[1][1] = ndc[ia][0] - p[0];
	};
	float s0[2][2], s1[2][2], s2[2][2];
	sub(1, 2, s0); sub(2, 0, s1); sub(0, 1, s2);
	for (int c = 0; c < 2; c++) {
		D[0][0][c] = (-a[0] * dA[0][c]) / den;
		D[1][0][c] = (A * s0[0][c] - a[0] * dA[1][c]) / den;
		D[2][0][c] = (A * s0[1][c] - a[0] * dA[2][c]) / den;
		D[0][1][c] = (A * s1[1][c] - a[1] * dA[0][c]) / den;
		D[1][1][c] = (-a[1] * dA[1][c]) / den;
		D[2][1][c] = (A * s1[0][c] - a[1] * dA[2][c]) / den;
		D[0][2][c] = (A * s2[0][c] - a[2] * dA[0][c]) / den;
		D[1][2][c] = (A * s2[1][c] - a[2] * dA[1][c]) / den;
		D[2][2][c] = (-a[2] * dA[2][c]) / den;
	}
}
} // namespace

// cpp/alignment/functional/kernel/RasterizedSurfaceJacobiansImpl.h:114-200 (+BarycentricCoordinateJacobians.h:185-419,
// ProjectionJacobians.h:26-38). pixel_faces/bary: first face per pixel ([H,W,Kf], [H,W,Kf,3]).
// out_vj [H,W,3,9]; out_nj [H,W,3,10] (last 3 = barycentrics)
ORC_API void orc_rasterized_surface_jacobians(const float* verts, const float* normals, const int64_t* faces, const int64_t* pixel_faces,
                                              const float* pixel_bary, int H, int W, int Kf, const double* K, int perspective_correct,
                                              float* out_vj, float* out_nj) {
	double ndcK[9];
	Box2 range;
	IntrinsicsToNdc(K, H, W, ndcK, &range);
	NdcCamera cam{static_cast<float>(ndcK[0]), static_cast<float>(ndcK[4]), static_cast<float>(ndcK[2]), static_cast<float>(ndcK[5])};
	const int64_t P = static_cast<int64_t>(H) * W;
	std::memset(out_vj, 0, sizeof(float) * P * 27);
	std::memset(out_nj, 0, sizeof(float) * P * 30);
#pragma omp parallel for schedule(static)
	for (int64_t pix = 0; pix < P; pix++) {
		int v = static_cast<int>(pix / W), u = static_cast<int>(pix % W);
		float p[2] = {PixelToNdc(u, W, H), PixelToNdc(v, H, W)};
		int64_t f = pixel_faces[pix * Kf];
		if (f == -1) continue;
		const float* V3[3] = {verts + 3 * faces[3 * f], verts + 3 * faces[3 * f + 1], verts + 3 * faces[3 * f + 2]};
		const float* N3[3] = {normals + 3 * faces[3 * f], normals + 3 * faces[3 * f + 1], normals + 3 * faces[3 * f + 2]};
		const float* rho = pixel_bary + pix * Kf * 3;
		float ndc[3][2];
		for (int i = 0; i < 3; i++) cam.Project(V3[i][0], V3[i][1], V3[i][2], &ndc[i][0], &ndc[i][1]);
		float A, a[3], dist_rho[3] = {0.f, 0.f, 0.f};
		if (perspective_correct) {
			A = SPA_CW(ndc[0][0], ndc[0][1], ndc[1][0], ndc[1][1], ndc[2][0], ndc[2][1]) + K_EPSILON;
			a[0] = SPA_CW(p[0], p[1], ndc[1][0], ndc[1][1], ndc[2][0], ndc[2][1]);
			a[1] = SPA_CW(p[0], p[1], ndc[2][0], ndc[2][1], ndc[0][0], ndc[0][1]);
			a[2] = SPA_CW(p[0], p[1], ndc[0][0], ndc[0][1], ndc[1][0], ndc[1][1]);
			for (int i = 0; i < 3; i++) dist_rho[i] = a[i] / A;
		} else {
			A = SPA_CW(ndc[0][0], ndc[0][1], ndc[1][0], ndc[1][1], ndc[2][0], ndc[2][1]) + K_EPSILON;
			for (int i = 0; i < 3; i++) a[i] = rho[i] * A;
		}
		float Dn[3][3][2];
		BaryWrtNdc(p, ndc, A, a, Dn);
		float J[3][9];   // d rho / d V (camera space)
		for (int i = 0; i < 3; i++) {
			const float z = V3[i][2];
			const float z2 = z * z;
			float Pj[2][3] = {{cam.fx / z, 0.f, -cam.fx * V3[i][0] / z2}, {0.f, cam.fy / z, -cam.fy * V3[i][1] / z2}};
			for (int r = 0; r < 3; r++)
				for (int c = 0; c < 3; c++) J[r][3 * i + c] = Dn[i][r][0] * Pj[0][c] + Dn[i][r][1] * Pj[1][c];
		}
		if (perspective_correct) {
			const float z0 = V3[0][2], z1 = V3[1][2], z2 = V3[2][2];
			const float v12 = z1 * z2, v02 = z0 * z2, v01 = z0 * z1;
			const float n0 = dist_rho[0] * v12, n1 = dist_rho[1] * v02, n2 = dist_rho[2] * v01;
			const float den = fmaxf(n0 + n1 + n2, K_EPSILON);
			const float den2 = den * den;
			float Pd[3][3] = {{(den - n0) * v12, -n0 * v02, -n0 * v01},
			                  {-n1 * v12, (den - n1) * v02, -n1 * v01},
			                  {-n2 * v12, -n2 * v02, (den - n2) * v01}};
			const float pz0 = dist_rho[1] * z2 + z1 * dist_rho[2];
			const float pz1 = dist_rho[0] * z2 + z0 * dist_rho[2];
			const float pz2 = dist_rho[0] * z1 + z0 * dist_rho[1];
			float Pz[3][3] = {{-n0 * pz0, den * dist_rho[0] * z2 - n0 * pz1, den * dist_rho[0] * z1 - n0 * pz2},
			                  {den * dist_rho[1] * z2 - n1 * pz0, -n1 * pz1, den * dist_rho[1] * z0 - n1 * pz2},
			                  {den * dist_rho[2] * z1 - n2 * pz0, den * dist_rho[2] * z0 - n2 * pz1, -n2 * pz2}};
			for (int r = 0; r < 3; r++) for (int c = 0; c < 3; c++) { Pd[r][c] /= den2; Pz[r][c] /= den2; }
			float J2[3][9];
			for (int r = 0; r < 3; r++)
				for (int c = 0; c < 9; c++) J2[r][c] = (Pd[r][0] * J[0][c] + Pd[r][1] * J[1][c]) + Pd[r][2] * J[2][c];
			for (int r = 0; r < 3; r++) for (int i = 0; i < 3; i++) J2[r][3 * i + 2] += Pz[r][i];
			std::memcpy(J, J2, sizeof(J));
		}
		float* ov = out_vj + pix * 27;
		float* on = out_nj + pix * 30;
		for (int r = 0; r < 3; r++) {
			for (int c = 0; c < 9; c++) {
				ov[9 * r + c] = (V3[0][r] * J[0][c] + V3[1][r] * J[1][c]) + V3[2][r] * J[2][c];
				on[9 * r + c] = (N3[0][r] * J[0][c] + N3[1][r] * J[1][c]) + N3[2][r] * J[2][c];
			}
			for (int i = 0; i < 3; i++) ov[9 * r + 3 * i + r] += rho[i];   // + rho (x) I_3 (KroneckerTensorProduct.h)
		}
		for (int i = 0; i < 3; i++) on[27 + i] = rho[i];
	}
}

// cpp/alignment/functional/kernel/AssociateFacesWithAnchorsImpl.h:34-107. out_nodes [F,3K], out_vertex_slots [F,3K,3] (-1 = none)
ORC_API void orc_associate_faces_with_anchors(const int64_t* faces, int64_t F, const int32_t* anchors, int K, int32_t* out_nodes,
                                              int32_t* out_vertex_slots, int32_t* out_counts) {
	const int M = 3 * K;
#pragma omp parallel for schedule(static)
	for (int64_t f = 0; f < F; f++) {
		int32_t* nodes = out_nodes + f * M;
		int32_t* slots = out_vertex_slots + f * M * 3;
		for (int i = 0; i < M; i++) { nodes[i] = -1; slots[3 * i] = slots[3 * i + 1] = slots[3 * i + 2] = -1; }
		int count = 0;
		for (int fv = 0; fv < 3; fv++) {
			int64_t v = faces[3 * f + fv];
			for (int k = 0; k < K; k++) {
				int32_t n = anchors[v * K + k];
				if (n == -1) continue;
				int i = 0;
				int inspected = nodes[i];
				while (inspected != n && inspected != -1 && i + 1 < M) { i++; inspected = nodes[i]; }
				if (inspected != n) { count++; nodes[i] = n; }
				slots[3 * i + fv] = k;
			}
		}
		out_counts[f] = count;
	}
}

// cpp/alignment/functional/kernel/PixelVertexAnchorJacobiansImpl.h:179-363.
// mode: 0 ALL (stride 6), 1 TRANSLATION_ONLY (stride 3, warped_vj = weights [V,K]), 2 ROTATION_ONLY (stride 3)
// out_pixel_jacobians [P, 3K, stride]; out_pixel_counts [P]
ORC_API void orc_pixel_vertex_anchor_jacobians(const float* rast_vj, const float* rast_nj, const float* warped_vj, const float* warped_nj,
                                               int K, const float* point_map_vectors, const float* rasterized_normals,
                                               const uint8_t* residual_mask, const int64_t* pixel_faces, int Kf, const int64_t* faces,
                                               const int32_t* face_nodes, const int32_t* face_slots, const int32_t* face_counts, int64_t P,
                                               int use_tukey, float tukey_cutoff, int mode, float* out_pixel_jacobians,
                                               int32_t* out_pixel_counts) {
	const int stride = mode == 0 ? 6 : 3;
	const int M = 3 * K;
	std::memset(out_pixel_jacobians, 0, sizeof(float) * P * M * stride);
	std::memset(out_pixel_counts, 0, sizeof(int32_t) * P);
#pragma omp parallel for schedule(static)
	for (int64_t pix = 0; pix < P; pix++) {
		if (!residual_mask[pix]) continue;
		const float* d = point_map_vectors + 3 * pix;
		const float* nl = rasterized_normals + 3 * pix;
		float dr_dnl[3], dr_dwl[3];
		if (use_tukey) {
			float r = dot3(nl, d);
			if (fabsf(r) > tukey_cutoff) continue;
			float q = r / tukey_cutoff;
			float psi = 1 - q * q;
			psi = r * psi * psi;
			for (int c = 0; c < 3; c++) { dr_dnl[c] = psi * d[c]; dr_dwl[c] = psi * nl[c]; }
		} else {
			for (int c = 0; c < 3; c++) { dr_dnl[c] = d[c]; dr_dwl[c] = nl[c]; }
		}
		const float* Jw = rast_vj + pix * 27;
		const float* Jn = rast_nj + pix * 30;
		float dr_dV[9], dr_dN[9];
		for (int c = 0; c < 9; c++) {
			float a = (dr_dwl[0] * Jw[c] + dr_dwl[1] * Jw[9 + c]) + dr_dwl[2] * Jw[18 + c];
			float b = (dr_dnl[0] * Jn[c] + dr_dnl[1] * Jn[9 + c]) + dr_dnl[2] * Jn[18 + c];
			dr_dV[c] = a + b;
		}
		for (int i = 0; i < 3; i++) for (int c = 0; c < 3; c++) dr_dN[3 * i + c] = dr_dnl[c] * Jn[27 + i];
		int64_t f = pixel_faces[pix * Kf];
		int count = face_counts[f];
		out_pixel_counts[pix] = count;
		float* pj = out_pixel_jacobians + pix * M * stride;
		for (int ia = 0; ia < count; ia++) {
			float* rot = mode == 1 ? nullptr : pj + ia * stride;
			float* tr = mode == 0 ? pj + ia * stride + 3 : (mode == 1 ? pj + ia * stride : nullptr);
			for (int fv = 0; fv < 3; fv++) {
				int32_t slot = face_slots[(f * M + ia) * 3 + fv];
				if (slot == -1) continue;
				int64_t vtx = faces[3 * f + fv];
				const float* dv = dr_dV + 3 * fv;
				float w = mode == 1 ? warped_vj[vtx * K + slot] : warped_vj[(vtx * K + slot) * 4 + 3];
				if (g_jac_fma) {   // fused mode (see g_jac_fma): the GPU's FMA order, term for term
					if (tr) for (int c = 0; c < 3; c++) tr[c] = std::fmaf(dv[c], w, tr[c]);
					if (rot) {
						const float* dn = dr_dN + 3 * fv;
						const float* p = warped_vj + (vtx * K + slot) * 4;
						const float* q = warped_nj + (vtx * K + slot) * 3;
						const float cr[3] = {std::fmaf(dv[1], p[2], std::fmaf(-dv[2], p[1], std::fmaf(dn[1], q[2], -dn[2] * q[1]))),
						                     std::fmaf(dv[2], p[0], std::fmaf(-dv[0], p[2], std::fmaf(dn[2], q[0], -dn[0] * q[2]))),
						                     std::fmaf(dv[0], p[1], std::fmaf(-dv[1], p[0], std::fmaf(dn[0], q[1], -dn[1] * q[0])))};
						for (int c = 0; c < 3; c++) rot[c] = std::fmaf(-w, cr[c], rot[c]);
					}
					continue;
				}
				if (tr) for (int c = 0; c < 3; c++) tr[c] += dv[c] * w;
				if (rot) {
					const float* dn = dr_dN + 3 * fv;
					float t1[3], t2[3];
					row_times_skew(dv, warped_vj + (vtx * K + slot) * 4, t1);
					row_times_skew(dn, warped_nj + (vtx * K + slot) * 3, t2);
					for (int c = 0; c < 3; c++) rot[c] += t1[c] + t2[c];
				}
			}
		}
	}
}

// Summation precision of the data-term JtJ / Jt r. The reference sums the float products serially in float
// (DeformableMeshToImageFitterImpl.h:199-456); on ill-conditioned node blocks that rounding alone moves the solved
// update by up to ~4e-4 relative (C2), so the checker sums the same float products in double (default, = the exactly
// summed reference data term) and keeps the float-serial order available to measure that noise.
static int g_acc_double = 1;
ORC_API void orc_set_accumulate_double(int on) { g_acc_double = on; }

// DeformableMeshToImageFitterImpl.h:199-456 : block-diagonal data JtJ and -Jt r, node lists in ascending (pixel, slot) order.
// out_H [N, s, s], out_g [N*s]
ORC_API void orc_data_hessian_gradient(const float* pixel_jacobians, const int32_t* pixel_counts, const int64_t* pixel_faces, int Kf,
                                       const int32_t* face_nodes, int K, const float* residuals, const uint8_t* residual_mask, int64_t P, int N,
                                       int mode, float* out_H, float* out_g) {
	const int s = mode == 0 ? 6 : 3;
	const int M = 3 * K;
	std::vector<int64_t> offsets(N + 1, 0);
	for (int64_t p = 0; p < P; p++) {
		int c = pixel_counts[p];
		if (c == 0) continue;
		int64_t f = pixel_faces[p * Kf];
		for (int ia = 0; ia < c; ia++) offsets[face_nodes[f * M + ia] + 1]++;
	}
	for (int n = 0; n < N; n++) offsets[n + 1] += offsets[n];
	std::vector<int64_t> addr(offsets[N]);
	std::vector<int64_t> fill(offsets.begin(), offsets.end() - 1);
	for (int64_t p = 0; p < P; p++) {
		int c = pixel_counts[p];
		if (c == 0) continue;
		int64_t f = pixel_faces[p * Kf];
		for (int ia = 0; ia < c; ia++) addr[fill[face_nodes[f * M + ia]]++] = p * M + ia;
	}
#pragma omp parallel for schedule(dynamic, 4)
	for (int n = 0; n < N; n++) {
		for (int c0 = 0; c0 < s; c0++) {
			for (int c1 = c0; c1 < s; c1++) {
				float acc = 0.0f;
				double accd = 0.0;
				for (int64_t e = offsets[n]; e < offsets[n + 1]; e++) {
					const float* J = pixel_jacobians + addr[e] * s;
					if (g_acc_double) accd += static_cast<double>(J[c0] * J[c1]);
					else acc += J[c0] * J[c1];
				}
				if (g_acc_double) acc = static_cast<float>(accd);
				out_H[n * s * s + c0 * s + c1] = acc;
				out_H[n * s * s + c1 * s + c0] = acc;
			}
		}
		float gsum[6] = {0, 0, 0, 0, 0, 0};
		double gsumd[6] = {0, 0, 0, 0, 0, 0};
		for (int64_t e = offsets[n]; e < offsets[n + 1]; e++) {
			int64_t p = addr[e] / M;
			if (!residual_mask[p]) continue;
			const float* J = pixel_jacobians + addr[e] * s;
			for (int c = 0; c < s; c++) {
				if (g_acc_double) gsumd[c] += static_cast<double>(J[c] * residuals[p]);
				else gsum[c] += J[c] * residuals[p];
			}
		}
		if (g_acc_double) for (int c = 0; c < s; c++) gsum[c] = static_cast<float>(gsumd[c]);
		for (int c = 0; c < s; c++) out_g[n * s + c] = 0.f - gsum[c];
	}
}

// =====================================================================================================================
// ARAP: residuals DeformableMeshToImageFitterImpl.h:644-784 (fixed-coverage weight indexed by node_j: A3),
// Huber DeformableMeshToImageFitter.cpp:434-444, edge Jacobians ArapJacobianImpl.h:35-209,
// Hessian ArapHessianImpl.h:44-195, gradient DeformableMeshToImageFitterImpl.h:464-563 (mode ALL).
// node_weights == nullptr -> fixed coverage (radii + edge layers), else variable (max of node c^2).
// =====================================================================================================================
ORC_API int orc_arap_residuals(const int32_t* edges, int E, const int8_t* edge_layers, const float* radii, const float* node_weights,
                               const float* nodes, const float* rotations, const float* translations, float lambda, int use_huber,
                               float huber_delta, float* out_res) {
	for (int e = 0; e < E; e++) {
		int i = edges[2 * e], j = edges[2 * e + 1];
		float w;
		if (node_weights) w = fmaxf(node_weights[i], node_weights[j]);
		else {
			if (j >= E) { g_error = "fixed-coverage ARAP residual indexes edge_layer_indices[node_j] out of bounds (reference A3)"; return 1; }
			w = radii[edge_layers[j]];
		}
		const float *gi = nodes + 3 * i, *gj = nodes + 3 * j, *ti = translations + 3 * i, *tj = translations + 3 * j;
		float d[3] = {gi[0] - gj[0], gi[1] - gj[1], gi[2] - gj[2]}, Rd[3];
		matvec3(rotations + 9 * i, d, Rd);
		float lw = lambda * w;
		for (int c = 0; c < 3; c++) out_res[3 * e + c] = lw * (((gi[c] + ti[c]) - (gj[c] + tj[c])) - Rd[c]);
	}
	if (use_huber) {
		float half = 0.5f * huber_delta * huber_delta;
		for (int e = 0; e < 3 * E; e++) {
			float r = out_res[e];
			out_res[e] = (r >= huber_delta) ? fabsf(r) - half : 0.5f * r * r;
		}
	}
	return 0;
}

ORC_API void orc_arap_edge_jacobians(const int32_t* edges, int E, const int8_t* edge_layers, const float* radii, const float* node_weights,
                                     const float* nodes, const float* rotations, float lambda, float* out_j) {
	for (int e = 0; e < E; e++) {
		int i = edges[2 * e], j = edges[2 * e + 1];
		float w = node_weights ? fmaxf(node_weights[i], node_weights[j]) : radii[edge_layers[e]];
		out_j[5 * e + 3] = lambda * w;
		out_j[5 * e + 4] = -lambda * w;
		float d[3] = {nodes[3 * i] - nodes[3 * j], nodes[3 * i + 1] - nodes[3 * j + 1], nodes[3 * i + 2] - nodes[3 * j + 2]}, Rd[3];
		matvec3(rotations + 9 * i, d, Rd);
		float s = -lambda * w;
		for (int c = 0; c < 3; c++) out_j[5 * e + c] = s * Rd[c];
	}
}

namespace {
void EdgeDE(const float* j5, float dEi[3][6], float dEj[3][6]) {
	const float* a = j5;
	float sk[3][3] = {{0, -a[2], a[1]}, {a[2], 0, -a[0]}, {-a[1], a[0], 0}};
	for (int r = 0; r < 3; r++) for (int c = 0; c < 6; c++) { dEi[r][c] = 0; dEj[r][c] = 0; }
	for (int r = 0; r < 3; r++) { for (int c = 0; c < 3; c++) dEi[r][c] = sk[r][c]; dEi[r][3 + r] = j5[3]; dEj[r][3 + r] = j5[4]; }
}
void AtB36(const float A[3][6], const float B[3][6], float* out) {
	for (int r = 0; r < 6; r++) for (int c = 0; c < 6; c++) out[6 * r + c] = (A[0][r] * B[0][c] + A[1][r] * B[1][c]) + A[2][r] * B[2][c];
}
} // namespace

// out_diag [N,6,6] (ARAP part only), out_wing [E,6,6] (dEi^T dEj for every edge, at block (i, j))
ORC_API void orc_arap_hessian(const int32_t* edges, int E, const float* edge_j, int N, float* out_diag, float* out_wing) {
	std::memset(out_diag, 0, sizeof(float) * N * 36);
	for (int e = 0; e < E; e++) {
		float dEi[3][6], dEj[3][6];
		EdgeDE(edge_j + 5 * e, dEi, dEj);
		AtB36(dEi, dEj, out_wing + 36 * e);
	}
	for (int w = 0; w < 2 * E; w++) {
		int e = w / 2;
		float dEi[3][6], dEj[3][6], blk[36];
		EdgeDE(edge_j + 5 * e, dEi, dEj);
		if (w % 2 == 0) AtB36(dEi, dEi, blk); else AtB36(dEj, dEj, blk);
		int n = edges[w];
		for (int k = 0; k < 36; k++) out_diag[36 * n + k] += blk[k];
	}
}

// adds -J_arap^T e into g (mode ALL, stride 6)
ORC_API void orc_arap_gradient(const int32_t* edges, int E, const float* edge_j, const float* res, float* g) {
	for (int wk = 0; wk < 3 * E; wk++) {
		int e = wk / 3, part = wk % 3;
		const float* a = edge_j + 5 * e;
		const float* r = res + 3 * e;
		float add[3];
		int node, off;
		if (part == 0) {
			float skT[3][3] = {{0, a[2], -a[1]}, {-a[2], 0, a[0]}, {a[1], -a[0], 0}};
			for (int c = 0; c < 3; c++) add[c] = (skT[c][0] * r[0] + skT[c][1] * r[1]) + skT[c][2] * r[2];
			node = edges[2 * e]; off = 0;
		} else if (part == 1) {
			for (int c = 0; c < 3; c++) add[c] = a[3] * r[c];
			node = edges[2 * e]; off = 3;
		} else {
			for (int c = 0; c < 3; c++) add[c] = a[4] * r[c];
			node = edges[2 * e + 1]; off = 3;
		}
		for (int c = 0; c < 3; c++) g[node * 6 + off + c] -= add[c];
	}
}

// =====================================================================================================================
// Solvers: cpp/core/linalg/SolveBlockDiagonalCholeskyCPU.cpp:30-96 (potrf + 2 trsm per block),
// SolveBlockSparseArrowheadCholesky.cpp:30-95 + SchurComplement.cpp:44-79 (uncapped math; corner off-diagonal
// blocks included for >=3-layer graphs as apps/math_experimental_scripts/sparse_block_cholesky_scripts.py:106-160).
// =====================================================================================================================
namespace {
// in-place lower Cholesky of row-major n x n SPD matrix (LAPACK potrf semantics); returns false if not PD
bool CholeskyInPlace(float* A, int n) {
	for (int j = 0; j < n; j++) {
		float s = A[j * n + j];
		for (int k = 0; k < j; k++) s -= A[j * n + k] * A[j * n + k];
		if (!(s > 0.f)) return false;
		float l = sqrtf(s);
		A[j * n + j] = l;
		for (int i = j + 1; i < n; i++) {
			float t = A[i * n + j];
			for (int k = 0; k < j; k++) t -= A[i * n + k] * A[j * n + k];
			A[i * n + j] = t / l;
		}
	}
	for (int i = 0; i < n; i++) for (int j = i + 1; j < n; j++) A[i * n + j] = 0.f;
	return true;
}
void CholeskySolveInPlace(const float* L, int n, float* b) {
	for (int i = 0; i < n; i++) { float s = b[i]; for (int k = 0; k < i; k++) s -= L[i * n + k] * b[k]; b[i] = s / L[i * n + i]; }
	for (int i = n - 1; i >= 0; i--) { float s = b[i]; for (int k = i + 1; k < n; k++) s -= L[k * n + i] * b[k]; b[i] = s / L[i * n + i]; }
}
} // namespace

// InvertBlocks.cpp:82-126 (InvertPositiveSemidefiniteBlocks): potrf, then potrs against the identity, per block.
// Returns 0, or 1 + the first block whose potrf fails.
ORC_API int orc_invert_psd_blocks(const float* blocks, int N, int s, float* out) {
	int fail = 0;
	for (int n = 0; n < N; n++) {
		float L[36];
		for (int i = 0; i < s * s; i++) L[i] = blocks[static_cast<int64_t>(n) * s * s + i];
		if (!CholeskyInPlace(L, s)) {
			if (!fail) fail = n + 1;
			continue;
		}
		for (int c = 0; c < s; c++) {
			float col[6] = {0, 0, 0, 0, 0, 0};
			col[c] = 1.f;
			CholeskySolveInPlace(L, s, col);
			for (int r = 0; r < s; r++) out[static_cast<int64_t>(n) * s * s + r * s + c] = col[r];
		}
	}
	return fail;
}

// lm: added to block diagonals first (PreconditionDiagonalBlocksImpl.h), if > 0. Returns 0, or 1 + failing block.
ORC_API int orc_solve_block_diagonal(const float* H, const float* g, int N, int s, float lm, float* x) {
	int fail = 0;
	for (int n = 0; n < N; n++) {
		float A[36];
		std::memcpy(A, H + n * s * s, sizeof(float) * s * s);
		if (lm > 0.f) for (int i = 0; i < s; i++) A[i * s + i] += lm;
		if (!CholeskyInPlace(A, s)) { if (!fail) fail = n + 1; for (int i = 0; i < s; i++) x[n * s + i] = NAN; continue; }
		for (int i = 0; i < s; i++) x[n * s + i] = g[n * s + i];
		CholeskySolveInPlace(A, s, x + n * s);
	}
	if (fail) g_error = "potrf failed in SolveBlockDiagonalCholesky (block not positive-definite)";
	return fail;
}

// H = diag blocks [N,6,6] (already including LM), wing blocks [E,6,6] at (edges[e][0], edges[e][1]); stem = first n0 blocks.
ORC_API int orc_solve_arrowhead(const float* diag, const float* wing, const int32_t* edges, int E, int N, int n0, const float* g, float* x) {
	const int n1 = N - n0, m = 6 * n1;
	std::vector<float> Dinv(static_cast<size_t>(n0) * 36);
	for (int i = 0; i < n0; i++) {
		float L[36];
		std::memcpy(L, diag + 36 * i, sizeof(L));
		if (!CholeskyInPlace(L, 6)) { g_error = "stem block not positive-definite"; return 1; }
		for (int c = 0; c < 6; c++) {
			float col[6] = {0, 0, 0, 0, 0, 0};
			col[c] = 1.f;
			CholeskySolveInPlace(L, 6, col);
			for (int r = 0; r < 6; r++) Dinv[36 * i + 6 * r + c] = col[r];
		}
	}
	// dense corner C
	std::vector<float> S(static_cast<size_t>(m) * m, 0.f);
	for (int j = 0; j < n1; j++) for (int r = 0; r < 6; r++) for (int c = 0; c < 6; c++) S[(6 * j + r) * m + 6 * j + c] = diag[36 * (n0 + j) + 6 * r + c];
	std::vector<std::vector<int>> stem_edges(n0);
	for (int e = 0; e < E; e++) {
		int i = edges[2 * e], j = edges[2 * e + 1];
		if (i < n0) stem_edges[i].push_back(e);
		else {   // corner off-diagonal block (>=3 layers)
			int a = i - n0, b = j - n0;
			for (int r = 0; r < 6; r++) for (int c = 0; c < 6; c++) {
				S[(6 * a + r) * m + 6 * b + c] += wing[36 * e + 6 * r + c];
				S[(6 * b + c) * m + 6 * a + r] += wing[36 * e + 6 * r + c];
			}
		}
	}
	// DinvB per stem edge, S -= B^T Dinv B
	std::vector<float> DB(static_cast<size_t>(E) * 36, 0.f);
	for (int i = 0; i < n0; i++) {
		for (int e : stem_edges[i]) {
			for (int r = 0; r < 6; r++) for (int c = 0; c < 6; c++) {
				float acc = 0.f;
				for (int k = 0; k < 6; k++) acc += Dinv[36 * i + 6 * r + k] * wing[36 * e + 6 * k + c];
				DB[36 * e + 6 * r + c] = acc;
			}
		}
		for (int e1 : stem_edges[i]) for (int e2 : stem_edges[i]) {
			int a = edges[2 * e1 + 1] - n0, b = edges[2 * e2 + 1] - n0;
			for (int r = 0; r < 6; r++) for (int c = 0; c < 6; c++) {
				float acc = 0.f;
				for (int k = 0; k < 6; k++) acc += wing[36 * e1 + 6 * k + r] * DB[36 * e2 + 6 * k + c];
				S[(6 * a + r) * m + 6 * b + c] -= acc;
			}
		}
	}
	// b_C' = b_C - B^T Dinv b_D
	std::vector<float> bc(m);
	for (int k = 0; k < m; k++) bc[k] = g[6 * n0 + k];
	for (int i = 0; i < n0; i++) for (int e : stem_edges[i]) {
		int a = edges[2 * e + 1] - n0;
		for (int c = 0; c < 6; c++) {
			float acc = 0.f;
			for (int k = 0; k < 6; k++) acc += DB[36 * e + 6 * k + c] * g[6 * i + k];
			bc[6 * a + c] -= acc;
		}
	}
	if (m > 0) {
		if (!CholeskyInPlace(S.data(), m)) { g_error = "Schur complement not positive-definite"; return 2; }
		CholeskySolveInPlace(S.data(), m, bc.data());
	}
	for (int k = 0; k < m; k++) x[6 * n0 + k] = bc[k];
	for (int i = 0; i < n0; i++) {
		float rhs[6];
		for (int c = 0; c < 6; c++) rhs[c] = g[6 * i + c];
		for (int e : stem_edges[i]) {
			int a = edges[2 * e + 1] - n0;
			for (int r = 0; r < 6; r++) {
				float acc = 0.f;
				for (int k = 0; k < 6; k++) acc += wing[36 * e + 6 * r + k] * bc[6 * a + k];
				rhs[r] -= acc;
			}
		}
		for (int r = 0; r < 6; r++) {
			float acc = 0.f;
			for (int k = 0; k < 6; k++) acc += Dinv[36 * i + 6 * r + k] * rhs[k];
			x[6 * i + r] = acc;
		}
	}
	return 0;
}

// cpp/core/linalg/RodriguesImpl.h:66-88 (NaN at |w| = 0 reproduced: A7)
ORC_API void orc_rodrigues(const float* w, int N, float* R) {
	for (int n = 0; n < N; n++) {
		const float* a = w + 3 * n;
		float ang = sqrtf((a[0] * a[0] + a[1] * a[1]) + a[2] * a[2]);
		float ax[3] = {a[0] / ang, a[1] / ang, a[2] / ang};
		float K[3][3] = {{0, -ax[2], ax[1]}, {ax[2], 0, -ax[0]}, {-ax[1], ax[0], 0}};
		float s = sin_cr(ang), c1 = 1 - cos_cr(ang);
		for (int r = 0; r < 3; r++) for (int c = 0; c < 3; c++) {
			float K2 = (K[r][0] * K[0][c] + K[r][1] * K[1][c]) + K[r][2] * K[2][c];
			R[9 * n + 3 * r + c] = ((r == c ? 1.f : 0.f) + s * K[r][c]) + c1 * K2;
		}
	}
}

// =====================================================================================================================
// FitToImage driver: cpp/alignment/DeformableMeshToImageFitter.cpp:85-390 (loop 111-275), operating in virtual node
// order (A5). The warp field arrays (nodes, R, t) are in virtual order and updated in place.
// =====================================================================================================================
struct OrcFitParams {
	int max_iterations;
	int mode_count;
	int modes[16];
	int use_perspective_correction;
	float max_depth;
	int use_tukey;
	float tukey_cutoff;
	float lm_factor;
	float arap_weight;
	int use_huber;
	float huber_delta;
	int ndc_consistent;   // NNRT_NDC_CONSISTENT: see IntrinsicsToNdc
};

struct OrcWarpField {
	int N, K;
	float coverage;
	int coverage_method;          // 0 FIXED_NODE_COVERAGE, 1 MINIMAL_K_NEIGHBOR_NODE_DISTANCE
	int min_valid_anchors;
	const float* nodes;           // [N,3] virtual order
	float* rotations;             // [N,9]
	float* translations;          // [N,3]
	const float* node_weights;    // [N] (coverage_method 1)
	int E;
	const int32_t* edges;         // [E,2]
	const int8_t* edge_layers;    // [E]
	const float* radii;           // [layers]
	int first_layer_count;        // n0
};

struct OrcFitOutputs {            // optional diagnostics of the LAST iteration (nullable)
	float* residuals;             // [P]
	uint8_t* residual_mask;       // [P]
	int64_t* pixel_faces;         // [P]
	float* updates;               // [N*6]
	float* gradient;              // [N*6]
	float* hessian_diag;          // [N*36]
	double* stage_seconds;        // [8]
};

namespace {
double Now() {
#ifdef _OPENMP
	return omp_get_wtime();
#else
	return 0.0;
#endif
}
} // namespace

ORC_API int orc_fit(const OrcFitParams* prm, OrcWarpField* wf, const float* mesh_points, const float* mesh_normals, int64_t V,
                    const int64_t* faces, int64_t F, const float* ref_points, const uint8_t* ref_mask, int H, int W, const double* K,
                    const double* extrinsics, int fast_raster, OrcFitOutputs* outs) {
	const int64_t P = static_cast<int64_t>(H) * W;
	const int N = wf->N, KA = wf->K;
	const bool use_reg = wf->E > 0;
	// consistent NDC: rows keep image order, which negates NDC face areas; swapping two corners keeps front faces front
	struct NdcModeGuard { NdcModeGuard(bool on) { g_ndc_consistent = on; } ~NdcModeGuard() { g_ndc_consistent = false; } } ndc_mode(prm->ndc_consistent != 0);
	std::vector<int64_t> swapped;
	if (prm->ndc_consistent) {
		swapped.assign(faces, faces + 3 * F);
		for (int64_t f = 0; f < F; f++) std::swap(swapped[3 * f + 1], swapped[3 * f + 2]);
		faces = swapped.data();
	}
	if (prm->lm_factor < 0.f || prm->lm_factor > 1.f) { g_error = "`preconditioning_dampening_factor` should be between 0 and 1"; return 10; }
	std::vector<int32_t> anchors(V * KA);
	std::vector<float> weights(V * KA);
	orc_compute_anchors(mesh_points, V, wf->nodes, N, KA, wf->coverage, wf->coverage_method == 1 ? wf->node_weights : nullptr,
	                    wf->min_valid_anchors, anchors.data(), weights.data());
	const int M = 3 * KA;
	std::vector<int32_t> fnodes(F * M), fslots(F * M * 3), fcounts(F);
	orc_associate_faces_with_anchors(faces, F, anchors.data(), KA, fnodes.data(), fslots.data(), fcounts.data());

	std::vector<float> wpts(V * 3), wnrm(V * 3), fndc(F * 9), depth(P), bary(P * 3), dist(P), rnorm(P * 3), rpts(P * 3), res(P), pmv(P * 3);
	std::vector<uint8_t> fmask(F), rmask(P), resmask(P);
	std::vector<int64_t> pface(P);
	std::vector<float> face_nrm(F * 9), vj(V * KA * 4), nj(V * KA * 3), rvj(P * 27), rnj(P * 30), pj(P * M * 6), Hd(N * 36), g(N * 6), x(N * 6);
	std::vector<int32_t> pcounts(P);
	double tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
	int s = 6;
	auto write_outs = [&]() {
		if (!outs) return;
		if (outs->residuals) std::memcpy(outs->residuals, res.data(), sizeof(float) * P);
		if (outs->residual_mask) std::memcpy(outs->residual_mask, resmask.data(), P);
		if (outs->pixel_faces) std::memcpy(outs->pixel_faces, pface.data(), sizeof(int64_t) * P);
		if (outs->updates) std::memcpy(outs->updates, x.data(), sizeof(float) * N * s);
		if (outs->gradient) std::memcpy(outs->gradient, g.data(), sizeof(float) * N * s);
		if (outs->hessian_diag) std::memcpy(outs->hessian_diag, Hd.data(), sizeof(float) * N * s * s);
	};
	for (int it = 0; it < prm->max_iterations; it++) {
		const int mode = prm->modes[it % prm->mode_count];
		s = mode == 0 ? 6 : 3;
		double t0 = Now();
		orc_warp_mesh(mesh_points, mesh_normals, V, wf->nodes, wf->rotations, wf->translations, anchors.data(), weights.data(), KA, extrinsics,
		              wpts.data(), wnrm.data());
		orc_extract_face_ndc(wpts.data(), faces, F, K, H, W, 0.0f, 10.0f, fndc.data(), fmask.data());
		double t1 = Now();
		int rc = fast_raster ? orc_rasterize_k1_fast(fndc.data(), fmask.data(), F, H, W, 0.5f, prm->use_perspective_correction, 1, pface.data(),
		                                             depth.data(), bary.data(), dist.data())
		                     : orc_rasterize(fndc.data(), fmask.data(), F, H, W, 0.5f, 1, -1, -1, prm->use_perspective_correction, 0, 1,
		                                     pface.data(), depth.data(), bary.data(), dist.data());
		if (rc) return rc;
		double t2 = Now();
		// ComputeDepthResiduals (:331-390)
		for (int64_t f = 0; f < F; f++) for (int i = 0; i < 3; i++) for (int c = 0; c < 3; c++) face_nrm[9 * f + 3 * i + c] = wnrm[3 * faces[3 * f + i] + c];
		orc_interpolate_face_attributes(pface.data(), bary.data(), P, 1, face_nrm.data(), 3, rnorm.data());
		orc_unproject(depth.data(), H, W, K, 1.0f, prm->max_depth, rpts.data(), rmask.data());
		for (int64_t p = 0; p < P; p++) {
			float dd[3] = {rpts[3 * p] - ref_points[3 * p], rpts[3 * p + 1] - ref_points[3 * p + 1], rpts[3 * p + 2] - ref_points[3 * p + 2]};
			for (int c = 0; c < 3; c++) pmv[3 * p + c] = dd[c];
			float dist_p = dot3(&rnorm[3 * p], dd);
			resmask[p] = ref_mask[p] && rmask[p];
			if (!resmask[p]) dist_p = 0.0f;
			if (prm->use_tukey) {
				float c = prm->tukey_cutoff;
				float c6 = (c * c / 6.f);
				float q = dist_p / c;
				float left = 1.f - (q * q);
				float r = c6 * (1.f - left * left * left);
				if (dist_p <= c) r = c6;   // (:384-385, as written: A8)
				res[p] = r;
			} else res[p] = dist_p;
		}
		double t3 = Now();
		// Jacobians
		if (mode == 1) {
			orc_warped_surface_jacobians(mesh_points, mesh_normals, V, wf->nodes, wf->rotations, anchors.data(), weights.data(), KA, vj.data(), nj.data());
		} else {
			orc_warped_surface_jacobians(mesh_points, mesh_normals, V, wf->nodes, wf->rotations, anchors.data(), weights.data(), KA, vj.data(), nj.data());
		}
		orc_rasterized_surface_jacobians(wpts.data(), wnrm.data(), faces, pface.data(), bary.data(), H, W, 1, K, prm->use_perspective_correction,
		                                 rvj.data(), rnj.data());
		orc_pixel_vertex_anchor_jacobians(rvj.data(), rnj.data(), mode == 1 ? weights.data() : vj.data(), nj.data(), KA, pmv.data(), rnorm.data(),
		                                  resmask.data(), pface.data(), 1, faces, fnodes.data(), fslots.data(), fcounts.data(), P, prm->use_tukey,
		                                  prm->tukey_cutoff, mode, pj.data(), pcounts.data());
		double t4 = Now();
		orc_data_hessian_gradient(pj.data(), pcounts.data(), pface.data(), 1, fnodes.data(), KA, res.data(), resmask.data(), P, N, mode, Hd.data(),
		                          g.data());
		double t5 = Now();
		int frc = 0;
		if (use_reg) {
			if (mode != 0) { g_error = "regularized (ARAP) solve supports IterationMode ALL only (reference A15)"; return 11; }
			std::vector<float> eres(wf->E * 3), ej(wf->E * 5), adiag(N * 36), wing(wf->E * 36);
			const float* nw = wf->coverage_method == 1 ? wf->node_weights : nullptr;
			if (orc_arap_residuals(wf->edges, wf->E, wf->edge_layers, wf->radii, nw, wf->nodes, wf->rotations, wf->translations, prm->arap_weight,
			                       prm->use_huber, prm->huber_delta, eres.data())) return 12;
			orc_arap_edge_jacobians(wf->edges, wf->E, wf->edge_layers, wf->radii, nw, wf->nodes, wf->rotations, prm->arap_weight, ej.data());
			orc_arap_hessian(wf->edges, wf->E, ej.data(), N, adiag.data(), wing.data());
			for (int k = 0; k < N * 36; k++) adiag[k] += Hd[k];
			if (prm->lm_factor > 0.f) for (int n = 0; n < N; n++) for (int i = 0; i < 6; i++) adiag[36 * n + 7 * i] += prm->lm_factor;
			orc_arap_gradient(wf->edges, wf->E, ej.data(), eres.data(), g.data());
			frc = orc_solve_arrowhead(adiag.data(), wing.data(), wf->edges, wf->E, N, wf->first_layer_count, g.data(), x.data());
			if (frc) return 20 + frc;
		} else {
			frc = orc_solve_block_diagonal(Hd.data(), g.data(), N, s, prm->lm_factor, x.data());
			if (frc) {   // the reference throws here (NNRT_LAPACK_CHECK); the diagnostics keep this iteration (NaN updates on the failed blocks)
				write_outs();
				return 30;
			}
		}
		double t6 = Now();
		// S12 update (:257-273): R <- R * Rodrigues(w), t <- t + dt
		std::vector<float> w3(N * 3), dR(N * 9);
		if (mode == 0 || mode == 2) {
			for (int n = 0; n < N; n++) for (int c = 0; c < 3; c++) w3[3 * n + c] = x[n * s + c];
			orc_rodrigues(w3.data(), N, dR.data());
		}
		for (int n = 0; n < N; n++) {
			if (mode == 0) for (int c = 0; c < 3; c++) wf->translations[3 * n + c] += x[6 * n + 3 + c];
			if (mode == 1) for (int c = 0; c < 3; c++) wf->translations[3 * n + c] += x[3 * n + c];
			if (mode == 0 || mode == 2) {
				float R[9];
				const float* A = wf->rotations + 9 * n;
				const float* B = dR.data() + 9 * n;
				for (int r = 0; r < 3; r++) for (int c = 0; c < 3; c++) R[3 * r + c] = (A[3 * r] * B[c] + A[3 * r + 1] * B[3 + c]) + A[3 * r + 2] * B[6 + c];
				std::memcpy(wf->rotations + 9 * n, R, sizeof(R));
			}
		}
		double t7 = Now();
		tacc[0] += t1 - t0; tacc[1] += t2 - t1; tacc[2] += t3 - t2; tacc[3] += t4 - t3; tacc[4] += t5 - t4; tacc[5] += t6 - t5; tacc[6] += t7 - t6;
		tacc[7] += t7 - t0;
		if (it == prm->max_iterations - 1) write_outs();
	}
	if (outs && outs->stage_seconds) std::memcpy(outs->stage_seconds, tacc, sizeof(tacc));
	return 0;
}

// ---- block-sparse stages of the arrowhead solve (SolveBlockSparseArrowheadCholesky.cpp:30-95, SchurComplement.cpp:43-78).
// Every block product entry is a float sum over the inner index in ascending order starting from 0; products of several
// block pairs are added in ascending inner-block order (the first one taken as is). Returns 0, or 1 on a coordinate /
// block index outside the operands (the reference reads out of bounds there).

// MatmulBlockSparseImpl.h:39-157 (padded form): c_i = a[row_i] b_i, zero block + mask 0 where row_i >= a_count
ORC_API int orc_matmul_block_sparse_row_wise(const float* a, int a_count, const float* b, const int32_t* coords, int count, int s, float* c,
                                             uint8_t* mask) {
	const int64_t ss = static_cast<int64_t>(s) * s;
	int bad = 0;
	for (int i = 0; i < count; i++) {
		const int row = coords[2 * i];
		bad |= row < 0;
		const bool ok = row >= 0 && row < a_count;
		mask[i] = ok;
		for (int r = 0; r < s; r++)
			for (int q = 0; q < s; q++) {
				float acc = 0.f;
				if (ok)
					for (int l = 0; l < s; l++) acc += a[row * ss + r * s + l] * b[i * ss + l * s + q];
				c[i * ss + r * s + q] = acc;
			}
	}
	return bad;
}

// MatmulBlockSparseImpl.h:160-391: dense [out_rows * out_cols] output blocks + mask (the reference's meshgrid order)
ORC_API int orc_matmul_block_sparse(const float* a, int a_count, const int16_t* a_board, int a_rows, int a_cols, int ta, const float* b,
                                    int b_count, const int16_t* b_board, int b_rows, int b_cols, int tb, int s, float* c, uint8_t* mask) {
	const int out_rows = ta ? a_cols : a_rows, out_cols = tb ? b_rows : b_cols, inner = ta ? a_rows : a_cols;
	const int64_t ss = static_cast<int64_t>(s) * s;
	int bad = 0;
	for (int oi = 0; oi < out_rows; oi++)
		for (int oj = 0; oj < out_cols; oj++) {
			const int64_t ob = static_cast<int64_t>(oi) * out_cols + oj;
			std::vector<float> acc(ss, 0.f);
			bool any = false;
			for (int k = 0; k < inner; k++) {
				const int ia = ta ? a_board[k * a_cols + oi] : a_board[oi * a_cols + k];
				if (ia == -1) continue;
				const int ib = tb ? b_board[oj * b_cols + k] : b_board[k * b_cols + oj];
				if (ib == -1) continue;
				if (ia < 0 || ia >= a_count || ib < 0 || ib >= b_count) {
					bad = 1;
					continue;
				}
				for (int r = 0; r < s; r++)
					for (int q = 0; q < s; q++) {
						float p = 0.f;
						for (int l = 0; l < s; l++) {
							const float av = ta ? a[ia * ss + l * s + r] : a[ia * ss + r * s + l];
							const float bv = tb ? b[ib * ss + q * s + l] : b[ib * ss + l * s + q];
							p += av * bv;
						}
						acc[r * s + q] = any ? acc[r * s + q] + p : p;
					}
				any = true;
			}
			for (int e = 0; e < ss; e++) c[ob * ss + e] = acc[e];
			mask[ob] = any;
		}
	return bad;
}

// MatmulBlockSparseImpl.h:441-582: out[m] = op(A) v; per-block products added to their rows in block order
ORC_API int orc_block_sparse_vector(const float* blocks, const int32_t* coords, int count, int s, int row_off, int col_off, int ta,
                                    const float* v, int64_t n_v, float* out, int64_t m) {
	const int64_t ss = static_cast<int64_t>(s) * s;
	for (int64_t i = 0; i < m; i++) out[i] = 0.f;
	int bad = 0;
	for (int i = 0; i < count; i++) {
		const int64_t br = ta ? coords[2 * i + 1] + col_off : coords[2 * i] + row_off;
		const int64_t bc = ta ? coords[2 * i] + row_off : coords[2 * i + 1] + col_off;
		if (br < 0 || (br + 1) * s > m || bc < 0 || (bc + 1) * s > n_v) {
			bad = 1;
			continue;
		}
		for (int r = 0; r < s; r++) {
			float p = 0.f;
			for (int l = 0; l < s; l++) p += (ta ? blocks[i * ss + l * s + r] : blocks[i * ss + r * s + l]) * v[bc * s + l];
			out[br * s + r] += p;
		}
	}
	return bad;
}

// MatmulBlockSparseImpl.h:604-690
ORC_API void orc_diagonal_block_vector(const float* blocks, int count, int s, const float* v, float* out) {
	const int64_t ss = static_cast<int64_t>(s) * s;
	for (int i = 0; i < count; i++)
		for (int r = 0; r < s; r++) {
			float p = 0.f;
			for (int l = 0; l < s; l++) p += blocks[i * ss + r * s + l] * v[static_cast<int64_t>(i) * s + l];
			out[static_cast<int64_t>(i) * s + r] = p;
		}
}

// SparseBlocksImpl.h:30-190 (op 0 fill, 1 add, 2 subtract); coords == NULL: block i at (i, i) (FillInDiagonalBlocks)
ORC_API int orc_sparse_blocks_op(float* matrix, int64_t rows, int64_t cols, const float* blocks, const int32_t* coords, int count, int s,
                                 int64_t row_off, int64_t col_off, int transpose, int op) {
	const int64_t ss = static_cast<int64_t>(s) * s;
	int bad = 0;
	for (int64_t blk = 0; blk < count; blk++) {
		const int64_t ci = coords ? coords[2 * blk] : blk, cj = coords ? coords[2 * blk + 1] : blk;
		const int64_t br = (transpose ? cj : ci) + row_off, bc = (transpose ? ci : cj) + col_off;
		for (int e = 0; e < ss; e++) {
			const int64_t i = br * s + (transpose ? e % s : e / s), j = bc * s + (transpose ? e / s : e % s);
			if (br < 0 || bc < 0 || i >= rows || j >= cols) {
				bad = 1;
				continue;
			}
			float& d = matrix[i * cols + j];
			const float x = blocks[blk * ss + e];
			d = op == 0 ? x : op == 1 ? d + x : d - x;
		}
	}
	return bad;
}

// SparseBlocksImpl.h:192-230; coords == NULL: GetDiagonalBlocks
ORC_API int orc_get_sparse_blocks(const float* matrix, int64_t rows, int64_t cols, int s, const int32_t* coords, int count, float* blocks) {
	const int64_t ss = static_cast<int64_t>(s) * s;
	int bad = 0;
	for (int64_t blk = 0; blk < count; blk++) {
		const int64_t br = coords ? coords[2 * blk] : blk, bc = coords ? coords[2 * blk + 1] : blk;
		for (int e = 0; e < ss; e++) {
			const int64_t i = br * s + e / s, j = bc * s + e % s;
			if (br < 0 || bc < 0 || i >= rows || j >= cols) {
				bad = 1;
				blocks[blk * ss + e] = NAN;
				continue;
			}
			blocks[blk * ss + e] = matrix[i * cols + j];
		}
	}
	return bad;
}

// InvertBlocksCPU.cpp (trtri per block): column j of the inverse by substitution; returns 1 on a zero diagonal entry
ORC_API int orc_invert_triangular_blocks(const float* blocks, int count, int s, int upper, float* out) {
	const int64_t ss = static_cast<int64_t>(s) * s;
	int bad = 0;
	for (int64_t blk = 0; blk < count; blk++) {
		const float* A = blocks + blk * ss;
		float* X = out + blk * ss;
		for (int j = 0; j < s; j++) {
			if (!upper) {
				for (int i = 0; i < j; i++) X[i * s + j] = 0.f;
				for (int i = j; i < s; i++) {
					float acc = 0.f;
					for (int k = j; k < i; k++) acc += A[i * s + k] * X[k * s + j];
					const float d = A[i * s + i];
					bad |= d == 0.f;
					X[i * s + j] = i == j ? 1.f / d : -acc / d;
				}
			} else {
				for (int i = j + 1; i < s; i++) X[i * s + j] = 0.f;
				for (int i = j; i >= 0; i--) {
					float acc = 0.f;
					for (int k = i + 1; k <= j; k++) acc += A[i * s + k] * X[k * s + j];
					const float d = A[i * s + i];
					bad |= d == 0.f;
					X[i * s + j] = i == j ? 1.f / d : -acc / d;
				}
			}
		}
	}
	return bad;
}
