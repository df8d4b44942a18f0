// Warp-field construction on the GPU ("hierarchy construction"): the O(n^2) parts of
// HierarchicalGraphWarpField::RebuildRegularizationLayers (cpp/geometry/HierarchicalGraphWarpField.cpp:74-199) and of the
// MINIMAL_K_NEIGHBOR_NODE_DISTANCE coverage weights (cpp/geometry/WarpField.cpp:249-263). The layer bookkeeping (which
// node goes to which layer, virtual order, edge layout) stays in warp_field.cpp; it consumes the three results below.
//   * k_grid_keys / k_medoid_sums / k_medoid_flags: median-grid subsampling (GeometrySamplingMedian.h:260-290,
//     GeometrySamplingGridBinning.h:27-46): per grid cell the member whose summed distance to the cell's members is
//     smallest (first such member in ascending point order). Sums run over the members in ascending point order, so
//     the float sums -- and the chosen medoids -- are those of the sequential restatement, bit for bit.
//   * k_knn_rows: K nearest coarse-layer nodes of every finer-layer node (KdTree K-NN in the reference,
//     HierarchicalGraphWarpFieldImpl.h:218-297), ordered by (squared distance, index) like std::partial_sort over pairs,
//     then each row sorted by descending index (-1 padding last).
//   * k_node_coverage: squared distance to the nearest other node, replaying WarpField.cpp:249-263's replace-the-larger
//     two-slot scan in ascending node order.
// Every kernel scans the candidate set in LDS tiles of HB nodes, each lane owning one query node. All float expressions
// keep the restatement's order (-ffp-contract=off, correctly rounded sqrt).
#include <algorithm>
#include <cfloat>

#include <hipcub/hipcub.hpp>

#include "common.hpp"
#include "warp_field.hpp"

namespace nnrt {

namespace {
constexpr int HB = 256;          // threads per workgroup = candidates staged per LDS tile
constexpr int KNN_MAX = 16;      // max_vertex_degree cap of the device K-NN

__global__ __launch_bounds__(HB) void k_grid_keys(const float* __restrict__ pts, int n, float cell, int4* __restrict__ keys) {
	const int i = blockIdx.x * HB + threadIdx.x;
	if (i >= n) return;
	keys[i] = make_int4(static_cast<int>(floorf(pts[3 * i] / cell)), static_cast<int>(floorf(pts[3 * i + 1] / cell)),
	                    static_cast<int>(floorf(pts[3 * i + 2] / cell)), 0);
}

__device__ inline bool same_cell(int4 a, int4 b) { return a.x == b.x && a.y == b.y && a.z == b.z; }

// sums[a] = sum over members b of a's cell, ascending b, of |p_b - p_a|
__global__ __launch_bounds__(HB) void k_medoid_sums(const float* __restrict__ pts, const int4* __restrict__ keys, int n, float* __restrict__ sums) {
	__shared__ float s_p[3 * HB];
	__shared__ int4 s_k[HB];
	const int a = blockIdx.x * HB + threadIdx.x;
	const bool live = a < n;
	const int4 ka = live ? keys[a] : make_int4(0, 0, 0, 0);
	const float ax = live ? pts[3 * a] : 0.f, ay = live ? pts[3 * a + 1] : 0.f, az = live ? pts[3 * a + 2] : 0.f;
	float sum = 0.f;
	for (int t0 = 0; t0 < n; t0 += HB) {
		__syncthreads();
		const int b = t0 + threadIdx.x;
		if (b < n) {
			s_k[threadIdx.x] = keys[b];
			s_p[3 * threadIdx.x] = pts[3 * b];
			s_p[3 * threadIdx.x + 1] = pts[3 * b + 1];
			s_p[3 * threadIdx.x + 2] = pts[3 * b + 2];
		}
		__syncthreads();
		const int m = min(HB, n - t0);
		for (int j = 0; j < m; j++) {
			if (!same_cell(s_k[j], ka)) continue;
			const float dx = s_p[3 * j] - ax, dy = s_p[3 * j + 1] - ay, dz = s_p[3 * j + 2] - az;
			sum += sqrtf((dx * dx + dy * dy) + dz * dz);
		}
	}
	if (live) sums[a] = sum;
}

// flag[a] = 1 iff a is its cell's medoid: the first member (ascending) with the smallest sum below FLT_MAX, or -- when no
// member's sum is below FLT_MAX -- the cell's first member (the restatement's `best = FLT_MAX, best_i = members[0]`)
__global__ __launch_bounds__(HB) void k_medoid_flags(const float* __restrict__ sums, const int4* __restrict__ keys, int n, uint8_t* __restrict__ flags) {
	__shared__ float s_s[HB];
	__shared__ int4 s_k[HB];
	const int a = blockIdx.x * HB + threadIdx.x;
	const bool live = a < n;
	const int4 ka = live ? keys[a] : make_int4(0, 0, 0, 0);
	const float sa = live ? sums[a] : 0.f;
	const bool va = sa < FLT_MAX;
	bool beaten = false, any_valid = false, first = true;
	for (int t0 = 0; t0 < n; t0 += HB) {
		__syncthreads();
		const int b = t0 + threadIdx.x;
		if (b < n) {
			s_k[threadIdx.x] = keys[b];
			s_s[threadIdx.x] = sums[b];
		}
		__syncthreads();
		const int m = min(HB, n - t0);
		for (int j = 0; j < m; j++) {
			if (!same_cell(s_k[j], ka)) continue;
			const int b2 = t0 + j;
			const float sb = s_s[j];
			const bool vb = sb < FLT_MAX;
			any_valid |= vb;
			first &= b2 >= a;
			beaten |= vb && (sb < sa || (sb == sa && b2 < a));
		}
	}
	if (live) flags[a] = static_cast<uint8_t>(va ? !beaten : (!any_valid && first));
}

// rows[s] = the k nearest coarse nodes of fine node s by (squared distance, index), sorted by descending index, -1 last
__global__ __launch_bounds__(HB) void k_knn_rows(const float* __restrict__ fine, int ns, const float* __restrict__ coarse, int nc, int k,
                                                 int32_t* __restrict__ rows) {
	__shared__ float s_p[3 * HB];
	const int s = blockIdx.x * HB + threadIdx.x;
	const bool live = s < ns;
	const float qx = live ? fine[3 * s] : 0.f, qy = live ? fine[3 * s + 1] : 0.f, qz = live ? fine[3 * s + 2] : 0.f;
	float bd[KNN_MAX];
	int bi[KNN_MAX];
#pragma unroll
	for (int q = 0; q < KNN_MAX; q++) {
		bd[q] = INFINITY;
		bi[q] = INT_MAX;
	}
	float worst_d = INFINITY;
	bool worst_empty = true;
	for (int t0 = 0; t0 < nc; t0 += HB) {
		__syncthreads();
		const int b = t0 + threadIdx.x;
		if (b < nc) {
			s_p[3 * threadIdx.x] = coarse[3 * b];
			s_p[3 * threadIdx.x + 1] = coarse[3 * b + 1];
			s_p[3 * threadIdx.x + 2] = coarse[3 * b + 2];
		}
		__syncthreads();
		const int m = min(HB, nc - t0);
		for (int j = 0; j < m; j++) {
			const float dx = s_p[3 * j] - qx, dy = s_p[3 * j + 1] - qy, dz = s_p[3 * j + 2] - qz;
			const float d = (dx * dx + dy * dy) + dz * dz;
			const int idx = t0 + j;
			// candidates arrive in ascending index: (d, idx) beats slot q iff d < bd[q] or the slot is still empty
			if (!(d < worst_d || worst_empty)) continue;
			float cd = d;
			int ci = idx;
			bool shifting = false;
#pragma unroll
			for (int q = 0; q < KNN_MAX; q++) {   // insertion: every slot from the insertion point on moves one down
				if (q >= k) break;
				const bool take = shifting || cd < bd[q] || bi[q] == INT_MAX;
				shifting = take;
				const float td = bd[q];
				const int ti = bi[q];
				bd[q] = take ? cd : bd[q];
				bi[q] = take ? ci : bi[q];
				cd = take ? td : cd;
				ci = take ? ti : ci;
			}
#pragma unroll
			for (int q = 0; q < KNN_MAX; q++)   // slot k - 1 by a static-index select chain (no scratch indexing)
				if (q == k - 1) {
					worst_d = bd[q];
					worst_empty = bi[q] == INT_MAX;
				}
		}
	}
	if (!live) return;
	int out[KNN_MAX];
#pragma unroll
	for (int q = 0; q < KNN_MAX; q++) out[q] = (q < k && q < nc) ? bi[q] : -1;
	// descending index sort of the row (k <= 16: insertion sort in registers)
#pragma unroll
	for (int q = 1; q < KNN_MAX; q++) {
#pragma unroll
		for (int r = q; r > 0; r--) {
			const int hi = max(out[r - 1], out[r]), lo = min(out[r - 1], out[r]);
			out[r - 1] = hi;
			out[r] = lo;
		}
	}
#pragma unroll
	for (int q = 0; q < KNN_MAX; q++)
		if (q < k) rows[static_cast<int64_t>(s) * k + q] = out[q];
}

__global__ __launch_bounds__(HB) void k_node_coverage(const float* __restrict__ nodes, int n, float* __restrict__ out) {
	__shared__ float s_p[3 * HB];
	const int i = blockIdx.x * HB + threadIdx.x;
	const bool live = i < n;
	const float xi = live ? nodes[3 * i] : 0.f, yi = live ? nodes[3 * i + 1] : 0.f, zi = live ? nodes[3 * i + 2] : 0.f;
	float d0 = INFINITY, d1 = INFINITY, maxd = INFINITY;
	int max_at = 0;
	for (int t0 = 0; t0 < n; t0 += HB) {
		__syncthreads();
		const int b = t0 + threadIdx.x;
		if (b < n) {
			s_p[3 * threadIdx.x] = nodes[3 * b];
			s_p[3 * threadIdx.x + 1] = nodes[3 * b + 1];
			s_p[3 * threadIdx.x + 2] = nodes[3 * b + 2];
		}
		__syncthreads();
		const int m = min(HB, n - t0);
		for (int j = 0; j < m; j++) {
			const float dx = s_p[3 * j] - xi, dy = s_p[3 * j + 1] - yi, dz = s_p[3 * j + 2] - zi;
			const float sq = (dx * dx + dy * dy) + dz * dz;
			if (sq < maxd) {
				if (max_at) d1 = sq;
				else d0 = sq;
				max_at = d1 > d0 ? 1 : 0;
				maxd = max_at ? d1 : d0;
			}
		}
	}
	if (!live) return;
	const float m = d0 < d1 ? d1 : d0;   // std::max(d0, d1)
	const float d = sqrtf(m);
	out[i] = d * d;
}

template <typename T>
struct Scratch {
	T* p = nullptr;
	~Scratch() {
		if (p) (void)hipFree(p);
	}
	nnrt_status alloc(size_t n) {
		NNRT_HIP(hipMalloc(&p, sizeof(T) * (n ? n : 1)));
		return NNRT_OK;
	}
};

unsigned blocks(int n) { return static_cast<unsigned>(ceil_div(n, HB)); }
} // namespace

// HierarchyOps over the current HIP device, on the null stream (construction is once per warp field, synchronous)
class DeviceHierarchyOps final : public HierarchyOps {
public:
	nnrt_status medoid_flags(const std::vector<float>& pts, float cell, std::vector<uint8_t>& flags) override {
		const int n = static_cast<int>(pts.size() / 3);
		flags.assign(n, 0);
		if (n == 0) return NNRT_OK;
		Scratch<float> d_pts, d_sums;
		Scratch<int4> d_keys;
		Scratch<uint8_t> d_flags;
		nnrt_status st;
		if ((st = d_pts.alloc(3 * static_cast<size_t>(n))) || (st = d_sums.alloc(n)) || (st = d_keys.alloc(n)) || (st = d_flags.alloc(n))) return st;
		NNRT_HIP(hipMemcpy(d_pts.p, pts.data(), sizeof(float) * pts.size(), hipMemcpyHostToDevice));
		k_grid_keys<<<blocks(n), HB>>>(d_pts.p, n, cell, d_keys.p);
		NNRT_LAUNCH_CHECK();
		k_medoid_sums<<<blocks(n), HB>>>(d_pts.p, d_keys.p, n, d_sums.p);
		NNRT_LAUNCH_CHECK();
		k_medoid_flags<<<blocks(n), HB>>>(d_sums.p, d_keys.p, n, d_flags.p);
		NNRT_LAUNCH_CHECK();
		NNRT_HIP(hipMemcpy(flags.data(), d_flags.p, n, hipMemcpyDeviceToHost));
		return NNRT_OK;
	}
	nnrt_status knn_rows(const std::vector<float>& fine, const std::vector<float>& coarse, int k, std::vector<int32_t>& rows) override {
		NNRT_CHECK_ARG(k >= 1 && k <= KNN_MAX, "max_vertex_degree must be in [1, 16]");
		const int ns = static_cast<int>(fine.size() / 3), nc = static_cast<int>(coarse.size() / 3);
		rows.assign(static_cast<size_t>(ns) * k, -1);
		if (ns == 0) return NNRT_OK;
		Scratch<float> d_f, d_c;
		Scratch<int32_t> d_rows;
		nnrt_status st;
		if ((st = d_f.alloc(fine.size())) || (st = d_c.alloc(coarse.size())) || (st = d_rows.alloc(rows.size()))) return st;
		NNRT_HIP(hipMemcpy(d_f.p, fine.data(), sizeof(float) * fine.size(), hipMemcpyHostToDevice));
		if (nc > 0) NNRT_HIP(hipMemcpy(d_c.p, coarse.data(), sizeof(float) * coarse.size(), hipMemcpyHostToDevice));
		k_knn_rows<<<blocks(ns), HB>>>(d_f.p, ns, d_c.p, nc, k, d_rows.p);
		NNRT_LAUNCH_CHECK();
		NNRT_HIP(hipMemcpy(rows.data(), d_rows.p, sizeof(int32_t) * rows.size(), hipMemcpyDeviceToHost));
		return NNRT_OK;
	}
	nnrt_status coverage_weights(const float* nodes, int n, float coverage, std::vector<float>& out) override {
		out.assign(n, 0.f);
		if (n == 1) {   // WarpField.cpp:249-263: a single node keeps the coverage, un-squared as written
			out[0] = coverage;
			return NNRT_OK;
		}
		if (n == 0) return NNRT_OK;
		Scratch<float> d_n, d_out;
		nnrt_status st;
		if ((st = d_n.alloc(3 * static_cast<size_t>(n))) || (st = d_out.alloc(n))) return st;
		NNRT_HIP(hipMemcpy(d_n.p, nodes, sizeof(float) * 3 * n, hipMemcpyHostToDevice));
		k_node_coverage<<<blocks(n), HB>>>(d_n.p, n, d_out.p);
		NNRT_LAUNCH_CHECK();
		NNRT_HIP(hipMemcpy(out.data(), d_out.p, sizeof(float) * n, hipMemcpyDeviceToHost));
		return NNRT_OK;
	}
};

// nnrt.geometry.functional.median_grid_subsample_3d_points (MedianGridSubsample3dPoints, GeometrySampling.cpp:62-68 ->
// GeometrySamplingMedian.h:264-296): one medoid per occupied grid cell, as indices into `pts`. The reference emits them in
// its hash map's bin order (not deterministic on the GPU); here in ascending point index (DeviceSelect over the flags).
nnrt_status launch_median_grid_subsample(const float* pts, int n, float cell, int64_t* out, int64_t* h_count, hipStream_t s) {
	*h_count = 0;
	if (n == 0) return NNRT_OK;
	Scratch<float> d_sums;
	Scratch<int4> d_keys;
	Scratch<uint8_t> d_flags;
	Scratch<int64_t> d_count;
	nnrt_status st;
	if ((st = d_sums.alloc(n)) || (st = d_keys.alloc(n)) || (st = d_flags.alloc(n)) || (st = d_count.alloc(1))) return st;
	k_grid_keys<<<blocks(n), HB, 0, s>>>(pts, n, cell, d_keys.p);
	NNRT_LAUNCH_CHECK();
	k_medoid_sums<<<blocks(n), HB, 0, s>>>(pts, d_keys.p, n, d_sums.p);
	NNRT_LAUNCH_CHECK();
	k_medoid_flags<<<blocks(n), HB, 0, s>>>(d_sums.p, d_keys.p, n, d_flags.p);
	NNRT_LAUNCH_CHECK();
	hipcub::CountingInputIterator<int64_t> idx(0);
	size_t bytes = 0;
	NNRT_HIP(hipcub::DeviceSelect::Flagged(nullptr, bytes, idx, d_flags.p, out, d_count.p, n, s));
	Scratch<uint8_t> tmp;
	if ((st = tmp.alloc(std::max<size_t>(bytes, 1)))) return st;
	NNRT_HIP(hipcub::DeviceSelect::Flagged(tmp.p, bytes, idx, d_flags.p, out, d_count.p, n, s));
	NNRT_HIP(hipMemcpyAsync(h_count, d_count.p, sizeof(int64_t), hipMemcpyDeviceToHost, s));
	NNRT_HIP(hipStreamSynchronize(s));
	return NNRT_OK;
}

HierarchyOps& device_hierarchy_ops() {
	static DeviceHierarchyOps ops;
	return ops;
}

} // namespace nnrt
