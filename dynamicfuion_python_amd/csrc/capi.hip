// Host orchestration and the C-ABI (include/nnrt_mi355x.h).
//
// FitToImage (cpp/alignment/DeformableMeshToImageFitter.cpp:85-276) as a static-shape loop: every buffer is sized at
// prepare() time, nothing in the iteration synchronizes with the host or allocates, so one GN iteration per iteration
// mode is captured into a hipGraph and replayed (the reference's per-stage host syncs: SURVEY.md section 3 CS-1).
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstring>
#include <memory>
#include <mutex>
#include <list>
#include <vector>

#include "fitter_kernels.hpp"
#include "warp_field.hpp"
#include "nnrt_dlpack.h"

namespace nnrt {

namespace {
thread_local std::string g_error;
std::atomic<uint64_t> g_next_warp_field_id{1};
}
void set_error(const std::string& message) { g_error = message; }
const std::string& get_error() { return g_error; }

NdcSetup make_ndc_setup(const double* K, int height, int width, bool consistent) {
	// CoordinateSystemConversions.h:109-146. consistent = false reproduces the reference (A11: rows mirrored about cy, columns
	// shifted by w - 2cx, clip window centred on the NDC principal point); consistent = true maps pixel (u, v) of the
	// intrinsics K onto the centre of raster pixel (u, v), the clip window being the image.
	const double fx = K[0], fy = K[4], cx = K[2], cy = K[5];
	const double h = height, w = width;
	const double s = std::min(w, h);
	const float range_x = ndc_range(width, height);
	const float range_y = ndc_range(height, width);
	const double fx_ndc = 2.0 * fx / s, fy_ndc = (consistent ? 2.0 : -2.0) * fy / s;
	const double cx_ndc = consistent ? (2.0 * cx + 1.0 - w) / s : -(2.0 * cx - w) / s;
	const double cy_ndc = consistent ? (2.0 * cy + 1.0 - h) / s : (2.0 * cy - h) / s;
	const double wx = consistent ? 0.0 : cx_ndc, wy = consistent ? 0.0 : cy_ndc;
	NdcSetup r;
	r.ndc = Camera{static_cast<float>(fx_ndc), static_cast<float>(fy_ndc), static_cast<float>(cx_ndc), static_cast<float>(cy_ndc)};
	r.min_x = static_cast<float>(wx - range_x / 2.f);
	r.max_x = static_cast<float>(wx + range_x / 2.f);
	r.min_y = static_cast<float>(wy - range_y / 2.f);
	r.max_y = static_cast<float>(wy + range_y / 2.f);
	return r;
}

WarpExtrinsics make_extrinsics(const double* E) {
	WarpExtrinsics r{};
	r.identity = 1;
	const double I[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
	for (int i = 0; i < 12; i++) {
		const double v = E ? E[i] : I[i];
		r.m[i] = static_cast<float>(v);
		if (v != I[i]) r.identity = 0;
	}
	return r;
}

Camera pixel_camera(const double* K) {
	return Camera{static_cast<float>(K[0]), static_cast<float>(K[4]), static_cast<float>(K[2]), static_cast<float>(K[5])};
}

// ---- device buffer helper ----
template <typename T>
struct DeviceBuffer {
	T* ptr = nullptr;
	size_t count = 0;
	nnrt_status ensure(size_t n) {
		if (n <= count && ptr) return NNRT_OK;
		if (ptr) hipFree(ptr);
		ptr = nullptr;
		count = 0;
		const size_t bytes = sizeof(T) * std::max<size_t>(n, 1);
		hipError_t e = hipMalloc(reinterpret_cast<void**>(&ptr), bytes);
		if (e != hipSuccess) {
			set_error(std::string("hipMalloc failed: ") + hipGetErrorString(e));
			ptr = nullptr;
			return NNRT_ERROR_HIP;
		}
		count = std::max<size_t>(n, 1);
		return NNRT_OK;
	}
	void release() {
		if (ptr) hipFree(ptr);
		ptr = nullptr;
		count = 0;
	}
};

template <typename T>
nnrt_status upload(DeviceBuffer<T>& buf, const std::vector<T>& host) {
	nnrt_status st = buf.ensure(host.size());
	if (st) return st;
	if (!host.empty() && hipMemcpy(buf.ptr, host.data(), sizeof(T) * host.size(), hipMemcpyHostToDevice) != hipSuccess) {
		set_error("hipMemcpy failed");
		return NNRT_ERROR_HIP;
	}
	return NNRT_OK;
}

struct DeviceGuard {
	int prev = -1;
	explicit DeviceGuard(int device) {
		hipGetDevice(&prev);
		if (device >= 0 && device != prev) hipSetDevice(device);
	}
	~DeviceGuard() {
		int cur = -1;
		hipGetDevice(&cur);
		if (prev >= 0 && cur != prev) hipSetDevice(prev);
	}
};

} // namespace nnrt

using namespace nnrt;

// =====================================================================================================================
// warp field
// =====================================================================================================================
struct nnrt_warp_field {
	int device = 0;
	int N = 0;
	float coverage = 0.05f;
	int threshold = 0;
	int anchor_count = 4;
	int minimum_valid = 0;
	int coverage_method = NNRT_MINIMAL_K_NEIGHBOR_NODE_DISTANCE;
	Hierarchy h;
	std::vector<float> nodes_original;     // [N,3] original order
	std::vector<float> weights_virtual;    // [N] coverage weights, virtual order
	DeviceBuffer<float> state;             // [N,16] virtual order
	DeviceBuffer<float> node_positions;    // [N,3] virtual order (anchor computation input)
	DeviceBuffer<float> node_weights;      // [N] virtual order
	DeviceBuffer<int32_t> edges;           // [E,2]
	DeviceBuffer<int8_t> edge_layers;      // [E]
	DeviceBuffer<float> radii;             // [layers]
	uint64_t id = 0;                       // unique per created warp field (a fitter's cached graphs capture its buffers)
	int E() const { return static_cast<int>(h.edge_layers.size()); }
};

namespace nnrt {
WarpFieldView warp_field_view(const void* handle) {
	const nnrt_warp_field* wf = static_cast<const nnrt_warp_field*>(handle);
	WarpFieldView v{};
	v.N = wf->N;
	v.anchor_count = wf->anchor_count;
	v.minimum_valid = wf->minimum_valid;
	v.fixed_coverage = wf->coverage_method == NNRT_MINIMAL_K_NEIGHBOR_NODE_DISTANCE ? 0 : 1;
	v.coverage = wf->coverage;
	v.state = wf->state.ptr;
	v.node_weights = wf->node_weights.ptr;
	v.device = wf->device;
	return v;
}
} // namespace nnrt

namespace {
nnrt_status wf_download_state(const nnrt_warp_field* wf, std::vector<float>& host) {
	host.resize(static_cast<size_t>(wf->N) * NODE_STRIDE);
	NNRT_HIP(hipMemcpy(host.data(), wf->state.ptr, sizeof(float) * host.size(), hipMemcpyDeviceToHost));
	return NNRT_OK;
}
nnrt_status wf_upload_state(nnrt_warp_field* wf, const std::vector<float>& host) {
	NNRT_HIP(hipMemcpy(wf->state.ptr, host.data(), sizeof(float) * host.size(), hipMemcpyHostToDevice));
	return NNRT_OK;
}
} // namespace

extern "C" {

const char* nnrt_last_error(void) { return get_error().c_str(); }

int32_t nnrt_runtime_version(void) {
	int v = 0;
	if (hipRuntimeGetVersion(&v) != hipSuccess) return -1;
	return v;
}

int32_t nnrt_device_count(void) {
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess) return -1;
	return n;
}

nnrt_status nnrt_warp_field_create(const float* h_nodes, int32_t node_count, float node_coverage, int32_t threshold_nodes_by_distance,
                                   int32_t anchor_count, int32_t minimum_valid_anchor_count, int32_t coverage_method, int32_t layer_count,
                                   int32_t max_vertex_degree, const float* h_layer_radii, int32_t device, nnrt_warp_field** out) {
	NNRT_CHECK_ARG(out != nullptr && h_nodes != nullptr, "null pointer");
	NNRT_CHECK_ARG(node_count >= 1, "node_count must be positive");
	NNRT_CHECK_ARG(anchor_count >= 1 && anchor_count <= MAX_ANCHORS, "anchor_count must be in [1, 8]");
	if (node_count < anchor_count) {
		set_error("Anchor count for warp field exceeds node count (WarpField.cpp:57-61)");
		return NNRT_ERROR_ARGUMENT;
	}
	NNRT_CHECK_ARG(minimum_valid_anchor_count >= 0 && minimum_valid_anchor_count <= anchor_count, "minimum_valid_anchor_count > anchor_count");
	NNRT_CHECK_ARG(coverage_method == NNRT_FIXED_NODE_COVERAGE || coverage_method == NNRT_MINIMAL_K_NEIGHBOR_NODE_DISTANCE,
	               "unknown coverage method");
	DeviceGuard guard(device);
	auto wf = std::make_unique<nnrt_warp_field>();
	wf->device = device;
	wf->id = g_next_warp_field_id.fetch_add(1);
	wf->N = node_count;
	wf->coverage = node_coverage;
	wf->threshold = threshold_nodes_by_distance;
	wf->anchor_count = anchor_count;
	wf->minimum_valid = minimum_valid_anchor_count;
	wf->coverage_method = coverage_method;
	wf->nodes_original.assign(h_nodes, h_nodes + 3 * static_cast<size_t>(node_count));
	HierarchyOps& ops = device_hierarchy_ops();
	nnrt_status st = build_hierarchy(h_nodes, node_count, node_coverage, layer_count, max_vertex_degree, h_layer_radii, ops, wf->h);
	if (st) return st;
	std::vector<float> weights_original;
	if ((st = ops.coverage_weights(h_nodes, node_count, node_coverage, weights_original))) return st;
	std::vector<float> state(static_cast<size_t>(node_count) * NODE_STRIDE, 0.f), pos(3 * static_cast<size_t>(node_count));
	wf->weights_virtual.resize(node_count);
	for (int v = 0; v < node_count; v++) {
		const int64_t o = wf->h.virtual_indices[v];
		float* s = &state[static_cast<size_t>(v) * NODE_STRIDE];
		for (int c = 0; c < 3; c++) {
			s[c] = h_nodes[3 * o + c];
			pos[3 * v + c] = h_nodes[3 * o + c];
		}
		s[6] = s[10] = s[14] = 1.f;   // identity rotation (WarpField::ResetRotations)
		wf->weights_virtual[v] = weights_original[o];
	}
	if ((st = wf->state.ensure(state.size()))) return st;
	if ((st = wf->node_positions.ensure(pos.size()))) return st;
	if ((st = wf->node_weights.ensure(node_count))) return st;
	const int E = wf->E();
	if ((st = wf->edges.ensure(2 * static_cast<size_t>(E)))) return st;
	if ((st = wf->edge_layers.ensure(E))) return st;
	if ((st = wf->radii.ensure(wf->h.radii.size()))) return st;
	NNRT_HIP(hipMemcpy(wf->state.ptr, state.data(), sizeof(float) * state.size(), hipMemcpyHostToDevice));
	NNRT_HIP(hipMemcpy(wf->node_positions.ptr, pos.data(), sizeof(float) * pos.size(), hipMemcpyHostToDevice));
	NNRT_HIP(hipMemcpy(wf->node_weights.ptr, wf->weights_virtual.data(), sizeof(float) * node_count, hipMemcpyHostToDevice));
	if (E > 0) {
		NNRT_HIP(hipMemcpy(wf->edges.ptr, wf->h.edges.data(), sizeof(int32_t) * 2 * E, hipMemcpyHostToDevice));
		NNRT_HIP(hipMemcpy(wf->edge_layers.ptr, wf->h.edge_layers.data(), sizeof(int8_t) * E, hipMemcpyHostToDevice));
	}
	NNRT_HIP(hipMemcpy(wf->radii.ptr, wf->h.radii.data(), sizeof(float) * wf->h.radii.size(), hipMemcpyHostToDevice));
	*out = wf.release();
	return NNRT_OK;
}

void nnrt_warp_field_destroy(nnrt_warp_field* wf) {
	if (!wf) return;
	DeviceGuard guard(wf->device);
	wf->state.release();
	wf->node_positions.release();
	wf->node_weights.release();
	wf->edges.release();
	wf->edge_layers.release();
	wf->radii.release();
	delete wf;
}

int32_t nnrt_warp_field_node_count(const nnrt_warp_field* wf) { return wf ? wf->N : -1; }
int32_t nnrt_warp_field_edge_count(const nnrt_warp_field* wf) { return wf ? wf->E() : -1; }
int32_t nnrt_warp_field_layer_counts(const nnrt_warp_field* wf, int32_t* h_counts) {
	if (!wf) return -1;
	for (size_t i = 0; i < wf->h.layer_counts.size(); i++)
		if (h_counts) h_counts[i] = wf->h.layer_counts[i];
	return static_cast<int32_t>(wf->h.layer_counts.size());
}

nnrt_status nnrt_warp_field_get_virtual_node_indices(const nnrt_warp_field* wf, int64_t* h_out) {
	NNRT_CHECK_ARG(wf && h_out, "null pointer");
	std::memcpy(h_out, wf->h.virtual_indices.data(), sizeof(int64_t) * wf->N);
	return NNRT_OK;
}

nnrt_status nnrt_warp_field_get_edges(const nnrt_warp_field* wf, int32_t* h_edges, int8_t* h_edge_layers) {
	NNRT_CHECK_ARG(wf, "null pointer");
	if (h_edges) std::memcpy(h_edges, wf->h.edges.data(), sizeof(int32_t) * wf->h.edges.size());
	if (h_edge_layers) std::memcpy(h_edge_layers, wf->h.edge_layers.data(), wf->h.edge_layers.size());
	return NNRT_OK;
}

static nnrt_status wf_get(const nnrt_warp_field* wf, float* h_out, int virtual_order, int offset, int width) {
	NNRT_CHECK_ARG(wf && h_out, "null pointer");
	DeviceGuard guard(wf->device);
	std::vector<float> s;
	nnrt_status st = wf_download_state(wf, s);
	if (st) return st;
	for (int v = 0; v < wf->N; v++) {
		const int64_t dst = virtual_order ? v : wf->h.virtual_indices[v];
		for (int c = 0; c < width; c++) h_out[dst * width + c] = s[static_cast<size_t>(v) * NODE_STRIDE + offset + c];
	}
	return NNRT_OK;
}

static nnrt_status wf_set(nnrt_warp_field* wf, const float* h_in, int virtual_order, int offset, int width) {
	NNRT_CHECK_ARG(wf && h_in, "null pointer");
	DeviceGuard guard(wf->device);
	std::vector<float> s;
	nnrt_status st = wf_download_state(wf, s);
	if (st) return st;
	for (int v = 0; v < wf->N; v++) {
		const int64_t src = virtual_order ? v : wf->h.virtual_indices[v];
		for (int c = 0; c < width; c++) s[static_cast<size_t>(v) * NODE_STRIDE + offset + c] = h_in[src * width + c];
	}
	return wf_upload_state(wf, s);
}

nnrt_status nnrt_warp_field_get_node_positions(const nnrt_warp_field* wf, float* h_out, int32_t virtual_order) {
	return wf_get(wf, h_out, virtual_order, 0, 3);
}
nnrt_status nnrt_warp_field_get_node_translations(const nnrt_warp_field* wf, float* h_out, int32_t virtual_order) {
	return wf_get(wf, h_out, virtual_order, 3, 3);
}
nnrt_status nnrt_warp_field_get_node_rotations(const nnrt_warp_field* wf, float* h_out, int32_t virtual_order) {
	return wf_get(wf, h_out, virtual_order, 6, 9);
}
nnrt_status nnrt_warp_field_set_node_translations(nnrt_warp_field* wf, const float* h_in, int32_t virtual_order) {
	return wf_set(wf, h_in, virtual_order, 3, 3);
}
nnrt_status nnrt_warp_field_set_node_rotations(nnrt_warp_field* wf, const float* h_in, int32_t virtual_order) {
	return wf_set(wf, h_in, virtual_order, 6, 9);
}
__global__ void k_reset_motion(float* state, int N) {
	const int n = blockIdx.x * blockDim.x + threadIdx.x;
	if (n >= N) return;
	float* s = state + static_cast<int64_t>(n) * NODE_STRIDE;
	for (int c = 3; c < 15; c++) s[c] = 0.f;
	s[6] = s[10] = s[14] = 1.f;
}

// node-state copy (snapshot / restore): one float4 per lane; a 1500-node state is 96 KB (a runtime blit kernel costs
// several microseconds more inside a graph)
__global__ void k_copy_state(const float4* __restrict__ src, float4* __restrict__ dst, int count) {
	const int i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i < count) dst[i] = src[i];
}

nnrt_status nnrt_warp_field_reset_motion(nnrt_warp_field* wf, void* stream) {
	NNRT_CHECK_ARG(wf, "null pointer");
	DeviceGuard guard(wf->device);
	k_reset_motion<<<static_cast<unsigned>(ceil_div(wf->N, 256)), 256, 0, static_cast<hipStream_t>(stream)>>>(wf->state.ptr, wf->N);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

nnrt_status nnrt_warp_field_get_node_coverage_weights(const nnrt_warp_field* wf, float* h_out) {
	NNRT_CHECK_ARG(wf && h_out, "null pointer");
	std::memcpy(h_out, wf->weights_virtual.data(), sizeof(float) * wf->N);
	return NNRT_OK;
}

} // extern "C"

// =====================================================================================================================
// fitter
// =====================================================================================================================
struct nnrt_fitter {
	nnrt_fitter_params p{};
	int device = 0;
	hipStream_t work = nullptr;
	hipEvent_t ev_in = nullptr, ev_out = nullptr;
	// frame dims
	int64_t V = 0, F = 0;
	int H = 0, W = 0, N = 0, K = 0, E = 0;
	bool prepared = false;
	const nnrt_warp_field* wf = nullptr;
	uint64_t wf_id = 0;   // id of the warp field whose buffers the cached graphs captured
	// frame constants
	NdcSetup ndc{};
	Camera pix{};
	WarpExtrinsics extr{};
	// buffers
	DeviceBuffer<float> mesh_p, mesh_n;
	DeviceBuffer<int4> faces4;
	DeviceBuffer<int32_t> anchors;
	DeviceBuffer<uint2> anchors16;   // [V] the anchors as 4 x 16 bits (K = 4, N < 65535): the vertex warp's loads
	bool use_anchors16 = false;
	DeviceBuffer<float> weights;
	DeviceBuffer<uint32_t> face_nodes;   // [F, face_node_slots(K)] distinct anchor nodes per face (once per frame)
	DeviceBuffer<float4> wpos, wnrm;
	DeviceBuffer<float2> jrows;        // [V,K,3] warped-Jacobian rows (store_jacobian_row; NNRT_GATHER_ROWS builds only)
	DeviceBuffer<float4> mesh_p4, mesh_n4;   // [V] canonical positions / normals as float4 (pass 2 forms the Jacobian rows)
	DeviceBuffer<float4> ref_points;   // [P] reference point (x, y, z, valid)
	DeviceBuffer<int> tile_flags, tile_order;   // the pixel launch's per-frame workgroup -> tile table (launch_tile_order)
	bool use_tile_order = false;
	bool pix_low_occupancy = false;   // the pixel launch's 4-waves-per-SIMD build (launches of several residency rounds)
	DeviceBuffer<float4> records;      // [P, 4] pixel Jacobian records
	DeviceBuffer<uint64_t> keys;
	DeviceBuffer<float> residuals;
	DeviceBuffer<uint8_t> residual_mask;
	DeviceBuffer<int32_t> pixel_face;
	DeviceBuffer<double> acc;       // [N, ACC_STRIDE] data term (fp64)
	DeviceBuffer<float> edge_jr;   // [E,8] ARAP edge Jacobian + residual
	DeviceBuffer<float> updates, gradient, hessian;
	DeviceBuffer<int> error_flag;
	// ARAP / arrowhead
	DeviceBuffer<float> wing, edge_residuals, a_diag, a_dinv, a_dinvb, a_rhs, a_x, a_res, a_dx;
	CornerSolver corner;   // Schur corner of the arrowhead solve (tile-sparse Cholesky plan + storage)
	DeviceBuffer<int> a_offsets, a_list, a_tgt_off, a_rhs_off, a_rhs_edges, a_inc_off, a_inc_list, a_inc_slot;
	DeviceBuffer<int2> a_tgt_ab, a_pairs;
	ArrowheadWorkspace aw;
	float refine_ratio = NNRT_REFINE_PIVOT_RATIO;   // refinement gate threshold (nnrt_fitter_set_refine_ratio)
	float refine_ratio_used = NNRT_REFINE_PIVOT_RATIO;   // the threshold the last launched iterations ran with (refine_info)
	int n0 = 0;
	int last_mode = 0;
	DeviceBuffer<float> snapshot;   // [N,16] node state stored by nnrt_fitter_snapshot_motion (restore-before-iteration runs)
	bool snapshot_valid = false;    // cleared by prepare() (the warp field or the node count may have changed)
	// graphs: one per iteration sequence (the modes of the `count` iterations of an iterate() call, and what each
	// iteration restarts from: RESET_NONE / RESET_IDENTITY / RESET_SNAPSHOT), captured once and replayed as ONE launch; the
	// most recent few are kept. exec == nullptr records a sequence that ran eagerly once (use_hip_graph = 1 captures a
	// sequence on its second request only, so a sequence launched once per frame never pays capture + instantiate).
	struct SeqGraph {
		std::vector<int> modes;
		int reset = 0;
		hipGraphExec_t exec = nullptr;
	};
	std::vector<SeqGraph> graphs;

	void drop_graphs() {
		for (auto& g : graphs)
			if (g.exec) hipGraphExecDestroy(g.exec);
		graphs.clear();
	}
};

namespace {

// depth overload (DeformableMeshToImageFitter.cpp:278-314): UnprojectDepthImageWithoutFiltering with the pixel intrinsics
// (PerspectiveProjectionImpl.h:60-146): d = depth / scale, valid iff 0 < d < max_depth (AND the optional image mask)
__global__ void k_prepare_reference_depth(const float* __restrict__ depth, const uint8_t* __restrict__ mask, int H, int W, float scale,
                                          float max_depth, Camera pix, float4* __restrict__ out) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= static_cast<int64_t>(H) * W) return;
	const int u = static_cast<int>(i % W), v = static_cast<int>(i / W);
	const float d = depth[i] / scale;
	const bool valid = d > 0 && d < max_depth && (mask == nullptr || mask[i] != 0);
	out[i] = valid ? make_float4((static_cast<float>(u) - pix.cx) * d / pix.fx, (static_cast<float>(v) - pix.cy) * d / pix.fy, d, 1.f)
	               : make_float4(0.f, 0.f, 0.f, 0.f);
}

// point-cloud overload (:85-95): organized reference points [P,3] and their mask
__global__ void k_prepare_reference_points(const float* __restrict__ points, const uint8_t* __restrict__ mask, int64_t P,
                                           float4* __restrict__ out) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= P) return;
	const bool valid = mask == nullptr || mask[i] != 0;
	out[i] = valid ? make_float4(points[3 * i], points[3 * i + 1], points[3 * i + 2], 1.f) : make_float4(0.f, 0.f, 0.f, 0.f);
}

// canonical vertices / normals [V,3] -> float4 [V] (w = 0): pass 2 forms the warped-surface Jacobian rows from them
__global__ void k_to_float4(const float* __restrict__ p, const float* __restrict__ n, int64_t V, float4* __restrict__ p4, float4* __restrict__ n4) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= V) return;
	p4[i] = make_float4(p[3 * i], p[3 * i + 1], p[3 * i + 2], 0.f);
	n4[i] = make_float4(n[3 * i], n[3 * i + 1], n[3 * i + 2], 0.f);
}

// faces -> int4; an index outside [0, V) becomes the degenerate face (0, 0, 0) (never rasterized, never gathered out of
// bounds) and sets error bit 4, which nnrt_fitter_check reports
// flip_winding: the consistent NDC convention keeps rows in image order, which negates every face's NDC area relative to
// the reference's mirrored image; swapping two corners restores the orientation the back-face test expects.
__global__ void k_faces_to_int4(const int64_t* __restrict__ faces, int64_t F, int64_t V, int flip_winding, int4* __restrict__ out,
                                int* error_flag) {
	const int64_t f = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (f >= F) return;
	const int64_t i0 = faces[3 * f], i1 = faces[3 * f + 1], i2 = faces[3 * f + 2];
	if (i0 < 0 || i0 >= V || i1 < 0 || i1 >= V || i2 < 0 || i2 >= V) {
		atomicOr(error_flag, 4);
		out[f] = make_int4(0, 0, 0, 0);
		return;
	}
	out[f] = flip_winding ? make_int4(static_cast<int>(i0), static_cast<int>(i2), static_cast<int>(i1), 0)
	                      : make_int4(static_cast<int>(i0), static_cast<int>(i1), static_cast<int>(i2), 0);
}

// from_identity: the warp and the update treat every node's motion as R = I, t = 0 without reading it (only on the
// block-diagonal path with <= 4 anchors, see fold_reset); the result equals a reset followed by the iteration.
// state_in (default: the warp field's state): where the warp and the update read the node motion the iteration starts
// from; the update always writes the warp field's state (a restore-from-snapshot folded into the iteration reads the
// snapshot directly instead of copying it first).
// stages of one iteration (nnrt_fitter_time_kernels launches subsets of them)
enum : unsigned { STAGE_WARP = 1u, STAGE_RASTER = 2u, STAGE_PIXEL = 4u, STAGE_SOLVE = 8u, STAGE_ALL = 15u };

nnrt_status enqueue_iteration(nnrt_fitter* ft, const nnrt_warp_field* wf, int mode, hipStream_t s, hipEvent_t* marks = nullptr,
                              bool from_identity = false, const float* state_in = nullptr, unsigned stages = STAGE_ALL) {
	if (!state_in) state_in = wf->state.ptr;
	nnrt_status st;
	auto mark = [&](int i) -> nnrt_status {
		if (marks) NNRT_HIP(hipEventRecord(marks[i], s));
		return NNRT_OK;
	};
	if ((st = mark(0))) return st;
	const bool with_jacobians = NNRT_GATHER_ROWS != 0;
	if ((stages & STAGE_WARP) &&
	    (st = launch_warp_mesh(ft->mesh_p.ptr, ft->mesh_n.ptr, ft->V, state_in, ft->anchors.ptr, ft->weights.ptr, ft->K, ft->extr,
	                           ft->wpos.ptr, ft->wnrm.ptr, with_jacobians ? ft->jrows.ptr : nullptr, s, from_identity,
	                           ft->use_anchors16 ? ft->anchors16.ptr : nullptr)))
		return st;
	if ((st = mark(1))) return st;
	const RasterOptions ro = make_raster_options(ft->H, ft->W, 0.5f / (static_cast<float>(fminf(ft->H, ft->W)) / 2.0f), ft->p.use_perspective_correction, 0, 1);
	if ((stages & STAGE_RASTER) && (st = launch_raster_scatter_mesh(ft->wpos.ptr, ft->faces4.ptr, ft->F, ft->ndc, 0.0f, 10.0f, ro, ft->keys.ptr, s))) return st;
	if ((st = mark(2))) return st;
	FitPixelArgs fa{};
	fa.H = ft->H;
	fa.W = ft->W;
	fa.tiles_x = static_cast<int>(ceil_div(ft->W, 16));
	fa.tiles_y = static_cast<int>(ceil_div(ft->H, 16));
	fa.tile_row0 = 0;
	fa.pix = ft->pix;
	fa.ndc = ft->ndc;
	fa.blur = ro.blur;
	fa.ax = ro.ax;
	fa.ay = ro.ay;
	fa.perspective = ft->p.use_perspective_correction;
	fa.max_depth = ft->p.max_depth;
	fa.use_tukey = ft->p.use_tukey_penalty_for_data_term;
	fa.tukey_c = ft->p.tukey_penalty_cutoff_cm;
	fa.anchor_count = ft->K;
	fa.keys = ft->keys.ptr;
	fa.faces4 = ft->faces4.ptr;
	fa.wpos = ft->wpos.ptr;
	fa.wnrm = ft->wnrm.ptr;
	fa.anchors = ft->anchors.ptr;
	fa.face_nodes = ft->face_nodes.ptr;
	fa.jrows = ft->jrows.ptr;
	fa.state_in = reinterpret_cast<const float4*>(state_in);
	fa.state_identity = from_identity;
	fa.cmesh_p = ft->mesh_p4.ptr;
	fa.cmesh_n = ft->mesh_n4.ptr;
	fa.weights = ft->weights.ptr;
	fa.ref_points = ft->ref_points.ptr;
	if (ft->use_tile_order) {
		fa.tile_order = ft->tile_order.ptr;
		fa.order_blocks = tile_order_blocks(fa.tiles_x * fa.tiles_y);
	}
	fa.records = ft->records.ptr;
	fa.low_occupancy = ft->pix_low_occupancy ? 1 : 0;
	fa.residuals = ft->residuals.ptr;
	fa.residual_mask = ft->residual_mask.ptr;
	fa.pixel_face = ft->pixel_face.ptr;
	fa.acc = ft->acc.ptr;
	if (ft->E > 0) {   // the ARAP edge terms ride in the pixel launch's extra workgroups
		ArapArgs& aa = fa.arap;
		aa.E = ft->E;
		aa.N = ft->N;
		aa.n0 = ft->n0;
		aa.lambda = ft->p.arap_term_weight;
		aa.use_huber = ft->p.use_huber_penalty_for_arap_term;
		aa.huber_delta = ft->p.huber_penalty_constant;
		aa.coverage_variable = wf->coverage_method == NNRT_MINIMAL_K_NEIGHBOR_NODE_DISTANCE;
		aa.edges = wf->edges.ptr;
		aa.edge_layers = wf->edge_layers.ptr;
		aa.radii = wf->radii.ptr;
		aa.node_weights = wf->node_weights.ptr;
		aa.node_state = state_in;
		aa.edge_jr = ft->edge_jr.ptr;
		aa.inc_slot = ft->a_inc_slot.ptr;
		aa.wing = ft->wing.ptr;
		aa.edge_residuals = ft->edge_residuals.ptr;
		aa.error_flag = ft->error_flag.ptr;
		fa.arap_blocks = fit_pixels_arap_blocks(ft->E);
	}
	if ((stages & STAGE_PIXEL) && (st = launch_fit_pixels(mode, fa, s, marks ? marks[3] : nullptr))) return st;
	if ((st = mark(4))) return st;
	if (!(stages & STAGE_SOLVE)) return mark(6);
	if (ft->E > 0) {
		if ((st = mark(5))) return st;
		const float lm = ft->p.preconditioning_dampening_factor;
		if ((st = launch_arrowhead_iteration(ft->aw, ft->acc.ptr, lm, wf->edges.ptr, ft->wing.ptr, wf->state.ptr, ft->edge_jr.ptr,
		                                     ft->updates.ptr, ft->gradient.ptr, ft->hessian.ptr, ft->error_flag.ptr, s, state_in)))
			return st;
	} else {
		if ((st = mark(5))) return st;
		SolveArgs sa{};
		sa.N = ft->N;
		sa.lm = ft->p.preconditioning_dampening_factor;
		sa.acc = ft->acc.ptr;
		sa.state_in = state_in;
		sa.node_state = wf->state.ptr;
		sa.updates_out = ft->updates.ptr;
		sa.gradient_out = ft->gradient.ptr;
		sa.hessian_out = ft->hessian.ptr;
		sa.error_flag = ft->error_flag.ptr;
		if ((st = launch_solve_update(mode, sa, s, from_identity))) return st;
	}
	return mark(6);
}

} // namespace

// [a, a + na) and [b, b + nb) share a byte
inline bool ranges_overlap(const void* a, size_t na, const void* b, size_t nb) {
	const uintptr_t x = reinterpret_cast<uintptr_t>(a), y = reinterpret_cast<uintptr_t>(b);
	return na > 0 && nb > 0 && x < y + nb && y < x + na;
}

extern "C" {

void nnrt_fitter_default_params(nnrt_fitter_params* p) {
	if (!p) return;
	std::memset(p, 0, sizeof(*p));
	p->max_iteration_count = 100;
	p->iteration_mode_count = 1;
	p->iteration_modes[0] = NNRT_ITERATION_ALL;
	p->minimal_update_threshold = 1e-6f;
	p->use_perspective_correction = 1;
	p->max_depth = 10.f;
	p->use_tukey_penalty_for_data_term = 0;
	p->tukey_penalty_cutoff_cm = 0.01f;
	p->preconditioning_dampening_factor = 0.f;
	p->arap_term_weight = 200.f;
	p->use_huber_penalty_for_arap_term = 0;
	p->huber_penalty_constant = 1e-4f;
	p->use_hip_graph = 1;
	p->ndc_convention = NNRT_NDC_REFERENCE;
}

nnrt_status nnrt_fitter_create(const nnrt_fitter_params* params, int32_t device, nnrt_fitter** out) {
	NNRT_CHECK_ARG(params && out, "null pointer");
	if (params->preconditioning_dampening_factor < 0.f || params->preconditioning_dampening_factor > 1.f) {
		set_error("`preconditioning_dampening_factor` should be a small non-negative value between 0 and 1 (DeformableMeshToImageFitter.cpp:79-82)");
		return NNRT_ERROR_ARGUMENT;
	}
	NNRT_CHECK_ARG(params->iteration_mode_count >= 1 && params->iteration_mode_count <= 16, "iteration_mode_count must be in [1, 16]");
	for (int i = 0; i < params->iteration_mode_count; i++)
		NNRT_CHECK_ARG(params->iteration_modes[i] >= 0 && params->iteration_modes[i] <= 2, "unknown iteration mode");
	NNRT_CHECK_ARG(params->ndc_convention == NNRT_NDC_REFERENCE || params->ndc_convention == NNRT_NDC_CONSISTENT, "unknown ndc_convention");
	DeviceGuard guard(device);
	auto ft = std::make_unique<nnrt_fitter>();
	ft->p = *params;
	ft->device = device;
	NNRT_HIP(hipStreamCreateWithFlags(&ft->work, hipStreamNonBlocking));
	NNRT_HIP(hipEventCreateWithFlags(&ft->ev_in, hipEventDisableTiming));
	NNRT_HIP(hipEventCreateWithFlags(&ft->ev_out, hipEventDisableTiming));

	nnrt_status st = ft->error_flag.ensure(1);
	if (st) return st;
	NNRT_HIP(hipMemset(ft->error_flag.ptr, 0, sizeof(int)));
	*out = ft.release();
	return NNRT_OK;
}

void nnrt_fitter_destroy(nnrt_fitter* ft) {
	if (!ft) return;
	DeviceGuard guard(ft->device);
	hipStreamSynchronize(ft->work);
	ft->drop_graphs();
	ft->acc.release();
	ft->ref_points.release();
	ft->tile_flags.release();
	ft->tile_order.release();
	ft->records.release();
	for (auto* b : {&ft->mesh_p, &ft->mesh_n, &ft->weights, &ft->residuals, &ft->edge_jr, &ft->updates, &ft->gradient,
	                &ft->hessian, &ft->wing, &ft->edge_residuals, &ft->a_diag, &ft->a_dinv, &ft->a_dinvb, &ft->a_rhs, &ft->a_x, &ft->a_res, &ft->a_dx})
		b->release();
	ft->faces4.release();
	ft->anchors.release();
	ft->anchors16.release();
	ft->face_nodes.release();
	ft->wpos.release();
	ft->wnrm.release();
	ft->jrows.release();
	ft->mesh_p4.release();
	ft->mesh_n4.release();
	ft->keys.release();
	ft->residual_mask.release();
	ft->pixel_face.release();
	ft->error_flag.release();
	ft->a_offsets.release();
	ft->a_list.release();
	ft->a_tgt_off.release();
	ft->a_rhs_off.release();
	ft->a_rhs_edges.release();
	ft->a_tgt_ab.release();
	ft->a_pairs.release();
	ft->a_inc_off.release();
	ft->a_inc_list.release();
	ft->a_inc_slot.release();
	if (ft->ev_in) hipEventDestroy(ft->ev_in);
	if (ft->ev_out) hipEventDestroy(ft->ev_out);

	if (ft->work) hipStreamDestroy(ft->work);
	delete ft;
}

namespace {
// reference input of one frame: either a depth image (+ scale) or an organized point cloud, with an optional mask
struct FrameReference {
	const float* depth = nullptr;
	const float* points = nullptr;
	const uint8_t* mask = nullptr;
	float depth_scale = 1.f;
};

nnrt_status prepare_frame(nnrt_fitter* ft, nnrt_warp_field* wf, const float* d_vertices, const float* d_normals, int64_t V,
                          const int64_t* d_faces, int64_t F, const FrameReference& ref, int32_t H, int32_t W, const double* h_K,
                          const double* h_E, void* stream) {
	NNRT_CHECK_ARG(ft && wf && d_vertices && d_normals && d_faces && (ref.depth || ref.points) && h_K, "null pointer");
	NNRT_CHECK_ARG(V > 0 && F > 0 && H > 0 && W > 0, "empty mesh or image");
	NNRT_CHECK_ARG(V < (int64_t(1) << 31) && F < (int64_t(1) << 31), "mesh too large for int32 indexing");
	NNRT_CHECK_ARG(ref.depth_scale > 0.f, "depth_scale must be positive");
	NNRT_CHECK_ARG(wf->device == ft->device, "the warp field and the fitter live on different devices");
	DeviceGuard guard(ft->device);
	// until this frame is fully prepared the fitter is not: a failure below (allocation, corner plan) leaves iterate()
	// refusing rather than replaying graphs over buffers that may have been released
	ft->prepared = false;
	hipStream_t us = static_cast<hipStream_t>(stream);
	const int64_t P = static_cast<int64_t>(H) * W;
	const int N = wf->N, K = wf->anchor_count, E = wf->E();
	NNRT_CHECK_ARG(N >= K, "the warp field has fewer nodes than anchors per vertex");
	NNRT_CHECK_ARG(N < FACE_NODE_MAX_NODES, "node count exceeds the face-node table's 20-bit node field");
	if (E > 0) {
		for (int i = 0; i < ft->p.iteration_mode_count; i++)
			if (ft->p.iteration_modes[i] != NNRT_ITERATION_ALL) {
				set_error("the regularized (ARAP) solve supports IterationMode ALL only (reference A15: the ARAP Hessian is 6x6-only)");
				return NNRT_ERROR_UNSUPPORTED;
			}
	}
	// (re)allocate; any reallocation invalidates captured graphs
	const auto before = std::make_tuple(ft->mesh_p.ptr, ft->faces4.ptr, ft->anchors.ptr, ft->keys.ptr, ft->acc.ptr, ft->wing.ptr, ft->corner.generation,
	                                    ft->face_nodes.ptr, ft->wpos.ptr, ft->mesh_p4.ptr, ft->tile_order.ptr, ft->anchors16.ptr);
	nnrt_status st;
	if ((st = ft->mesh_p.ensure(3 * V)) || (st = ft->mesh_n.ensure(3 * V)) || (st = ft->faces4.ensure(F)) ||
	    (st = ft->anchors.ensure(static_cast<size_t>(V) * K)) || (st = ft->weights.ensure(static_cast<size_t>(V) * K)) ||
	    (st = ft->face_nodes.ensure(static_cast<size_t>(F) * face_node_slots(K))) ||
	    (st = ft->wpos.ensure(V)) || (st = ft->wnrm.ensure(V)) ||
	    (st = ft->jrows.ensure(NNRT_GATHER_ROWS ? 3 * static_cast<size_t>(V) * K : 1)) || (st = ft->mesh_p4.ensure(V)) ||
	    (st = ft->mesh_n4.ensure(V)) || (st = ft->anchors16.ensure(K == 4 && N < 65535 ? static_cast<size_t>(V) : 1)) ||
	    (st = ft->ref_points.ensure(P)) || (st = ft->records.ensure(4 * P)) || (st = ft->keys.ensure(P)) ||
	    (st = ft->residuals.ensure(P)) || (st = ft->residual_mask.ensure(P)) || (st = ft->pixel_face.ensure(P)) ||
	    (st = ft->acc.ensure(static_cast<size_t>(N) * ACC_STRIDE)) ||
	    (st = ft->updates.ensure(static_cast<size_t>(N) * 6)) || (st = ft->gradient.ensure(static_cast<size_t>(N) * 6)) ||
	    (st = ft->hessian.ensure(static_cast<size_t>(N) * 36)))
		return st;
	// the pixel launch's per-frame tile order, for launches of more than one residency round (5 waves per SIMD): their
	// last round's workgroups decide the tail, and the order gives those the tiles without reference pixels (C3 fused
	// launch 214 -> 197 us). In one round every wave starts at once and the table load only delays it (C2 40.2 -> 41.8).
	// NNRT_TILE_ORDER=0: never, =2: always.
	const size_t tiles = static_cast<size_t>(ceil_div(W, 16)) * static_cast<size_t>(ceil_div(H, 16));
	int cus = 0;
	if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, ft->device) != hipSuccess || cus <= 0) cus = 256;
	const bool multi_round = 4 * tiles > static_cast<size_t>(5 * 4 * cus);
	const bool tile_order = fit_pixels_tile_order_supported() && [&] {
		const char* v = std::getenv("NNRT_TILE_ORDER");
		if (v && *v == '0') return false;
		if (v && *v == '2') return true;
		return multi_round;
	}();
	// the same launches take the pixel kernel's 4-waves-per-SIMD build: their pass-2 gathers miss L2 (C3's 72-MB
	// canonical mesh) and fewer, spill-free waves congest the memory pipeline less (C3 fused launch 198.6 -> 188 us; at C2,
	// one round, 40.4 -> 47.2). NNRT_PIX_WPE4=0 / 1 forces.
	const bool pix_low = [&] {
		const char* v = std::getenv("NNRT_PIX_WPE4");
		if (v) return *v == '1';
		return multi_round;
	}();
	{
		if (tile_order && ((st = ft->tile_flags.ensure(tiles)) || (st = ft->tile_order.ensure(static_cast<size_t>(tile_order_blocks(static_cast<int>(tiles)))))))
			return st;
	}
	// ARAP workspace
	ft->E = E;
	ft->n0 = wf->h.layer_counts.empty() ? N : wf->h.layer_counts[0];
	if (E > 0) {
		const int n0 = ft->n0, m = 6 * (N - n0);
		{   // corner node positions (virtual order) for the nested-dissection bisection
			std::vector<float> cpos(3 * static_cast<size_t>(N - n0));
			for (int a = 0; a < N - n0; a++) {
				const int64_t o = wf->h.virtual_indices.empty() ? n0 + a : wf->h.virtual_indices[static_cast<size_t>(n0 + a)];
				for (int c = 0; c < 3; c++) cpos[3 * static_cast<size_t>(a) + c] = wf->nodes_original[3 * static_cast<size_t>(o) + c];
			}
			if ((st = ft->corner.prepare(wf->h.edges.data(), E, n0, N, cpos.data()))) {
				ft->drop_graphs();
				return st;
			}
		}
		if ((st = ft->wing.ensure(static_cast<size_t>(E) * 36)) || (st = ft->edge_residuals.ensure(3 * static_cast<size_t>(E))) ||
		    (st = ft->a_diag.ensure(static_cast<size_t>(N) * 36)) || (st = ft->a_dinv.ensure(static_cast<size_t>(n0) * 36)) ||
		    (st = ft->a_dinvb.ensure(static_cast<size_t>(E) * 36)) ||
		    (st = ft->edge_jr.ensure(2 * static_cast<size_t>(E) * EDGE_TERMS)) ||
		    (st = ft->a_rhs.ensure(6 * static_cast<size_t>(N))) || (st = ft->a_x.ensure(6 * static_cast<size_t>(N))) ||
		    (st = ft->a_res.ensure(6 * static_cast<size_t>(N))) || (st = ft->a_dx.ensure(6 * static_cast<size_t>(N))) ||
		    (st = ft->a_offsets.ensure(n0 + 1)) || (st = ft->a_list.ensure(E)))
			return st;
		// CSR of stem edges by source node
		std::vector<int> counts(n0 + 1, 0), list(E), fill;
		for (int e = 0; e < E; e++) {
			const int i = wf->h.edges[2 * e];
			if (i < n0) counts[i + 1]++;
		}
		for (int i = 0; i < n0; i++) counts[i + 1] += counts[i];
		fill.assign(counts.begin(), counts.end() - 1);
		for (int e = 0; e < E; e++) {
			const int i = wf->h.edges[2 * e];
			if (i < n0) list[fill[i]++] = e;
		}
		NNRT_HIP(hipMemcpy(ft->a_offsets.ptr, counts.data(), sizeof(int) * (n0 + 1), hipMemcpyHostToDevice));
		NNRT_HIP(hipMemcpy(ft->a_list.ptr, list.data(), sizeof(int) * E, hipMemcpyHostToDevice));
		// CSR of edge incidences by node (source: 2 e, target: 2 e + 1), ascending e per node
		std::vector<int> inc_off(static_cast<size_t>(N) + 1, 0), inc_list(2 * static_cast<size_t>(E));
		for (int e = 0; e < E; e++) {
			inc_off[static_cast<size_t>(wf->h.edges[2 * e]) + 1]++;
			inc_off[static_cast<size_t>(wf->h.edges[2 * e + 1]) + 1]++;
		}
		for (int n = 0; n < N; n++) inc_off[static_cast<size_t>(n) + 1] += inc_off[static_cast<size_t>(n)];
		{
			std::vector<int> fill_inc(inc_off.begin(), inc_off.end() - 1);
			for (int e = 0; e < E; e++) {
				inc_list[static_cast<size_t>(fill_inc[static_cast<size_t>(wf->h.edges[2 * e])]++)] = 2 * e;
				inc_list[static_cast<size_t>(fill_inc[static_cast<size_t>(wf->h.edges[2 * e + 1])]++)] = 2 * e + 1;
			}
		}
		// the slot of each incidence in that order: the ARAP edge kernel writes its two nodes' terms there (node-major, so
		// k_arrow_prepare reads each node's terms contiguously, without the incidence list)
		std::vector<int> inc_slot(2 * static_cast<size_t>(E));
		for (size_t q = 0; q < inc_list.size(); q++) inc_slot[static_cast<size_t>(inc_list[q])] = static_cast<int>(q);
		if ((st = upload(ft->a_inc_off, inc_off)) || (st = upload(ft->a_inc_list, inc_list)) || (st = upload(ft->a_inc_slot, inc_slot))) return st;
		ft->aw.inc_off = ft->a_inc_off.ptr;
		ft->aw.inc_list = ft->a_inc_list.ptr;
		const StemSchurLists sl = build_stem_schur_lists(wf->h.edges.data(), E, n0, N);
		if ((st = upload(ft->a_tgt_off, sl.tgt_off)) || (st = upload(ft->a_tgt_ab, sl.tgt_ab)) || (st = upload(ft->a_pairs, sl.pairs)) ||
		    (st = upload(ft->a_rhs_off, sl.rhs_off)) || (st = upload(ft->a_rhs_edges, sl.rhs_edges)))
			return st;
		ft->aw.targets = static_cast<int>(sl.tgt_ab.size());
		ft->aw.tgt_off = ft->a_tgt_off.ptr;
		ft->aw.tgt_ab = ft->a_tgt_ab.ptr;
		ft->aw.pairs = ft->a_pairs.ptr;
		ft->aw.rhs_off = ft->a_rhs_off.ptr;
		ft->aw.rhs_edges = ft->a_rhs_edges.ptr;
		ft->aw.N = N;
		ft->aw.n0 = n0;
		ft->aw.E = E;
		ft->aw.m = m;
		ft->aw.corner = &ft->corner;
		ft->aw.diag = ft->a_diag.ptr;
		ft->aw.dinv = ft->a_dinv.ptr;
		ft->aw.dinv_b = ft->a_dinvb.ptr;
		ft->aw.rhs = ft->a_rhs.ptr;
		ft->aw.x = ft->a_x.ptr;
		ft->aw.refine = NNRT_ARAP_REFINE != 0;
		ft->aw.refine_ratio = ft->refine_ratio;
		ft->aw.res = ft->a_res.ptr;
		ft->aw.dx = ft->a_dx.ptr;
		ft->aw.edge_offsets = ft->a_offsets.ptr;
		ft->aw.edge_list = ft->a_list.ptr;
	}
	const auto after = std::make_tuple(ft->mesh_p.ptr, ft->faces4.ptr, ft->anchors.ptr, ft->keys.ptr, ft->acc.ptr, ft->wing.ptr, ft->corner.generation,
	                                   ft->face_nodes.ptr, ft->wpos.ptr, ft->mesh_p4.ptr, ft->tile_order.ptr, ft->anchors16.ptr);
	// Captured graphs bake every buffer pointer and the per-frame constants (NDC setup, pixel camera, extrinsics) into
	// their kernel arguments: any change drops them. The warp field is recognised by its unique id, not its address.
	const NdcSetup nndc = make_ndc_setup(h_K, H, W, ft->p.ndc_convention == NNRT_NDC_CONSISTENT);
	const Camera npix = pixel_camera(h_K);
	const WarpExtrinsics ne = make_extrinsics(h_E);
	// the warp's 16-bit anchor copy (every index fits: N < 65535; -1 as 0xFFFF), filled with the anchors below
	const bool anchors16 = K == 4 && N < 65535 && [] {
		const char* v = std::getenv("NNRT_ANCHORS16");   // development switch: 0 = the int32 anchors
		return !(v && *v == '0');
	}();
	if (before != after || ft->use_tile_order != tile_order || ft->pix_low_occupancy != pix_low || ft->use_anchors16 != anchors16 || ft->wf != wf || ft->wf_id != wf->id || ft->V != V || ft->F != F || ft->H != H || ft->W != W || ft->N != N ||
	    ft->K != K || std::memcmp(&nndc, &ft->ndc, sizeof(nndc)) != 0 || std::memcmp(&npix, &ft->pix, sizeof(npix)) != 0 ||
	    std::memcmp(&ne, &ft->extr, sizeof(ne)) != 0)
		ft->drop_graphs();
	ft->use_tile_order = tile_order;
	ft->pix_low_occupancy = pix_low;
	ft->use_anchors16 = anchors16;
	ft->V = V;
	ft->F = F;
	ft->H = H;
	ft->W = W;
	ft->N = N;
	ft->K = K;
	ft->wf = wf;
	ft->wf_id = wf->id;
	ft->ndc = nndc;
	ft->pix = npix;
	ft->extr = ne;
	ft->snapshot_valid = false;
	// order the work stream after the caller's stream
	NNRT_HIP(hipEventRecord(ft->ev_in, us));
	NNRT_HIP(hipStreamWaitEvent(ft->work, ft->ev_in, 0));
	hipStream_t s = ft->work;
	NNRT_HIP(hipMemcpyAsync(ft->mesh_p.ptr, d_vertices, sizeof(float) * 3 * V, hipMemcpyDeviceToDevice, s));
	NNRT_HIP(hipMemcpyAsync(ft->mesh_n.ptr, d_normals, sizeof(float) * 3 * V, hipMemcpyDeviceToDevice, s));
	k_faces_to_int4<<<static_cast<unsigned>(ceil_div(F, 256)), 256, 0, s>>>(d_faces, F, V, ft->p.ndc_convention == NNRT_NDC_CONSISTENT,
	                                                                        ft->faces4.ptr, ft->error_flag.ptr);
	NNRT_LAUNCH_CHECK();
	k_to_float4<<<static_cast<unsigned>(ceil_div(V, 256)), 256, 0, s>>>(d_vertices, d_normals, V, ft->mesh_p4.ptr, ft->mesh_n4.ptr);
	NNRT_LAUNCH_CHECK();
	// once per frame (:96-106): anchors & weights on the canonical mesh in virtual node order
	if ((st = launch_compute_anchors(ft->mesh_p.ptr, V, wf->node_positions.ptr, N, K, wf->coverage,
	                                 wf->coverage_method == NNRT_MINIMAL_K_NEIGHBOR_NODE_DISTANCE ? wf->node_weights.ptr : nullptr,
	                                 wf->threshold ? wf->minimum_valid : 0, ft->anchors.ptr, ft->weights.ptr, s)))
		return st;
	// the faces' distinct anchor nodes (AssociateFacesWithAnchors, :105), consumed by the node pass of every iteration
	if ((st = launch_face_node_table(ft->faces4.ptr, F, ft->anchors.ptr, K, ft->face_nodes.ptr, s))) return st;
	if (ft->use_anchors16 && (st = launch_pack_anchors16(ft->anchors.ptr, V, ft->anchors16.ptr, s))) return st;
	// reference point cloud (:289-306): depth / scale with 0 < d < max_depth, AND the user mask; stored as depth (0 = masked)
	if (ref.depth)
		k_prepare_reference_depth<<<static_cast<unsigned>(ceil_div(P, 256)), 256, 0, s>>>(ref.depth, ref.mask, H, W, ref.depth_scale,
		                                                                                  ft->p.max_depth, ft->pix, ft->ref_points.ptr);
	else
		k_prepare_reference_points<<<static_cast<unsigned>(ceil_div(P, 256)), 256, 0, s>>>(ref.points, ref.mask, P, ft->ref_points.ptr);
	NNRT_LAUNCH_CHECK();
	// the pixel launch's tile order for this frame's reference points
	if (ft->use_tile_order &&
	    (st = launch_tile_order(ft->ref_points.ptr, H, W, static_cast<int>(ceil_div(W, 16)), static_cast<int>(ceil_div(H, 16)), ft->tile_flags.ptr,
	                            ft->tile_order.ptr, s)))
		return st;
	NNRT_HIP(hipMemsetAsync(ft->keys.ptr, 0xff, sizeof(uint64_t) * P, s));
	NNRT_HIP(hipMemsetAsync(ft->acc.ptr, 0, sizeof(double) * N * ACC_STRIDE, s));
	NNRT_HIP(hipEventRecord(ft->ev_out, s));
	NNRT_HIP(hipStreamWaitEvent(us, ft->ev_out, 0));
	ft->prepared = true;
	return NNRT_OK;
}
} // namespace

nnrt_status nnrt_fitter_prepare(nnrt_fitter* ft, nnrt_warp_field* wf, const float* d_vertices, const float* d_normals, int64_t V,
                                const int64_t* d_faces, int64_t F, const float* d_depth, const uint8_t* d_mask, int32_t H, int32_t W,
                                const double* h_K, const double* h_E, float depth_scale, void* stream) {
	FrameReference ref;
	ref.depth = d_depth;
	ref.mask = d_mask;
	ref.depth_scale = depth_scale;
	NNRT_CHECK_ARG(d_depth, "null depth image");
	return prepare_frame(ft, wf, d_vertices, d_normals, V, d_faces, F, ref, H, W, h_K, h_E, stream);
}

nnrt_status nnrt_fitter_prepare_point_cloud(nnrt_fitter* ft, nnrt_warp_field* wf, const float* d_vertices, const float* d_normals,
                                            int64_t V, const int64_t* d_faces, int64_t F, const float* d_points, const uint8_t* d_point_mask,
                                            int32_t H, int32_t W, const double* h_K, const double* h_E, void* stream) {
	FrameReference ref;
	ref.points = d_points;
	ref.mask = d_point_mask;
	NNRT_CHECK_ARG(d_points, "null reference point cloud");
	return prepare_frame(ft, wf, d_vertices, d_normals, V, d_faces, F, ref, H, W, h_K, h_E, stream);
}

namespace {
constexpr int MAX_GRAPH_ITERATIONS = 64;   // iterations per captured sequence graph (longer runs replay several)
constexpr size_t MAX_CACHED_GRAPHS = 8;
// what the iterations of a sequence restart from: nothing; the identity warp (every iteration); the stored snapshot (every
// iteration); the stored snapshot before the first iteration of the call only (a whole frame fit from a stored state)
enum { RESET_NONE = 0, RESET_IDENTITY = 1, RESET_SNAPSHOT = 2, RESET_SNAPSHOT_FIRST = 3 };

// A restart folded into the iteration's kernels where they support it: from the identity (block-diagonal path, <= 4
// anchors: the identity-specialised warp / update), or from the snapshot (every path: the warp, the ARAP edge terms and
// the update read the snapshot as the starting state). Otherwise a separate kernel restarts.
bool fold_reset(const nnrt_fitter* ft) { return ft->E == 0 && ft->K <= 4; }
bool fold_snapshot(const nnrt_fitter*) { return true; }

nnrt_status check_frame(const nnrt_fitter* ft, const nnrt_warp_field* wf, const char* who) {
	if (!ft->prepared || ft->wf != wf || ft->wf_id != wf->id) {
		set_error(std::string("nnrt_fitter_prepare must be called with this warp field before ") + who);
		return NNRT_ERROR_ARGUMENT;
	}
	if (wf->device != ft->device) {
		set_error("the warp field and the fitter live on different devices");
		return NNRT_ERROR_ARGUMENT;
	}
	return NNRT_OK;
}

// how iteration i of a sequence starts
struct Restart {   // internal (static helpers below), not part of the C-ABI
	int kernel = RESET_NONE;         // restart launched before the iteration (RESET_NONE: none)
	bool from_identity = false;      // folded identity start
	const float* state_in = nullptr; // folded snapshot start
};

static Restart restart_plan(const nnrt_fitter* ft, int r) {
	Restart p;
	if (r == RESET_IDENTITY) {
		if (fold_reset(ft)) p.from_identity = true;
		else p.kernel = RESET_IDENTITY;
	} else if (r == RESET_SNAPSHOT) {
		if (fold_snapshot(ft)) p.state_in = ft->snapshot.ptr;
		else p.kernel = RESET_SNAPSHOT;
	}
	return p;
}

// a restart launched on s (inside or outside a capture)
nnrt_status enqueue_restart(nnrt_fitter* ft, nnrt_warp_field* wf, int kernel, hipStream_t s) {
	if (kernel == RESET_IDENTITY) {
		k_reset_motion<<<static_cast<unsigned>(ceil_div(wf->N, 256)), 256, 0, s>>>(wf->state.ptr, wf->N);
		if (hipGetLastError() != hipSuccess) {
			set_error("kernel launch failed (k_reset_motion)");
			return NNRT_ERROR_HIP;
		}
	} else if (kernel == RESET_SNAPSHOT) {
		const int count = wf->N * (NODE_STRIDE / 4);
		k_copy_state<<<static_cast<unsigned>(ceil_div(count, 256)), 256, 0, s>>>(reinterpret_cast<const float4*>(ft->snapshot.ptr),
		                                                                        reinterpret_cast<float4*>(wf->state.ptr), count);
		if (hipGetLastError() != hipSuccess) {
			set_error("kernel launch failed (k_copy_state)");
			return NNRT_ERROR_HIP;
		}
	}
	return NNRT_OK;
}

nnrt_status enqueue_step(nnrt_fitter* ft, nnrt_warp_field* wf, int mode, int restart, hipStream_t s) {
	const Restart p = restart_plan(ft, restart);
	nnrt_status st = enqueue_restart(ft, wf, p.kernel, s);
	if (st) return st;
	return enqueue_iteration(ft, wf, mode, s, nullptr, p.from_identity, p.state_in);
}

int restart_of(int reset, bool first_of_call) {
	return reset == RESET_SNAPSHOT_FIRST ? (first_of_call ? RESET_SNAPSHOT : RESET_NONE) : reset;
}

nnrt_status iterate_impl(nnrt_fitter* ft, nnrt_warp_field* wf, int32_t first_iteration, int32_t count, int reset, hipStream_t us) {
	ft->refine_ratio_used = ft->refine_ratio;
	nnrt_status st;
	for (int it0 = first_iteration; it0 < first_iteration + count; it0 += MAX_GRAPH_ITERATIONS) {
		const int n = std::min(MAX_GRAPH_ITERATIONS, first_iteration + count - it0);
		std::vector<int> modes(static_cast<size_t>(n));
		for (int i = 0; i < n; i++) modes[static_cast<size_t>(i)] = ft->p.iteration_modes[(it0 + i) % ft->p.iteration_mode_count];
		ft->last_mode = modes.back();
		// a sequence graph is keyed by its modes and by what each of its iterations restarts from
		const int key_reset = reset == RESET_SNAPSHOT_FIRST && it0 != first_iteration ? RESET_NONE : reset;
		nnrt_fitter::SeqGraph* seen = nullptr;
		for (auto& g : ft->graphs)
			if (g.reset == key_reset && g.modes == modes) seen = &g;
		const bool capture = ft->p.use_hip_graph == NNRT_GRAPH_ALWAYS || (ft->p.use_hip_graph == NNRT_GRAPH_AUTO && seen != nullptr);
		if (!capture) {
			// eager launches on the caller's stream
			for (int i = 0; i < n; i++)
				if ((st = enqueue_step(ft, wf, modes[static_cast<size_t>(i)], restart_of(reset, it0 + i == first_iteration), us))) return st;
			if (ft->p.use_hip_graph == NNRT_GRAPH_AUTO && !seen) {
				if (ft->graphs.size() >= MAX_CACHED_GRAPHS) {
					if (ft->graphs.front().exec) hipGraphExecDestroy(ft->graphs.front().exec);
					ft->graphs.erase(ft->graphs.begin());
				}
				ft->graphs.push_back({modes, key_reset, nullptr});
			}
			continue;
		}
		// Graphs are captured on the fitter's private stream (capture needs a non-legacy stream) and replayed on the
		// caller's: a whole run of iterations is one launch.
		if (!seen || !seen->exec) {
			hipGraph_t g = nullptr;
			NNRT_HIP(hipStreamBeginCapture(ft->work, hipStreamCaptureModeThreadLocal));
			st = NNRT_OK;
			for (int i = 0; i < n && !st; i++)
				st = enqueue_step(ft, wf, modes[static_cast<size_t>(i)], restart_of(reset, it0 + i == first_iteration), ft->work);
			hipError_t ce = hipStreamEndCapture(ft->work, &g);
			if (st) {
				if (g) hipGraphDestroy(g);
				if (st == NNRT_ERROR_HIP) set_error("kernel launch failed during graph capture");
				return st;
			}
			NNRT_HIP(ce);
			hipGraphExec_t exec = nullptr;
			hipError_t ie = hipGraphInstantiate(&exec, g, nullptr, nullptr, 0);
			hipGraphDestroy(g);
			NNRT_HIP(ie);
			if (seen) {
				seen->exec = exec;
			} else {
				if (ft->graphs.size() >= MAX_CACHED_GRAPHS) {
					if (ft->graphs.front().exec) hipGraphExecDestroy(ft->graphs.front().exec);
					ft->graphs.erase(ft->graphs.begin());
				}
				ft->graphs.push_back({modes, key_reset, exec});
				seen = &ft->graphs.back();
			}
		}
		NNRT_HIP(hipGraphLaunch(seen->exec, us));
	}
	return NNRT_OK;
}
} // namespace

nnrt_status nnrt_fitter_iterate(nnrt_fitter* ft, nnrt_warp_field* wf, int32_t first_iteration, int32_t count, void* stream) {
	NNRT_CHECK_ARG(ft && wf && count >= 0, "invalid arguments");
	nnrt_status st = check_frame(ft, wf, "nnrt_fitter_iterate");
	if (st) return st;
	DeviceGuard guard(ft->device);
	return iterate_impl(ft, wf, first_iteration, count, RESET_NONE, static_cast<hipStream_t>(stream));
}

nnrt_status nnrt_fitter_iterate_from_identity(nnrt_fitter* ft, nnrt_warp_field* wf, int32_t first_iteration, int32_t count, void* stream) {
	NNRT_CHECK_ARG(ft && wf && count >= 0, "invalid arguments");
	nnrt_status st = check_frame(ft, wf, "nnrt_fitter_iterate_from_identity");
	if (st) return st;
	DeviceGuard guard(ft->device);
	return iterate_impl(ft, wf, first_iteration, count, RESET_IDENTITY, static_cast<hipStream_t>(stream));
}

nnrt_status nnrt_fitter_corner_info(const nnrt_fitter* ft, int64_t* h_out) {
	NNRT_CHECK_ARG(ft && h_out, "null pointer");
	const CornerSolver& c = ft->corner;
	const bool on = ft->E > 0;
	h_out[0] = on ? ft->N - ft->n0 : 0;
	h_out[1] = on ? c.tile_columns() : 0;
	h_out[2] = on ? c.levels() : 0;
	h_out[3] = on ? c.back_launches() : 0;
	h_out[4] = on ? c.stored_tiles() : 0;
	h_out[5] = on ? c.dense_lower_tiles() : 0;
	return NNRT_OK;
}

nnrt_status nnrt_fitter_get_warped_mesh(nnrt_fitter* ft, float* h_positions, float* h_normals, int64_t vertex_count, void* stream) {
	NNRT_CHECK_ARG(ft && h_positions && h_normals, "null pointer");
	NNRT_CHECK_ARG(ft->V > 0 && ft->wpos.ptr, "no prepared frame");
	// the host buffers hold vertex_count rows: a mismatch with the prepared mesh is refused, not written past
	NNRT_CHECK_ARG(vertex_count == ft->V, "vertex_count differs from the prepared mesh's vertex count");
	DeviceGuard guard(ft->device);
	NNRT_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
	NNRT_HIP(hipStreamSynchronize(ft->work));
	std::vector<float4> p(static_cast<size_t>(ft->V)), n(static_cast<size_t>(ft->V));
	NNRT_HIP(hipMemcpy(p.data(), ft->wpos.ptr, sizeof(float4) * p.size(), hipMemcpyDeviceToHost));
	NNRT_HIP(hipMemcpy(n.data(), ft->wnrm.ptr, sizeof(float4) * n.size(), hipMemcpyDeviceToHost));
	for (size_t v = 0; v < p.size(); v++) {
		h_positions[3 * v] = p[v].x;
		h_positions[3 * v + 1] = p[v].y;
		h_positions[3 * v + 2] = p[v].z;
		h_normals[3 * v] = n[v].x;
		h_normals[3 * v + 1] = n[v].y;
		h_normals[3 * v + 2] = n[v].z;
	}
	return NNRT_OK;
}

nnrt_status nnrt_fitter_get_arrowhead_system(nnrt_fitter* ft, float* h_diag, float* h_wing, float* h_rhs, int64_t node_count, int64_t edge_count,
                                             void* stream) {
	NNRT_CHECK_ARG(ft && h_diag && h_wing && h_rhs, "null pointer");
	NNRT_CHECK_ARG(ft->E > 0 && ft->a_diag.ptr && ft->wing.ptr && ft->a_rhs.ptr, "no prepared ARAP frame (the arrowhead system needs layer_count > 1)");
	NNRT_CHECK_ARG(node_count == ft->N && edge_count == ft->E, "node_count / edge_count differ from the prepared frame's");
	DeviceGuard guard(ft->device);
	NNRT_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
	NNRT_HIP(hipStreamSynchronize(ft->work));
	NNRT_HIP(hipMemcpy(h_diag, ft->a_diag.ptr, sizeof(float) * 36 * static_cast<size_t>(ft->N), hipMemcpyDeviceToHost));
	NNRT_HIP(hipMemcpy(h_wing, ft->wing.ptr, sizeof(float) * 36 * static_cast<size_t>(ft->E), hipMemcpyDeviceToHost));
	NNRT_HIP(hipMemcpy(h_rhs, ft->a_rhs.ptr, sizeof(float) * 6 * static_cast<size_t>(ft->N), hipMemcpyDeviceToHost));
	return NNRT_OK;
}

nnrt_status nnrt_fitter_corner_work(const nnrt_fitter* ft, int64_t* h_out) {
	NNRT_CHECK_ARG(ft && h_out, "null pointer");
	const CornerSolver& c = ft->corner;
	const bool on = ft->E > 0;
	h_out[0] = on ? c.mfma_flops() : 0;
	h_out[1] = on ? c.update_terms() : 0;
	h_out[2] = on ? c.eliminated_columns() : 0;
	return NNRT_OK;
}

nnrt_status nnrt_fitter_refine_info(nnrt_fitter* ft, float* h_out, void* stream) {
	NNRT_CHECK_ARG(ft && h_out, "null pointer");
	DeviceGuard guard(ft->device);
	// the gate as the last launched solve applied it: its device pivot word and the threshold it ran with (a later
	// nnrt_fitter_set_refine_ratio changes the next solve, not the report of this one: ADVICE r4)
	h_out[0] = 1.f;
	h_out[1] = ft->refine_ratio_used;
	h_out[2] = 0.f;
	h_out[3] = 0.f;
	h_out[4] = 0.f;
	if (ft->E > 0 && ft->corner.pivot_ratio()) {
		NNRT_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
		NNRT_HIP(hipStreamSynchronize(ft->work));
		unsigned w[REFINE_WORDS] = {};
		NNRT_HIP(hipMemcpy(w, ft->corner.pivot_ratio(), sizeof(w), hipMemcpyDeviceToHost));
		float r, dm, xm;
		std::memcpy(&r, &w[0], sizeof(r));
		std::memcpy(&dm, &w[REFINE_GUARD_D], sizeof(dm));
		std::memcpy(&xm, &w[REFINE_GUARD_X], sizeof(xm));
		const bool ran = NNRT_ARAP_REFINE != 0 && refine_window(r, ft->refine_ratio_used);
		h_out[0] = r;
		h_out[2] = ran ? 1.f : 0.f;
		h_out[3] = ran ? (xm > 0.f ? dm / xm : dm) : 0.f;
		h_out[4] = ran && refine_accept(dm, xm) ? 1.f : 0.f;
	}
	return NNRT_OK;
}

nnrt_status nnrt_fitter_set_refine_ratio(nnrt_fitter* ft, float ratio) {
	NNRT_CHECK_ARG(ft, "null pointer");
	NNRT_CHECK_ARG(ratio >= 0.f, "refine ratio must be >= 0 (0: never refine)");
	if (ratio == ft->refine_ratio) return NNRT_OK;
	DeviceGuard guard(ft->device);
	NNRT_HIP(hipStreamSynchronize(ft->work));
	ft->refine_ratio = ratio;
	ft->aw.refine_ratio = ratio;
	ft->drop_graphs();   // the threshold is a launch argument of the captured sequences
	return NNRT_OK;
}

int32_t nnrt_fitter_graph_count(const nnrt_fitter* ft) {
	if (!ft) return -1;
	int32_t n = 0;
	for (const auto& g : ft->graphs) n += g.exec != nullptr;
	return n;
}

nnrt_status nnrt_fitter_snapshot_motion(nnrt_fitter* ft, nnrt_warp_field* wf, void* stream) {
	NNRT_CHECK_ARG(ft && wf, "null pointer");
	nnrt_status st = check_frame(ft, wf, "nnrt_fitter_snapshot_motion");
	if (st) return st;
	DeviceGuard guard(ft->device);
	const auto before = ft->snapshot.ptr;
	if ((st = ft->snapshot.ensure(static_cast<size_t>(wf->N) * NODE_STRIDE))) return st;
	if (ft->snapshot.ptr != before) ft->drop_graphs();
	const int count = wf->N * (NODE_STRIDE / 4);
	k_copy_state<<<static_cast<unsigned>(ceil_div(count, 256)), 256, 0, static_cast<hipStream_t>(stream)>>>(
	    reinterpret_cast<const float4*>(wf->state.ptr), reinterpret_cast<float4*>(ft->snapshot.ptr), count);
	NNRT_LAUNCH_CHECK();
	ft->snapshot_valid = true;
	return NNRT_OK;
}

static nnrt_status from_snapshot(nnrt_fitter* ft, nnrt_warp_field* wf, int32_t first_iteration, int32_t count, int reset, void* stream,
                                 const char* who) {
	NNRT_CHECK_ARG(ft && wf && count >= 0, "invalid arguments");
	nnrt_status st = check_frame(ft, wf, who);
	if (st) return st;
	if (!ft->snapshot_valid) {
		set_error(std::string("nnrt_fitter_snapshot_motion must be called after prepare() before ") + who);
		return NNRT_ERROR_ARGUMENT;
	}
	DeviceGuard guard(ft->device);
	return iterate_impl(ft, wf, first_iteration, count, reset, static_cast<hipStream_t>(stream));
}

nnrt_status nnrt_fitter_iterate_from_snapshot(nnrt_fitter* ft, nnrt_warp_field* wf, int32_t first_iteration, int32_t count, void* stream) {
	return from_snapshot(ft, wf, first_iteration, count, RESET_SNAPSHOT, stream, "nnrt_fitter_iterate_from_snapshot");
}

nnrt_status nnrt_fitter_fit_from_snapshot(nnrt_fitter* ft, nnrt_warp_field* wf, int32_t count, void* stream) {
	return from_snapshot(ft, wf, 0, count, RESET_SNAPSHOT_FIRST, stream, "nnrt_fitter_fit_from_snapshot");
}

nnrt_status nnrt_fitter_restore_motion(nnrt_fitter* ft, nnrt_warp_field* wf, void* stream) {
	NNRT_CHECK_ARG(ft && wf, "null pointer");
	nnrt_status st = check_frame(ft, wf, "nnrt_fitter_restore_motion");
	if (st) return st;
	if (!ft->snapshot_valid) {
		set_error("nnrt_fitter_snapshot_motion must be called after prepare() before nnrt_fitter_restore_motion");
		return NNRT_ERROR_ARGUMENT;
	}
	DeviceGuard guard(ft->device);
	return enqueue_restart(ft, wf, RESET_SNAPSHOT, static_cast<hipStream_t>(stream));
}

nnrt_status nnrt_fitter_iterate_timed(nnrt_fitter* ft, nnrt_warp_field* wf, int32_t first_iteration, int32_t count, float* h_stage_ms,
                                      void* stream) {
	NNRT_CHECK_ARG(ft && wf && h_stage_ms && count > 0, "invalid arguments");
	if (nnrt_status cst = check_frame(ft, wf, "nnrt_fitter_iterate_timed")) return cst;
	DeviceGuard guard(ft->device);
	ft->refine_ratio_used = ft->refine_ratio;
	hipStream_t us = static_cast<hipStream_t>(stream);
	NNRT_HIP(hipEventRecord(ft->ev_in, us));
	NNRT_HIP(hipStreamWaitEvent(ft->work, ft->ev_in, 0));
	constexpr int NS = NNRT_TIMED_STAGES;
	std::vector<hipEvent_t> ev(static_cast<size_t>(count) * (NS + 1), nullptr);
	for (auto& e : ev) NNRT_HIP(hipEventCreate(&e));
	nnrt_status st = NNRT_OK;
	for (int i = 0; i < count && !st; i++) {
		const int it = first_iteration + i;
		const int mode = ft->p.iteration_modes[it % ft->p.iteration_mode_count];
		ft->last_mode = mode;
		st = enqueue_iteration(ft, wf, mode, ft->work, &ev[static_cast<size_t>(i) * (NS + 1)]);
	}
	if (!st) {
		NNRT_HIP(hipStreamSynchronize(ft->work));
		for (int k = 0; k < NS; k++) h_stage_ms[k] = 0.f;
		for (int i = 0; i < count; i++)
			for (int k = 0; k < NS; k++) {
				float ms = 0.f;
				NNRT_HIP(hipEventElapsedTime(&ms, ev[static_cast<size_t>(i) * (NS + 1) + k], ev[static_cast<size_t>(i) * (NS + 1) + k + 1]));
				h_stage_ms[k] += ms / count;
			}
	}
	for (auto& e : ev)
		if (e) hipEventDestroy(e);
	NNRT_HIP(hipEventRecord(ft->ev_out, ft->work));
	NNRT_HIP(hipStreamWaitEvent(us, ft->ev_out, 0));
	return st;
}

nnrt_status nnrt_fitter_time_kernels(nnrt_fitter* ft, nnrt_warp_field* wf, int32_t reps, int32_t trials, float* h_kernel_ms, void* stream) {
	NNRT_CHECK_ARG(ft && wf && h_kernel_ms && reps > 0 && trials > 0, "invalid arguments");
	if (nnrt_status cst = check_frame(ft, wf, "nnrt_fitter_time_kernels")) return cst;
	if (!ft->snapshot_valid) {
		set_error("nnrt_fitter_snapshot_motion must be called after prepare() before nnrt_fitter_time_kernels");
		return NNRT_ERROR_ARGUMENT;
	}
	DeviceGuard guard(ft->device);
	hipStream_t us = static_cast<hipStream_t>(stream);
	hipStream_t s = ft->work;
	NNRT_HIP(hipEventRecord(ft->ev_in, us));
	NNRT_HIP(hipStreamWaitEvent(s, ft->ev_in, 0));
	ft->refine_ratio_used = ft->refine_ratio;
	// an error the caller's own earlier iterations raised and has not checked yet survives the timing replays (their
	// flags are discarded below): saved here, restored at the end
	int pending_flag = 0;
	NNRT_HIP(hipStreamSynchronize(s));
	NNRT_HIP(hipMemcpy(&pending_flag, ft->error_flag.ptr, sizeof(int), hipMemcpyDeviceToHost));
	// prefix sequences, each `reps` iterations from the snapshot state in one graph: every kernel runs after the launch
	// it follows in a real iteration (the raster alone excepted, which repeats its own idempotent scatter)
	const unsigned seq[4] = {STAGE_ALL, STAGE_RASTER | STAGE_PIXEL | STAGE_SOLVE, STAGE_RASTER | STAGE_PIXEL, STAGE_RASTER};
	const int mode = ft->p.iteration_modes[0];
	hipGraphExec_t exec[4] = {};
	hipEvent_t ev[2] = {};
	std::vector<float> per_rep[4];
	nnrt_status st = NNRT_OK;
	const size_t P = static_cast<size_t>(ft->H) * ft->W;
	auto run = [&]() -> nnrt_status {
		for (auto& e : ev) NNRT_HIP(hipEventCreate(&e));
		for (int q = 0; q < 4; q++) {
			hipGraph_t g = nullptr;
			NNRT_HIP(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
			nnrt_status cs = NNRT_OK;
			for (int i = 0; i < reps && !cs; i++) cs = enqueue_iteration(ft, wf, mode, s, nullptr, false, ft->snapshot.ptr, seq[q]);
			hipError_t ce = hipStreamEndCapture(s, &g);
			if (cs || ce != hipSuccess) {   // a partially returned graph is destroyed on every early exit
				if (g) hipGraphDestroy(g);
				if (cs) return cs;
				NNRT_HIP(ce);
			}
			hipError_t ie = hipGraphInstantiate(&exec[q], g, nullptr, nullptr, 0);
			hipGraphDestroy(g);
			NNRT_HIP(ie);
		}
		// trials interleave the four sequences (clock drift cancels); consumers' state (raster keys, accumulators) is
		// reset outside the timed region before every replay
		for (int t = -1; t < trials; t++)
			for (int q = 0; q < 4; q++) {
				NNRT_HIP(hipMemsetAsync(ft->keys.ptr, 0xff, sizeof(uint64_t) * P, s));
				NNRT_HIP(hipMemsetAsync(ft->acc.ptr, 0, sizeof(double) * static_cast<size_t>(ft->N) * ACC_STRIDE, s));
				NNRT_HIP(hipEventRecord(ev[0], s));
				NNRT_HIP(hipGraphLaunch(exec[q], s));
				NNRT_HIP(hipEventRecord(ev[1], s));
				NNRT_HIP(hipEventSynchronize(ev[1]));
				float ms = 0.f;
				NNRT_HIP(hipEventElapsedTime(&ms, ev[0], ev[1]));
				if (t >= 0) per_rep[q].push_back(ms / reps);   // trial -1 warms the graph
			}
		return NNRT_OK;
	};
	st = run();
	for (auto& e : exec)
		if (e) hipGraphExecDestroy(e);
	for (auto& e : ev)
		if (e) hipEventDestroy(e);
	if (!st) {
		float med[4];
		for (int q = 0; q < 4; q++) {
			std::vector<float> v = per_rep[q];
			std::sort(v.begin(), v.end());
			med[q] = v[v.size() / 2];
		}
		h_kernel_ms[0] = med[0] - med[1];   // warp
		h_kernel_ms[1] = med[3];            // raster
		h_kernel_ms[2] = med[2] - med[3];   // fused pixel launch
		h_kernel_ms[3] = med[1] - med[2];   // solve + update (ARAP: the whole arrowhead chain)
		h_kernel_ms[4] = med[0];            // whole iteration
		// leave the fitter as an iteration would: raster keys empty, accumulators zero, motion = the snapshot's result;
		// the device error flag goes back to what the caller's own iterations left (the replays' flags are dropped:
		// nnrt_fitter_check reports the caller's iterations only)
		NNRT_HIP(hipMemsetAsync(ft->keys.ptr, 0xff, sizeof(uint64_t) * P, s));
		NNRT_HIP(hipMemsetAsync(ft->acc.ptr, 0, sizeof(double) * static_cast<size_t>(ft->N) * ACC_STRIDE, s));
		NNRT_HIP(hipStreamSynchronize(s));
		NNRT_HIP(hipMemcpy(ft->error_flag.ptr, &pending_flag, sizeof(int), hipMemcpyHostToDevice));
	}
	NNRT_HIP(hipEventRecord(ft->ev_out, s));
	NNRT_HIP(hipStreamWaitEvent(us, ft->ev_out, 0));
	return st;
}

nnrt_status nnrt_fitter_check(nnrt_fitter* ft, void* stream) {
	NNRT_CHECK_ARG(ft, "null pointer");
	DeviceGuard guard(ft->device);
	NNRT_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
	NNRT_HIP(hipStreamSynchronize(ft->work));
	int flag = 0;
	NNRT_HIP(hipMemcpy(&flag, ft->error_flag.ptr, sizeof(int), hipMemcpyDeviceToHost));
	NNRT_HIP(hipMemset(ft->error_flag.ptr, 0, sizeof(int)));
	if (flag & 8) {
		set_error("the corner's dataflow substitution launch gave up waiting on a dependency (k_corner_flow spin bound)");
		return NNRT_ERROR_HIP;
	}
	if (flag & 1) {
		set_error("potrf failed: a Hessian block (or the Schur complement) is not positive-definite (reference NNRT_LAPACK_CHECK, "
		          "SolveBlockDiagonalCholeskyCPU.cpp:48-51)");
		return NNRT_ERROR_NOT_POSITIVE_DEFINITE;
	}
	if (flag & 2) {
		set_error("fixed-coverage ARAP residual indexes edge_layer_indices[node_j] out of bounds (reference quirk A3)");
		return NNRT_ERROR_UNSUPPORTED;
	}
	if (flag & 4) {
		set_error("mesh triangle index out of range (faces must index [0, vertex_count))");
		return NNRT_ERROR_ARGUMENT;
	}
	return NNRT_OK;
}

nnrt_status nnrt_fitter_fit_to_image(nnrt_fitter* ft, nnrt_warp_field* wf, const float* d_vertices, const float* d_normals, int64_t V,
                                     const int64_t* d_faces, int64_t F, const float* d_depth, const uint8_t* d_mask, int32_t H, int32_t W,
                                     const double* h_K, const double* h_E, float depth_scale, void* stream) {
	nnrt_status st = nnrt_fitter_prepare(ft, wf, d_vertices, d_normals, V, d_faces, F, d_depth, d_mask, H, W, h_K, h_E, depth_scale, stream);
	if (st) return st;
	// A14: the reference never updates `maximum_update`, so the loop always runs max_iteration_count iterations
	if ((st = nnrt_fitter_iterate(ft, wf, 0, ft->p.max_iteration_count, stream))) return st;
	return nnrt_fitter_check(ft, stream);
}

nnrt_status nnrt_fitter_fit_to_point_cloud(nnrt_fitter* ft, nnrt_warp_field* wf, const float* d_vertices, const float* d_normals, int64_t V,
                                           const int64_t* d_faces, int64_t F, const float* d_points, const uint8_t* d_point_mask, int32_t H,
                                           int32_t W, const double* h_K, const double* h_E, void* stream) {
	nnrt_status st = nnrt_fitter_prepare_point_cloud(ft, wf, d_vertices, d_normals, V, d_faces, F, d_points, d_point_mask, H, W, h_K, h_E, stream);
	if (st) return st;
	if ((st = nnrt_fitter_iterate(ft, wf, 0, ft->p.max_iteration_count, stream))) return st;
	return nnrt_fitter_check(ft, stream);
}

nnrt_status nnrt_fitter_get_diagnostics(nnrt_fitter* ft, float* h_residuals, uint8_t* h_mask, int32_t* h_faces, float* h_updates,
                                        float* h_gradient, float* h_hessian, void* stream) {
	NNRT_CHECK_ARG(ft && ft->prepared, "fitter not prepared");
	DeviceGuard guard(ft->device);
	NNRT_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
	NNRT_HIP(hipStreamSynchronize(ft->work));
	const int64_t P = static_cast<int64_t>(ft->H) * ft->W;
	const int s = ft->last_mode == NNRT_ITERATION_ALL ? 6 : 3;
	if (h_residuals) NNRT_HIP(hipMemcpy(h_residuals, ft->residuals.ptr, sizeof(float) * P, hipMemcpyDeviceToHost));
	if (h_mask) NNRT_HIP(hipMemcpy(h_mask, ft->residual_mask.ptr, P, hipMemcpyDeviceToHost));
	if (h_faces) NNRT_HIP(hipMemcpy(h_faces, ft->pixel_face.ptr, sizeof(int32_t) * P, hipMemcpyDeviceToHost));
	if (h_updates) NNRT_HIP(hipMemcpy(h_updates, ft->updates.ptr, sizeof(float) * ft->N * s, hipMemcpyDeviceToHost));
	if (h_gradient) NNRT_HIP(hipMemcpy(h_gradient, ft->gradient.ptr, sizeof(float) * ft->N * s, hipMemcpyDeviceToHost));
	if (h_hessian) NNRT_HIP(hipMemcpy(h_hessian, ft->hessian.ptr, sizeof(float) * ft->N * s * s, hipMemcpyDeviceToHost));
	return NNRT_OK;
}

nnrt_status nnrt_fitter_get_anchors(nnrt_fitter* ft, int32_t* h_anchors, float* h_weights, void* stream) {
	NNRT_CHECK_ARG(ft && ft->prepared, "fitter not prepared");
	DeviceGuard guard(ft->device);
	NNRT_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
	NNRT_HIP(hipStreamSynchronize(ft->work));
	if (h_anchors) NNRT_HIP(hipMemcpy(h_anchors, ft->anchors.ptr, sizeof(int32_t) * ft->V * ft->K, hipMemcpyDeviceToHost));
	if (h_weights) NNRT_HIP(hipMemcpy(h_weights, ft->weights.ptr, sizeof(float) * ft->V * ft->K, hipMemcpyDeviceToHost));
	return NNRT_OK;
}

// ---------------------------------------------------------------------------------------------------------------------
// stage entry points
// ---------------------------------------------------------------------------------------------------------------------
nnrt_status nnrt_compute_anchors_and_weights(const float* d_points, int64_t V, const float* d_nodes, int32_t N, int32_t K, float coverage,
                                             const float* d_node_weights, int32_t minimum_valid, int32_t* d_anchors, float* d_weights,
                                             void* stream) {
	NNRT_CHECK_ARG(minimum_valid <= K, "minimum_valid_anchor_count has to be <= anchor_count (WarpAnchorComputation.cpp:92-95)");
	return launch_compute_anchors(d_points, V, d_nodes, N, K, coverage, d_node_weights, minimum_valid, d_anchors, d_weights,
	                              static_cast<hipStream_t>(stream));
}

nnrt_status nnrt_warp_mesh(const float* d_vertices, const float* d_normals, int64_t V, const float* d_nodes, const float* d_rotations,
                           const float* d_translations, int32_t N, const int32_t* d_anchors, const float* d_weights, int32_t K,
                           const double* h_E, float* d_out_vertices, float* d_out_normals, void* stream) {
	NNRT_CHECK_ARG(d_vertices && d_normals && d_nodes && d_anchors && d_weights && d_out_vertices && d_out_normals, "null pointer");
	hipStream_t s = static_cast<hipStream_t>(stream);
	float* state = nullptr;
	float4 *wp = nullptr, *wn = nullptr;
	NNRT_HIP(hipMallocAsync(reinterpret_cast<void**>(&state), sizeof(float) * NODE_STRIDE * std::max(N, 1), s));
	NNRT_HIP(hipMallocAsync(reinterpret_cast<void**>(&wp), sizeof(float4) * std::max<int64_t>(V, 1), s));
	NNRT_HIP(hipMallocAsync(reinterpret_cast<void**>(&wn), sizeof(float4) * std::max<int64_t>(V, 1), s));
	nnrt_status st = launch_pack_nodes(d_nodes, d_rotations, d_translations, N, state, s);
	if (!st) st = launch_warp_mesh(d_vertices, d_normals, V, state, d_anchors, d_weights, K, make_extrinsics(h_E), wp, wn, nullptr, s);
	if (!st) st = launch_unpack_float4x3(wp, V, d_out_vertices, s);
	if (!st) st = launch_unpack_float4x3(wn, V, d_out_normals, s);
	hipFreeAsync(state, s);
	hipFreeAsync(wp, s);
	hipFreeAsync(wn, s);
	return st;
}

nnrt_status nnrt_warp_points(const float* d_points, const float* d_normals, int64_t V, const float* d_nodes, const float* d_rotations,
                             const float* d_translations, int32_t N, const int32_t* d_anchors, const float* d_weights, int32_t K, float coverage,
                             int32_t threshold, int32_t minimum_valid, const double* h_E, float* d_out_points, float* d_out_normals,
                             void* stream) {
	NNRT_CHECK_ARG((d_points && d_nodes && d_rotations && d_translations && d_out_points) || V == 0, "null pointer");
	NNRT_CHECK_ARG(!d_normals == !d_out_normals, "normals in and out must both be given or both be NULL");
	NNRT_CHECK_ARG(K >= 1 && K <= MAX_ANCHORS, "anchor_count needs to satisfy 0 < anchor_count <= 8 (Warping.cpp:70-75)");
	NNRT_CHECK_ARG(minimum_valid >= 0 && minimum_valid <= K,
	               "minimum_valid_anchor_count is required to satisfy 0 <= minimum_valid_anchor_count <= anchor_count (Warping.cpp:76-79)");
	NNRT_CHECK_ARG(!d_anchors == !d_weights, "anchors and anchor_weights must both be given");
	if (V == 0) return NNRT_OK;
	hipStream_t s = static_cast<hipStream_t>(stream);
	float* state = nullptr;
	int32_t* anchors = nullptr;
	float* weights = nullptr;
	NNRT_HIP(hipMallocAsync(reinterpret_cast<void**>(&state), sizeof(float) * NODE_STRIDE * std::max(N, 1), s));
	nnrt_status st = launch_pack_nodes(d_nodes, d_rotations, d_translations, N, state, s);
	const int32_t* a = d_anchors;
	const float* w = d_weights;
	if (!st && !d_anchors) {   // online anchors: FindAnchorsAndWeightsForPoint_Euclidean[_Threshold]_FixedNodeCoverageWeight
		NNRT_HIP(hipMallocAsync(reinterpret_cast<void**>(&anchors), sizeof(int32_t) * V * K, s));
		NNRT_HIP(hipMallocAsync(reinterpret_cast<void**>(&weights), sizeof(float) * V * K, s));
		st = launch_compute_anchors(d_points, V, d_nodes, N, K, coverage, nullptr, minimum_valid, anchors, weights, s, threshold ? 1 : 0);
		a = anchors;
		w = weights;
	}
	if (!st) st = launch_warp_points(d_points, d_normals, V, state, a, w, K, threshold ? minimum_valid : -1, make_extrinsics(h_E), d_out_points,
	                                 d_out_normals, s);
	hipFreeAsync(state, s);
	if (anchors) hipFreeAsync(anchors, s);
	if (weights) hipFreeAsync(weights, s);
	return st;
}

nnrt_status nnrt_compute_point_to_plane_distances(const float* d_normals1, const float* d_vertices1, const float* d_vertices2, int64_t count,
                                                  float* d_out, void* stream) {
	NNRT_CHECK_ARG((d_normals1 && d_vertices1 && d_vertices2 && d_out) || count == 0, "null pointer");
	return launch_point_to_plane(d_normals1, d_vertices1, d_vertices2, count, d_out, static_cast<hipStream_t>(stream));
}

nnrt_status nnrt_get_meshes_ndc_face_vertices_and_clip_mask(const float* const* h_vertex_sets, const int64_t* const* h_face_sets,
                                                            const int64_t* h_face_counts, int32_t mesh_count, const double* h_K, int32_t H,
                                                            int32_t W, float near_clip, float far_clip, float* d_face_ndc, uint8_t* d_clip_mask,
                                                            void* stream) {
	NNRT_CHECK_ARG(h_K && h_vertex_sets && h_face_sets && h_face_counts && mesh_count >= 0, "null pointer");
	NNRT_CHECK_ARG(near_clip >= 0.f, "near_clipping_distance cannot be less than 0 (ExtractFaceVertices.cpp:40-44)");
	NNRT_CHECK_ARG(near_clip <= far_clip, "near_clipping_distance cannot be greater than far_clipping_distance");
	const NdcSetup ndc = make_ndc_setup(h_K, H, W, false);
	int64_t offset = 0;
	for (int m = 0; m < mesh_count; m++) {   // face f of mesh m -> output row offset(m) + f (ExtractClippedFaceVerticesImpl.h:111-116)
		const int64_t F = h_face_counts[m];
		NNRT_CHECK_ARG(F >= 0 && (F == 0 || (h_vertex_sets[m] && h_face_sets[m])), "mesh needs both triangle indices and vertex positions");
		nnrt_status st = launch_extract_face_ndc(h_vertex_sets[m], h_face_sets[m], F, ndc, near_clip, far_clip, d_face_ndc + 9 * offset,
		                                         d_clip_mask + offset, static_cast<hipStream_t>(stream));
		if (st) return st;
		offset += F;
	}
	return NNRT_OK;
}

nnrt_status nnrt_get_mesh_ndc_face_vertices_and_clip_mask(const float* d_vertices, const int64_t* d_faces, int64_t F, const double* h_K, int32_t H,
                                                          int32_t W, float near_clip, float far_clip, float* d_face_ndc, uint8_t* d_clip_mask,
                                                          void* stream) {
	NNRT_CHECK_ARG(h_K && d_vertices && d_faces && d_face_ndc && d_clip_mask, "null pointer");
	NNRT_CHECK_ARG(near_clip >= 0.f, "near_clipping_distance cannot be less than 0 (ExtractFaceVertices.cpp:40-44)");
	NNRT_CHECK_ARG(near_clip <= far_clip, "near_clipping_distance cannot be greater than far_clipping_distance");
	return launch_extract_face_ndc(d_vertices, d_faces, F, make_ndc_setup(h_K, H, W, false), near_clip, far_clip, d_face_ndc, d_clip_mask,
	                               static_cast<hipStream_t>(stream));
}

nnrt_status nnrt_rasterize_ndc_triangles(const float* d_face_ndc, const uint8_t* d_clip_mask, int64_t F, int32_t H, int32_t W,
                                         float blur_radius_pixels, int32_t faces_per_pixel, int32_t bin_size, int32_t max_faces_per_bin,
                                         int32_t perspective, int32_t clip_barycentric, int32_t cull_back_faces, int64_t* d_faces_out,
                                         float* d_depth_out, float* d_bary_out, float* d_dist_out, void* stream) {
	(void) max_faces_per_bin;
	NNRT_CHECK_ARG(H > 0 && W > 0, "image_size must be positive");
	if (faces_per_pixel > MAX_FACES_PER_PIXEL || faces_per_pixel < 1) {
		set_error("Need faces_per_pixel <= 8 (RasterizeNdcTriangles.cpp:45-47)");
		return NNRT_ERROR_ARGUMENT;
	}
	// bin-size validation kept for error parity (RasterizeNdcTriangles.cpp:53-76); bins themselves are not needed here
	const int max_dim = std::max(H, W);
	if (bin_size == -1) bin_size = max_dim <= 64 ? 8 : static_cast<int>(std::pow(2, std::max(static_cast<int>(std::ceil(std::log2(static_cast<double>(max_dim)))) - 4, 4)));
	if (bin_size != 0 && 1 + (max_dim - 1) / bin_size >= 22) {
		set_error("The provided bin_size is too small (RasterizeNdcTriangles.cpp:70-76)");
		return NNRT_ERROR_ARGUMENT;
	}
	hipStream_t s = static_cast<hipStream_t>(stream);
	const RasterOptions o = make_raster_options(H, W, blur_radius_pixels / (static_cast<float>(fminf(H, W)) / 2.0f), perspective, clip_barycentric, cull_back_faces);
	if (faces_per_pixel == 1) {
		const int64_t P = static_cast<int64_t>(H) * W;
		uint64_t* keys = nullptr;
		NNRT_HIP(hipMallocAsync(reinterpret_cast<void**>(&keys), sizeof(uint64_t) * P, s));
		NNRT_HIP(hipMemsetAsync(keys, 0xff, sizeof(uint64_t) * P, s));
		nnrt_status st = launch_raster_scatter_ndc(d_face_ndc, d_clip_mask, F, o, keys, s);
		if (!st) st = launch_raster_resolve(d_face_ndc, F, o, keys, d_faces_out, d_depth_out, d_bary_out, d_dist_out, s);
		hipFreeAsync(keys, s);
		return st;
	}
	return launch_raster_multi(d_face_ndc, d_clip_mask, F, o, faces_per_pixel, d_faces_out, d_depth_out, d_bary_out, d_dist_out, s);
}

nnrt_status nnrt_interpolate_face_attributes(const int64_t* d_pixel_faces, const float* d_bary, int64_t P, int32_t Kf, const float* d_attrs,
                                             int32_t C, float* d_out, void* stream) {
	return launch_interpolate(d_pixel_faces, d_bary, P, Kf, d_attrs, C, d_out, static_cast<hipStream_t>(stream));
}

nnrt_status nnrt_unproject_depth(const float* d_depth, int32_t H, int32_t W, const double* h_K, float depth_scale, float depth_max,
                                 float* d_points, uint8_t* d_mask, void* stream) {
	NNRT_CHECK_ARG(h_K, "null intrinsics");
	return launch_unproject(d_depth, NNRT_DTYPE_FLOAT32, H, W, pixel_camera(h_K), make_extrinsics(nullptr), depth_scale, depth_max, d_points,
	                        d_mask, static_cast<hipStream_t>(stream));
}

nnrt_status nnrt_unproject_depth_image(const void* d_depth, int32_t depth_dtype, int32_t H, int32_t W, const double* h_K, const double* h_E,
                                       float depth_scale, float depth_max, float* d_points, uint8_t* d_mask, void* stream) {
	NNRT_CHECK_ARG(h_K, "null intrinsics");
	NNRT_CHECK_ARG(depth_dtype == NNRT_DTYPE_UINT16 || depth_dtype == NNRT_DTYPE_FLOAT32, "depth must be uint16 or float32");
	NNRT_CHECK_ARG(H >= 0 && W >= 0, "negative image size");
	NNRT_CHECK_ARG((d_depth && d_points && d_mask) || static_cast<int64_t>(H) * W == 0, "null pointer");
	double pose[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
	if (h_E) {   // Open3D InverseTransformation: [R^T | -R^T t], computed in double, rounded once into TransformIndexer's floats
		for (int r = 0; r < 3; r++) {
			double tr = 0.0;
			for (int c = 0; c < 3; c++) {
				pose[4 * r + c] = h_E[4 * c + r];
				tr += h_E[4 * c + r] * h_E[4 * c + 3];
			}
			pose[4 * r + 3] = -tr;
		}
	}
	return launch_unproject(d_depth, depth_dtype, H, W, pixel_camera(h_K), make_extrinsics(h_E ? pose : nullptr), depth_scale, depth_max,
	                        d_points, d_mask, static_cast<hipStream_t>(stream));
}

nnrt_status nnrt_backproject_depth_ushort(const uint16_t* d_depth, int32_t height, int32_t width, float fx, float fy, float cx, float cy,
                                          float normalizer, float* d_points, void* stream) {
	NNRT_CHECK_ARG(height >= 0 && width >= 0, "negative image size");
	NNRT_CHECK_ARG((d_depth && d_points) || height * static_cast<int64_t>(width) == 0, "null image");
	return launch_backproject_depth_u16(d_depth, height, width, BackprojectCamera{fx, fy, cx, cy, normalizer}, d_points,
	                                    static_cast<hipStream_t>(stream));
}

nnrt_status nnrt_backproject_depth_float(const float* d_depth, int32_t height, int32_t width, float fx, float fy, float cx, float cy,
                                         float* d_points, void* stream) {
	NNRT_CHECK_ARG(height >= 0 && width >= 0, "negative image size");
	NNRT_CHECK_ARG((d_depth && d_points) || height * static_cast<int64_t>(width) == 0, "null image");
	return launch_backproject_depth_f32(d_depth, height, width, BackprojectCamera{fx, fy, cx, cy, 1.0f}, d_points,
	                                    static_cast<hipStream_t>(stream));
}

nnrt_status nnrt_matmul3d(const float* d_a, const float* d_b, int64_t batch, int32_t m, int32_t k, int32_t n, float* d_c, void* stream) {
	NNRT_CHECK_ARG(batch >= 0 && m >= 0 && k >= 0 && n >= 0, "negative dimension");
	NNRT_CHECK_ARG((d_a && d_b && d_c) || batch * m * n == 0, "null pointer");
	return launch_matmul3d(d_a, d_b, batch, m, k, n, d_c, static_cast<hipStream_t>(stream));
}

nnrt_status nnrt_median_grid_subsample_3d_points(const float* d_points, int64_t n, float cell, int64_t* d_out, int64_t* h_count, void* stream) {
	NNRT_CHECK_ARG(h_count && (n == 0 || (d_points && d_out)), "null pointer");
	NNRT_CHECK_ARG(n >= 0 && n < (int64_t(1) << 31), "point count out of range");
	NNRT_CHECK_ARG(cell > 0.f, "grid_cell_size must be positive");
	return launch_median_grid_subsample(d_points, static_cast<int>(n), cell, d_out, h_count, static_cast<hipStream_t>(stream));
}

nnrt_status nnrt_axis_angle_to_matrices_rodrigues(const float* d_vectors, int32_t count, float* d_matrices, void* stream) {
	return launch_rodrigues(d_vectors, count, d_matrices, static_cast<hipStream_t>(stream));
}

nnrt_status nnrt_solve_block_diagonal_cholesky(const float* d_blocks, const float* d_b, int32_t count, int32_t block_size, float* d_x,
                                               void* stream) {
	hipStream_t s = static_cast<hipStream_t>(stream);
	int* flag = nullptr;
	NNRT_HIP(hipMallocAsync(reinterpret_cast<void**>(&flag), sizeof(int), s));
	NNRT_HIP(hipMemsetAsync(flag, 0, sizeof(int), s));
	nnrt_status st = launch_solve_block_diagonal(d_blocks, d_b, count, block_size, d_x, flag, s);
	int host_flag = 0;
	if (!st) {
		NNRT_HIP(hipMemcpyAsync(&host_flag, flag, sizeof(int), hipMemcpyDeviceToHost, s));
		NNRT_HIP(hipStreamSynchronize(s));
	}
	hipFreeAsync(flag, s);
	if (st) return st;
	if (host_flag) {
		set_error("potrf failed in SolveBlockDiagonalCholesky (block not positive-definite)");
		return NNRT_ERROR_NOT_POSITIVE_DEFINITE;
	}
	return NNRT_OK;
}

nnrt_status nnrt_invert_positive_semidefinite_blocks(const float* d_blocks, int32_t count, int32_t block_size, float* d_out, void* stream) {
	hipStream_t s = static_cast<hipStream_t>(stream);
	NNRT_CHECK_ARG(count >= 0, "negative block count");
	int* flag = nullptr;
	NNRT_HIP(hipMallocAsync(reinterpret_cast<void**>(&flag), sizeof(int), s));
	NNRT_HIP(hipMemsetAsync(flag, 0, sizeof(int), s));
	nnrt_status st = launch_invert_psd_blocks(d_blocks, count, block_size, d_out, flag, s);
	int host_flag = 0;
	if (!st) {
		NNRT_HIP(hipMemcpyAsync(&host_flag, flag, sizeof(int), hipMemcpyDeviceToHost, s));
		NNRT_HIP(hipStreamSynchronize(s));
	}
	hipFreeAsync(flag, s);
	if (st) return st;
	if (host_flag) {
		set_error("potrf failed in InvertPositiveSemidefiniteBlocks (block not positive-definite)");
		return NNRT_ERROR_NOT_POSITIVE_DEFINITE;
	}
	return NNRT_OK;
}

extern "C++" {
// runs launch(flag) on the stream with a zeroed device flag; a raised flag becomes `code` with `message`
template <typename F>
nnrt_status with_device_flag(hipStream_t s, nnrt_status code, const char* message, F&& launch) {
	int* flag = nullptr;
	NNRT_HIP(hipMallocAsync(reinterpret_cast<void**>(&flag), sizeof(int), s));
	NNRT_HIP(hipMemsetAsync(flag, 0, sizeof(int), s));
	nnrt_status st = launch(flag);
	int host_flag = 0;
	if (!st) {
		NNRT_HIP(hipMemcpyAsync(&host_flag, flag, sizeof(int), hipMemcpyDeviceToHost, s));
		NNRT_HIP(hipStreamSynchronize(s));
	}
	hipFreeAsync(flag, s);
	if (st) return st;
	if (host_flag) {
		set_error(message);
		return code;
	}
	return NNRT_OK;
}
} // extern "C++"

nnrt_status nnrt_matmul_block_sparse_row_wise(const float* d_a_blocks, int32_t a_block_count, const float* d_b_blocks,
                                              const int32_t* d_b_coordinates, int32_t b_block_count, int32_t block_size, float* d_c_blocks,
                                              uint8_t* d_c_mask, void* stream) {
	NNRT_CHECK_ARG(a_block_count >= 0 && b_block_count >= 0 && block_size > 0, "bad block count or block size");
	NNRT_CHECK_ARG(b_block_count == 0 || (d_b_blocks && d_b_coordinates && d_c_blocks && d_c_mask), "null pointer");
	NNRT_CHECK_ARG(a_block_count == 0 || d_a_blocks, "null pointer");
	hipStream_t s = static_cast<hipStream_t>(stream);
	return with_device_flag(s, NNRT_ERROR_ARGUMENT, "negative block row coordinate in MatmulBlockSparseRowWise", [&](int* flag) {
		return launch_matmul_block_sparse_row_wise(d_a_blocks, a_block_count, d_b_blocks, d_b_coordinates, b_block_count, block_size, d_c_blocks,
		                                           d_c_mask, flag, s);
	});
}

nnrt_status nnrt_matmul_block_sparse(const float* d_a_blocks, int32_t a_block_count, const int16_t* d_a_breadboard, int32_t a_block_rows,
                                     int32_t a_block_columns, int32_t transpose_a, const float* d_b_blocks, int32_t b_block_count,
                                     const int16_t* d_b_breadboard, int32_t b_block_rows, int32_t b_block_columns, int32_t transpose_b,
                                     int32_t block_size, float* d_c_blocks, uint8_t* d_c_mask, void* stream) {
	NNRT_CHECK_ARG(a_block_count >= 0 && b_block_count >= 0 && block_size > 0, "bad block count or block size");
	NNRT_CHECK_ARG(a_block_rows >= 0 && a_block_columns >= 0 && b_block_rows >= 0 && b_block_columns >= 0, "negative breadboard size");
	const int32_t a_inner = transpose_a ? a_block_rows : a_block_columns, b_inner = transpose_b ? b_block_columns : b_block_rows;
	NNRT_CHECK_ARG(a_inner == b_inner, "Matrix inner dimensions must but do not match.");
	const int64_t out_blocks = static_cast<int64_t>(transpose_a ? a_block_columns : a_block_rows) * (transpose_b ? b_block_rows : b_block_columns);
	NNRT_CHECK_ARG(out_blocks == 0 || (d_c_blocks && d_c_mask && d_a_breadboard && d_b_breadboard), "null pointer");
	NNRT_CHECK_ARG((a_block_count == 0 || d_a_blocks) && (b_block_count == 0 || d_b_blocks), "null pointer");
	hipStream_t s = static_cast<hipStream_t>(stream);
	return with_device_flag(s, NNRT_ERROR_ARGUMENT, "breadboard block index out of range in MatmulBlockSparse", [&](int* flag) {
		return launch_matmul_block_sparse(d_a_blocks, a_block_count, d_a_breadboard, a_block_rows, a_block_columns, transpose_a != 0, d_b_blocks,
		                                  b_block_count, d_b_breadboard, b_block_rows, b_block_columns, transpose_b != 0, block_size, d_c_blocks,
		                                  d_c_mask, flag, s);
	});
}

nnrt_status nnrt_block_sparse_and_vector_product(const float* d_blocks, const int32_t* d_coordinates, int32_t block_count, int32_t block_size,
                                                 int32_t block_row_offset, int32_t block_column_offset, int32_t transpose,
                                                 const float* d_vector, int64_t vector_length, int64_t m, float* d_out, void* stream) {
	NNRT_CHECK_ARG(block_count >= 0 && block_size > 0 && vector_length >= 0 && m >= 0, "bad size");
	NNRT_CHECK_ARG(m % block_size == 0, "output length m must be a multiple of the block size");
	NNRT_CHECK_ARG((m == 0 || d_out) && (block_count == 0 || (d_blocks && d_coordinates && d_vector)), "null pointer");
	NNRT_CHECK_ARG(m == 0 || block_count == 0 || !ranges_overlap(d_out, sizeof(float) * m, d_vector, sizeof(float) * vector_length),
	               "d_out must not overlap d_vector (it is zeroed first)");
	hipStream_t s = static_cast<hipStream_t>(stream);
	return with_device_flag(s, NNRT_ERROR_ARGUMENT, "block coordinate outside the matrix in BlockSparseAndVectorProduct", [&](int* flag) {
		return launch_block_sparse_vector(d_blocks, d_coordinates, block_count, block_size, block_row_offset, block_column_offset, transpose != 0,
		                                  d_vector, vector_length, d_out, m, flag, s);
	});
}

nnrt_status nnrt_diagonal_block_sparse_and_vector_product(const float* d_blocks, int32_t block_count, int32_t block_size, const float* d_vector,
                                                          float* d_out, void* stream) {
	NNRT_CHECK_ARG(block_count >= 0 && block_size > 0, "bad block count or block size");
	NNRT_CHECK_ARG(block_count == 0 || (d_blocks && d_vector && d_out), "null pointer");
	return launch_diagonal_block_vector(d_blocks, block_count, block_size, d_vector, d_out, static_cast<hipStream_t>(stream));
}

nnrt_status nnrt_sparse_blocks_op(float* d_matrix, int64_t rows, int64_t columns, const float* d_blocks, const int32_t* d_coordinates,
                                  int32_t block_count, int32_t block_size, int64_t block_row_offset, int64_t block_column_offset,
                                  int32_t transpose, int32_t op, void* stream) {
	NNRT_CHECK_ARG(rows >= 0 && columns >= 0 && block_count >= 0 && block_size > 0, "bad size");
	NNRT_CHECK_ARG(op >= 0 && op <= 2, "op must be 0 (fill), 1 (add) or 2 (subtract)");
	NNRT_CHECK_ARG(block_count == 0 || (d_matrix && d_blocks), "null pointer");
	hipStream_t s = static_cast<hipStream_t>(stream);
	return with_device_flag(s, NNRT_ERROR_ARGUMENT, "block placed outside the matrix", [&](int* flag) {
		return launch_sparse_blocks_op(d_matrix, rows, columns, d_blocks, d_coordinates, block_count, block_size, block_row_offset,
		                               block_column_offset, transpose != 0, op, flag, s);
	});
}

nnrt_status nnrt_get_sparse_blocks(const float* d_matrix, int64_t rows, int64_t columns, int32_t block_size, const int32_t* d_coordinates,
                                   int32_t block_count, float* d_blocks, void* stream) {
	NNRT_CHECK_ARG(rows >= 0 && columns >= 0 && block_count >= 0 && block_size > 0, "bad size");
	NNRT_CHECK_ARG(block_count == 0 || (d_matrix && d_blocks), "null pointer");
	hipStream_t s = static_cast<hipStream_t>(stream);
	return with_device_flag(s, NNRT_ERROR_ARGUMENT, "block coordinate outside the matrix", [&](int* flag) {
		return launch_get_sparse_blocks(d_matrix, rows, columns, block_size, d_coordinates, block_count, d_blocks, flag, s);
	});
}

nnrt_status nnrt_transpose_blocks_in_place(float* d_blocks, int32_t block_count, int32_t block_size, void* stream) {
	NNRT_CHECK_ARG(block_count >= 0 && block_size > 0, "bad block count or block size");
	NNRT_CHECK_ARG(block_count == 0 || d_blocks, "null pointer");
	return launch_transpose_blocks(d_blocks, block_count, block_size, static_cast<hipStream_t>(stream));
}

nnrt_status nnrt_invert_triangular_blocks(const float* d_blocks, int32_t block_count, int32_t block_size, int32_t upper, float* d_out,
                                          void* stream) {
	NNRT_CHECK_ARG(block_count >= 0 && block_size > 0, "bad block count or block size");
	NNRT_CHECK_ARG(block_count == 0 || (d_blocks && d_out), "null pointer");
	const size_t bytes = sizeof(float) * static_cast<size_t>(block_count) * block_size * block_size;
	NNRT_CHECK_ARG(block_count == 0 || !ranges_overlap(d_out, bytes, d_blocks, bytes),
	               "d_out must not overlap d_blocks (each block's inverse is built column by column while its entries are read)");
	hipStream_t s = static_cast<hipStream_t>(stream);
	return with_device_flag(s, NNRT_ERROR_NOT_POSITIVE_DEFINITE, "trtri failed in InvertTriangularBlocks (zero on a block diagonal)",
	                        [&](int* flag) { return launch_invert_triangular_blocks(d_blocks, block_count, block_size, upper != 0, d_out, flag, s); });
}

} // extern "C"

namespace {
// Everything the arrowhead solve derives from the wing structure alone -- the stem CSR, the target-grouped Schur lists,
// the tile-sparse corner plan and its buffers, the per-call scratch -- kept per (device, N, n0, coordinates) so a
// repeated structure (a fixed hierarchy, solved every iteration) skips the host planning and the allocations. An entry
// is owned by one call at a time (taken out of the pool, returned after the call has synchronised its stream), so
// concurrent calls never share device scratch; the pool holds the ARROW_POOL_MAX most recently used structures.
struct ArrowheadPlan {
	int device = -1, N = 0, n0 = 0, E = 0, targets = 0;
	std::vector<int32_t> coords;
	CornerSolver corner;
	DeviceBuffer<float> dinv, dinv_b;
	DeviceBuffer<int> edge_offsets, edge_list, flag, tgt_off, rhs_off, rhs_edges;
	DeviceBuffer<int2> tgt_ab, pairs;
	~ArrowheadPlan() {
		for (auto* b : {&dinv, &dinv_b}) b->release();
		for (auto* b : {&edge_offsets, &edge_list, &flag, &tgt_off, &rhs_off, &rhs_edges}) b->release();
		for (auto* b : {&tgt_ab, &pairs}) b->release();
	}
	bool matches(int dev, int32_t n, int32_t base, const std::vector<int32_t>& c) const {
		return device == dev && N == n && n0 == base && coords == c;
	}
	nnrt_status build(int dev, int32_t n, int32_t base, std::vector<int32_t> c) {
		device = dev;
		N = n;
		n0 = base;
		coords = std::move(c);
		E = static_cast<int>(coords.size() / 2);
		std::vector<int> counts(n0 + 1, 0), list(std::max(E, 1)), fill;
		for (int e = 0; e < E; e++)
			if (coords[2 * e] < n0) counts[coords[2 * e] + 1]++;
		for (int i = 0; i < n0; i++) counts[i + 1] += counts[i];
		fill.assign(counts.begin(), counts.end() - 1);
		for (int e = 0; e < E; e++)
			if (coords[2 * e] < n0) list[fill[coords[2 * e]]++] = e;
		nnrt_status st = corner.prepare(coords.data(), E, n0, N);
		if (st) return st;
		const StemSchurLists sl = build_stem_schur_lists(coords.data(), E, n0, N);
		targets = static_cast<int>(sl.tgt_ab.size());
		if ((st = dinv.ensure(36 * static_cast<size_t>(std::max(n0, 1)))) || (st = dinv_b.ensure(36 * static_cast<size_t>(std::max(E, 1)))) ||
		    (st = flag.ensure(1)) || (st = upload(edge_offsets, counts)) || (st = upload(edge_list, list)) || (st = upload(tgt_off, sl.tgt_off)) ||
		    (st = upload(tgt_ab, sl.tgt_ab)) || (st = upload(pairs, sl.pairs)) || (st = upload(rhs_off, sl.rhs_off)) ||
		    (st = upload(rhs_edges, sl.rhs_edges)))
			return st;
		return NNRT_OK;
	}
};
constexpr size_t ARROW_POOL_MAX = 4;
std::mutex g_arrow_mu;
// heap-allocated and never destroyed: device memory must not be released by static destructors after the HIP runtime
// has shut down at process exit
std::list<std::unique_ptr<ArrowheadPlan>>& arrow_pool() {
	static auto* pool = new std::list<std::unique_ptr<ArrowheadPlan>>();
	return *pool;
}

} // namespace

extern "C" {

nnrt_status nnrt_solve_block_sparse_arrowhead_cholesky(const float* d_diag, const float* d_wing, const int32_t* d_coords, int32_t E, int32_t N,
                                                       int32_t n0, const float* d_b, float* d_x, void* stream) {
	NNRT_CHECK_ARG(n0 >= 0 && n0 <= N, "arrow_base_block_index out of range");
	NNRT_CHECK_ARG((reinterpret_cast<uintptr_t>(d_diag) & 15) == 0 && (reinterpret_cast<uintptr_t>(d_wing) & 15) == 0,
	               "diagonal and wing blocks must be 16-byte aligned (the stem reads 6x6 blocks as float4)");
	NNRT_CHECK_ARG((reinterpret_cast<uintptr_t>(d_x) & 7) == 0, "x must be 8-byte aligned");
	hipStream_t s = static_cast<hipStream_t>(stream);
	std::vector<int32_t> coords(2 * static_cast<size_t>(E));
	if (E > 0) {
		NNRT_HIP(hipMemcpyAsync(coords.data(), d_coords, sizeof(int32_t) * 2 * E, hipMemcpyDeviceToHost, s));
		NNRT_HIP(hipStreamSynchronize(s));
	}
	for (int e = 0; e < E; e++) {   // before any allocation: the host lists index by these
		const int i = coords[2 * e], j = coords[2 * e + 1];
		NNRT_CHECK_ARG(i >= 0 && i < N && j >= 0 && j < N, "wing block coordinate outside [0, diagonal_block_count)");
		NNRT_CHECK_ARG(i != j, "wing block on the block diagonal");
		NNRT_CHECK_ARG(j >= n0, "wing block column inside the arrow stem (the stem is block-diagonal)");
	}
	int device = 0;
	NNRT_HIP(hipGetDevice(&device));
	std::unique_ptr<ArrowheadPlan> plan;
	{
		std::lock_guard<std::mutex> lock(g_arrow_mu);
		auto& pool = arrow_pool();
		for (auto it = pool.begin(); it != pool.end(); ++it)
			if ((*it)->matches(device, N, n0, coords)) {
				plan = std::move(*it);
				pool.erase(it);
				break;
			}
	}
	nnrt_status st = NNRT_OK;
	if (!plan) {
		plan = std::make_unique<ArrowheadPlan>();
		if ((st = plan->build(device, N, n0, std::move(coords)))) return st;
	}
	ArrowheadWorkspace ws;
	ws.N = N;
	ws.n0 = n0;
	ws.E = E;
	ws.m = 6 * (N - n0);
	ws.corner = &plan->corner;
	ws.dinv = plan->dinv.ptr;
	ws.dinv_b = plan->dinv_b.ptr;
	ws.edge_offsets = plan->edge_offsets.ptr;
	ws.edge_list = plan->edge_list.ptr;
	ws.targets = plan->targets;
	ws.tgt_off = plan->tgt_off.ptr;
	ws.tgt_ab = plan->tgt_ab.ptr;
	ws.pairs = plan->pairs.ptr;
	ws.rhs_off = plan->rhs_off.ptr;
	ws.rhs_edges = plan->rhs_edges.ptr;
	ws.diag = const_cast<float*>(d_diag);
	ws.rhs = const_cast<float*>(d_b);
	ws.x = d_x;
	int host_flag = 0;
	if (hipMemsetAsync(plan->flag.ptr, 0, sizeof(int), s) != hipSuccess) {
		set_error("hipMemsetAsync failed");
		return NNRT_ERROR_HIP;
	}
	st = arrowhead_solve_core(ws, d_coords, d_wing, plan->flag.ptr, s);
	if (!st) {
		if (hipMemcpyAsync(&host_flag, plan->flag.ptr, sizeof(int), hipMemcpyDeviceToHost, s) != hipSuccess ||
		    hipStreamSynchronize(s) != hipSuccess) {
			set_error("arrowhead solve: stream synchronisation failed");
			return NNRT_ERROR_HIP;   // the plan is dropped (its device work state is unknown)
		}
		// the stream is drained: the plan's scratch is free for the next call with this structure; evicted plans are
		// destroyed after the lock is released (hipFree synchronises the device and must not block other threads' lookups)
		std::list<std::unique_ptr<ArrowheadPlan>> evicted;
		{
			std::lock_guard<std::mutex> lock(g_arrow_mu);
			auto& pool = arrow_pool();
			pool.push_front(std::move(plan));
			while (pool.size() > ARROW_POOL_MAX) {
				evicted.push_back(std::move(pool.back()));
				pool.pop_back();
			}
		}
	}
	if (st) return st;
	if (host_flag & 8) {
		set_error("arrowhead solve: the corner's dataflow substitution launch gave up waiting on a dependency (k_corner_flow spin bound)");
		return NNRT_ERROR_HIP;
	}
	if (host_flag) {
		set_error("arrowhead solve: a stem block or the Schur complement is not positive-definite");
		return NNRT_ERROR_NOT_POSITIVE_DEFINITE;
	}
	return NNRT_OK;
}

void nnrt_release_arrowhead_plans(void) {
	std::list<std::unique_ptr<ArrowheadPlan>> released;   // freed after the lock is dropped (hipFree synchronises)
	{
		std::lock_guard<std::mutex> lock(g_arrow_mu);
		released.swap(arrow_pool());
	}
}

// ---- DLPack entry points (include/nnrt_dlpack.h): validate, then forward to the pointer entry points ----------------
namespace {
enum class Mem { device, host };
// dtypes: list of (code, bits); dims: -1 = any extent (returned through `dims_out`)
nnrt_status dl_check(const DLManagedTensor* mt, const char* name, std::initializer_list<std::pair<int, int>> dtypes, int ndim,
                     std::initializer_list<int64_t> dims, Mem mem, int device, const void** data, int64_t* dims_out) {
	if (!mt) {
		set_error(std::string("invalid argument: ") + name + ": null tensor");
		return NNRT_ERROR_ARGUMENT;
	}
	const DLTensor& t = mt->dl_tensor;
	bool dtype_ok = false;
	for (const auto& d : dtypes) dtype_ok |= t.dtype.code == d.first && t.dtype.bits == d.second && t.dtype.lanes == 1;
	if (!dtype_ok) {
		set_error(std::string("invalid argument: ") + name + ": unsupported dtype (code " + std::to_string(t.dtype.code) + ", bits " +
		          std::to_string(t.dtype.bits) + ")");
		return NNRT_ERROR_ARGUMENT;
	}
	if (t.ndim != ndim) {
		set_error(std::string("invalid argument: ") + name + ": expected " + std::to_string(ndim) + " dimensions, got " + std::to_string(t.ndim));
		return NNRT_ERROR_ARGUMENT;
	}
	int k = 0;
	for (int64_t want : dims) {
		if (want >= 0 && t.shape[k] != want) {
			set_error(std::string("invalid argument: ") + name + ": dimension " + std::to_string(k) + " is " + std::to_string(t.shape[k]) +
			          ", expected " + std::to_string(want));
			return NNRT_ERROR_ARGUMENT;
		}
		dims_out[k] = t.shape[k];
		k++;
	}
	if (t.strides) {   // compact row-major only
		int64_t expect = 1;
		for (int d = ndim - 1; d >= 0; d--) {
			if (t.shape[d] > 1 && t.strides[d] != expect) {
				set_error(std::string("invalid argument: ") + name + ": not a compact row-major tensor");
				return NNRT_ERROR_ARGUMENT;
			}
			expect *= t.shape[d];
		}
	}
	const bool on_device = t.device.device_type == kDLROCM;
	const bool on_host = t.device.device_type == kDLCPU || t.device.device_type == kDLROCMHost;
	if (mem == Mem::device && !(on_device && t.device.device_id == device)) {
		set_error(std::string("invalid argument: ") + name + ": must be a ROCm device tensor on device " + std::to_string(device));
		return NNRT_ERROR_ARGUMENT;
	}
	if (mem == Mem::host && !on_host) {
		set_error(std::string("invalid argument: ") + name + ": must be a host (CPU) tensor");
		return NNRT_ERROR_ARGUMENT;
	}
	*data = static_cast<const char*>(t.data) + t.byte_offset;
	return NNRT_OK;
}
constexpr std::pair<int, int> F32{kDLFloat, 32}, F64{kDLFloat, 64}, I64{kDLInt, 64}, U8{kDLUInt, 8}, B8{kDLBool, 8};
} // namespace

nnrt_status nnrt_warp_field_create_dlpack(const DLManagedTensor* nodes, float node_coverage, int32_t threshold_nodes_by_distance,
                                          int32_t anchor_count, int32_t minimum_valid_anchor_count, int32_t coverage_method,
                                          int32_t layer_count, int32_t max_vertex_degree, const float* h_layer_radii, int32_t device,
                                          nnrt_warp_field** out) {
	NNRT_CHECK_ARG(nodes != nullptr, "nodes: null tensor");
	const bool on_device = nodes->dl_tensor.device.device_type == kDLROCM;
	const void* data = nullptr;
	int64_t dims[2];
	nnrt_status st = dl_check(nodes, "nodes", {F32}, 2, {-1, 3}, on_device ? Mem::device : Mem::host,
	                          on_device ? nodes->dl_tensor.device.device_id : device, &data, dims);
	if (st) return st;
	NNRT_CHECK_ARG(dims[0] <= INT32_MAX, "nodes: too many nodes");
	std::vector<float> host;
	const float* h_nodes = static_cast<const float*>(data);
	if (on_device) {
		DeviceGuard guard(nodes->dl_tensor.device.device_id);
		host.resize(3 * static_cast<size_t>(dims[0]));
		NNRT_HIP(hipMemcpy(host.data(), data, sizeof(float) * host.size(), hipMemcpyDeviceToHost));
		h_nodes = host.data();
	}
	return nnrt_warp_field_create(h_nodes, static_cast<int32_t>(dims[0]), node_coverage, threshold_nodes_by_distance, anchor_count,
	                              minimum_valid_anchor_count, coverage_method, layer_count, max_vertex_degree, h_layer_radii, device, out);
}

nnrt_status nnrt_fitter_fit_to_image_dlpack(nnrt_fitter* ft, nnrt_warp_field* wf, const DLManagedTensor* vertices, const DLManagedTensor* normals,
                                            const DLManagedTensor* faces, const DLManagedTensor* depth, const DLManagedTensor* mask,
                                            const DLManagedTensor* K, const DLManagedTensor* E, float depth_scale, void* stream) {
	NNRT_CHECK_ARG(ft && wf, "null handle");
	NNRT_CHECK_ARG(wf->device == ft->device, "the warp field and the fitter live on different devices");
	const int dev = ft->device;
	const void *pv, *pn, *pf, *pd, *pm = nullptr, *pk, *pe;
	int64_t dv[2], dn[2], df[2], dd[2], dm[2], dk[2], de[2];
	nnrt_status st;
	if ((st = dl_check(vertices, "vertices", {F32}, 2, {-1, 3}, Mem::device, dev, &pv, dv))) return st;
	if ((st = dl_check(normals, "normals", {F32}, 2, {dv[0], 3}, Mem::device, dev, &pn, dn))) return st;
	if ((st = dl_check(faces, "faces", {I64}, 2, {-1, 3}, Mem::device, dev, &pf, df))) return st;
	if ((st = dl_check(depth, "depth", {F32}, 2, {-1, -1}, Mem::device, dev, &pd, dd))) return st;
	if (mask && (st = dl_check(mask, "mask", {B8, U8}, 2, {dd[0], dd[1]}, Mem::device, dev, &pm, dm))) return st;
	if ((st = dl_check(K, "K", {F64}, 2, {3, 3}, Mem::host, dev, &pk, dk))) return st;
	if ((st = dl_check(E, "E", {F64}, 2, {4, 4}, Mem::host, dev, &pe, de))) return st;
	NNRT_CHECK_ARG(dd[0] <= INT32_MAX && dd[1] <= INT32_MAX, "depth: image too large");
	return nnrt_fitter_fit_to_image(ft, wf, static_cast<const float*>(pv), static_cast<const float*>(pn), dv[0], static_cast<const int64_t*>(pf),
	                                df[0], static_cast<const float*>(pd), static_cast<const uint8_t*>(pm), static_cast<int32_t>(dd[0]),
	                                static_cast<int32_t>(dd[1]), static_cast<const double*>(pk), static_cast<const double*>(pe), depth_scale, stream);
}

nnrt_status nnrt_rasterize_ndc_triangles_dlpack(const DLManagedTensor* face_ndc, const DLManagedTensor* clip_mask, float blur_radius_pixels,
                                                int32_t perspective_correct_barycentric_coordinates, int32_t clip_barycentric_coordinates,
                                                int32_t cull_back_faces, const DLManagedTensor* pixel_faces, const DLManagedTensor* depths,
                                                const DLManagedTensor* barycentrics, const DLManagedTensor* distances, void* stream) {
	NNRT_CHECK_ARG(face_ndc != nullptr, "face_ndc: null tensor");
	const int dev = face_ndc->dl_tensor.device.device_id;
	const void *pn, *pm = nullptr, *pf, *pd, *pb, *ps;
	int64_t dn[3], dm[1], df[3], dd[3], db[4], ds[3];
	nnrt_status st;
	if ((st = dl_check(face_ndc, "face_ndc", {F32}, 3, {-1, 3, 3}, Mem::device, dev, &pn, dn))) return st;
	if (clip_mask && (st = dl_check(clip_mask, "clip_mask", {B8, U8}, 1, {dn[0]}, Mem::device, dev, &pm, dm))) return st;
	if ((st = dl_check(pixel_faces, "pixel_faces", {I64}, 3, {-1, -1, -1}, Mem::device, dev, &pf, df))) return st;
	if ((st = dl_check(depths, "depths", {F32}, 3, {df[0], df[1], df[2]}, Mem::device, dev, &pd, dd))) return st;
	if ((st = dl_check(barycentrics, "barycentrics", {F32}, 4, {df[0], df[1], df[2], 3}, Mem::device, dev, &pb, db))) return st;
	if ((st = dl_check(distances, "distances", {F32}, 3, {df[0], df[1], df[2]}, Mem::device, dev, &ps, ds))) return st;
	NNRT_CHECK_ARG(df[0] <= INT32_MAX && df[1] <= INT32_MAX && df[2] <= INT32_MAX, "pixel_faces: image too large");
	DeviceGuard guard(dev);
	return nnrt_rasterize_ndc_triangles(static_cast<const float*>(pn), static_cast<const uint8_t*>(pm), dn[0], static_cast<int32_t>(df[0]),
	                                    static_cast<int32_t>(df[1]), blur_radius_pixels, static_cast<int32_t>(df[2]), -1, -1,
	                                    perspective_correct_barycentric_coordinates, clip_barycentric_coordinates, cull_back_faces,
	                                    static_cast<int64_t*>(const_cast<void*>(pf)), static_cast<float*>(const_cast<void*>(pd)),
	                                    static_cast<float*>(const_cast<void*>(pb)), static_cast<float*>(const_cast<void*>(ps)), stream);
}

} // extern "C"
