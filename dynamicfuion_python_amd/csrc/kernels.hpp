// Kernel launchers shared between the HIP translation units.
#pragma once

#include "common.hpp"

namespace nnrt {

struct WarpExtrinsics {
	float m[12];     // rows 0..2 of the 4x4 extrinsic matrix (float, as Open3D TransformIndexer)
	int identity;
};
WarpExtrinsics make_extrinsics(const double* E);

// One (vertex, anchor) term of the blended warp (WarpUtilities.h:448-467) and its Jacobian rows
// (WarpedSurfaceJacobiansImpl.h:33-158): cp = w (g + R (pc - g) + t), cn = w R nc, jv = (-w R (p - g), w), jn = (-w R n, 0).
// p / n: the vertex as stored; pc / nc: after the extrinsics. IDENTITY: R = I, t = 0 without reading them. Shared by
// the warp kernels.
template <bool IDENTITY>
__device__ inline void warp_slot_state(const float4 (&ns)[4], float w, f3 p, f3 n, f3 pc, f3 nc, int extr_identity, f3& cp, f3& cn, float4& ojv,
                                       float4& ojn) {
	f3 g, t;
	float R[9];
	if constexpr (IDENTITY) {
		const float4 s0 = ns[0];
		g = make3(s0.x, s0.y, s0.z);
		t = make3(0.f, 0.f, 0.f);
#pragma unroll
		for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0) ? 1.f : 0.f;
	} else {
		const float4 s0 = ns[0], s1 = ns[1], s2 = ns[2], s3 = ns[3];   // g, t, R (row-major), pad
		g = make3(s0.x, s0.y, s0.z);
		t = make3(s0.w, s1.x, s1.y);
		const float Rl[9] = {s1.z, s1.w, s2.x, s2.y, s2.z, s2.w, s3.x, s3.y, s3.z};
#pragma unroll
		for (int i = 0; i < 9; i++) R[i] = Rl[i];
	}
	const f3 Rd = matvec3(R, sub3(pc, g));
	cp = make3(w * ((g.x + Rd.x) + t.x), w * ((g.y + Rd.y) + t.y), w * ((g.z + Rd.z) + t.z));
	const f3 Rn = matvec3(R, nc);
	cn = make3(w * Rn.x, w * Rn.y, w * Rn.z);
	const f3 Rj = extr_identity ? Rd : matvec3(R, sub3(p, g));
	const f3 Rnj = extr_identity ? Rn : matvec3(R, n);
	ojv = make_float4(-w * Rj.x, -w * Rj.y, -w * Rj.z, w);
	ojn = make_float4(-w * Rnj.x, -w * Rnj.y, -w * Rnj.z, 0.f);
}
// the node's state rows (g, t, R: one 64-B line; IDENTITY: g only), loaded ahead of warp_slot_state by callers that keep
// several slots' gathers in flight
template <bool IDENTITY>
__device__ inline void load_warp_state(const float* __restrict__ node_state, int32_t a, float4 (&ns)[4]) {
	const float4* q = reinterpret_cast<const float4*>(node_state + static_cast<int64_t>(a) * NODE_STRIDE);
	ns[0] = q[0];
	if constexpr (!IDENTITY) {
		ns[1] = q[1];
		ns[2] = q[2];
		ns[3] = q[3];
	} else {
		ns[1] = ns[2] = ns[3] = make_float4(0.f, 0.f, 0.f, 0.f);
	}
}
template <bool IDENTITY>
__device__ inline void warp_slot(const float* __restrict__ node_state, int32_t a, float w, f3 p, f3 n, f3 pc, f3 nc, int extr_identity, f3& cp,
                                 f3& cn, float4& ojv, float4& ojn) {
	float4 ns[4];
	load_warp_state<IDENTITY>(node_state, a, ns);
	warp_slot_state<IDENTITY>(ns, w, p, n, pc, nc, extr_identity, cp, cn, ojv, ojn);
}

// one (vertex, anchor) slot's warped-Jacobian row as 24 B: (jv.x, jv.y) (jv.z, jn.x) (jn.y, jn.z); the weight w is not
// repeated here (the fitter reads it from the anchor weights)
__device__ inline void store_jacobian_row(float2* __restrict__ jrows, int64_t slot, float4 ojv, float4 ojn) {
	float2* o = jrows + 3 * slot;
	o[0] = make_float2(ojv.x, ojv.y);
	o[1] = make_float2(ojv.z, ojn.x);
	o[2] = make_float2(ojn.y, ojn.z);
}

__device__ inline f3 apply_extrinsics_point(const WarpExtrinsics& E, f3 p) {
	return make3(((p.x * E.m[0] + p.y * E.m[1]) + p.z * E.m[2]) + E.m[3], ((p.x * E.m[4] + p.y * E.m[5]) + p.z * E.m[6]) + E.m[7],
	             ((p.x * E.m[8] + p.y * E.m[9]) + p.z * E.m[10]) + E.m[11]);
}
__device__ inline f3 apply_extrinsics_normal(const WarpExtrinsics& E, f3 n) {
	return make3((n.x * E.m[0] + n.y * E.m[1]) + n.z * E.m[2], (n.x * E.m[4] + n.y * E.m[5]) + n.z * E.m[6], (n.x * E.m[8] + n.y * E.m[9]) + n.z * E.m[10]);
}

nnrt_status launch_compute_anchors(const float* points, int64_t V, const float* nodes, int N, int K, float coverage,
                                   const float* node_weights, int minimum_valid, int32_t* anchors, float* weights, hipStream_t stream,
                                   int threshold = -1);   // -1: threshold iff minimum_valid > 0 (the anchor API); 0 / 1: forced
nnrt_status launch_warp_mesh(const float* points, const float* normals, int64_t V, const float* node_state, const int32_t* anchors,
                             const float* weights, int K, const WarpExtrinsics& E, float4* out_p, float4* out_n, float2* jrows,
                             hipStream_t stream, bool from_identity = false, const uint2* anchors16 = nullptr);
// K = 4 anchors with every index below 65535 as 4 x 16 bits per vertex (the lane-per-vertex warp's anchors16)
nnrt_status launch_pack_anchors16(const int32_t* anchors, int64_t V, uint2* out, hipStream_t stream);
nnrt_status launch_pack_nodes(const float* nodes, const float* R, const float* t, int N, float* state, hipStream_t stream);
nnrt_status launch_unpack_float4x3(const float4* in, int64_t count, float* out, hipStream_t stream);
nnrt_status launch_extract_face_ndc(const float* verts, const int64_t* faces, int64_t F, const NdcSetup& s, float near_clip, float far_clip,
                                    float* out, uint8_t* mask, hipStream_t stream);
struct BackprojectCamera {
	float fx, fy, cx, cy, normalizer;
};
nnrt_status launch_backproject_depth_u16(const uint16_t* depth, int H, int W, const BackprojectCamera& c, float* out, hipStream_t stream);
nnrt_status launch_backproject_depth_f32(const float* depth, int H, int W, const BackprojectCamera& c, float* out, hipStream_t stream);
nnrt_status launch_unproject(const void* depth, int depth_dtype, int H, int W, const Camera& K, const WarpExtrinsics& pose, float scale,
                             float depth_max, float* pts, uint8_t* mask, hipStream_t stream);
nnrt_status launch_warp_points(const float* points, const float* normals, int64_t V, const float* node_state, const int32_t* anchors,
                               const float* weights, int K, int minimum_valid, const WarpExtrinsics& E, float* out_p, float* out_n,
                               hipStream_t stream);
nnrt_status launch_matmul3d(const float* A, const float* B, int64_t batch, int m, int k, int n, float* C, hipStream_t stream);
nnrt_status launch_median_grid_subsample(const float* pts, int n, float cell, int64_t* out, int64_t* h_count, hipStream_t s);
nnrt_status launch_point_to_plane(const float* n1, const float* v1, const float* v2, int64_t count, float* out, hipStream_t stream);
nnrt_status launch_interpolate(const int64_t* pixel_faces, const float* bary, int64_t P, int Kf, const float* attrs, int C, float* out,
                               hipStream_t stream);
nnrt_status launch_rodrigues(const float* w, int N, float* R, hipStream_t stream);

// rasterizer
struct RasterOptions {
	int H, W;
	float blur;          // NDC units (compared against squared distances: A13)
	int perspective;
	int clip_barycentric;
	int cull_back_faces;
	PixelAxis ax, ay;    // pixel-centre NDC constants of the x (W over H) and y (H over W) axes: set by make_raster_options
};
RasterOptions make_raster_options(int H, int W, float blur, int perspective, int clip_barycentric, int cull_back_faces);
nnrt_status launch_raster_scatter_ndc(const float* face_ndc, const uint8_t* mask, int64_t F, const RasterOptions& o, uint64_t* keys,
                                      hipStream_t stream);
nnrt_status launch_raster_resolve(const float* face_ndc, int64_t F, const RasterOptions& o, uint64_t* keys, int64_t* out_face,
                                  float* out_depth, float* out_bary, float* out_dist, hipStream_t stream);
nnrt_status launch_raster_scatter_mesh(const float4* wpos, const int4* faces4, int64_t F, const NdcSetup& s, float near_clip, float far_clip,
                                       const RasterOptions& o, uint64_t* keys, hipStream_t stream);
nnrt_status launch_raster_multi(const float* face_ndc, const uint8_t* mask, int64_t F, const RasterOptions& o, int faces_per_pixel,
                                int64_t* out_face, float* out_depth, float* out_bary, float* out_dist, hipStream_t stream);

// read-only device view of a warp field (capi.hip owns the handle; the TSDF kernels warp voxels with it)
struct WarpFieldView {
	int N, anchor_count, minimum_valid, fixed_coverage;
	float coverage;                 // node coverage (fixed-coverage weights use coverage^2)
	const float* state;             // [N,16] virtual order: g(3) t(3) R(9, row-major) pad
	const float* node_weights;      // [N] squared coverage per node (variable coverage)
	int device;
};
WarpFieldView warp_field_view(const void* warp_field_handle);

// float transcendentals evaluated in double and rounded once: bit-identical with the host restatement (oracle/) and
// within 1 ulp of the reference's expf/sinf/cosf
__host__ __device__ inline float exp_cr(float x) { return static_cast<float>(exp(static_cast<double>(x))); }
__host__ __device__ inline float sin_cr(float x) { return static_cast<float>(sin(static_cast<double>(x))); }
__host__ __device__ inline float cos_cr(float x) { return static_cast<float>(cos(static_cast<double>(x))); }

// shared device helper: RodriguesImpl.h:66-88 (|w| = 0 -> NaN, reference quirk A7)
__device__ inline void rodrigues_device(float w0, float w1, float w2, float* R) {
	const float ang = sqrtf((w0 * w0 + w1 * w1) + w2 * w2);
	const float ax = w0 / ang, ay = w1 / ang, az = w2 / ang;
	const float Km[3][3] = {{0.f, -az, ay}, {az, 0.f, -ax}, {-ay, ax, 0.f}};
#ifdef __HIP_DEVICE_COMPILE__
	// one shared argument reduction for both (the device library's sin and cos evaluate the same reduction and
	// polynomials: bit-identical to sin_cr / cos_cr)
	double sd, cd;
	sincos(static_cast<double>(ang), &sd, &cd);
	const float s = static_cast<float>(sd), c1 = 1 - static_cast<float>(cd);
#else
	const float s = sin_cr(ang), c1 = 1 - cos_cr(ang);
#endif
#pragma unroll
	for (int r = 0; r < 3; r++) {
#pragma unroll
		for (int c = 0; c < 3; c++) {
			const float K2 = (Km[r][0] * Km[0][c] + Km[r][1] * Km[1][c]) + Km[r][2] * Km[2][c];
			R[3 * r + c] = ((r == c ? 1.f : 0.f) + s * Km[r][c]) + c1 * K2;
		}
	}
}

// lower Cholesky of an n x n (n <= 6) row-major SPD matrix in registers (LAPACK potrf semantics); false if not PD
template <int n>
__host__ __device__ inline bool cholesky_small(float (&A)[n][n]) {
#pragma unroll
	for (int j = 0; j < n; j++) {
		float s = A[j][j];
#pragma unroll
		for (int k = 0; k < j; k++) s -= A[j][k] * A[j][k];
		if (!(s > 0.f)) return false;
		const float l = sqrtf(s);
		A[j][j] = l;
#pragma unroll
		for (int i = j + 1; i < n; i++) {
			float t = A[i][j];
#pragma unroll
			for (int k = 0; k < j; k++) t -= A[i][k] * A[j][k];
			A[i][j] = t / l;
		}
	}
	return true;
}
template <int n>
__host__ __device__ inline void cholesky_solve_small(const float (&L)[n][n], float (&b)[n]) {
#pragma unroll
	for (int i = 0; i < n; i++) {
		float s = b[i];
#pragma unroll
		for (int k = 0; k < i; k++) s -= L[i][k] * b[k];
		b[i] = s / L[i][i];
	}
#pragma unroll
	for (int i = n - 1; i >= 0; i--) {
		float s = b[i];
#pragma unroll
		for (int k = i + 1; k < n; k++) s -= L[k][i] * b[k];
		b[i] = s / L[i][i];
	}
}

// A^-1 from the lower Cholesky factor L of an SPD block: one potrs per identity column (InvertBlocks.cpp:82-126,
// potrf + potrs against the identity); the arrowhead stem's D^-1 and nnrt_invert_positive_semidefinite_blocks
template <int n>
__host__ __device__ inline void invert_from_cholesky_small(const float (&L)[n][n], float (&Ai)[n][n]) {
#pragma unroll
	for (int c = 0; c < n; c++) {
		float col[n];
#pragma unroll
		for (int r = 0; r < n; r++) col[r] = r == c ? 1.f : 0.f;
		cholesky_solve_small<n>(L, col);
#pragma unroll
		for (int r = 0; r < n; r++) Ai[r][c] = col[r];
	}
}

nnrt_status launch_solve_block_diagonal(const float* blocks, const float* b, int count, int s, float* x, int* error_flag, hipStream_t stream);
nnrt_status launch_invert_psd_blocks(const float* blocks, int count, int s, float* out, int* error_flag, hipStream_t stream);
// block_sparse.hip: the arrowhead's block-sparse stages as API entry points (nnrt.core.linalg)
nnrt_status launch_matmul_block_sparse_row_wise(const float* a, int a_count, const float* b, const int32_t* b_coords, int64_t count, int s,
                                                float* c, uint8_t* mask, int* error_flag, hipStream_t stream);
nnrt_status launch_matmul_block_sparse(const float* a, int a_count, const int16_t* a_board, int a_rows, int a_cols, bool ta, const float* b,
                                       int b_count, const int16_t* b_board, int b_rows, int b_cols, bool tb, int s, float* c, uint8_t* mask,
                                       int* error_flag, hipStream_t stream);
nnrt_status launch_block_sparse_vector(const float* blocks, const int32_t* coords, int64_t count, int s, int row_off, int col_off, bool ta,
                                       const float* v, int64_t n_v, float* out, int64_t m, int* error_flag, hipStream_t stream);
nnrt_status launch_diagonal_block_vector(const float* blocks, int64_t count, int s, const float* v, float* out, hipStream_t stream);
nnrt_status launch_sparse_blocks_op(float* matrix, int64_t rows, int64_t cols, const float* blocks, const int32_t* coords, int64_t count, int s,
                                    int64_t row_off, int64_t col_off, bool transpose, int op, int* error_flag, hipStream_t stream);
nnrt_status launch_get_sparse_blocks(const float* matrix, int64_t rows, int64_t cols, int s, const int32_t* coords, int64_t count, float* blocks,
                                     int* error_flag, hipStream_t stream);
nnrt_status launch_transpose_blocks(float* blocks, int64_t count, int s, hipStream_t stream);
nnrt_status launch_invert_triangular_blocks(const float* blocks, int64_t count, int s, bool upper, float* out, int* error_flag,
                                            hipStream_t stream);

} // namespace nnrt
