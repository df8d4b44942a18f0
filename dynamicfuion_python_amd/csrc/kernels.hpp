// Kernel launchers shared between the HIP translation units.
#pragma once

#include "common.hpp"

namespace nnrt {

struct WarpExtrinsics {
	float m[12];     // rows 0..2 of the 4x4 extrinsic matrix (float, as Open3D TransformIndexer)
	int identity;
};
WarpExtrinsics make_extrinsics(const double* E);

nnrt_status launch_compute_anchors(const float* points, int64_t V, const float* nodes, int N, int K, float coverage,
                                   const float* node_weights, int minimum_valid, int32_t* anchors, float* weights, hipStream_t stream);
nnrt_status launch_warp_mesh(const float* points, const float* normals, int64_t V, const float* node_state, const int32_t* anchors,
                             const float* weights, int K, const WarpExtrinsics& E, float4* out_p, float4* out_n, float4* jv, float4* jn,
                             hipStream_t stream, bool from_identity = false);
nnrt_status launch_pack_nodes(const float* nodes, const float* R, const float* t, int N, float* state, hipStream_t stream);
nnrt_status launch_unpack_float4x3(const float4* in, int64_t count, float* out, hipStream_t stream);
nnrt_status launch_extract_face_ndc(const float* verts, const int64_t* faces, int64_t F, const NdcSetup& s, float near_clip, float far_clip,
                                    float* out, uint8_t* mask, hipStream_t stream);
struct BackprojectCamera {
	float fx, fy, cx, cy, normalizer;
};
nnrt_status launch_backproject_depth_u16(const uint16_t* depth, int H, int W, const BackprojectCamera& c, float* out, hipStream_t stream);
nnrt_status launch_backproject_depth_f32(const float* depth, int H, int W, const BackprojectCamera& c, float* out, hipStream_t stream);
nnrt_status launch_unproject(const float* depth, int H, int W, const Camera& K, float scale, float depth_max, float* pts, uint8_t* mask,
                             hipStream_t stream);
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
};
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
	const float s = sin_cr(ang), c1 = 1 - cos_cr(ang);
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

nnrt_status launch_solve_block_diagonal(const float* blocks, const float* b, int count, int s, float* x, int* error_flag, hipStream_t stream);
nnrt_status solve_arrowhead(const float* diag, const float* wing, const int32_t* coords, int E, int N, int n0, const float* b, float* x,
                            int* error_flag, hipStream_t stream);

} // namespace nnrt
