// Shared device/host helpers for the MI355X (gfx950) DeformableMeshToImageFitter hot path.
// Built with -ffp-contract=off so float expression order matches the documented restatement (DESIGN.md "Numerics").
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "nnrt_mi355x.h"

namespace nnrt {

// -------- error plumbing (C-ABI: return codes + thread-local message) --------
void set_error(const std::string& message);
const std::string& get_error();

struct Status {
	nnrt_status code = NNRT_OK;
	explicit operator bool() const { return code != NNRT_OK; }
};

#define NNRT_HIP(expr)                                                                                                   \
	do {                                                                                                                 \
		hipError_t _e = (expr);                                                                                          \
		if (_e != hipSuccess) {                                                                                          \
			::nnrt::set_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + __FILE__ + ":" +            \
			                  std::to_string(__LINE__) + " (" #expr ")");                                              \
			return NNRT_ERROR_HIP;                                                                                       \
		}                                                                                                                \
	} while (0)

#define NNRT_CHECK_ARG(cond, msg)                                                                                        \
	do {                                                                                                                 \
		if (!(cond)) {                                                                                                   \
			::nnrt::set_error(std::string("invalid argument: ") + (msg));                                              \
			return NNRT_ERROR_ARGUMENT;                                                                                  \
		}                                                                                                                \
	} while (0)

#define NNRT_LAUNCH_CHECK() NNRT_HIP(hipGetLastError())

// Development timing builds only (-DNNRT_KERNEL_STAMPS, tools/dev/stamps_build.sh): per wave of a stamped launch, the
// constant-rate clock (100 MHz) at its start and end and its hardware id (XCC << 32 | HW_ID), into a per-file __device__
// array read back by that file's nnrt_dev_<name>_stamps export. The product build compiles the macros to nothing.
#ifdef NNRT_KERNEL_STAMPS
#define NNRT_WAVE_STAMP(arr, slot, value)                                                                                  \
	do {                                                                                                                   \
		const int wid_ = static_cast<int>(blockIdx.x) * static_cast<int>(blockDim.x >> 6) + static_cast<int>(threadIdx.x >> 6); \
		if ((threadIdx.x & 63) == 0 && wid_ < 16384) arr[wid_][slot] = (value);                                                \
	} while (0)
#define NNRT_STAMP_HWID()                                                                                                  \
	(static_cast<unsigned long long>(__builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11))) |                            \
	 (static_cast<unsigned long long>(__builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11))) << 32))
#else
#define NNRT_WAVE_STAMP(arr, slot, value) \
	do {                                  \
	} while (0)
#endif

constexpr float K_EPSILON = 1e-8f;        // cpp/rendering/kernel/RasterizationConstants.h:24
constexpr int MAX_ANCHORS = 8;            // cpp/geometry/functional/kernel/Defines.h MAX_ANCHOR_COUNT
constexpr int MAX_FACES_PER_PIXEL = 8;    // RasterizationConstants.h:20

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// -------- node state layout: one 64-byte record per node (virtual order) --------
// [0..2] position g, [3..5] translation t, [6..14] rotation R (row-major), [15] pad
constexpr int NODE_STRIDE = 16;

// -------- small vector math (float expression order mirrors the Eigen expressions of the reference) --------
struct f3 {
	float x, y, z;
};
__host__ __device__ inline f3 make3(float x, float y, float z) { return {x, y, z}; }
__host__ __device__ inline f3 sub3(f3 a, f3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
__host__ __device__ inline float dot3(f3 a, f3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__host__ __device__ inline f3 matvec3(const float* R, f3 v) {
	return {(R[0] * v.x + R[1] * v.y) + R[2] * v.z, (R[3] * v.x + R[4] * v.y) + R[5] * v.z, (R[6] * v.x + R[7] * v.y) + R[8] * v.z};
}
// row vector r times skew(a) == r x a
__host__ __device__ inline f3 row_times_skew(f3 r, f3 a) {
	return {r.y * a.z - r.z * a.y, r.z * a.x - r.x * a.z, r.x * a.y - r.y * a.x};
}
__host__ __device__ inline float fmin3f(float a, float b, float c) { return fminf(fminf(a, b), c); }
__host__ __device__ inline float fmax3f(float a, float b, float c) { return fmaxf(fmaxf(a, b), c); }

// cpp/rendering/kernel/CoordinateSystemConversions.h:45-73
__host__ __device__ inline float ndc_range(int d1, int d2) {
	float range = 2.0f;
	if (d1 > d2) range = (static_cast<float>(d1) * range) / static_cast<float>(d2);
	return range;
}
__host__ __device__ inline float pixel_to_ndc(int i, int d1, int d2) {
	float range = ndc_range(d1, d2);
	const float offset = (range / 2.0f);
	return -offset + (range * static_cast<float>(i) + offset) / static_cast<float>(d1);
}

// ---- correctly rounded division through a shared reciprocal (Markstein) ----
// y = RN(1/b) from the double quotient (double rounding is innocuous for a float reciprocal), q = RN(a*y),
// r = a - b*q exact by FMA, RN(q + r*y) = RN(a/b) for normal-range operands (Markstein's theorem); other operands fall
// back to the division. Bit-identical to a/b with -fhip-fp32-correctly-rounded-divide-sqrt, at 3 instructions per
// quotient once the reciprocal of a shared denominator is known.
// RN(1/b) for |b| in [2^-125, 2^125] from the hardware estimate and one Newton step with FMA (3 instructions): equal
// to the correctly rounded reciprocal for every float in that range, verified exhaustively on gfx950
// (tools/dev/rcp_check.hip, all 2^32 patterns); outside it the double quotient.
__device__ inline float rcp_rn_normal(float b) {
	const float y = __builtin_amdgcn_rcpf(b);
	return __builtin_fmaf(__builtin_fmaf(-b, y, 1.0f), y, y);
}
__device__ inline float rcp_rn(float b) {
	const float ab = fabsf(b);
	if (ab >= 0x1p-125f && ab <= 0x1p125f) return rcp_rn_normal(b);
	return static_cast<float>(1.0 / static_cast<double>(b));
}
__device__ inline float div_rn(float a, float b, float y) {
	const float aa = fabsf(a), ab = fabsf(b);
	if (!(aa > 1e-30f && aa < 1e30f && ab > 1e-30f && ab < 1e30f)) return a / b;
	const float q = a * y;
	const float r = fmaf(-b, q, a);
	return fmaf(r, y, q);
}
// pixel_to_ndc with the reciprocal of d1 precomputed (rcp_rn(d1))
__device__ inline float pixel_to_ndc_r(int i, int d1, int d2, float inv_d1) {
	float range = ndc_range(d1, d2);
	const float offset = (range / 2.0f);
	return -offset + div_rn(range * static_cast<float>(i) + offset, static_cast<float>(d1), inv_d1);
}

// pixel_to_ndc(i, d1, d2) along one image axis with its constants precomputed on the host: range = ndc_range(d1, d2),
// offset = range / 2 (exact), inv = RN(1/d1). The numerator range * i + offset lies in [offset, range * d1] for pixel
// indices 0 <= i < d1 (normal floats), so the Markstein quotient needs no range guard: bit-identical to pixel_to_ndc.
struct PixelAxis {
	int dim;
	float dimf, range, offset, inv, scale;   // scale = d1 / range (estimates only)
};
inline PixelAxis make_pixel_axis(int d1, int d2) {
	PixelAxis a;
	a.dim = d1;
	a.dimf = static_cast<float>(d1);
	a.range = ndc_range(d1, d2);
	a.offset = a.range / 2.0f;
	a.inv = static_cast<float>(1.0 / static_cast<double>(d1));
	a.scale = a.dimf / a.range;
	return a;
}
__device__ inline float pixel_ndc(int i, const PixelAxis& a) {
	const float n = a.range * static_cast<float>(i) + a.offset;
	const float q = n * a.inv;
	const float r = fmaf(-a.dimf, q, n);
	return -a.offset + fmaf(r, a.inv, q);
}

// Open3D TransformIndexer::Project with float intrinsics
struct Camera {
	float fx, fy, cx, cy;
	__host__ __device__ inline void project(float x, float y, float z, float* u, float* v) const {
		float inv_z = 1.0f / z;
		*u = fx * x * inv_z + cx;
		*v = fy * y * inv_z + cy;
	}
	// project with RN(1/z) from rcp_rn (3 instructions in its range instead of a correctly rounded division):
	// bit-identical to project
	__device__ inline void project_rn(float x, float y, float z, float* u, float* v) const {
		const float inv_z = rcp_rn(z);
		*u = fx * x * inv_z + cx;
		*v = fy * y * inv_z + cy;
	}
};

struct NdcSetup {
	Camera ndc;            // NDC intrinsics (float)
	float min_x, max_x, min_y, max_y;   // NDC clip range
};
// CoordinateSystemConversions.h:109-146 ImageSpaceIntrinsicsToNdc (double on host, stored as float like TransformIndexer)
NdcSetup make_ndc_setup(const double* K, int height, int width, bool consistent);

__host__ __device__ inline float spa_cw(float px, float py, float v0x, float v0y, float v1x, float v1y) {
	// cpp/rendering/functional/kernel/BarycentricCoordinates.h:35-47 (ClockWise)
	return (px - v0x) * (v0y - v1y) - (py - v0y) * (v0x - v1x);
}

// ---- per-face raster test shared by the scatter pass and the resolve pass (bit-identical in both) ----
// cpp/rendering/kernel/RayFaceIntersection.h:162-255 minus the queue logic.
struct FaceNdc {
	float x[3], y[3], z[3];
};
struct RasterHit {
	float depth, dist, b0, b1, b2;
};

__device__ inline float point_segment_sq(float px, float py, float ax, float ay, float bx, float by) {
	float sx = bx - ax, sy = by - ay;
	float l2 = sx * sx + sy * sy;
	float t = (sx * (px - ax) + sy * (py - ay)) / l2;
	if (l2 <= K_EPSILON) {
		float dx = px - bx, dy = py - by;
		return dx * dx + dy * dy;
	}
	t = fminf(fmaxf(t, 0.f), 1.f);
	float cx = ax + t * sx, cy = ay + t * sy;
	float dx = cx - px, dy = cy - py;
	return dx * dx + dy * dy;
}

// Ray-face test of one pixel centre (RayFaceIntersection.h:162-255 semantics). Returns true if accepted.
// DIST = false skips the point-to-edge distance: valid only where the caller knows the distance test passes (a face
// whose box diagonal is far below the blur radius, or a winner re-resolved after a full test); h.dist is then unset.
__device__ inline float face_area_cw(const FaceNdc& f) { return spa_cw(f.x[0], f.y[0], f.x[1], f.y[1], f.x[2], f.y[2]); }
// reciprocal of the barycentric denominator (area + K_EPSILON) of a face, for face_test's shared-reciprocal division
__device__ inline float face_inv_area(const FaceNdc& f) { return rcp_rn(face_area_cw(f) + K_EPSILON); }

// The per-pixel part of the test once the box, culling and degeneracy checks have passed: barycentrics from the three
// signed parallelogram areas s_i of the pixel centre against the edges opposite vertex i (A = area + K_EPSILON,
// inv_area = rcp_rn(A)), perspective correction, clipping, depth and the blur-distance test. Shared by face_test and
// the rasterizer's row walk (which forms the s_i from row-shared terms with the same operations), so both are bit-identical.
template <bool DIST>
__device__ inline bool face_hit_from_spa(const FaceNdc& f, float s0, float s1, float s2, float A, float inv_area, float px, float py, float blur,
                                         bool persp, bool clip, RasterHit& h) {
	float b0 = div_rn(s0, A, inv_area);
	float b1 = div_rn(s1, A, inv_area);
	float b2 = div_rn(s2, A, inv_area);
	if (persp) {
		const float n0 = b0 * f.z[1] * f.z[2], n1 = f.z[0] * b1 * f.z[2], n2 = f.z[0] * f.z[1] * b2;
		const float den = fmaxf(n0 + n1 + n2, K_EPSILON);
		b0 = n0 / den;
		b1 = n1 / den;
		b2 = n2 / den;
	}
	float c0 = b0, c1 = b1, c2 = b2;
	if (clip) {
		c0 = fmaxf(b0, 0.f);
		c1 = fmaxf(b1, 0.f);
		c2 = fmaxf(b2, 0.f);
		float zz = (c0 * c0 + c1 * c1) + c2 * c2;
		if (zz > 0.f) {
			float s = sqrtf(zz);
			c0 /= s;
			c1 /= s;
			c2 /= s;
		}
	}
	const float depth = c0 * f.z[0] + c1 * f.z[1] + c2 * f.z[2];
	if (depth < 0.f) return false;
	if constexpr (DIST) {
		const float d = fmin3f(point_segment_sq(px, py, f.x[0], f.y[0], f.x[1], f.y[1]), point_segment_sq(px, py, f.x[0], f.y[0], f.x[2], f.y[2]),
		                       point_segment_sq(px, py, f.x[1], f.y[1], f.x[2], f.y[2]));
		const bool inside = b0 > 0.f && b1 > 0.f && b2 > 0.f;
		if (!inside && d >= blur) return false;
		h.dist = inside ? -d : d;
	}
	h.depth = depth;
	h.b0 = c0;
	h.b1 = c1;
	h.b2 = c2;
	return true;
}

template <bool DIST = true>
__device__ inline bool face_test(const FaceNdc& f, float px, float py, float blur, bool persp, bool clip, bool cull, RasterHit& h,
                                 float inv_area) {
	const float area = spa_cw(f.x[0], f.y[0], f.x[1], f.y[1], f.x[2], f.y[2]);
	const bool back = area < 0.f;
	const bool zero_area = (area <= K_EPSILON && area >= -1.f * K_EPSILON);
	const float xmin = fmin3f(f.x[0], f.x[1], f.x[2]) - blur;
	const float xmax = fmax3f(f.x[0], f.x[1], f.x[2]) + blur;
	const float ymin = fmin3f(f.y[0], f.y[1], f.y[2]) - blur;
	const float ymax = fmax3f(f.y[0], f.y[1], f.y[2]) + blur;
	const bool zinv = fmax3f(f.z[0], f.z[1], f.z[2]) < K_EPSILON;
	if ((px > xmax || px < xmin || py > ymax || py < ymin || zinv) || (cull && back) || zero_area) return false;
	return face_hit_from_spa<DIST>(f, spa_cw(px, py, f.x[1], f.y[1], f.x[2], f.y[2]), spa_cw(px, py, f.x[2], f.y[2], f.x[0], f.y[0]),
	                               spa_cw(px, py, f.x[0], f.y[0], f.x[1], f.y[1]), area + K_EPSILON, inv_area, px, py, blur, persp, clip, h);
}
template <bool DIST = true>
__device__ inline bool face_test(const FaceNdc& f, float px, float py, float blur, bool persp, bool clip, bool cull, RasterHit& h) {
	return face_test<DIST>(f, px, py, blur, persp, clip, cull, h, face_inv_area(f));
}

// 64-bit (depth, face) key: non-negative float depth bits are order-preserving; ties resolve to the lower face index
// (the reference's operator<, RayFaceIntersection.h:42-45).
__device__ inline uint64_t raster_key(float depth, int32_t face) {
	float d = depth + 0.0f;   // canonicalize -0 to +0
	return (static_cast<uint64_t>(__float_as_uint(d)) << 32) | static_cast<uint32_t>(face);
}
constexpr uint64_t EMPTY_KEY = ~0ull;

// pixel index range possibly covered by a bounding box along one image axis (widened by one pixel; exact test follows)
__host__ __device__ inline void pixel_span(float lo, float hi, int dim, int other, int* first, int* last) {
	const double r = static_cast<double>(ndc_range(dim, other));
	double a = floor((static_cast<double>(lo) + r / 2.0) * dim / r - 0.5) - 1.0;
	double b = ceil((static_cast<double>(hi) + r / 2.0) * dim / r - 0.5) + 1.0;
	if (!(a <= dim - 1) || !(b >= 0.0)) {   // empty (also NaN / inf bounds)
		*first = 1;
		*last = 0;
		return;
	}
	if (a < 0.0) a = 0.0;
	if (b > dim - 1) b = dim - 1;
	*first = static_cast<int>(a);
	*last = static_cast<int>(b);
}

} // namespace nnrt
