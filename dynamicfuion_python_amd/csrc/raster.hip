// Rasterizer for gfx950. Semantics: cpp/rendering/RasterizeNdcTriangles.cpp:33-129 and RayFaceIntersection.h:162-255
// (perspective-correct barycentrics, back-face culling, blur radius compared against the squared point-face distance: A13).
//
// faces_per_pixel == 1 (the fitter's call, DeformableMeshToImageFitter.cpp:125): instead of the reference's coarse
// grid bins + per-pixel bin walk, each face scatters into the pixels of its bounding box a 64-bit key
// (float depth bits << 32 | face) with a global atomicMin. The minimum key is exactly the lexicographic (depth, face)
// winner that the reference's queue logic selects, so no bin capacity (and no silent truncation) exists. A resolve pass
// recomputes the winner's barycentrics/depth with the same device function, bit-identically.
// faces_per_pixel > 1 (API only): per-pixel lists of the faces that pass the full test at the pixel centre (count, scan,
// fill), each replayed in ascending face order through the reference's bounded queue.
#include "kernels.hpp"

#include <hipcub/hipcub.hpp>
#include <cstdlib>

namespace nnrt {

__device__ inline FaceNdc load_face_ndc(const float* face_ndc, int64_t f) {
	FaceNdc r;
	const float* p = face_ndc + 9 * f;
#pragma unroll
	for (int i = 0; i < 3; i++) {
		r.x[i] = p[3 * i];
		r.y[i] = p[3 * i + 1];
		r.z[i] = p[3 * i + 2];
	}
	return r;
}

RasterOptions make_raster_options(int H, int W, float blur, int perspective, int clip_barycentric, int cull_back_faces) {
	RasterOptions o{H, W, blur, perspective, clip_barycentric, cull_back_faces, make_pixel_axis(W, H), make_pixel_axis(H, W)};
	return o;
}

// First pixel index i in [0, dim] whose centre pixel_ndc(i) >= lo (dim: none) and last index in [-1, dim) whose centre is
// <= hi (-1: none). pixel_ndc is non-decreasing in i; a float estimate lands at most a step away and the walks make it
// exact (typically one evaluation each). lo, hi finite.
__device__ inline int pixel_first(float lo, const PixelAxis& a) {
	const float e = fminf(fmaxf(ceilf((lo + a.offset) * a.scale - 0.5f), 0.f), a.dimf);
	int i = static_cast<int>(e);
#pragma clang loop unroll(disable) vectorize(disable)
	while (i > 0 && pixel_ndc(i - 1, a) >= lo) i--;
#pragma clang loop unroll(disable) vectorize(disable)
	while (i < a.dim && pixel_ndc(i, a) < lo) i++;
	return i;
}
__device__ inline int pixel_last(float hi, const PixelAxis& a) {
	const float e = fminf(fmaxf(floorf((hi + a.offset) * a.scale - 0.5f), -1.f), a.dimf - 1.f);
	int i = static_cast<int>(e);
#pragma clang loop unroll(disable) vectorize(disable)
	while (i < a.dim - 1 && pixel_ndc(i + 1, a) <= hi) i++;
#pragma clang loop unroll(disable) vectorize(disable)
	while (i >= 0 && pixel_ndc(i, a) > hi) i--;
	return i;
}

// A face with a non-finite vertex coordinate is never rasterized (the sum of the nine coordinates is non-finite iff one
// is, for NDC-sized values). Such faces only arise from the reference's A7 NaN rotations; the reference's queue then
// depends on its face processing order (NaN fails every comparison), so both implementations here reject them.
__device__ inline bool face_finite(const FaceNdc& fn) {
	const float s = ((fn.x[0] + fn.x[1]) + (fn.x[2] + fn.y[0])) + ((fn.y[1] + fn.y[2]) + (fn.z[0] + fn.z[1])) + fn.z[2];
	return __builtin_isfinite(s);
}

// Exact pixel range of a face: the pixels whose centres pass face_test's bounding-box check (box widened by the blur
// radius). Returns false for faces face_test rejects for every pixel (culled, zero-area, behind the camera, off-image,
// non-finite).
__device__ inline bool face_pixel_range(const FaceNdc& fn, const RasterOptions& o, int& u0, int& u1, int& v0, int& v1) {
	if (!face_finite(fn)) return false;
	const float area = spa_cw(fn.x[0], fn.y[0], fn.x[1], fn.y[1], fn.x[2], fn.y[2]);
	const bool back = area < 0.f;
	const bool zero_area = (area <= K_EPSILON && area >= -1.f * K_EPSILON);
	const bool zinv = fmax3f(fn.z[0], fn.z[1], fn.z[2]) < K_EPSILON;
	if ((o.cull_back_faces && back) || zero_area || zinv) return false;
	const float xmin = fmin3f(fn.x[0], fn.x[1], fn.x[2]) - o.blur;
	const float xmax = fmax3f(fn.x[0], fn.x[1], fn.x[2]) + o.blur;
	const float ymin = fmin3f(fn.y[0], fn.y[1], fn.y[2]) - o.blur;
	const float ymax = fmax3f(fn.y[0], fn.y[1], fn.y[2]) + o.blur;
	if (!(xmax >= xmin) || !(ymax >= ymin)) return false;
	u0 = pixel_first(xmin, o.ax);
	u1 = pixel_last(xmax, o.ax);
	v0 = pixel_first(ymin, o.ay);
	v1 = pixel_last(ymax, o.ay);
	return u0 <= u1 && v0 <= v1;
}

// K = 1 scatter. Each wave owns SCATTER_FPW consecutive faces. Consecutive faces of a mesh are spatially coherent, so
// the wave's pixel boxes share a small bounding rectangle, held as a wave-private tile of (depth, face) keys in LDS; the
// tile is merged into the image with one global atomicMin per touched pixel, row-contiguous across lanes (memory-side
// global atomics cost one request per scattered lane: MI355X_MICROARCH.md "Global float atomics"). A wave whose rectangle
// exceeds the tile (e.g. a face run that wraps to the next mesh row) scatters straight to the image instead. Either way
// the result is the minimum key over all faces, i.e. identical to a direct scatter.
// Load balance: a face's work is its box rows. The wave lists its faces' rows (a wave-wide prefix sum of row counts)
// and deals them out one row per lane, so lanes walk rows of ~equal length instead of whole boxes of unequal size. A
// row shares its pixel-row NDC coordinate and the y-terms of the three edge functions across its pixels.
constexpr int SCATTER_BLOCK = 256;
constexpr int SCATTER_WAVES = SCATTER_BLOCK / 64;
constexpr int SCATTER_FPW = 32;                                          // faces per wave
constexpr int SCATTER_FACES_PER_BLOCK = SCATTER_WAVES * SCATTER_FPW;
constexpr int SCATTER_TILE_KEYS = 512;                                   // 4 KiB per wave

template <int FPW, int KEYS>
struct ScatterLds {
	static constexpr int faces = FPW, tile_keys = KEYS;
	uint64_t keys[KEYS];
	float4 rec[FPW][4];           // x0 x1 x2 y0 | y1 y2 z0 z1 | z2 inv_area (u0 | span_u << 16) (v0 | fast << 30 | near_all << 31) |
	                              // A x1-x2 x2-x0 x0-x1 (the rows' face constants: face_row_constants)
	uint32_t row[64];             // one round of row tasks: face slot | row << 8
};
using ScatterWaveLds = ScatterLds<SCATTER_FPW, SCATTER_TILE_KEYS>;
// Dense meshes (more faces than pixels, e.g. C3's 4.5 M mostly sub-pixel triangles at 1280 x 960): one face per lane, 64
// per wave -- the wave's fixed costs (face loads in flight, box reductions, row dealing, tile clear and merge) serve
// twice the faces, and half the waves run the launch's latency rounds -- with a 256-key tile (64 consecutive sub-pixel
// faces cover a small pixel box), which keeps six waves per SIMD. The per-face operations are face_pixel_range's, the
// scatter the same keyed minimum: results identical to the lane-pair path (round 6).
constexpr int DENSE_FPW = 64;
constexpr int DENSE_TILE_KEYS = 256;
using DenseWaveLds = ScatterLds<DENSE_FPW, DENSE_TILE_KEYS>;

__device__ inline void scatter_wave_sync() {
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// one face row: pixels u0 .. u0 + span - 1 of image row v
// Markstein quotient a / b through y = RN(1/b), without div_rn's operand-range guard (see depth_near_all_fast)
__device__ inline float div_mk(float a, float b, float y) {
	const float q = a * y;
	const float r = fmaf(-b, q, a);
	return fmaf(r, y, q);
}

// Depth at a pixel of a face whose every box pixel passes the distance test (A13 near_all), fast path. The reference
// forms the barycentrics and the perspective weights as correctly rounded quotients; here they are Markstein quotients
// through the correctly rounded reciprocals of A and of the perspective denominator, without div_rn's guard. The guard
// exists for numerators outside [1e-30, 1e30]. Above: excluded (the caller admits faces with |A| in [1e-30, 1e30],
// |z| < 1e10 and a box within the blur radius, blur < 1e20, so |s_i| stays far below 1e30; the perspective numerators are
// checked here). Below: such a quotient can differ from the correctly rounded one only in the sign of a zero or in
// subnormal digits, i.e. by < 1e-35 after the |z| < 1e10 weighting, which cannot change the bits of a depth of
// magnitude >= 1e-20; smaller depths are recomputed on the guarded path. Returns false where face_hit_from_spa rejects.
__device__ inline bool depth_near_all_fast(const FaceNdc& f, float s0, float s1, float s2, float A, float inv_area, float px, float py,
                                           const RasterOptions& o, float& depth) {
	float b0 = div_mk(s0, A, inv_area), b1 = div_mk(s1, A, inv_area), b2 = div_mk(s2, A, inv_area);
	if (o.perspective) {
		const float n0 = b0 * f.z[1] * f.z[2], n1 = f.z[0] * b1 * f.z[2], n2 = f.z[0] * f.z[1] * b2;
		const float den = fmaxf(n0 + n1 + n2, K_EPSILON);
		if (fmaxf(fmaxf(fabsf(n0), fabsf(n1)), fabsf(n2)) < 1e29f && den < 1e30f) {
			const float y = rcp_rn_normal(den);   // den in [K_EPSILON, 1e30): rcp_rn_normal's exact range
			b0 = div_mk(n0, den, y);
			b1 = div_mk(n1, den, y);
			b2 = div_mk(n2, den, y);
		} else {
			b0 = n0 / den;
			b1 = n1 / den;
			b2 = n2 / den;
		}
	}
	depth = b0 * f.z[0] + b1 * f.z[1] + b2 * f.z[2];
	if (!(fabsf(depth) >= 1e-20f)) {
		RasterHit h;
		if (!face_hit_from_spa<false>(f, s0, s1, s2, A, inv_area, px, py, o.blur, o.perspective, 0, h)) return false;
		depth = h.depth;
		return true;
	}
	return !(depth < 0.f);
}

// A face's row-invariant terms, formed once per face in the wave's setup instead of once per row: (A = spa_cw(v0, v1, v2)
// + K_EPSILON, x1 - x2, x2 - x0, x0 - x1) -- the same operations scatter_row used to repeat per row -- and whether a
// near_all face's rows take depth_near_all_fast (its conditions on A, the depths and the options).
__device__ inline float4 face_row_constants(const FaceNdc& fn) {
	return make_float4(spa_cw(fn.x[0], fn.y[0], fn.x[1], fn.y[1], fn.x[2], fn.y[2]) + K_EPSILON, fn.x[1] - fn.x[2], fn.x[2] - fn.x[0], fn.x[0] - fn.x[1]);
}
__device__ inline bool face_rows_fast(const FaceNdc& fn, float A, const RasterOptions& o) {
	return !o.clip_barycentric && o.blur < 1e20f && fabsf(A) > 1e-30f && fabsf(A) < 1e30f &&
	       fmaxf(fmaxf(fabsf(fn.z[0]), fabsf(fn.z[1])), fabsf(fn.z[2])) < 1e10f;
}

// one face row: pixels u0 .. u0 + span - 1 of image row v. MODE 0: full test (distance included); 1: near_all face
// (guarded quotients); 2: near_all face on the fast path (depth_near_all_fast's conditions hold).
template <int MODE>
__device__ inline void scatter_row(const FaceNdc& fn, float inv_area, float4 k, int u0, int span, int v, int32_t face, const RasterOptions& o,
                                   bool staged, uint64_t* tile, int tu0, int tv0, int tw, uint64_t* keys) {
	const float py = pixel_ndc(v, o.ay);
	const float A = k.x;
	// spa_cw(p, a, b) = (px - ax) * (ay - by) - (py - ay) * (ax - bx), edges (v1, v2), (v2, v0), (v0, v1)
	const float c0 = fn.y[1] - fn.y[2], c1 = fn.y[2] - fn.y[0], c2 = fn.y[0] - fn.y[1];
	const float r0 = (py - fn.y[1]) * k.y, r1 = (py - fn.y[2]) * k.z, r2 = (py - fn.y[0]) * k.w;
	uint64_t* trow = tile + (v - tv0) * tw - tu0;
#pragma clang loop unroll(disable) vectorize(disable)
	for (int u = u0; u < u0 + span; u++) {
		const float px = pixel_ndc(u, o.ax);
		const float s0 = (px - fn.x[1]) * c0 - r0, s1 = (px - fn.x[2]) * c1 - r1, s2 = (px - fn.x[0]) * c2 - r2;
		float depth;
		if constexpr (MODE == 2) {
			if (!depth_near_all_fast(fn, s0, s1, s2, A, inv_area, px, py, o, depth)) continue;
		} else {
			RasterHit h;
			if (!face_hit_from_spa<MODE == 0>(fn, s0, s1, s2, A, inv_area, px, py, o.blur, o.perspective, o.clip_barycentric, h)) continue;
			depth = h.depth;
		}
		const unsigned long long key = raster_key(depth, face);
		if (staged)
			__hip_atomic_fetch_min(reinterpret_cast<unsigned long long*>(trow + u), key, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
		else
			atomicMin(reinterpret_cast<unsigned long long*>(keys + static_cast<int64_t>(v) * o.W + u), key);
	}
}

template <class W>
__device__ inline void scatter_rows(int rows, int slot, int32_t face0, const RasterOptions& o, uint64_t* keys, W& w, bool staged,
                                    int bu0, int bv0, int tw, int th);
#ifdef NNRT_KERNEL_STAMPS
__device__ unsigned long long g_raster_stamps[16384][8];   // start, setup end, end, hwid, rows, tile, pixels, max pixels per lane
#endif

// lane < W::faces holds face face0 + lane (ok = it exists and is not masked out); all 64 lanes of the wave call this
template <class W>
__device__ inline void scatter_wave(const FaceNdc& fn, bool ok, int32_t face0, const RasterOptions& o, uint64_t* keys, W& w) {
	const int lane = static_cast<int>(threadIdx.x & 63);
	int u0 = 0, u1 = -1, v0 = 0, v1 = -1;
	if (ok) ok = face_pixel_range(fn, o, u0, u1, v0, v1);
	int bu0 = ok ? u0 : 0x7fffffff, bu1 = ok ? u1 : -1, bv0 = ok ? v0 : 0x7fffffff, bv1 = ok ? v1 : -1;
#pragma unroll
	for (int d = 32; d >= 1; d >>= 1) {
		bu0 = min(bu0, __shfl_xor(bu0, d));
		bu1 = max(bu1, __shfl_xor(bu1, d));
		bv0 = min(bv0, __shfl_xor(bv0, d));
		bv1 = max(bv1, __shfl_xor(bv1, d));
	}
	if (bu1 < 0) return;   // wave-uniform: none of the wave's faces covers a pixel
	const int tw = bu1 - bu0 + 1, th = bv1 - bv0 + 1;
	const bool staged = tw * th <= W::tile_keys;
	if (staged)
		for (int i = lane; i < tw * th; i += 64) w.keys[i] = EMPTY_KEY;
	const int rows = ok ? v1 - v0 + 1 : 0;
	if (ok) {
		// A13: the blur radius is compared against SQUARED NDC distances, so for a face whose blur-widened box has a
		// squared diagonal well below the radius every pixel in the box passes the distance test: skip computing it.
		const float bw = (fmax3f(fn.x[0], fn.x[1], fn.x[2]) - fmin3f(fn.x[0], fn.x[1], fn.x[2])) + 2.f * o.blur;
		const float bh = (fmax3f(fn.y[0], fn.y[1], fn.y[2]) - fmin3f(fn.y[0], fn.y[1], fn.y[2])) + 2.f * o.blur;
		const bool near_all = (bw * bw + bh * bh) < 0.5f * o.blur;
		w.rec[lane][0] = make_float4(fn.x[0], fn.x[1], fn.x[2], fn.y[0]);
		w.rec[lane][1] = make_float4(fn.y[1], fn.y[2], fn.z[0], fn.z[1]);
		const float4 k = face_row_constants(fn);
		const bool fast = face_rows_fast(fn, k.x, o);
		w.rec[lane][2] = make_float4(fn.z[2], face_inv_area(fn), __uint_as_float(static_cast<uint32_t>(u0) | static_cast<uint32_t>(u1 - u0 + 1) << 16),
		                             __uint_as_float(static_cast<uint32_t>(v0) | (fast ? 0x40000000u : 0u) | (near_all ? 0x80000000u : 0u)));
		w.rec[lane][3] = k;
	}
	scatter_rows(rows, lane, face0, o, keys, w, staged, bu0, bv0, tw, th);
}

// Deals the wave's face rows one per lane (rows: this lane's face's box rows, slot: its face's record) and scatters
// them, then merges the staged tile into the image. All 64 lanes call this.
template <class W>
__device__ inline void scatter_rows(int rows, int slot, int32_t face0, const RasterOptions& o, uint64_t* keys, W& w, bool staged,
                                    int bu0, int bv0, int tw, int th) {
	const int lane = static_cast<int>(threadIdx.x & 63);
	int incl = rows;
#pragma unroll
	for (int d = 1; d < 64; d <<= 1) {
		const int t = __shfl_up(incl, d);
		if (lane >= d) incl += t;
	}
	const int total = __shfl(incl, 63);
	const int start = incl - rows;
#ifdef NNRT_KERNEL_STAMPS
	int px_lane = 0;
#endif
	for (int base = 0; base < total; base += 64) {
#pragma clang loop unroll(disable) vectorize(disable)
		for (int t = max(start, base); t < min(start + rows, base + 64); t++) w.row[t - base] = static_cast<uint32_t>(slot) | static_cast<uint32_t>(t - start) << 8;
		scatter_wave_sync();
		if (base + lane < total) {
			const uint32_t e = w.row[lane];
			const int slot = static_cast<int>(e & 255u), r = static_cast<int>(e >> 8);
			const float4 q0 = w.rec[slot][0], q1 = w.rec[slot][1], q2 = w.rec[slot][2], q3 = w.rec[slot][3];
			FaceNdc g;
			g.x[0] = q0.x;
			g.x[1] = q0.y;
			g.x[2] = q0.z;
			g.y[0] = q0.w;
			g.y[1] = q1.x;
			g.y[2] = q1.y;
			g.z[0] = q1.z;
			g.z[1] = q1.w;
			g.z[2] = q2.x;
			const uint32_t ui = __float_as_uint(q2.z), vi = __float_as_uint(q2.w);
			const int fu0 = static_cast<int>(ui & 0xffffu), span = static_cast<int>(ui >> 16);
			const int v = static_cast<int>(vi & 0x3fffffffu) + r;
#ifdef NNRT_KERNEL_STAMPS
			px_lane += span;
#endif
			if (!(vi >> 31))
				scatter_row<0>(g, q2.y, q3, fu0, span, v, face0 + slot, o, staged, w.keys, bu0, bv0, tw, keys);
			else if ((vi >> 30) & 1u)
				scatter_row<2>(g, q2.y, q3, fu0, span, v, face0 + slot, o, staged, w.keys, bu0, bv0, tw, keys);
			else
				scatter_row<1>(g, q2.y, q3, fu0, span, v, face0 + slot, o, staged, w.keys, bu0, bv0, tw, keys);
		}
		scatter_wave_sync();
	}
#ifdef NNRT_KERNEL_STAMPS
	{
		int px_sum = px_lane, px_max = px_lane;
		for (int d = 32; d >= 1; d >>= 1) {
			px_sum += __shfl_xor(px_sum, d);
			px_max = max(px_max, __shfl_xor(px_max, d));
		}
		NNRT_WAVE_STAMP(g_raster_stamps, 4, static_cast<unsigned long long>(total));
		NNRT_WAVE_STAMP(g_raster_stamps, 5, static_cast<unsigned long long>(tw * th) << 1 | (staged ? 1ull : 0ull));
		NNRT_WAVE_STAMP(g_raster_stamps, 6, static_cast<unsigned long long>(px_sum));
		NNRT_WAVE_STAMP(g_raster_stamps, 7, static_cast<unsigned long long>(px_max));
	}
#endif
	if (!staged) return;
	// merge the tile row by row: i = y * tw + x, y from a float quotient corrected to the exact one
	const float inv_tw = 1.0f / static_cast<float>(tw);
	for (int i = lane; i < tw * th; i += 64) {
		const uint64_t k = w.keys[i];
		if (k == EMPTY_KEY) continue;
		int y = static_cast<int>(static_cast<float>(i) * inv_tw);
		if (y * tw > i) y--;
		if ((y + 1) * tw <= i) y++;
		const int64_t p = static_cast<int64_t>(bv0 + y) * o.W + bu0 + (i - y * tw);
		atomicMin(reinterpret_cast<unsigned long long*>(keys + p), static_cast<unsigned long long>(k));
	}
}

// value of the partner lane of a lane pair (lane ^ 1): DPP quad permutation [1, 0, 3, 2]
__device__ inline int pair_swap(int v) { return __builtin_amdgcn_update_dpp(0, v, 0xB1, 0xf, 0xf, false); }
__device__ inline float pair_swap(float v) { return __builtin_bit_cast(float, pair_swap(__builtin_bit_cast(int, v))); }

// Mesh path: lane pair (2f, 2f + 1) holds face face0 + f, f < SCATTER_FPW (both lanes hold the whole projected face, ok
// alike). The per-face setup is split between the pair -- the even lane works the x axis (the face's pixel columns),
// the odd lane the y axis (its rows) -- so one instruction stream covers both axes (face_pixel_range's operations,
// per axis, unchanged); the row dealing and scatter are scatter_wave's (scatter_rows).
__device__ inline void scatter_wave_pairs(const FaceNdc& fn, bool ok, int32_t face0, const RasterOptions& o, uint64_t* keys, ScatterWaveLds& w) {
	const int lane = static_cast<int>(threadIdx.x & 63);
	const bool odd = lane & 1;
	// face_pixel_range's face checks (both lanes)
	if (ok) {
		if (!face_finite(fn)) ok = false;
		const float area = spa_cw(fn.x[0], fn.y[0], fn.x[1], fn.y[1], fn.x[2], fn.y[2]);
		const bool back = area < 0.f;
		const bool zero_area = (area <= K_EPSILON && area >= -1.f * K_EPSILON);
		const bool zinv = fmax3f(fn.z[0], fn.z[1], fn.z[2]) < K_EPSILON;
		if ((o.cull_back_faces && back) || zero_area || zinv) ok = false;
	}
	// this lane's axis: box (widened by the blur radius) and its exact pixel range
	const float c0 = odd ? fn.y[0] : fn.x[0], c1 = odd ? fn.y[1] : fn.x[1], c2 = odd ? fn.y[2] : fn.x[2];
	const PixelAxis ax = odd ? o.ay : o.ax;
	const float cmin = fmin3f(c0, c1, c2), cmax = fmax3f(c0, c1, c2);
	const float lo = cmin - o.blur, hi = cmax + o.blur;
	int a0 = 0, a1 = -1;
	const bool axis_ok = ok && hi >= lo;
	if (axis_ok) {
		a0 = pixel_first(lo, ax);
		a1 = pixel_last(hi, ax);
	}
	// the pair's verdict: both boxes non-empty (face_pixel_range: the two extent checks, then u0 <= u1 && v0 <= v1)
	const bool both_extents = axis_ok && pair_swap(static_cast<int>(axis_ok)) != 0;
	const bool mine_nonempty = a0 <= a1;
	ok = both_extents && mine_nonempty && pair_swap(static_cast<int>(mine_nonempty)) != 0;
	// wave box: min / max of the valid faces' ranges per axis (butterfly over the lanes of the same parity)
	int blo = ok ? a0 : 0x7fffffff, bhi = ok ? a1 : -1;
#pragma unroll
	for (int d = 32; d >= 2; d >>= 1) {
		blo = min(blo, __shfl_xor(blo, d));
		bhi = max(bhi, __shfl_xor(bhi, d));
	}
	const int bu0 = __builtin_amdgcn_readlane(blo, 0), bu1 = __builtin_amdgcn_readlane(bhi, 0);
	const int bv0 = __builtin_amdgcn_readlane(blo, 1), bv1 = __builtin_amdgcn_readlane(bhi, 1);
	if (bu1 < 0) return;   // wave-uniform: none of the wave's faces covers a pixel
	const int tw = bu1 - bu0 + 1, th = bv1 - bv0 + 1;
	const bool staged = tw * th <= SCATTER_TILE_KEYS;
	if (staged)
		for (int i = lane; i < tw * th; i += 64) w.keys[i] = EMPTY_KEY;
	// the partner's range: the even lane gets (v0, v1), the odd lane (u0, u1)
	const int p0 = pair_swap(a0), p1 = pair_swap(a1);
	const int u0 = odd ? p0 : a0, u1 = odd ? p1 : a1, v0 = odd ? a0 : p0, v1 = odd ? a1 : p1;
	const int slot = lane >> 1;
	const int rows = ok && !odd ? v1 - v0 + 1 : 0;   // a face's rows are dealt from its even lane
	// A13 near_all (as in scatter_wave): squared blur-widened box diagonal, each lane its own axis' side
	const float side = (cmax - cmin) + 2.f * o.blur;
	const float other = pair_swap(side);
	const float bw = odd ? other : side, bh = odd ? side : other;
	const bool near_all = (bw * bw + bh * bh) < 0.5f * o.blur;
	if (ok) {
		const float4 k = face_row_constants(fn);   // both lanes (one instruction stream); the odd lane stores it
		if (!odd) {
			const bool fast = face_rows_fast(fn, k.x, o);
			w.rec[slot][0] = make_float4(fn.x[0], fn.x[1], fn.x[2], fn.y[0]);
			w.rec[slot][2] = make_float4(fn.z[2], face_inv_area(fn), __uint_as_float(static_cast<uint32_t>(u0) | static_cast<uint32_t>(u1 - u0 + 1) << 16),
			                             __uint_as_float(static_cast<uint32_t>(v0) | (fast ? 0x40000000u : 0u) | (near_all ? 0x80000000u : 0u)));
		} else {
			w.rec[slot][1] = make_float4(fn.y[1], fn.y[2], fn.z[0], fn.z[1]);
			w.rec[slot][3] = k;
		}
	}
	scatter_rows(rows, slot, face0, o, keys, w, staged, bu0, bv0, tw, th);
}

__global__ __launch_bounds__(SCATTER_BLOCK) void k_raster_scatter_ndc(const float* __restrict__ face_ndc, const uint8_t* __restrict__ mask,
                                                                      int64_t F, RasterOptions o, uint64_t* __restrict__ keys) {
	__shared__ ScatterWaveLds s_wave[SCATTER_WAVES];
	const int64_t face0 = (static_cast<int64_t>(blockIdx.x) * SCATTER_WAVES + (threadIdx.x >> 6)) * SCATTER_FPW;
	const int lane = static_cast<int>(threadIdx.x & 63);
	const int64_t f = face0 + lane;
	FaceNdc fn{};
	bool ok = lane < SCATTER_FPW && f < F && !(mask && !mask[f]);
	if (ok) fn = load_face_ndc(face_ndc, f);
	scatter_wave(fn, ok, static_cast<int32_t>(face0), o, keys, s_wave[threadIdx.x >> 6]);
}

nnrt_status launch_raster_scatter_ndc(const float* face_ndc, const uint8_t* mask, int64_t F, const RasterOptions& o, uint64_t* keys,
                                      hipStream_t stream) {
	if (F == 0) return NNRT_OK;
	NNRT_CHECK_ARG(o.W < 65536 && F < (int64_t(1) << 31), "image wider than 65535 pixels or more than 2^31 faces");
	k_raster_scatter_ndc<<<static_cast<unsigned>(ceil_div(F, SCATTER_FACES_PER_BLOCK)), SCATTER_BLOCK, 0, stream>>>(face_ndc, mask, F, o, keys);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

// fitter path: NDC extraction + clip test (ExtractClippedFaceVerticesImpl.h:108-179) fused with the scatter
__device__ inline bool project_mesh_face(const float4* __restrict__ wpos, int4 fi, const NdcSetup& s, float near_clip, float far_clip,
                                         FaceNdc& fn) {
	const int vi[3] = {fi.x, fi.y, fi.z};
	bool in_range = false, inlier = false;
	f3 v[3];
#pragma unroll
	for (int i = 0; i < 3; i++) {
		const float4 p = wpos[vi[i]];
		v[i] = make3(p.x, p.y, p.z);
		in_range |= v[i].z >= near_clip;
		in_range |= v[i].z <= far_clip;
	}
	if (!in_range) return false;
#pragma unroll
	for (int i = 0; i < 3; i++) {
		s.ndc.project_rn(v[i].x, v[i].y, v[i].z, &fn.x[i], &fn.y[i]);
		fn.z[i] = v[i].z;
		inlier |= (fn.y[i] >= s.min_y && fn.x[i] >= s.min_x && fn.y[i] <= s.max_y && fn.x[i] <= s.max_x);
	}
	return inlier;
}

#ifdef NNRT_KERNEL_STAMPS
extern "C" int nnrt_dev_raster_stamps(unsigned long long* out) {
	return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_raster_stamps), sizeof(g_raster_stamps)) == hipSuccess ? 0 : 1;
}
#endif

__global__ __launch_bounds__(SCATTER_BLOCK) void k_raster_scatter_mesh(const float4* __restrict__ wpos, const int4* __restrict__ faces4,
                                                                       int64_t F, NdcSetup s, float near_clip, float far_clip, RasterOptions o,
                                                                       uint64_t* __restrict__ keys) {
	__shared__ ScatterWaveLds s_wave[SCATTER_WAVES];
	const int64_t face0 = (static_cast<int64_t>(blockIdx.x) * SCATTER_WAVES + (threadIdx.x >> 6)) * SCATTER_FPW;
	const int lane = static_cast<int>(threadIdx.x & 63);
	const int64_t f = face0 + (lane >> 1);   // lane pairs (scatter_wave_pairs)
	FaceNdc fn{};
	NNRT_WAVE_STAMP(g_raster_stamps, 0, __builtin_amdgcn_s_memrealtime());
	NNRT_WAVE_STAMP(g_raster_stamps, 3, NNRT_STAMP_HWID());
	const bool ok = f < F && project_mesh_face(wpos, faces4[f], s, near_clip, far_clip, fn);
	NNRT_WAVE_STAMP(g_raster_stamps, 1, __builtin_amdgcn_s_memrealtime());
	scatter_wave_pairs(fn, ok, static_cast<int32_t>(face0), o, keys, s_wave[threadIdx.x >> 6]);
	NNRT_WAVE_STAMP(g_raster_stamps, 2, __builtin_amdgcn_s_memrealtime());
}

// dense meshes: one face per lane (DenseWaveLds)
__global__ __launch_bounds__(SCATTER_BLOCK) void k_raster_scatter_mesh_dense(const float4* __restrict__ wpos, const int4* __restrict__ faces4,
                                                                             int64_t F, NdcSetup s, float near_clip, float far_clip, RasterOptions o,
                                                                             uint64_t* __restrict__ keys) {
	__shared__ DenseWaveLds s_wave[SCATTER_WAVES];
	const int64_t face0 = (static_cast<int64_t>(blockIdx.x) * SCATTER_WAVES + (threadIdx.x >> 6)) * DENSE_FPW;
	const int64_t f = face0 + static_cast<int>(threadIdx.x & 63);
	FaceNdc fn{};
	const bool ok = f < F && project_mesh_face(wpos, faces4[f], s, near_clip, far_clip, fn);
	scatter_wave(fn, ok, static_cast<int32_t>(face0), o, keys, s_wave[threadIdx.x >> 6]);
}

bool raster_mesh_dense(int64_t F, const RasterOptions& o) {
	if (const char* v = std::getenv("NNRT_RASTER_DENSE")) return *v == '1';   // development switch: 0 / 1 force a path
	return F >= static_cast<int64_t>(o.H) * o.W;
}

nnrt_status launch_raster_scatter_mesh(const float4* wpos, const int4* faces4, int64_t F, const NdcSetup& s, float near_clip, float far_clip,
                                       const RasterOptions& o, uint64_t* keys, hipStream_t stream) {
	if (F == 0) return NNRT_OK;
	NNRT_CHECK_ARG(o.W < 65536 && F < (int64_t(1) << 31), "image wider than 65535 pixels or more than 2^31 faces");
	if (raster_mesh_dense(F, o)) {
		k_raster_scatter_mesh_dense<<<static_cast<unsigned>(ceil_div(F, SCATTER_WAVES * DENSE_FPW)), SCATTER_BLOCK, 0, stream>>>(wpos, faces4, F, s, near_clip,
		                                                                                                                   far_clip, o, keys);
		NNRT_LAUNCH_CHECK();
		return NNRT_OK;
	}
	k_raster_scatter_mesh<<<static_cast<unsigned>(ceil_div(F, SCATTER_FACES_PER_BLOCK)), SCATTER_BLOCK, 0, stream>>>(wpos, faces4, F, s, near_clip,
	                                                                                                                 far_clip, o, keys);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

// resolve the winner per pixel into reference-layout fragments ([H,W,1]); resets keys for the next call
__global__ __launch_bounds__(256) void k_raster_resolve(const float* __restrict__ face_ndc, RasterOptions o, uint64_t* __restrict__ keys,
                                                        int64_t* __restrict__ out_face, float* __restrict__ out_depth,
                                                        float* __restrict__ out_bary, float* __restrict__ out_dist) {
	const int64_t p = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (p >= static_cast<int64_t>(o.H) * o.W) return;
	const uint64_t key = keys[p];
	keys[p] = EMPTY_KEY;
	int64_t face = -1;
	RasterHit h{-1.f, -1.f, -1.f, -1.f, -1.f};
	if (key != EMPTY_KEY) {
		const int32_t f = static_cast<int32_t>(key & 0xffffffffu);
		const int v = static_cast<int>(p / o.W), u = static_cast<int>(p % o.W);
		if (face_test(load_face_ndc(face_ndc, f), pixel_to_ndc(u, o.W, o.H), pixel_to_ndc(v, o.H, o.W), o.blur, o.perspective,
		              o.clip_barycentric, o.cull_back_faces, h)) {
			face = f;
		} else {
			h = RasterHit{-1.f, -1.f, -1.f, -1.f, -1.f};
		}
	}
	out_face[p] = face;
	out_depth[p] = h.depth;
	out_dist[p] = h.dist;
	out_bary[3 * p] = h.b0;
	out_bary[3 * p + 1] = h.b1;
	out_bary[3 * p + 2] = h.b2;
}

nnrt_status launch_raster_resolve(const float* face_ndc, int64_t F, const RasterOptions& o, uint64_t* keys, int64_t* out_face, float* out_depth,
                                  float* out_bary, float* out_dist, hipStream_t stream) {
	(void) F;
	const int64_t P = static_cast<int64_t>(o.H) * o.W;
	if (P == 0) return NNRT_OK;
	k_raster_resolve<<<static_cast<unsigned>(ceil_div(P, 256)), 256, 0, stream>>>(face_ndc, o, keys, out_face, out_depth, out_bary, out_dist);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

// =====================================================================================================================
// faces_per_pixel > 1 (API path): per-pixel hit lists. Every face walks the exact pixel range of its box (as the K = 1
// scatter) running the full face test; pass A counts the hits per pixel, a scan places the lists, pass B appends the
// face indices. One lane per pixel then sorts its list by face index -- the ascending order in which the reference's
// bounded queue visits a bin's faces -- and replays that queue (RayFaceIntersection.h:162-255: the first K hits, then a
// hit replaces the current deepest only when strictly nearer), then orders the queue by (depth, face)
// (RayFaceIntersection.h:42-45). Work is proportional to the hits, not to the faces binned per tile, so dense meshes of
// tiny faces (millions of sub-pixel triangles) cost what the K = 1 scatter costs.
// =====================================================================================================================
template <bool FILL>
__global__ __launch_bounds__(256) void k_hit_lists(const float* __restrict__ face_ndc, const uint8_t* __restrict__ mask, int64_t F,
                                                   RasterOptions o, int* __restrict__ counts, const int* __restrict__ offsets,
                                                   int32_t* __restrict__ lists) {
	const int64_t f = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (f >= F || (mask && !mask[f])) return;
	const FaceNdc fn = load_face_ndc(face_ndc, f);
	int u0, u1, v0, v1;
	if (!face_pixel_range(fn, o, u0, u1, v0, v1)) return;
	const float w = (fmax3f(fn.x[0], fn.x[1], fn.x[2]) - fmin3f(fn.x[0], fn.x[1], fn.x[2])) + 2.f * o.blur;
	const float hh = (fmax3f(fn.y[0], fn.y[1], fn.y[2]) - fmin3f(fn.y[0], fn.y[1], fn.y[2])) + 2.f * o.blur;
	const bool near_all = (w * w + hh * hh) < 0.5f * o.blur;   // A13: every box pixel passes the distance test
	const float inv_area = face_inv_area(fn);
	for (int v = v0; v <= v1; v++) {
		const float py = pixel_ndc(v, o.ay);
		for (int u = u0; u <= u1; u++) {
			const float px = pixel_ndc(u, o.ax);
			RasterHit h;
			const bool hit = near_all ? face_test<false>(fn, px, py, o.blur, o.perspective, o.clip_barycentric, o.cull_back_faces, h, inv_area)
			                          : face_test<true>(fn, px, py, o.blur, o.perspective, o.clip_barycentric, o.cull_back_faces, h, inv_area);
			if (!hit) continue;
			const int64_t p = static_cast<int64_t>(v) * o.W + u;
			const int slot = atomicAdd(counts + p, 1);
			if constexpr (FILL) lists[offsets[p] + slot] = static_cast<int32_t>(f);
		}
	}
}

struct QEntry {
	float depth, dist, b0, b1, b2;
	int32_t face;
};

__global__ __launch_bounds__(256) void k_hit_resolve(const float* __restrict__ face_ndc, RasterOptions o, int K, const int* __restrict__ offsets,
                                                     int32_t* __restrict__ lists, int64_t* __restrict__ out_face, float* __restrict__ out_depth,
                                                     float* __restrict__ out_bary, float* __restrict__ out_dist) {
	const int64_t p = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (p >= static_cast<int64_t>(o.H) * o.W) return;
	const int v = static_cast<int>(p / o.W), u = static_cast<int>(p % o.W);
	const float px = pixel_to_ndc(u, o.W, o.H), py = pixel_to_ndc(v, o.H, o.W);
	int32_t* l = lists + offsets[p];
	const int n = offsets[p + 1] - offsets[p];
	for (int i = 1; i < n; i++) {   // ascending face index (the lists are short: the faces covering this pixel centre)
		const int32_t x = l[i];
		int j = i - 1;
		while (j >= 0 && l[j] > x) {
			l[j + 1] = l[j];
			j--;
		}
		l[j + 1] = x;
	}
	QEntry q[MAX_FACES_PER_PIXEL];
	int qs = 0, qat = -1;
	float qmax = -1000.f;
	for (int i = 0; i < n; i++) {
		const int32_t f = l[i];
		RasterHit h;
		if (!face_test(load_face_ndc(face_ndc, f), px, py, o.blur, o.perspective, o.clip_barycentric, o.cull_back_faces, h)) continue;
		const QEntry e{h.depth, h.dist, h.b0, h.b1, h.b2, f};
		if (qs < K) {
			q[qs] = e;
			if (e.depth > qmax) {
				qmax = e.depth;
				qat = qs;
			}
			qs++;
		} else if (e.depth < qmax) {
			q[qat] = e;
			qmax = e.depth;
			for (int j = 0; j < K; j++)
				if (q[j].depth > qmax) {
					qmax = q[j].depth;
					qat = j;
				}
		}
	}
	for (int i = 1; i < qs; i++) {   // (depth, face): RayFaceIntersection.h:42-45
		QEntry x = q[i];
		int j = i - 1;
		while (j >= 0 && (q[j].depth > x.depth || (q[j].depth == x.depth && q[j].face > x.face))) {
			q[j + 1] = q[j];
			j--;
		}
		q[j + 1] = x;
	}
	for (int i = 0; i < K; i++) {
		const int64_t o_ = p * K + i;
		if (i < qs) {
			out_face[o_] = q[i].face;
			out_depth[o_] = q[i].depth;
			out_dist[o_] = q[i].dist;
			out_bary[3 * o_] = q[i].b0;
			out_bary[3 * o_ + 1] = q[i].b1;
			out_bary[3 * o_ + 2] = q[i].b2;
		} else {
			out_face[o_] = -1;
			out_depth[o_] = -1.f;
			out_dist[o_] = -1.f;
			out_bary[3 * o_] = out_bary[3 * o_ + 1] = out_bary[3 * o_ + 2] = -1.f;
		}
	}
}

nnrt_status launch_raster_multi(const float* face_ndc, const uint8_t* mask, int64_t F, const RasterOptions& o, int faces_per_pixel,
                                int64_t* out_face, float* out_depth, float* out_bary, float* out_dist, hipStream_t stream) {
	const int64_t P = static_cast<int64_t>(o.H) * o.W;
	NNRT_CHECK_ARG(P < (int64_t(1) << 31), "image too large");
	int *counts = nullptr, *offsets = nullptr;
	int32_t* lists = nullptr;
	void* tmp = nullptr;
	size_t tmp_bytes = 0;
	NNRT_HIP(hipMallocAsync(reinterpret_cast<void**>(&counts), sizeof(int) * (P + 1), stream));
	NNRT_HIP(hipMallocAsync(reinterpret_cast<void**>(&offsets), sizeof(int) * (P + 1), stream));
	NNRT_HIP(hipMemsetAsync(counts, 0, sizeof(int) * (P + 1), stream));
	const unsigned fg = static_cast<unsigned>(ceil_div(F > 0 ? F : 1, 256));
	if (F > 0) k_hit_lists<false><<<fg, 256, 0, stream>>>(face_ndc, mask, F, o, counts, nullptr, nullptr);
	NNRT_LAUNCH_CHECK();
	NNRT_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, tmp_bytes, counts, offsets, static_cast<int>(P + 1), stream));
	NNRT_HIP(hipMallocAsync(&tmp, tmp_bytes, stream));
	NNRT_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, counts, offsets, static_cast<int>(P + 1), stream));
	int total = 0;
	NNRT_HIP(hipMemcpyAsync(&total, offsets + P, sizeof(int), hipMemcpyDeviceToHost, stream));
	NNRT_HIP(hipMemsetAsync(counts, 0, sizeof(int) * (P + 1), stream));
	NNRT_HIP(hipStreamSynchronize(stream));
	NNRT_HIP(hipMallocAsync(reinterpret_cast<void**>(&lists), sizeof(int32_t) * (total > 0 ? total : 1), stream));
	if (F > 0) k_hit_lists<true><<<fg, 256, 0, stream>>>(face_ndc, mask, F, o, counts, offsets, lists);
	NNRT_LAUNCH_CHECK();
	k_hit_resolve<<<static_cast<unsigned>(ceil_div(P, 256)), 256, 0, stream>>>(face_ndc, o, faces_per_pixel, offsets, lists, out_face, out_depth,
	                                                                          out_bary, out_dist);
	NNRT_LAUNCH_CHECK();
	NNRT_HIP(hipFreeAsync(counts, stream));
	NNRT_HIP(hipFreeAsync(offsets, stream));
	NNRT_HIP(hipFreeAsync(lists, stream));
	NNRT_HIP(hipFreeAsync(tmp, stream));
	return NNRT_OK;
}

} // namespace nnrt
