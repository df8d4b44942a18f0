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

// Conservative pixel index range of [lo, hi] along one image axis, in float (two pixels of margin absorb the rounding
// of the estimate; face_pixel_range trims it exactly). Empty for NaN / off-image bounds.
__device__ inline void pixel_span_f(float lo, float hi, int dim, int other, int* first, int* last) {
	const float r = ndc_range(dim, other);
	const float s = static_cast<float>(dim) / r;
	float a = floorf((lo + 0.5f * r) * s - 0.5f) - 2.f;
	float b = ceilf((hi + 0.5f * r) * s - 0.5f) + 2.f;
	if (!(a <= static_cast<float>(dim - 1)) || !(b >= 0.f)) {
		*first = 1;
		*last = 0;
		return;
	}
	a = fmaxf(a, 0.f);
	b = fminf(b, static_cast<float>(dim - 1));
	*first = static_cast<int>(a);
	*last = static_cast<int>(b);
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
	pixel_span_f(xmin, xmax, o.W, o.H, &u0, &u1);
	pixel_span_f(ymin, ymax, o.H, o.W, &v0, &v1);
	// pixel_to_ndc is monotone: trim the widening so only pixels inside the box remain
	const float inv_w = rcp_rn(static_cast<float>(o.W)), inv_h = rcp_rn(static_cast<float>(o.H));
	while (u0 <= u1 && pixel_to_ndc_r(u0, o.W, o.H, inv_w) < xmin) u0++;
	while (u1 >= u0 && pixel_to_ndc_r(u1, o.W, o.H, inv_w) > xmax) u1--;
	while (v0 <= v1 && pixel_to_ndc_r(v0, o.H, o.W, inv_h) < ymin) v0++;
	while (v1 >= v0 && pixel_to_ndc_r(v1, o.H, o.W, inv_h) > ymax) v1--;
	return u0 <= u1 && v0 <= v1;
}

// One workgroup = 64 consecutive faces, 4 lanes per face (the lanes of a quad split the face's pixel tests, so a launch
// has 4x the waves of a lane-per-face launch and each lane a quarter of the serial test loop). Consecutive faces of a
// mesh are spatially coherent, so their pixel boxes share a small bounding rectangle: the workgroup resolves its
// faces' (depth, face) minima in LDS with 64-bit LDS atomics and then merges the rectangle into the image with one
// global atomicMin per touched pixel, row-contiguous across lanes (memory-side global atomics cost one 64-B request
// per scattered lane: MI355X_MICROARCH.md "Global float atomics"). Workgroups whose rectangle exceeds the LDS tile fall
// back to per-pixel global atomics. Result = min over all faces of the key, i.e. identical to a direct scatter.
constexpr int SCATTER_BLOCK = 256;
constexpr int SCATTER_LANES_PER_FACE = 1;
constexpr int SCATTER_FACES_PER_BLOCK = SCATTER_BLOCK / SCATTER_LANES_PER_FACE;
constexpr int SCATTER_LDS_KEYS = 4096;   // 32 KiB


__device__ inline void scatter_block(const FaceNdc& fn, bool ok, int32_t face, const RasterOptions& o, uint64_t* keys) {
	__shared__ uint64_t s_keys[SCATTER_LDS_KEYS];
	__shared__ int s_box[4];
	int u0 = 0, u1 = -1, v0 = 0, v1 = -1;
	if (ok) ok = face_pixel_range(fn, o, u0, u1, v0, v1);
	if (threadIdx.x == 0) {
		s_box[0] = 0x7fffffff;
		s_box[1] = -1;
		s_box[2] = 0x7fffffff;
		s_box[3] = -1;
	}
	__syncthreads();
	{
		// wave-level min/max first: one LDS atomic per wave instead of 64 same-address atomics per wave
		int bu0 = ok ? u0 : 0x7fffffff, bu1 = ok ? u1 : -1, bv0 = ok ? v0 : 0x7fffffff, bv1 = ok ? v1 : -1;
#pragma unroll
		for (int d = 32; d >= 1; d >>= 1) {
			bu0 = min(bu0, __shfl_xor(bu0, d));
			bu1 = max(bu1, __shfl_xor(bu1, d));
			bv0 = min(bv0, __shfl_xor(bv0, d));
			bv1 = max(bv1, __shfl_xor(bv1, d));
		}
		if ((threadIdx.x & 63) == 0 && bu1 >= 0) {
			atomicMin(&s_box[0], bu0);
			atomicMax(&s_box[1], bu1);
			atomicMin(&s_box[2], bv0);
			atomicMax(&s_box[3], bv1);
		}
	}
	__syncthreads();
	const int bu0 = s_box[0], bv0 = s_box[2];
	const int bw = s_box[1] - bu0 + 1, bh = s_box[3] - bv0 + 1;
	if (bw <= 0 || bh <= 0) return;   // uniform: no face of this workgroup covers a pixel
	const bool staged = bw * bh <= SCATTER_LDS_KEYS;
	if (staged) {
		for (int i = threadIdx.x; i < bw * bh; i += SCATTER_BLOCK) s_keys[i] = EMPTY_KEY;
		__syncthreads();
	}
	// A13: the blur radius is compared against SQUARED NDC distances, so for a face whose blur-widened box has a squared
	// diagonal well below the radius every pixel in the box passes the distance test: skip computing it.
	bool near_all = false;
	if (ok) {
		const float w = (fmax3f(fn.x[0], fn.x[1], fn.x[2]) - fmin3f(fn.x[0], fn.x[1], fn.x[2])) + 2.f * o.blur;
		const float hh = (fmax3f(fn.y[0], fn.y[1], fn.y[2]) - fmin3f(fn.y[0], fn.y[1], fn.y[2])) + 2.f * o.blur;
		near_all = (w * w + hh * hh) < 0.5f * o.blur;
	}
	if (ok) {
		const float inv_w = rcp_rn(static_cast<float>(o.W)), inv_h = rcp_rn(static_cast<float>(o.H));
		const float inv_area = face_inv_area(fn);
		const int sub = static_cast<int>(threadIdx.x % SCATTER_LANES_PER_FACE);
		const int span_u = u1 - u0 + 1;
		const int count = span_u * (v1 - v0 + 1);
		for (int i = sub; i < count; i += SCATTER_LANES_PER_FACE) {
			const int v = v0 + i / span_u, u = u0 + i % span_u;
			{
				const float py = pixel_to_ndc_r(v, o.H, o.W, inv_h);
				const float px = pixel_to_ndc_r(u, o.W, o.H, inv_w);
				RasterHit h;
				const bool hit = near_all ? face_test<false>(fn, px, py, o.blur, o.perspective, o.clip_barycentric, o.cull_back_faces, h, inv_area)
				                          : face_test<true>(fn, px, py, o.blur, o.perspective, o.clip_barycentric, o.cull_back_faces, h, inv_area);
				if (!hit) continue;
				const unsigned long long key = raster_key(h.depth, face);
				if (staged)
					__hip_atomic_fetch_min(reinterpret_cast<unsigned long long*>(s_keys + (v - bv0) * bw + (u - bu0)), key, __ATOMIC_RELAXED,
					                       __HIP_MEMORY_SCOPE_WORKGROUP);
				else
					atomicMin(reinterpret_cast<unsigned long long*>(keys + static_cast<int64_t>(v) * o.W + u), key);
			}
		}
	}
	if (!staged) return;
	__syncthreads();
	for (int i = threadIdx.x; i < bw * bh; i += SCATTER_BLOCK) {
		const uint64_t k = s_keys[i];
		if (k == EMPTY_KEY) continue;
		const int64_t p = static_cast<int64_t>(bv0 + i / bw) * o.W + bu0 + i % bw;
		atomicMin(reinterpret_cast<unsigned long long*>(keys + p), static_cast<unsigned long long>(k));
	}
}

__global__ __launch_bounds__(SCATTER_BLOCK) void k_raster_scatter_ndc(const float* __restrict__ face_ndc, const uint8_t* __restrict__ mask,
                                                                      int64_t F, RasterOptions o, uint64_t* __restrict__ keys) {
	const int64_t f = static_cast<int64_t>(blockIdx.x) * SCATTER_FACES_PER_BLOCK + threadIdx.x / SCATTER_LANES_PER_FACE;
	FaceNdc fn{};
	bool ok = f < F && !(mask && !mask[f]);
	if (ok) fn = load_face_ndc(face_ndc, f);
	scatter_block(fn, ok, static_cast<int32_t>(f), o, keys);
}

nnrt_status launch_raster_scatter_ndc(const float* face_ndc, const uint8_t* mask, int64_t F, const RasterOptions& o, uint64_t* keys,
                                      hipStream_t stream) {
	if (F == 0) return NNRT_OK;
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
		s.ndc.project(v[i].x, v[i].y, v[i].z, &fn.x[i], &fn.y[i]);
		fn.z[i] = v[i].z;
		inlier |= (fn.y[i] >= s.min_y && fn.x[i] >= s.min_x && fn.y[i] <= s.max_y && fn.x[i] <= s.max_x);
	}
	return inlier;
}

__global__ __launch_bounds__(SCATTER_BLOCK) void k_raster_scatter_mesh(const float4* __restrict__ wpos, const int4* __restrict__ faces4,
                                                                       int64_t F, NdcSetup s, float near_clip, float far_clip, RasterOptions o,
                                                                       uint64_t* __restrict__ keys) {
	const int64_t f = static_cast<int64_t>(blockIdx.x) * SCATTER_FACES_PER_BLOCK + threadIdx.x / SCATTER_LANES_PER_FACE;
	FaceNdc fn{};
	const bool ok = f < F && project_mesh_face(wpos, faces4[f], s, near_clip, far_clip, fn);
	scatter_block(fn, ok, static_cast<int32_t>(f), o, keys);
}

nnrt_status launch_raster_scatter_mesh(const float4* wpos, const int4* faces4, int64_t F, const NdcSetup& s, float near_clip, float far_clip,
                                       const RasterOptions& o, uint64_t* keys, hipStream_t stream) {
	if (F == 0) return NNRT_OK;
	k_raster_scatter_mesh<<<static_cast<unsigned>(ceil_div(F, SCATTER_FACES_PER_BLOCK)), SCATTER_BLOCK, 0, stream>>>(wpos, faces4, F, s, near_clip, far_clip, o, keys);
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
	const float inv_w = rcp_rn(static_cast<float>(o.W)), inv_h = rcp_rn(static_cast<float>(o.H));
	const float inv_area = face_inv_area(fn);
	for (int v = v0; v <= v1; v++) {
		const float py = pixel_to_ndc_r(v, o.H, o.W, inv_h);
		for (int u = u0; u <= u1; u++) {
			const float px = pixel_to_ndc_r(u, o.W, o.H, inv_w);
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
