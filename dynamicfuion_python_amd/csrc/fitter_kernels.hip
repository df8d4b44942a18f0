// GN iteration kernels for gfx950 (DeformableMeshToImageFitter.cpp:111-275).
//
// k_fit_pixels fuses, per pixel, stages S3b-S10 of the reference loop: raster resolve, depth residual
// (ComputeDepthResiduals :331-390), rasterized-surface Jacobians (RasterizedSurfaceJacobiansImpl.h:114-200),
// pixel->node Jacobians (PixelVertexAnchorJacobiansImpl.h:179-363) and the block-diagonal data JtJ / Jt r reduction
// (DeformableMeshToImageFitterImpl.h:199-456). The reference materialises [P,12,6] pixel Jacobians, [P,3,19] rasterized
// Jacobians and [N,4000] node lists (capped: A4) and reduces each node serially. Here every 64-lane wavefront owns an
// 8x8 pixel block; it walks the distinct nodes its pixels touch (wave-uniform loop driven by a ballot), each lane builds
// its pixel's 6-dof Jacobian for that node, and the 27 products (21 JtJ upper-triangle entries + 6 J r) are summed over
// the wave in double with a transposing butterfly (permlane swaps + DPP, no LDS) and added to the node's fp64
// accumulator row with one 27-lane atomic. Products are rounded to float exactly as the reference forms them and
// summed in double, so the data term equals the exactly-summed reference data term (see DESIGN.md "Numerics") -- no
// intermediate tensors, no node-list cap, no LDS.
#include "fitter_kernels.hpp"

#ifndef NNRT_FIT_VARIANT
#define NNRT_FIT_VARIANT 0   // development timing builds only (tools/fit_variants.py): 0 = product
#endif

#if NNRT_FIT_VARIANT == 30
__device__ unsigned long long g_fit_stamps[2][1 << 17];
#define FSTAMP(k, i)                                                                                                          \
	do {                                                                                                                    \
		if ((threadIdx.x & 63) == 0) g_fit_stamps[k][(blockIdx.x * 4 + threadIdx.x / 64) * 8 + (i)] = __builtin_amdgcn_s_memrealtime(); \
	} while (0)
extern "C" int nnrt_dev_fit_stamps(int k, unsigned long long* host, int n) {
	return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_fit_stamps), sizeof(unsigned long long) * n, sizeof(unsigned long long) * (1 << 17) * k) ==
	               hipSuccess ? 0 : 1;
}
#else
#define FSTAMP(k, i) do {} while (0)
#endif

namespace nnrt {

constexpr int PIX_TILE = 16;
constexpr int PIX_BLOCK = PIX_TILE * PIX_TILE;

template <int MODE>
struct ModeTraits;
template <>
struct ModeTraits<NNRT_ITERATION_ALL> {
	static constexpr int S = 6, NH = 21, NACC = 27;
};
template <>
struct ModeTraits<NNRT_ITERATION_TRANSLATION_ONLY> {
	static constexpr int S = 3, NH = 6, NACC = 9;
};
template <>
struct ModeTraits<NNRT_ITERATION_ROTATION_ONLY> {
	static constexpr int S = 3, NH = 6, NACC = 9;
};

// ---- wavefront reduction helpers ----
template <int CTRL>
__device__ inline float dpp_f32(float x) {
	return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xf, 0xf, false));
}
template <int CTRL>
__device__ inline double dpp_f64(double x) {
	const uint64_t u = __builtin_bit_cast(uint64_t, x);
	const int lo = __builtin_amdgcn_update_dpp(0, static_cast<int>(u & 0xffffffffu), CTRL, 0xf, 0xf, false);
	const int hi = __builtin_amdgcn_update_dpp(0, static_cast<int>(u >> 32), CTRL, 0xf, 0xf, false);
	return __builtin_bit_cast(double, (static_cast<uint64_t>(static_cast<uint32_t>(hi)) << 32) | static_cast<uint32_t>(lo));
}
template <int CTRL, typename R>
__device__ inline R dpp_move(R x) {
	if constexpr (sizeof(R) == 4) return dpp_f32<CTRL>(x);
	else return dpp_f64<CTRL>(x);
}

// ---- wave sum of 32 per-lane values (transposing butterfly) ----
// Each exchange step halves the values a lane holds: lanes with the step's bit set keep the upper half of the values,
// the others the lower half, each adding its partner's copy. The two cross-row steps go first through gfx950's
// v_permlane32_swap / v_permlane16_swap
// swap(lo, hi) exchanges the upper half of `lo` with the lower half of `hi` (32 lanes, or the odd/even 16-lane rows),
// so after one add the lanes with the step's bit clear hold lo(l) + lo(l ^ d) and the others hi(l ^ d) + hi(l):
// a whole transposing step costs one swap per dword and one add, no selects. Rows then finish with DPP (8, 4, 2) and a
// quad_perm add (1). On return lanes 2i and 2i + 1 hold the wave total of value index i.
template <bool ROW16>
__device__ inline uint2 permlane_swap_u32(uint32_t lo, uint32_t hi) {
	if constexpr (ROW16) {
		const auto r = __builtin_amdgcn_permlane16_swap(lo, hi, false, false);
		return make_uint2(r[0], r[1]);
	} else {
		const auto r = __builtin_amdgcn_permlane32_swap(lo, hi, false, false);
		return make_uint2(r[0], r[1]);
	}
}
template <bool ROW16, typename R>
__device__ inline R swap_add(R lo, R hi) {
	if constexpr (sizeof(R) == 4) {
		const uint2 r = permlane_swap_u32<ROW16>(__builtin_bit_cast(uint32_t, lo), __builtin_bit_cast(uint32_t, hi));
		return __builtin_bit_cast(R, r.x) + __builtin_bit_cast(R, r.y);
	} else {
		const uint64_t a = __builtin_bit_cast(uint64_t, lo), b = __builtin_bit_cast(uint64_t, hi);
		const uint2 l = permlane_swap_u32<ROW16>(static_cast<uint32_t>(a), static_cast<uint32_t>(b));
		const uint2 h = permlane_swap_u32<ROW16>(static_cast<uint32_t>(a >> 32), static_cast<uint32_t>(b >> 32));
		const R x = __builtin_bit_cast(R, (static_cast<uint64_t>(h.x) << 32) | l.x);
		const R y = __builtin_bit_cast(R, (static_cast<uint64_t>(h.y) << 32) | l.y);
		return x + y;
	}
}

template <int D, int HALF, typename R>
__device__ inline void butterfly_row_step(R (&v)[32], bool upper) {
#pragma unroll
	for (int j = 0; j < HALF; j++) {
		const R lo = v[j], hi = v[j + HALF];
		const R from_above = dpp_move<0x100 + D>(lo);   // row_shl:D
		const R from_below = dpp_move<0x110 + D>(hi);   // row_shr:D
		v[j] = upper ? (hi + from_below) : (lo + from_above);
	}
}

template <typename R>
__device__ inline R wave_reduce32_swap(R (&v)[32], int lane) {
#pragma unroll
	for (int j = 0; j < 16; j++) v[j] = swap_add<false>(v[j], v[j + 16]);
#pragma unroll
	for (int j = 0; j < 8; j++) v[j] = swap_add<true>(v[j], v[j + 8]);
	butterfly_row_step<8, 4>(v, (lane & 8) != 0);
	butterfly_row_step<4, 2>(v, (lane & 4) != 0);
	butterfly_row_step<2, 1>(v, (lane & 2) != 0);
	return v[0] + dpp_move<0xB1>(v[0]);   // quad_perm [1,0,3,2]: lanes 2i, 2i+1 exchange
}

// ---- pass 1: per pixel (S3b-S9) -----------------------------------------------------------------------------------
// Resolves the raster winner, writes the residual / mask / face outputs and, for pixels that contribute to the data
// term, the compact per-pixel Jacobian record [dr/dV (9), dr/dn_l (3), rho (3), r] (4 x float4). The raster key is
// replaced by the contributing face (or EMPTY) for pass 2, which resets it.
template <int MODE>
__global__ __launch_bounds__(PIX_BLOCK) void k_pixel_jacobians(FitPixelArgs a) {

	// XCD-aware tile order: consecutive workgroups are dealt round-robin over the 8 XCDs, so give each XCD a contiguous
	// band of tiles (neighbouring tiles share vertices, anchors and nodes -> L2 reuse within the XCD).
	const int tiles = a.tiles_x * a.tiles_y;
	const int per_xcd = (tiles + 7) / 8;
	const int b = blockIdx.x;
	const int tile = (b % 8) * per_xcd + b / 8;
	const int tu = tile % a.tiles_x, tv = tile / a.tiles_x;
	// wave w of the workgroup owns the 8x8 quadrant (w & 1, w >> 1): compact pixel sets touch the fewest nodes
	const int lane = static_cast<int>(threadIdx.x & 63), wave = static_cast<int>(threadIdx.x >> 6);
	const int u = tu * PIX_TILE + (wave & 1) * 8 + (lane & 7);
	const int v = tv * PIX_TILE + (wave >> 1) * 8 + (lane >> 3);
	const bool in_image = tile < tiles && u < a.W && v < a.H;
	const int64_t p = static_cast<int64_t>(v) * a.W + u;

	int vid[3] = {0, 0, 0};
	float dr_dV[9];
	float rn[3] = {0.f, 0.f, 0.f}, rho[3] = {0.f, 0.f, 0.f};

	FSTAMP(0, 0);
	if (in_image) {
		const uint64_t key = a.keys[p];
		int32_t face = -1;
		RasterHit h{0.f, 0.f, 0.f, 0.f, 0.f};
		f3 V3[3], N3[3];
		FaceNdc fn;
		const float px = pixel_to_ndc(u, a.W, a.H), py = pixel_to_ndc(v, a.H, a.W);
		if (key != EMPTY_KEY) {
			face = static_cast<int32_t>(key & 0xffffffffu);
			const int4 fi = a.faces4[face];
			vid[0] = fi.x;
			vid[1] = fi.y;
			vid[2] = fi.z;
#pragma unroll
			for (int i = 0; i < 3; i++) {
				const float4 wp = a.wpos[vid[i]];
				const float4 wn = a.wnrm[vid[i]];
				V3[i] = make3(wp.x, wp.y, wp.z);
				N3[i] = make3(wn.x, wn.y, wn.z);
				a.ndc.ndc.project(V3[i].x, V3[i].y, V3[i].z, &fn.x[i], &fn.y[i]);
				fn.z[i] = V3[i].z;
			}
			// the scatter accepted this face for this pixel after the full test; re-resolving needs no distance test
			if (!face_test<false>(fn, px, py, a.blur, a.perspective, false, true, h)) face = -1;
		}
		FSTAMP(0, 1);
		// ---- ComputeDepthResiduals (:331-390) ----
		const float depth = face >= 0 ? h.depth : -1.f;
		const bool rendered_valid = depth > 0 && depth < a.max_depth;
		f3 nl = make3(0.f, 0.f, 0.f), prast = make3(0.f, 0.f, 0.f);
		if (face >= 0) {
			float acc;
			acc = 0.0f;
			acc += h.b0 * N3[0].x;
			acc += h.b1 * N3[1].x;
			acc += h.b2 * N3[2].x;
			nl.x = acc;
			acc = 0.0f;
			acc += h.b0 * N3[0].y;
			acc += h.b1 * N3[1].y;
			acc += h.b2 * N3[2].y;
			nl.y = acc;
			acc = 0.0f;
			acc += h.b0 * N3[0].z;
			acc += h.b1 * N3[1].z;
			acc += h.b2 * N3[2].z;
			nl.z = acc;
		}
		if (rendered_valid) {
			prast = make3((static_cast<float>(u) - a.pix.cx) * depth / a.pix.fx, (static_cast<float>(v) - a.pix.cy) * depth / a.pix.fy, depth);
		}
		const float4 qr = a.ref_points[p];
		const bool ref_valid = qr.w != 0.f;
		const f3 q = make3(qr.x, qr.y, qr.z);
		const bool mask = ref_valid && rendered_valid;
		const f3 d = sub3(prast, q);   // point map vector w_l - o_l
		float dist = dot3(nl, d);
		if (!mask) dist = 0.0f;
		float residual = dist;
		if (a.use_tukey) {
			const float c = a.tukey_c;
			const float c6 = (c * c / 6.f);
			const float qq = dist / c;
			const float left = 1.f - (qq * qq);
			residual = c6 * (1.f - left * left * left);
			if (dist <= c) residual = c6;   // (:384-385 as written: A8)
		}
		a.residuals[p] = residual;
		a.residual_mask[p] = mask ? 1 : 0;
		a.pixel_face[p] = face;

		bool contributes = mask;
		f3 dr_dwl = nl, dr_dnl = d;
		if (contributes && a.use_tukey) {
			const float r = dot3(nl, d);
			if (fabsf(r) > a.tukey_c) contributes = false;
			const float qq = r / a.tukey_c;
			float psi = 1 - qq * qq;
			psi = r * psi * psi;
			dr_dnl = make3(psi * d.x, psi * d.y, psi * d.z);
			dr_dwl = make3(psi * nl.x, psi * nl.y, psi * nl.z);
		}
		if (contributes) {
			// ---- rasterized surface Jacobians (RasterizedSurfaceJacobiansImpl.h:114-200) ----
			rho[0] = h.b0;
			rho[1] = h.b1;
			rho[2] = h.b2;
			float A, sa[3], drho[3] = {0.f, 0.f, 0.f};
			A = spa_cw(fn.x[0], fn.y[0], fn.x[1], fn.y[1], fn.x[2], fn.y[2]) + K_EPSILON;
			if (a.perspective) {
				sa[0] = spa_cw(px, py, fn.x[1], fn.y[1], fn.x[2], fn.y[2]);
				sa[1] = spa_cw(px, py, fn.x[2], fn.y[2], fn.x[0], fn.y[0]);
				sa[2] = spa_cw(px, py, fn.x[0], fn.y[0], fn.x[1], fn.y[1]);
				const float inv_A = rcp_rn(A);
#pragma unroll
				for (int i = 0; i < 3; i++) drho[i] = div_rn(sa[i], A, inv_A);
			} else {
#pragma unroll
				for (int i = 0; i < 3; i++) sa[i] = rho[i] * A;
			}
			// d rho / d ndc (BarycentricCoordinateJacobians.h:85-181)
			const float den = A * A + K_EPSILON;
			const float dA[3][2] = {{fn.y[1] - fn.y[2], fn.x[2] - fn.x[1]}, {fn.y[2] - fn.y[0], fn.x[0] - fn.x[2]}, {fn.y[0] - fn.y[1], fn.x[1] - fn.x[0]}};
			// sub-area derivatives: (p, va, vb) -> d/dva = (vb.y - p.y, p.x - vb.x), d/dvb = (p.y - va.y, va.x - p.x)
			const float s0a[2] = {fn.y[2] - py, px - fn.x[2]}, s0b[2] = {py - fn.y[1], fn.x[1] - px};   // (p, v1, v2)
			const float s1a[2] = {fn.y[0] - py, px - fn.x[0]}, s1b[2] = {py - fn.y[2], fn.x[2] - px};   // (p, v2, v0)
			const float s2a[2] = {fn.y[1] - py, px - fn.x[1]}, s2b[2] = {py - fn.y[0], fn.x[0] - px};   // (p, v0, v1)
			const float inv_den = rcp_rn(den);
			float Dn[3][3][2];
#pragma unroll
			for (int c = 0; c < 2; c++) {
				Dn[0][0][c] = div_rn(-sa[0] * dA[0][c], den, inv_den);
				Dn[1][0][c] = div_rn(A * s0a[c] - sa[0] * dA[1][c], den, inv_den);
				Dn[2][0][c] = div_rn(A * s0b[c] - sa[0] * dA[2][c], den, inv_den);
				Dn[0][1][c] = div_rn(A * s1b[c] - sa[1] * dA[0][c], den, inv_den);
				Dn[1][1][c] = div_rn(-sa[1] * dA[1][c], den, inv_den);
				Dn[2][1][c] = div_rn(A * s1a[c] - sa[1] * dA[2][c], den, inv_den);
				Dn[0][2][c] = div_rn(A * s2a[c] - sa[2] * dA[0][c], den, inv_den);
				Dn[1][2][c] = div_rn(A * s2b[c] - sa[2] * dA[1][c], den, inv_den);
				Dn[2][2][c] = div_rn(-sa[2] * dA[2][c], den, inv_den);
			}
			// perspective-correction factors first (RasterizedSurfaceJacobiansImpl.h:217-284), so the 3x9 Jacobian can be
			// streamed one face vertex (3 columns) at a time: same expressions, far fewer live registers
			float Pd[3][3], Pz[3][3];
			if (a.perspective) {
				const float z0 = V3[0].z, z1 = V3[1].z, z2 = V3[2].z;
				const float v12 = z1 * z2, v02 = z0 * z2, v01 = z0 * z1;
				const float n0 = drho[0] * v12, n1 = drho[1] * v02, n2 = drho[2] * v01;
				const float dd = fmaxf(n0 + n1 + n2, K_EPSILON);
				const float dd2 = dd * dd;
				const float pd[3][3] = {{(dd - n0) * v12, -n0 * v02, -n0 * v01}, {-n1 * v12, (dd - n1) * v02, -n1 * v01},
				                        {-n2 * v12, -n2 * v02, (dd - n2) * v01}};
				const float pz0 = drho[1] * z2 + z1 * drho[2];
				const float pz1 = drho[0] * z2 + z0 * drho[2];
				const float pz2 = drho[0] * z1 + z0 * drho[1];
				const float pz[3][3] = {{-n0 * pz0, dd * drho[0] * z2 - n0 * pz1, dd * drho[0] * z1 - n0 * pz2},
				                        {dd * drho[1] * z2 - n1 * pz0, -n1 * pz1, dd * drho[1] * z0 - n1 * pz2},
				                        {dd * drho[2] * z1 - n2 * pz0, dd * drho[2] * z0 - n2 * pz1, -n2 * pz2}};
				const float inv_dd2 = rcp_rn(dd2);
#pragma unroll
				for (int r = 0; r < 3; r++)
#pragma unroll
					for (int c = 0; c < 3; c++) {
						Pd[r][c] = div_rn(pd[r][c], dd2, inv_dd2);
						Pz[r][c] = div_rn(pz[r][c], dd2, inv_dd2);
					}
			}
			// dr/dV = dr/dwl * dwl/dV + dr/dnl * dnl/dV ; dr/dN = dr/dnl (rho (x) I)
			const float rw[3] = {dr_dwl.x, dr_dwl.y, dr_dwl.z};
			rn[0] = dr_dnl.x;
			rn[1] = dr_dnl.y;
			rn[2] = dr_dnl.z;
#pragma unroll
			for (int i = 0; i < 3; i++) {
				const float z = V3[i].z;
				const float z2 = z * z;
				const float P0[3] = {a.ndc.ndc.fx / z, 0.f, -a.ndc.ndc.fx * V3[i].x / z2};
				const float P1[3] = {0.f, a.ndc.ndc.fy / z, -a.ndc.ndc.fy * V3[i].y / z2};
				float Jc[3][3];   // rows of the 3x9 Jacobian, columns 3i .. 3i+2
#pragma unroll
				for (int r = 0; r < 3; r++)
#pragma unroll
					for (int c = 0; c < 3; c++) Jc[r][c] = Dn[i][r][0] * P0[c] + Dn[i][r][1] * P1[c];
				if (a.perspective) {
					float J2[3][3];
#pragma unroll
					for (int r = 0; r < 3; r++)
#pragma unroll
						for (int c = 0; c < 3; c++) J2[r][c] = (Pd[r][0] * Jc[0][c] + Pd[r][1] * Jc[1][c]) + Pd[r][2] * Jc[2][c];
#pragma unroll
					for (int r = 0; r < 3; r++) J2[r][2] += Pz[r][i];
#pragma unroll
					for (int r = 0; r < 3; r++)
#pragma unroll
						for (int c = 0; c < 3; c++) Jc[r][c] = J2[r][c];
				}
#pragma unroll
				for (int c = 0; c < 3; c++) {
					float w_rc[3], n_rc[3];
#pragma unroll
					for (int r = 0; r < 3; r++) {
						const f3 Vk[3] = {V3[0], V3[1], V3[2]};
						const f3 Nk[3] = {N3[0], N3[1], N3[2]};
						const float vr0 = r == 0 ? Vk[0].x : (r == 1 ? Vk[0].y : Vk[0].z);
						const float vr1 = r == 0 ? Vk[1].x : (r == 1 ? Vk[1].y : Vk[1].z);
						const float vr2 = r == 0 ? Vk[2].x : (r == 1 ? Vk[2].y : Vk[2].z);
						const float nr0 = r == 0 ? Nk[0].x : (r == 1 ? Nk[0].y : Nk[0].z);
						const float nr1 = r == 0 ? Nk[1].x : (r == 1 ? Nk[1].y : Nk[1].z);
						const float nr2 = r == 0 ? Nk[2].x : (r == 1 ? Nk[2].y : Nk[2].z);
						w_rc[r] = (vr0 * Jc[0][c] + vr1 * Jc[1][c]) + vr2 * Jc[2][c];
						if (c == r) w_rc[r] += rho[i];
						n_rc[r] = (nr0 * Jc[0][c] + nr1 * Jc[1][c]) + nr2 * Jc[2][c];
					}
					const float x = (rw[0] * w_rc[0] + rw[1] * w_rc[1]) + rw[2] * w_rc[2];
					const float y = (rn[0] * n_rc[0] + rn[1] * n_rc[1]) + rn[2] * n_rc[2];
					dr_dV[3 * i + c] = x + y;
				}
			}
			float4* rec = a.records + 4 * p;
			rec[0] = make_float4(dr_dV[0], dr_dV[1], dr_dV[2], dr_dV[3]);
			rec[1] = make_float4(dr_dV[4], dr_dV[5], dr_dV[6], dr_dV[7]);
			rec[2] = make_float4(dr_dV[8], rn[0], rn[1], rn[2]);
			rec[3] = make_float4(rho[0], rho[1], rho[2], residual);
		}
		a.keys[p] = contributes ? static_cast<uint64_t>(static_cast<uint32_t>(face)) : EMPTY_KEY;
	}
	FSTAMP(0, 2);
}

// ---- pass 2: per node (S10) ------------------------------------------------------------------------------------
// 8x8 pixels per wave. For each distinct node of the wave's pixels (wave-uniform loop driven by a ballot), every lane
// forms its pixel's 6-dof Jacobian for that node from the pass-1 record and the face vertices' warped-Jacobian rows;
// JJᵀ and J r are summed over the wave and added to the node's fp64 accumulator row.
template <int MODE, int MAXK>
__global__ __launch_bounds__(PIX_BLOCK) void k_node_reduce(FitPixelArgs a) {
	using T = ModeTraits<MODE>;
	constexpr int S = T::S;
	static_assert(T::NACC <= 32, "accumulator row must fit the 32-value wave reduction");

	// XCD-aware tile order: consecutive workgroups are dealt round-robin over the 8 XCDs, so give each XCD a contiguous
	// band of tiles (neighbouring tiles share vertices, anchors and nodes -> L2 reuse within the XCD).
	const int tiles = a.tiles_x * a.tiles_y;
	const int per_xcd = (tiles + 7) / 8;
	const int b = blockIdx.x;
	const int tile = (b % 8) * per_xcd + b / 8;
	const int tu = tile % a.tiles_x, tv = tile / a.tiles_x;
	// wave w of the workgroup owns the 8x8 quadrant (w & 1, w >> 1): compact pixel sets touch the fewest nodes
	const int lane = static_cast<int>(threadIdx.x & 63), wave = static_cast<int>(threadIdx.x >> 6);
	const int u = tu * PIX_TILE + (wave & 1) * 8 + (lane & 7);
	const int v = tv * PIX_TILE + (wave >> 1) * 8 + (lane >> 3);
	const bool in_image = tile < tiles && u < a.W && v < a.H;
	const int64_t p = static_cast<int64_t>(v) * a.W + u;

	// per-lane inputs of the wave-level node loop below
	uint32_t pending = 0;   // bit 8*fv + k: anchor k of face vertex fv still to be reduced
	int vid[3] = {0, 0, 0};
	int anc[3][MAXK];
	float dr_dV[9];
	float rn[3] = {0.f, 0.f, 0.f}, rho[3] = {0.f, 0.f, 0.f};
	float r_used = 0.f;
#if NNRT_FIT_VARIANT == 16 || NNRT_FIT_VARIANT == 17
	float cj[3][MAXK][S];   // per anchor slot: this pixel's contribution to the slot node's Jacobian
#pragma unroll
	for (int fv = 0; fv < 3; fv++)
#pragma unroll
		for (int k = 0; k < MAXK; k++)
#pragma unroll
			for (int c = 0; c < S; c++) cj[fv][k][c] = 0.f;
#endif
#pragma unroll
	for (int c = 0; c < 9; c++) dr_dV[c] = 0.f;
#pragma unroll
	for (int fv = 0; fv < 3; fv++)
#pragma unroll
		for (int k = 0; k < MAXK; k++) anc[fv][k] = -1;

	FSTAMP(1, 0);
	if (in_image) {
		const uint64_t key = a.keys[p];
		a.keys[p] = EMPTY_KEY;   // ready for the next iteration's scatter
		if (key != EMPTY_KEY) {
			const int face = static_cast<int>(key & 0xffffffffu);
			const int4 fi = a.faces4[face];
			vid[0] = fi.x;
			vid[1] = fi.y;
			vid[2] = fi.z;
			const int KA = a.anchor_count;
#pragma unroll
			for (int fv = 0; fv < 3; fv++)
#pragma unroll
				for (int k = 0; k < MAXK; k++) {
					const int n = (k < KA) ? a.anchors[static_cast<int64_t>(vid[fv]) * KA + k] : -1;
					anc[fv][k] = n;
					if (n >= 0) pending |= 1u << (8 * fv + k);
				}
			const float4* rec = a.records + 4 * p;
			const float4 r0 = rec[0], r1 = rec[1], r2 = rec[2], r3 = rec[3];
			dr_dV[0] = r0.x;
			dr_dV[1] = r0.y;
			dr_dV[2] = r0.z;
			dr_dV[3] = r0.w;
			dr_dV[4] = r1.x;
			dr_dV[5] = r1.y;
			dr_dV[6] = r1.z;
			dr_dV[7] = r1.w;
			dr_dV[8] = r2.x;
			rn[0] = r2.y;
			rn[1] = r2.z;
			rn[2] = r2.w;
			rho[0] = r3.x;
			rho[1] = r3.y;
			rho[2] = r3.z;
			r_used = r3.w;
#if NNRT_FIT_VARIANT == 16 || NNRT_FIT_VARIANT == 17
			pending = 0;
#pragma unroll
			for (int fv = 0; fv < 3; fv++) {
				const f3 dv = make3(dr_dV[3 * fv], dr_dV[3 * fv + 1], dr_dV[3 * fv + 2]);
				const f3 dn = make3(rn[0] * rho[fv], rn[1] * rho[fv], rn[2] * rho[fv]);
#pragma unroll
				for (int k = 0; k < MAXK; k++) {
					bool later_duplicate = false;
#pragma unroll
					for (int k2 = k + 1; k2 < MAXK; k2++) later_duplicate |= anc[fv][k2] == anc[fv][k];
					if (anc[fv][k] < 0 || later_duplicate) continue;
					pending |= 1u << (8 * fv + k);
					const int64_t vk = static_cast<int64_t>(vid[fv]) * KA + k;
					const float4 jv = a.jv[vk];
					float* c = cj[fv][k];
					if (MODE == NNRT_ITERATION_TRANSLATION_ONLY) {
						c[0] = dv.x * jv.w;
						c[1] = dv.y * jv.w;
						c[2] = dv.z * jv.w;
					} else {
						const float4 jn = a.jn[vk];
						const f3 t1 = row_times_skew(dv, make3(jv.x, jv.y, jv.z));
						const f3 t2 = row_times_skew(dn, make3(jn.x, jn.y, jn.z));
						c[0] = t1.x + t2.x;
						c[1] = t1.y + t2.y;
						c[2] = t1.z + t2.z;
						if (MODE == NNRT_ITERATION_ALL) {
							c[3 % S] = dv.x * jv.w;
							c[4 % S] = dv.y * jv.w;
							c[5 % S] = dv.z * jv.w;
						}
					}
				}
			}
#endif
		}
	}

	// ---- wave-level reduction over the distinct nodes of this wave's pixels ----
	// Per node, a pixel's Jacobian sums the contributions of every face vertex anchored to it (fv ascending, the
	// reference's association keeps the LAST matching anchor slot of a vertex: AssociateFacesWithAnchors), then JJ^T
	// and J r are added to the node's accumulator row.
	if (__ballot(r_used == 1.2345f) == 777ull) a.acc[0] = 0;   // anchors the stamp after the prologue loads
	FSTAMP(1, 1);
	const int KA = a.anchor_count;
	// this lane's Jacobian with respect to `node` (zero if none of its face's vertices is anchored to it); clears the
	// node's pending slots. Contributions are summed in face-vertex order, the reference's per-node accumulation order.
	// Slots of this lane anchored to `node`: per face vertex the LAST matching anchor slot (AssociateFacesWithAnchors),
	// -1 if none; clears them from `pending`.
	auto node_slots = [&](int node, int (&kk)[3]) {
#pragma unroll
		for (int fv = 0; fv < 3; fv++) {
			kk[fv] = -1;
#pragma unroll
			for (int k = 0; k < MAXK; k++) {
				const uint32_t bit = 1u << (8 * fv + k);
				if ((pending & bit) && anc[fv][k] == node) {
					pending &= ~bit;
					kk[fv] = k;
				}
			}
		}
	};
	struct SlotData {
		float4 jv[3], jn[3];
	};
	auto load_slots = [&](const int (&kk)[3], SlotData& d) {
#pragma unroll
		for (int fv = 0; fv < 3; fv++) {
			d.jv[fv] = make_float4(0.f, 0.f, 0.f, 0.f);
			d.jn[fv] = make_float4(0.f, 0.f, 0.f, 0.f);
			if (kk[fv] >= 0) {
				const int64_t vk = static_cast<int64_t>(vid[fv]) * KA + kk[fv];
				d.jv[fv] = a.jv[vk];
				if (MODE != NNRT_ITERATION_TRANSLATION_ONLY) d.jn[fv] = a.jn[vk];
			}
		}
	};
	// this lane's Jacobian with respect to the node whose slots are kk: contributions summed in face-vertex order,
	// the reference's per-node accumulation order; zero if no vertex of the lane's face is anchored to the node
	auto slot_jacobian = [&](const int (&kk)[3], const SlotData& d, float (&Jn)[S]) {
		float jr[3] = {0.f, 0.f, 0.f}, jt[3] = {0.f, 0.f, 0.f};
#pragma unroll
		for (int fv = 0; fv < 3; fv++) {
			if (kk[fv] < 0) continue;
			const float4 jv = d.jv[fv];
			const f3 dv = make3(dr_dV[3 * fv], dr_dV[3 * fv + 1], dr_dV[3 * fv + 2]);
			if (MODE != NNRT_ITERATION_ROTATION_ONLY) {
				jt[0] += dv.x * jv.w;
				jt[1] += dv.y * jv.w;
				jt[2] += dv.z * jv.w;
			}
			if (MODE != NNRT_ITERATION_TRANSLATION_ONLY) {
				const float4 jn = d.jn[fv];
				const f3 dn = make3(rn[0] * rho[fv], rn[1] * rho[fv], rn[2] * rho[fv]);
				const f3 t1 = row_times_skew(dv, make3(jv.x, jv.y, jv.z));
				const f3 t2 = row_times_skew(dn, make3(jn.x, jn.y, jn.z));
				jr[0] += t1.x + t2.x;
				jr[1] += t1.y + t2.y;
				jr[2] += t1.z + t2.z;
			}
		}
		if (MODE == NNRT_ITERATION_ALL) {
			Jn[0] = jr[0];
			Jn[1] = jr[1];
			Jn[2] = jr[2];
			Jn[3 % S] = jt[0];
			Jn[4 % S] = jt[1];
			Jn[5 % S] = jt[2];
		} else if (MODE == NNRT_ITERATION_TRANSLATION_ONLY) {
			Jn[0] = jt[0];
			Jn[1] = jt[1];
			Jn[2] = jt[2];
		} else {
			Jn[0] = jr[0];
			Jn[1] = jr[1];
			Jn[2] = jr[2];
		}
	};
	auto node_jacobian = [&](int node, float (&Jn)[S]) {
		int kk[3];
		SlotData d;
		node_slots(node, kk);
		load_slots(kk, d);
		slot_jacobian(kk, d, Jn);
	};
	// wave-uniform: the first pending node of the first lane that still has one (-1 when the wave is done)
	auto next_node = [&]() -> int {
		const uint64_t active = __ballot(pending != 0u);
		if (active == 0) return -1;
		const int leader = __ffsll(static_cast<unsigned long long>(active)) - 1;
		int mine = -1;
#pragma unroll
		for (int fv = 2; fv >= 0; fv--)
#pragma unroll
			for (int k = MAXK - 1; k >= 0; k--)
				if ((pending >> (8 * fv + k)) & 1u) mine = anc[fv][k];
		return __shfl(mine, leader);
	};
#if NNRT_FIT_VARIANT == 16 || NNRT_FIT_VARIANT == 17
	// Jacobian for `node` from the precomputed slot contributions (rotation part first for mode ALL, as cj is laid out)
	auto pre_jacobian = [&](int node, float (&Jn)[S]) {
		float Jv[S];
#pragma unroll
		for (int c = 0; c < S; c++) Jv[c] = 0.f;
#pragma unroll
		for (int fv = 0; fv < 3; fv++)
#pragma unroll
			for (int k = 0; k < MAXK; k++) {
				const uint32_t bit = 1u << (8 * fv + k);
				const bool m = (pending & bit) && anc[fv][k] == node;
				if (m) pending &= ~bit;
#pragma unroll
				for (int c = 0; c < S; c++) Jv[c] = m ? Jv[c] + cj[fv][k][c] : Jv[c];
			}
#pragma unroll
		for (int c = 0; c < S; c++) Jn[c] = Jv[c];
	};
#endif
#if NNRT_FIT_VARIANT == 19
	if (__ballot(pending != 0u) == 12345ull) a.acc[0] = r_used + dr_dV[0] + rn[0] + rho[0] + anc[0][0];   // keep loads live
	pending = 0;
#endif
#if NNRT_FIT_VARIANT == 16
	constexpr int XS16 = 17;
	__shared__ double s_x16[PIX_BLOCK / 64][64 * XS16];
	double* xw16 = s_x16[wave];
	while (true) {
		const int nodeA = next_node();
		if (nodeA < 0) break;
		float JA[S], JB[S];
		pre_jacobian(nodeA, JA);
		const int nodeB = next_node();
#pragma unroll
		for (int c = 0; c < S; c++) JB[c] = 0.f;
		if (nodeB >= 0) pre_jacobian(nodeB, JB);
		double* row = xw16 + lane * XS16;
#pragma unroll
		for (int c = 0; c < 8; c++) {
			row[c] = c < S ? static_cast<double>(JA[c < S ? c : 0]) : (c == S ? static_cast<double>(r_used) : 0.0);
			row[8 + c] = c < S ? static_cast<double>(JB[c < S ? c : 0]) : (c == S ? static_cast<double>(r_used) : 0.0);
		}
		__builtin_amdgcn_wave_barrier();
		typedef double d4 __attribute__((ext_vector_type(4)));
		d4 C = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
		for (int m = 0; m < 16; m++) {
			const double x = xw16[(4 * m + (lane >> 4)) * XS16 + (lane & 15)];
			C = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, C, 0, 0, 0);
		}
		__builtin_amdgcn_wave_barrier();
		const int col = lane & 15;
#pragma unroll
		for (int i = 0; i < 4; i++) {
			const int rw = (lane >> 4) + 4 * i;
			if ((rw >> 3) != (col >> 3)) continue;
			const int node = (rw >> 3) ? nodeB : nodeA;
			const int r0 = rw & 7, c0 = col & 7;
			int idx = -1;
			if (r0 < S && c0 < S && r0 <= c0) idx = r0 * S - (r0 * (r0 - 1)) / 2 + (c0 - r0);
			else if (r0 < S && c0 == S) idx = T::NH + r0;
			if (idx >= 0 && node >= 0) atomicAdd(a.acc + static_cast<int64_t>(node) * ACC_STRIDE + idx, C[i]);
		}
	}
#elif NNRT_FIT_VARIANT == 17
	while (true) {
		const int node = next_node();
		if (node < 0) break;
		float Jn[S];
		pre_jacobian(node, Jn);
		double vals[32];
		int e = 0;
#pragma unroll
		for (int c0 = 0; c0 < S; c0++)
#pragma unroll
			for (int c1 = c0; c1 < S; c1++) vals[e++] = static_cast<double>(Jn[c0] * Jn[c1]);
#pragma unroll
		for (int c = 0; c < S; c++) vals[T::NH + c] = static_cast<double>(Jn[c] * r_used);
#pragma unroll
		for (int c = T::NACC; c < 32; c++) vals[c] = 0.0;
		const double total = wave_reduce32_swap(vals, lane);
		const int idx = (lane & 1) ? 32 : (lane >> 1);
		if (idx < T::NACC) atomicAdd(a.acc + static_cast<int64_t>(node) * ACC_STRIDE + idx, total);
	}
#elif NNRT_FIT_VARIANT == 11
	// ---- node pairs through the FP64 matrix core ----
	// X (64 pixels x 16) = [J_A, r, 0 | J_B, r, 0] per lane, staged in LDS; XᵀX over the wave's 64 pixels by 16
	// v_mfma_f64_16x16x4_f64 (products of float Jacobian entries are exact in double, sums in double). Diagonal 8x8
	// blocks hold JJᵀ (rows/cols < S) and J r (column S) of node A and node B.
	constexpr int XS = 17;   // row stride in doubles (136 B: b64-aligned, spreads the rows over the LDS banks)
	__shared__ double s_x[PIX_BLOCK / 64][64 * XS];
	double* xw = s_x[wave];
	while (true) {
		const int nodeA = next_node();
		if (nodeA < 0) break;
		// both nodes' slot searches first, then all their loads in flight together
		int kkA[3], kkB[3] = {-1, -1, -1};
		node_slots(nodeA, kkA);
		const int nodeB = next_node();
		if (nodeB >= 0) node_slots(nodeB, kkB);
		SlotData dA, dB;
		load_slots(kkA, dA);
		load_slots(kkB, dB);
		float JA[S], JB[S];
		slot_jacobian(kkA, dA, JA);
		slot_jacobian(kkB, dB, JB);
		double* row = xw + lane * XS;
#pragma unroll
		for (int c = 0; c < 8; c++) {
			row[c] = c < S ? static_cast<double>(JA[c < S ? c : 0]) : (c == S ? static_cast<double>(r_used) : 0.0);
			row[8 + c] = c < S ? static_cast<double>(JB[c < S ? c : 0]) : (c == S ? static_cast<double>(r_used) : 0.0);
		}
		__builtin_amdgcn_wave_barrier();
		typedef double d4 __attribute__((ext_vector_type(4)));
		d4 C = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
		for (int m = 0; m < 16; m++) {
			const double x = xw[(4 * m + (lane >> 4)) * XS + (lane & 15)];
			C = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, C, 0, 0, 0);
		}
		__builtin_amdgcn_wave_barrier();
		// lane holds C[row = (lane >> 4) + 4 i][col = lane & 15], i = 0..3
		const int col = lane & 15;
#pragma unroll
		for (int i = 0; i < 4; i++) {
			const int rw = (lane >> 4) + 4 * i;
			if ((rw >> 3) != (col >> 3)) continue;
			const int node = (rw >> 3) ? nodeB : nodeA;
			const int r0 = rw & 7, c0 = col & 7;
			int idx = -1;
			if (r0 < S && c0 < S && r0 <= c0) idx = r0 * S - (r0 * (r0 - 1)) / 2 + (c0 - r0);
			else if (r0 < S && c0 == S) idx = T::NH + r0;
			if (idx >= 0 && node >= 0) atomicAdd(a.acc + static_cast<int64_t>(node) * ACC_STRIDE + idx, C[i]);
		}
	}
#elif NNRT_FIT_VARIANT == 13
	// software-pipelined: the next node's slot loads are in flight while the current node is reduced
	int nodeA = next_node();
	int kkA[3] = {-1, -1, -1};
	SlotData dA;
	if (nodeA >= 0) {
		node_slots(nodeA, kkA);
		load_slots(kkA, dA);
	}
	while (nodeA >= 0) {
		const int nodeB = next_node();
		int kkB[3] = {-1, -1, -1};
		SlotData dB;
		if (nodeB >= 0) {
			node_slots(nodeB, kkB);
			load_slots(kkB, dB);
		}
		float Jn[S];
		slot_jacobian(kkA, dA, Jn);
		double vals[32];
		int e = 0;
#pragma unroll
		for (int c0 = 0; c0 < S; c0++)
#pragma unroll
			for (int c1 = c0; c1 < S; c1++) vals[e++] = static_cast<double>(Jn[c0] * Jn[c1]);
#pragma unroll
		for (int c = 0; c < S; c++) vals[T::NH + c] = static_cast<double>(Jn[c] * r_used);
#pragma unroll
		for (int c = T::NACC; c < 32; c++) vals[c] = 0.0;
		const double total = wave_reduce32_swap(vals, lane);
		const int idx = (lane & 1) ? 32 : (lane >> 1);
		if (idx < T::NACC) atomicAdd(a.acc + static_cast<int64_t>(nodeA) * ACC_STRIDE + idx, total);
		nodeA = nodeB;
#pragma unroll
		for (int fv = 0; fv < 3; fv++) kkA[fv] = kkB[fv];
		dA = dB;
	}
#else
	while (true) {
		const int node = next_node();
		if (node < 0) break;
		float Jn[S];
		node_jacobian(node, Jn);
		// products rounded to float as the reference forms them (lanes without the node hold Jn = 0 -> 0 products),
		// summed in double over the wave and across waves
		double vals[32];
		int e = 0;
#pragma unroll
		for (int c0 = 0; c0 < S; c0++)
#pragma unroll
			for (int c1 = c0; c1 < S; c1++) vals[e++] = static_cast<double>(Jn[c0] * Jn[c1]);
#pragma unroll
		for (int c = 0; c < S; c++) vals[T::NH + c] = static_cast<double>(Jn[c] * r_used);
#pragma unroll
		for (int c = T::NACC; c < 32; c++) vals[c] = 0.0;
		const double total = wave_reduce32_swap(vals, lane);
		const int idx = (lane & 1) ? 32 : (lane >> 1);   // lanes 2i, 2i+1 hold entry i
#if NNRT_FIT_VARIANT == 18
		if (idx < T::NACC && total == 1234.5) a.acc[idx] = total;
#else
		if (idx < T::NACC) atomicAdd(a.acc + static_cast<int64_t>(node) * ACC_STRIDE + idx, total);
#endif
	}
#endif
	FSTAMP(1, 2);
}

nnrt_status launch_fit_pixels(int mode, const FitPixelArgs& args, hipStream_t stream) {
	const int tiles = args.tiles_x * args.tiles_y;
	const unsigned grid = static_cast<unsigned>(((tiles + 7) / 8) * 8);
	switch (mode) {
		case NNRT_ITERATION_ALL: k_pixel_jacobians<NNRT_ITERATION_ALL><<<grid, PIX_BLOCK, 0, stream>>>(args); break;
		case NNRT_ITERATION_TRANSLATION_ONLY: k_pixel_jacobians<NNRT_ITERATION_TRANSLATION_ONLY><<<grid, PIX_BLOCK, 0, stream>>>(args); break;
		case NNRT_ITERATION_ROTATION_ONLY: k_pixel_jacobians<NNRT_ITERATION_ROTATION_ONLY><<<grid, PIX_BLOCK, 0, stream>>>(args); break;
		default: set_error("unknown iteration mode"); return NNRT_ERROR_ARGUMENT;
	}
	NNRT_LAUNCH_CHECK();
	// anchor slots per vertex: the common 4-anchor configuration gets its own instantiation (half the slot logic)
	const bool k4 = args.anchor_count <= 4;
	switch (mode) {
		case NNRT_ITERATION_ALL:
			if (k4) k_node_reduce<NNRT_ITERATION_ALL, 4><<<grid, PIX_BLOCK, 0, stream>>>(args);
			else k_node_reduce<NNRT_ITERATION_ALL, MAX_ANCHORS><<<grid, PIX_BLOCK, 0, stream>>>(args);
			break;
		case NNRT_ITERATION_TRANSLATION_ONLY:
			if (k4) k_node_reduce<NNRT_ITERATION_TRANSLATION_ONLY, 4><<<grid, PIX_BLOCK, 0, stream>>>(args);
			else k_node_reduce<NNRT_ITERATION_TRANSLATION_ONLY, MAX_ANCHORS><<<grid, PIX_BLOCK, 0, stream>>>(args);
			break;
		case NNRT_ITERATION_ROTATION_ONLY:
			if (k4) k_node_reduce<NNRT_ITERATION_ROTATION_ONLY, 4><<<grid, PIX_BLOCK, 0, stream>>>(args);
			else k_node_reduce<NNRT_ITERATION_ROTATION_ONLY, MAX_ANCHORS><<<grid, PIX_BLOCK, 0, stream>>>(args);
			break;
		default: set_error("unknown iteration mode"); return NNRT_ERROR_ARGUMENT;
	}
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

// =====================================================================================================================
// Block-diagonal LM solve + update (S11 no-edge path + S12): PreconditionDiagonalBlocksImpl.h, SolveBlockDiagonalCholesky
// (potrf + 2 trsm per block), RodriguesImpl.h:66-88, HierarchicalGraphWarpField::TranslateNodes/RotateNodes (:261-282:
// t += dt, R <- R * dR). One thread per node; consumes and re-zeroes the accumulator row.
// =====================================================================================================================
template <int MODE>
__device__ inline void apply_update(float* ns, const float* x) {
	if (MODE == NNRT_ITERATION_ALL) {
		ns[3] += x[3];
		ns[4] += x[4];
		ns[5] += x[5];
	} else if (MODE == NNRT_ITERATION_TRANSLATION_ONLY) {
		ns[3] += x[0];
		ns[4] += x[1];
		ns[5] += x[2];
	}
	if (MODE != NNRT_ITERATION_TRANSLATION_ONLY) {
		float dR[9], R[9], o[9];
		rodrigues_device(x[0], x[1], x[2], dR);
#pragma unroll
		for (int i = 0; i < 9; i++) R[i] = ns[6 + i];
#pragma unroll
		for (int r = 0; r < 3; r++)
#pragma unroll
			for (int c = 0; c < 3; c++) o[3 * r + c] = (R[3 * r] * dR[c] + R[3 * r + 1] * dR[3 + c]) + R[3 * r + 2] * dR[6 + c];
#pragma unroll
		for (int i = 0; i < 9; i++) ns[6 + i] = o[i];
	}
}

template <int MODE>
__global__ void k_solve_update(SolveArgs a) {
	using T = ModeTraits<MODE>;
	constexpr int S = T::S;
	const int n = blockIdx.x * blockDim.x + threadIdx.x;
	if (n >= a.N) return;
	double* acc = a.acc + static_cast<int64_t>(n) * ACC_STRIDE;
	float H[S][S], g[S];
	int e = 0;
#pragma unroll
	for (int c0 = 0; c0 < S; c0++)
#pragma unroll
		for (int c1 = c0; c1 < S; c1++) {
			const float hv = static_cast<float>(acc[e]);
			H[c0][c1] = hv;
			H[c1][c0] = hv;
			e++;
		}
#pragma unroll
	for (int c = 0; c < S; c++) g[c] = 0.f - static_cast<float>(acc[T::NH + c]);
#pragma unroll
	for (int k = 0; k < T::NACC; k++) acc[k] = 0.0;
	if (a.hessian_out) {
#pragma unroll
		for (int r = 0; r < S; r++)
#pragma unroll
			for (int c = 0; c < S; c++) a.hessian_out[static_cast<int64_t>(n) * S * S + r * S + c] = H[r][c];
	}
#pragma unroll
	for (int c = 0; c < S; c++) a.gradient_out[static_cast<int64_t>(n) * S + c] = g[c];
	if (a.lm > 0.f) {
#pragma unroll
		for (int i = 0; i < S; i++) H[i][i] += a.lm;
	}
	float x[S];
	if (!cholesky_small<S>(H)) {
		atomicOr(a.error_flag, 1);
#pragma unroll
		for (int c = 0; c < S; c++) x[c] = NAN;
	} else {
#pragma unroll
		for (int c = 0; c < S; c++) x[c] = g[c];
		cholesky_solve_small<S>(H, x);
	}
#pragma unroll
	for (int c = 0; c < S; c++) a.updates_out[static_cast<int64_t>(n) * S + c] = x[c];
	apply_update<MODE>(a.node_state + static_cast<int64_t>(n) * NODE_STRIDE, x);
}

nnrt_status launch_solve_update(int mode, const SolveArgs& args, hipStream_t stream) {
	const unsigned grid = static_cast<unsigned>(ceil_div(args.N, 256));
	switch (mode) {
		case NNRT_ITERATION_ALL: k_solve_update<NNRT_ITERATION_ALL><<<grid, 256, 0, stream>>>(args); break;
		case NNRT_ITERATION_TRANSLATION_ONLY: k_solve_update<NNRT_ITERATION_TRANSLATION_ONLY><<<grid, 256, 0, stream>>>(args); break;
		case NNRT_ITERATION_ROTATION_ONLY: k_solve_update<NNRT_ITERATION_ROTATION_ONLY><<<grid, 256, 0, stream>>>(args); break;
		default: set_error("unknown iteration mode"); return NNRT_ERROR_ARGUMENT;
	}
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

// generic block-diagonal Cholesky solve (API stage entry point)
template <int S>
__global__ void k_block_diag_solve(const float* __restrict__ blocks, const float* __restrict__ b, int count, float* __restrict__ x,
                                   int* error_flag) {
	const int n = blockIdx.x * blockDim.x + threadIdx.x;
	if (n >= count) return;
	float H[S][S], y[S];
#pragma unroll
	for (int r = 0; r < S; r++) {
#pragma unroll
		for (int c = 0; c < S; c++) H[r][c] = blocks[static_cast<int64_t>(n) * S * S + r * S + c];
		y[r] = b[static_cast<int64_t>(n) * S + r];
	}
	if (!cholesky_small<S>(H)) {
		atomicOr(error_flag, 1);
#pragma unroll
		for (int r = 0; r < S; r++) y[r] = NAN;
	} else {
		cholesky_solve_small<S>(H, y);
	}
#pragma unroll
	for (int r = 0; r < S; r++) x[static_cast<int64_t>(n) * S + r] = y[r];
}

nnrt_status launch_solve_block_diagonal(const float* blocks, const float* b, int count, int s, float* x, int* error_flag, hipStream_t stream) {
	if (count == 0) return NNRT_OK;
	const unsigned grid = static_cast<unsigned>(ceil_div(count, 256));
	if (s == 6) k_block_diag_solve<6><<<grid, 256, 0, stream>>>(blocks, b, count, x, error_flag);
	else if (s == 3) k_block_diag_solve<3><<<grid, 256, 0, stream>>>(blocks, b, count, x, error_flag);
	else {
		set_error("block size must be 3 or 6");
		return NNRT_ERROR_ARGUMENT;
	}
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

} // namespace nnrt
