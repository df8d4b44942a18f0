// GN iteration kernels for gfx950 (DeformableMeshToImageFitter.cpp:111-275).
//
// The reference materialises [P,12,6] pixel Jacobians, [P,3,19] rasterized Jacobians and [N,4000] node lists
// (capped: A4) and reduces each node serially. Here the data term takes two passes over the pixels, run back to back by
// every wave of one launch (k_fit_pixels_fused):
//  * pass 1 (pixel_body, one lane per pixel): raster resolve, depth residual (ComputeDepthResiduals :331-390)
//    and the rasterized-surface chain (RasterizedSurfaceJacobiansImpl.h:114-284) folded with dr/dw_l, dr/dn_l into a
//    16-float record per contributing pixel (dr/dV 9, dr/dn_l 3, rho 3, r).
//  * pass 2 (node_body, one wave per 8x8 pixels): groups the block's (pixel, node) associations by node
//    (AssociateFacesWithAnchorsImpl.h semantics), forms each association's node Jacobian
//    (PixelVertexAnchorJacobiansImpl.h:179-363) and sums JJᵀ and J r per node (DeformableMeshToImageFitterImpl.h:199-456)
//    into fp64 accumulator rows.
// Products are rounded to float exactly as the reference forms them and summed in double, so the data term equals the
// exactly-summed reference data term (see DESIGN.md "Numerics"); no node-list cap.
#include "fitter_kernels.hpp"



namespace nnrt {

constexpr int PIX_TILE = 16;
// waves per workgroup of the fused launch; each wave owns one 8x8 quadrant of a 16x16 tile
#ifndef NNRT_PIX_WAVES
#define NNRT_PIX_WAVES 4
#endif
constexpr int PIX_WAVES = NNRT_PIX_WAVES;
constexpr int PIX_BLOCK = 64 * PIX_WAVES;
static_assert(PIX_WAVES == 1 || PIX_WAVES == 2 || PIX_WAVES == 4, "waves per workgroup");

// this wave's tile and quadrant (0..3: (q & 1, q >> 1) in 8-pixel steps). XCD-aware: consecutive workgroups are dealt
// round-robin over the 8 XCDs, so each XCD gets a contiguous band of quadrants (neighbouring pixels share vertices,
// anchors and nodes -> L2 reuse within the XCD).
__device__ inline int pix_quadrant(const FitPixelArgs& a) {
	if (PIX_WAVES == 4 && a.tile_order) {
		// the per-frame table holds XCD band x (the workgroups b = x + 8 k, dispatched round-robin over the XCDs) at
		// [x * per_band, (x + 1) * per_band), in k order (k_tile_order); one scalar load
		const int b = static_cast<int>(blockIdx.x), per_band = a.order_blocks >> 3;
		return a.tile_order[(b & 7) * per_band + (b >> 3)] * 4 + static_cast<int>(threadIdx.x >> 6);
	}
	const int blocks = (4 * a.tiles_x * a.tiles_y + PIX_WAVES - 1) / PIX_WAVES;
	const int per_xcd = (blocks + 7) / 8;
	const int b = static_cast<int>(blockIdx.x);
	return ((b % 8) * per_xcd + b / 8) * PIX_WAVES + static_cast<int>(threadIdx.x >> 6);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

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

// ---- pass 1: per pixel (S3b-S9) -----------------------------------------------------------------------------------
// Resolves the raster winner, writes the residual / mask / face outputs and, for pixels that contribute to the data
// term, the compact per-pixel Jacobian record [dr/dV (9), dr/dn_l (3), rho (3), r] (4 x float4). The raster key is
// reset to EMPTY for the next iteration's scatter; the contributing face goes to pass 2 in registers.
// dn: this lane's 27 parked floats at dn[i * dn_stride] (lane-private LDS column)
// out_face / out_vid: the pixel's contributing face (-1: none) and its vertices, handed to pass 2 in registers
// RK: the record stays in the pixel lane's registers (rk) instead of memory, and pass 2 takes it by cross-lane reads
// (the 4-wave build, whose 128-VGPR budget holds it: at C3 the launch is bound by its memory requests, 17 per
// association of which the record's were 4)
template <int MODE, bool RK>
__device__ __forceinline__ void pixel_body(const FitPixelArgs& a, float* dn, int dn_stride, int& out_face, int (&out_vid)[3], float (&rk)[16],
                                           int& out_nodes) {
	// one 8x8 quadrant per wave: compact pixel sets touch the fewest nodes
	const int tiles = a.tiles_x * a.tiles_y;
	const int qd = pix_quadrant(a), tile = qd >> 2, quad = qd & 3;
	const int tu = tile % a.tiles_x, tv = a.tile_row0 + tile / a.tiles_x;
	const int lane = static_cast<int>(threadIdx.x & 63);
	const int u = tu * PIX_TILE + (quad & 1) * 8 + (lane & 7);
	const int v = tv * PIX_TILE + (quad >> 1) * 8 + (lane >> 3);
	const bool in_image = tile < tiles && u < a.W && v < a.H;
	const int64_t p = static_cast<int64_t>(v) * a.W + u;

	int vid[3] = {0, 0, 0};
	float rn[3] = {0.f, 0.f, 0.f}, rho[3] = {0.f, 0.f, 0.f};

	if (in_image) {
		const uint64_t key = a.keys[p];
		int32_t face = -1;
		RasterHit h{0.f, 0.f, 0.f, 0.f, 0.f};
		f3 V3[3], N3[3];
		FaceNdc fn;
		const float px = pixel_ndc(u, a.ax), py = pixel_ndc(v, a.ay);
		if (key != EMPTY_KEY) {
			face = static_cast<int32_t>(key & 0xffffffffu);
			const int4 fi = a.faces4[face];
			out_nodes = fi.w;   // the face's distinct anchor nodes (k_face_node_table)
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
		a.keys[p] = EMPTY_KEY;   // ready for the next iteration's scatter (pass 2 takes the face from registers)
		out_face = contributes ? face : -1;
		out_vid[0] = vid[0];
		out_vid[1] = vid[1];
		out_vid[2] = vid[2];
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
				const float inv_A = rcp_rn_normal(A);   // consumed by div_rn only, which ignores it outside (1e-30, 1e30)
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
			const float inv_den = rcp_rn_normal(den);   // (div_rn only)
			// d rho_r / d ndc of face vertex i, component c, and (below) the perspective z-terms of vertex i: parked in LDS
			// (lane-private slots) until vertex i's columns are formed, which keeps the kernel at <= 96 VGPRs (5 waves/SIMD:
			// one residency round at 640x480)
#define DN(i, r, c) dn[(((i) * 3 + (r)) * 2 + (c)) * dn_stride]
#define PZ(r, i) dn[(18 + (r) * 3 + (i)) * dn_stride]
#pragma unroll
			for (int c = 0; c < 2; c++) {
				DN(0, 0, c) = div_rn(-sa[0] * dA[0][c], den, inv_den);
				DN(1, 0, c) = div_rn(A * s0a[c] - sa[0] * dA[1][c], den, inv_den);
				DN(2, 0, c) = div_rn(A * s0b[c] - sa[0] * dA[2][c], den, inv_den);
				DN(0, 1, c) = div_rn(A * s1b[c] - sa[1] * dA[0][c], den, inv_den);
				DN(1, 1, c) = div_rn(-sa[1] * dA[1][c], den, inv_den);
				DN(2, 1, c) = div_rn(A * s1a[c] - sa[1] * dA[2][c], den, inv_den);
				DN(0, 2, c) = div_rn(A * s2a[c] - sa[2] * dA[0][c], den, inv_den);
				DN(1, 2, c) = div_rn(A * s2b[c] - sa[2] * dA[1][c], den, inv_den);
				DN(2, 2, c) = div_rn(-sa[2] * dA[2][c], den, inv_den);
			}
			// perspective-correction factors first (RasterizedSurfaceJacobiansImpl.h:217-284), so the 3x9 Jacobian can be
			// streamed one face vertex (3 columns) at a time: same expressions, far fewer live registers
			float Pd[3][3];
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
				const float inv_dd2 = rcp_rn_normal(dd2);   // (div_rn only)
#pragma unroll
				for (int r = 0; r < 3; r++)
#pragma unroll
					for (int c = 0; c < 3; c++) {
						Pd[r][c] = div_rn(pd[r][c], dd2, inv_dd2);
						PZ(r, c) = div_rn(pz[r][c], dd2, inv_dd2);
					}
			}
			// record [dr/dV (9), dr/dn_l (3), rho (3), r]; everything but dr/dV first, so it is not held across the columns
			float* rec_f = reinterpret_cast<float*>(a.records + 4 * p);
			if constexpr (RK) {
				rk[9] = dr_dnl.x;
				rk[10] = dr_dnl.y;
				rk[11] = dr_dnl.z;
				rk[12] = rho[0];
				rk[13] = rho[1];
				rk[14] = rho[2];
				rk[15] = residual;
			} else {
				rec_f[9] = dr_dnl.x;
				rec_f[10] = dr_dnl.y;
				rec_f[11] = dr_dnl.z;
				reinterpret_cast<float4*>(rec_f)[3] = make_float4(rho[0], rho[1], rho[2], residual);
			}
			// dr/dV = dr/dwl * dwl/dV + dr/dnl * dnl/dV ; dr/dN = dr/dnl (rho (x) I)
			const float rw[3] = {dr_dwl.x, dr_dwl.y, dr_dwl.z};
			rn[0] = dr_dnl.x;
			rn[1] = dr_dnl.y;
			rn[2] = dr_dnl.z;
#pragma unroll
			for (int i = 0; i < 3; i++) {
				__builtin_amdgcn_sched_barrier(0);   // one face vertex's columns at a time: bounds the live registers
				const float z = V3[i].z;
				const float z2 = z * z;
				const float P0[3] = {a.ndc.ndc.fx / z, 0.f, -a.ndc.ndc.fx * V3[i].x / z2};
				const float P1[3] = {0.f, a.ndc.ndc.fy / z, -a.ndc.ndc.fy * V3[i].y / z2};
				float Jc[3][3];   // rows of the 3x9 Jacobian, columns 3i .. 3i+2
#pragma unroll
				for (int r = 0; r < 3; r++)
#pragma unroll
					for (int c = 0; c < 3; c++) Jc[r][c] = DN(i, r, 0) * P0[c] + DN(i, r, 1) * P1[c];
				if (a.perspective) {
					float J2[3][3];
#pragma unroll
					for (int r = 0; r < 3; r++)
#pragma unroll
						for (int c = 0; c < 3; c++) J2[r][c] = (Pd[r][0] * Jc[0][c] + Pd[r][1] * Jc[1][c]) + Pd[r][2] * Jc[2][c];
#pragma unroll
					for (int r = 0; r < 3; r++) J2[r][2] += PZ(r, i);
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
					if constexpr (RK) rk[3 * i + c] = x + y;
					else rec_f[3 * i + c] = x + y;   // stored as formed: no 9-float tail of live outputs
				}
			}
#undef DN
#undef PZ

		}
	}
}

// ---- once per frame: the face -> distinct anchor node table (AssociateFacesWithAnchorsImpl.h:34-107) --------------------
template <int MAXK>
// (also stores the face's distinct-node count in faces4[f].w, which the pixel launch reads with the face's vertices: its
// pass 2 then loads only the table row's used 16-B pieces)
__global__ __launch_bounds__(256) void k_face_node_table(int4* __restrict__ faces4, int64_t F, const int32_t* __restrict__ anchors, int K,
                                                         uint32_t* __restrict__ out) {
	constexpr int NS = 3 * MAXK;
	const int64_t f = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (f >= F) return;
	const int4 fi = faces4[f];
	const int vid[3] = {fi.x, fi.y, fi.z};
	int node[NS];
	uint32_t code[NS];
	int n = 0;
#pragma unroll
	for (int fv = 0; fv < 3; fv++)
		for (int k = 0; k < K; k++) {
			const int a = anchors[static_cast<int64_t>(vid[fv]) * K + k];
			if (a < 0) continue;
			int at = -1;
			for (int i = 0; i < n; i++)
				if (node[i] == a) at = i;
			if (at < 0) {
				at = n++;
				node[at] = a;
				code[at] = 0xFFFu;
			}
			// per face vertex the LAST slot holding the node (ascending k overwrites)
			code[at] = (code[at] & ~(0xFu << (4 * fv))) | (static_cast<uint32_t>(k) << (4 * fv));
		}
	for (int i = 1; i < n; i++) {   // ascending node
		const int x = node[i];
		const uint32_t c = code[i];
		int j = i - 1;
		while (j >= 0 && node[j] > x) {
			node[j + 1] = node[j];
			code[j + 1] = code[j];
			j--;
		}
		node[j + 1] = x;
		code[j + 1] = c;
	}
	uint32_t* o = out + f * NS;
	for (int i = 0; i < NS; i++) o[i] = i < n ? (static_cast<uint32_t>(node[i]) << FACE_NODE_SHIFT) | code[i] : FACE_NODE_NONE;
	reinterpret_cast<int*>(faces4)[4 * f + 3] = n;
}

nnrt_status launch_face_node_table(int4* faces4, int64_t F, const int32_t* anchors, int K, uint32_t* out, hipStream_t stream) {
	if (F == 0) return NNRT_OK;
	const unsigned grid = static_cast<unsigned>(ceil_div(F, 256));
	if (K <= 4) k_face_node_table<4><<<grid, 256, 0, stream>>>(faces4, F, anchors, K, out);
	else k_face_node_table<MAX_ANCHORS><<<grid, 256, 0, stream>>>(faces4, F, anchors, K, out);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

// minimum over the 64 lanes (DPP row shifts, then row broadcasts into lane 63), wave-uniform result
// (lanes without a DPP source read the identity INT_MAX, which lets the compiler fold each step into one v_min_i32_dpp)
__device__ inline int wave_min_i32(int v) {
	constexpr int ID = 0x7fffffff;
	v = min(v, __builtin_amdgcn_update_dpp(ID, v, 0x111, 0xf, 0xf, false));   // row_shr:1
	v = min(v, __builtin_amdgcn_update_dpp(ID, v, 0x112, 0xf, 0xf, false));   // row_shr:2
	v = min(v, __builtin_amdgcn_update_dpp(ID, v, 0x114, 0xf, 0xf, false));   // row_shr:4
	v = min(v, __builtin_amdgcn_update_dpp(ID, v, 0x118, 0xf, 0xf, false));   // row_shr:8
	v = min(v, __builtin_amdgcn_update_dpp(ID, v, 0x142, 0xa, 0xf, false));   // row_bcast:15
	v = min(v, __builtin_amdgcn_update_dpp(ID, v, 0x143, 0xc, 0xf, false));   // row_bcast:31
	return __builtin_amdgcn_readlane(v, 63);
}

// ---- pass 2, node-grouped per wave --------------------------------------------------------------------------------
// 8x8 pixels per wave (the K1 mapping); the wave's (pixel, node) associations are processed in chunks of NG_CAP.
// (1) Group: every contributing pixel lane holds its face's distinct anchor nodes in ascending order (the per-frame face
//     table), so the wave's next node is the minimum of the lanes' list heads (one DPP reduction); the lanes whose head it
//     is file one association each (pixel lane, face-table entry) at consecutive LDS positions (mbcnt) and advance their
//     list; the gather decodes the entry into the jv/jn row of every face vertex anchored to the node. A node that does
//     not fit the chunk continues in the next one.
// (2) Jacobians: one association per lane (no idle lanes); J (S floats, formed as the reference forms them) and r
//     overwrite the association's slot.
// (3) Sums: the wave splits into 64 / GROUP lane groups; lane e of a group owns accumulator entry e (JJᵀ upper
//     triangle, then J r) and walks its group's share of the chunk adding the float product J[c0] * J[c1] in double;
//     at a node change the group adds its totals to the node's fp64 row (one 27-lane atomic). No cross-lane reduction.
// Chunks are software-pipelined over two LDS buffers: the jv / jn row gathers of chunk c + 1 are in flight while
// chunk c is summed, and chunk c + 1 is grouped while chunk c's gathers land. Pixel records are staged in LDS.
constexpr int NG_CAP = 64;     // associations per chunk (one lane each in (2)); lane group g of (3) owns slots
                               // [g * NG_CAP / G, (g + 1) * NG_CAP / G), zero-padded past the chunk's count
// Slot buffers are component-major (word c of slot i at c * NG_STRIDE + i; odd stride: the words one lane group reads
// in (3) fall in distinct LDS banks). Words: (1) pixel lane, face-table entry; (2a) the node at word 7;
// (2) J[0..S-1], r at word S (zeros past the count, whose node word repeats the chunk's last node).
constexpr int NG_STRIDE = 65;

constexpr int NG_ROWS = 8;     // pixel rows per wave (8 x NG_ROWS pixels)
static_assert(2 * NG_ROWS == PIX_TILE, "pass 2 walks the pass-1 tiles");

__device__ inline void ng_flush(double* dst, double v) { atomicAdd(dst, v); }

// development timing build only (-DNNRT_FIT_STAMPS): per wave, shader cycles spent in pass 2's phases (group, gather +
// Jacobians, sums, and the chunk count), read back by nnrt_dev_fit_phases
#ifdef NNRT_FIT_STAMPS
__device__ unsigned long long g_fit_phases[16384][8];   // group, gather + Jacobians, sums cycles; chunks; serial batches; group steps
#define PHASE_CLOCK() __builtin_amdgcn_s_memtime()
#endif

// slots0 / slots1: this wave's two chunk buffers (8 * NG_STRIDE words each); ent: its face-table rows ([NSLOT][64])
// face_in / vid_in: this lane's pixel's contributing face (-1: none) and its vertices, from pass 1
template <int MODE, int MAXK, bool RK>
__device__ __forceinline__ void node_body(const FitPixelArgs& a, float* slots0, float* slots1, uint32_t* ent, int face_in,
                                          const int (&vid_in)[3], const float (&rk)[16], int nodes_in) {
	using T = ModeTraits<MODE>;
	constexpr int S = T::S;
	constexpr int NSLOT = 3 * MAXK;
	constexpr int GROUP = T::NACC > 16 ? 32 : 16;
	constexpr int G = 64 / GROUP;
	constexpr int SEG = NG_CAP / G;
	constexpr int NG_BATCH = SEG % 8 == 0 ? 8 : 6;   // associations per group read ahead in (3)
	static_assert(T::NACC <= GROUP && NG_CAP % G == 0 && SEG % NG_BATCH == 0 && NG_STRIDE >= NG_CAP && (NG_STRIDE & 1), "slot layout");
	static_assert(NSLOT % 4 == 0, "face table rows are loaded as int4");
	// tiles of 16 x 16 pixels (the pass-1 tiles), one 8 x 8 block per wave
	const int tiles = a.tiles_x * a.tiles_y;
	const int qd = pix_quadrant(a), tile = qd >> 2, quad = qd & 3;
	const int tu = tile % a.tiles_x, tv = a.tile_row0 + tile / a.tiles_x;
	const int lane = static_cast<int>(threadIdx.x & 63);
	const int u = tu * PIX_TILE + (quad & 1) * 8 + (lane & 7), v = tv * 2 * NG_ROWS + (quad >> 1) * NG_ROWS + (lane >> 3);
	const bool in_image = tile < tiles && (lane >> 3) < NG_ROWS && u < a.W && v < a.H;
	const int pu0 = tu * PIX_TILE + (quad & 1) * 8, pv0 = tv * 2 * NG_ROWS + (quad >> 1) * NG_ROWS;
	const int KA = a.anchor_count;

	// this pixel's face: distinct anchor nodes still to be filed, ascending; the row waits in LDS (s_ent[wave][.][lane]),
	// the current head in a register (head_at: its index)
	uint32_t head_e = FACE_NODE_NONE;
	int head_at = 0;
	int vid[3] = {0, 0, 0};
	if (in_image) {
		if (face_in >= 0) {
			const int face = face_in;
			const uint4* fn4 = reinterpret_cast<const uint4*>(a.face_nodes + static_cast<int64_t>(face) * NSLOT);
#pragma unroll
			for (int t = 0; t < NSLOT / 4; t++) {
				// pieces past the face's node count hold FACE_NODE_NONE only: not loaded
				const uint4 e4 = t == 0 || 4 * t < nodes_in ? fn4[t] : make_uint4(FACE_NODE_NONE, FACE_NODE_NONE, FACE_NODE_NONE, FACE_NODE_NONE);
				ent[(4 * t) * 64 + lane] = e4.x;
				ent[(4 * t + 1) * 64 + lane] = e4.y;
				ent[(4 * t + 2) * 64 + lane] = e4.z;
				ent[(4 * t + 3) * 64 + lane] = e4.w;
				if (t == 0) head_e = e4.x;
			}
			vid[0] = vid_in[0];
			vid[1] = vid_in[1];
			vid[2] = vid_in[2];
		}
	}

	const int vid_ka[3] = {vid[0] * KA, vid[1] * KA, vid[2] * KA};   // first Jacobian-row slot of each face vertex

	// accumulator entry of this lane within its group
	const int grp = lane / GROUP, e = lane % GROUP;
	const bool e_valid = e < T::NACC;
	int c0 = 0, c1 = 0;
	{
		int idx = 0;
#pragma unroll
		for (int r0 = 0; r0 < S; r0++)
#pragma unroll
			for (int r1 = r0; r1 < S; r1++) {
				if (idx == e) {
					c0 = r0;
					c1 = r1;
				}
				idx++;
			}
#pragma unroll
		for (int r0 = 0; r0 < S; r0++)
			if (T::NH + r0 == e) {
				c0 = r0;
				c1 = S;
			}
	}
	double acc = 0.0;
	int cur = -1;

#ifdef NNRT_FIT_STAMPS
	unsigned long long n_serial = 0, n_steps = 0;   // timing build: slot-serial sum batches, grouping steps
#endif
	// (1) file up to NG_CAP associations into `slots`; returns the count (0: nothing pending)
	const uint64_t lanes_below = (1ull << lane) - 1ull;
	auto group = [&](float* slots) -> int {
		int filed = 0;
		while (filed < NG_CAP) {
#ifdef NNRT_FIT_STAMPS
			n_steps++;
#endif
			const int head = static_cast<int>(head_e >> FACE_NODE_SHIFT);   // FACE_NODE_MAX_NODES: list exhausted
			const int X = wave_min_i32(head);
			if (X == FACE_NODE_MAX_NODES) break;
			const uint64_t M = __ballot(head == X);
			if (M == 0) break;   // unreachable (X is some lane's head); guarantees progress
			const int rank = __popcll(M & lanes_below);
			const int room = NG_CAP - filed;
			if (head == X && rank < room) {
				const int pos = filed + rank;
				// the pixel lane and the face-table entry (node, per-vertex slots): decoded per association in (2a)
				slots[pos] = __builtin_bit_cast(float, lane);
				slots[NG_STRIDE + pos] = __builtin_bit_cast(float, head_e);
				head_at++;
				head_e = head_at < NSLOT ? ent[head_at * 64 + lane] : FACE_NODE_NONE;
			}
			const int n_head = __popcll(M);
			filed += n_head < room ? n_head : room;   // (integer select: the generic min() overload went through double)
		}
		return filed;
	};

	// (2a) gather: association `lane` of a filed chunk -> its jv / jn rows (in flight until (2b))
	int4 d = make_int4(0, -1, -1, -1);
	float4 jv[3];
	[[maybe_unused]] float4 jn[3];   // the unfused / gathered rows only
	float4 rq[4];
#if !NNRT_GATHER_ROWS
	float4 ns4[4];   // the association's node state (g, t, R), and per face vertex its canonical position / normal
	float4 cp4[3], cn4[3];
#endif
	auto gather = [&](float* slots, int count) {
		d = make_int4(0, -1, -1, -1);
		int pl = 0;
		uint32_t code = FACE_NODE_NONE;
		if (lane < count) {
			pl = __builtin_bit_cast(int, slots[lane]);
			code = __builtin_bit_cast(uint32_t, slots[NG_STRIDE + lane]);
		}
		// the pixel lane's vertex rows (every lane takes part in the shuffles), then the anchor slot of each face vertex
		// holding the node (-1: none) and the node into word 7
		int vrow[3];
#pragma unroll
		for (int fv = 0; fv < 3; fv++) vrow[fv] = __shfl(vid_ka[fv], pl);
#if !NNRT_GATHER_ROWS
		int vtx[3];
#pragma unroll
		for (int fv = 0; fv < 3; fv++) vtx[fv] = __shfl(vid[fv], pl);
#endif
		if (lane < count) {
			int r3[3];
#pragma unroll
			for (int fv = 0; fv < 3; fv++) {
				const int k = static_cast<int>((code >> (4 * fv)) & 0xFu);
				r3[fv] = k != 0xF ? vrow[fv] + k : -1;
			}
			d = make_int4(pl, r3[0], r3[1], r3[2]);
			slots[7 * NG_STRIDE + lane] = __builtin_bit_cast(float, static_cast<int>(code >> FACE_NODE_SHIFT));
		}
		const int rows[3] = {d.y, d.z, d.w};
		// unconditional loads (row -1 reads row 0, ignored in (2b)): a branch per load would make the compiler wait for
		// each gather before issuing the next, serialising the chunk's six row fetches
#if NNRT_GATHER_ROWS
#pragma unroll
		for (int fv = 0; fv < 3; fv++) {
			const int r = rows[fv] >= 0 ? rows[fv] : 0;
			const float w = MODE != NNRT_ITERATION_ROTATION_ONLY ? a.weights[r] : 0.f;
			if (MODE != NNRT_ITERATION_TRANSLATION_ONLY) {
				const float2* row = a.jrows + 3 * static_cast<int64_t>(r);
				const float2 j0 = row[0], j1 = row[1], j2 = row[2];
				jv[fv] = make_float4(j0.x, j0.y, j1.x, w);
				jn[fv] = make_float4(j1.y, j2.x, j2.y, 0.f);
			} else {
				jv[fv] = make_float4(0.f, 0.f, 0.f, w);
				jn[fv] = make_float4(0.f, 0.f, 0.f, 0.f);
			}
		}
#else
		// the weight of every face vertex (translation terms) and, for the rotation terms, the node state and the
		// canonical vertex / normal: the rows are formed in (2b) exactly as the warp forms them (warp_slot)
		{
			const int node = lane < count ? static_cast<int>(code >> FACE_NODE_SHIFT) : 0;
#pragma unroll
			for (int fv = 0; fv < 3; fv++) {
				const int r = rows[fv] >= 0 ? rows[fv] : 0;
				jv[fv].w = a.weights[r];
			}
			if (MODE != NNRT_ITERATION_TRANSLATION_ONLY) {
				const float4* ns = a.state_in + 4 * static_cast<int64_t>(node);
				ns4[0] = ns[0];
				if (!a.state_identity) {
					ns4[1] = ns[1];
					ns4[2] = ns[2];
					ns4[3] = ns[3];
				}
#pragma unroll
				for (int fv = 0; fv < 3; fv++) {
					cp4[fv] = a.cmesh_p[vtx[fv]];
					cn4[fv] = a.cmesh_n[vtx[fv]];
				}
			}
		}
#endif
		if constexpr (RK) {   // the record from its pixel lane's registers
#pragma unroll
			for (int w = 0; w < 4; w++)
				rq[w] = make_float4(__shfl(rk[4 * w], d.x), __shfl(rk[4 * w + 1], d.x), __shfl(rk[4 * w + 2], d.x), __shfl(rk[4 * w + 3], d.x));
		} else {
			const int64_t pp = static_cast<int64_t>(min(pv0 + (d.x >> 3), a.H - 1)) * a.W + min(pu0 + (d.x & 7), a.W - 1);
#pragma unroll
			for (int w = 0; w < 4; w++) rq[w] = a.records[4 * pp + w];
		}
	};
	// (2b) J and r of association `lane` into its slot
	auto jacobians = [&](float* slots, int count) {
		if (lane >= count && lane < NG_CAP) {   // padding: zero products, continuing the chunk's last node
			const float last = slots[7 * NG_STRIDE + count - 1];
#pragma unroll
			for (int c = 0; c <= S; c++) slots[c * NG_STRIDE + lane] = 0.f;
			slots[7 * NG_STRIDE + lane] = last;
		}
		if (lane < count) {
			const int l = d.x;
			const int rows[3] = {d.y, d.z, d.w};
			(void)l;
			const float q[16] = {rq[0].x, rq[0].y, rq[0].z, rq[0].w, rq[1].x, rq[1].y, rq[1].z, rq[1].w,
			                     rq[2].x, rq[2].y, rq[2].z, rq[2].w, rq[3].x, rq[3].y, rq[3].z, rq[3].w};
			const float dr_dV[9] = {q[0], q[1], q[2], q[3], q[4], q[5], q[6], q[7], q[8]};
			const float rn[3] = {q[9], q[10], q[11]};
			const float rho[3] = {q[12], q[13], q[14]};
			float jr[3] = {0.f, 0.f, 0.f}, jt[3] = {0.f, 0.f, 0.f};
#if NNRT_JAC_FMA && !NNRT_GATHER_ROWS
			// Fused form (round 5): per face vertex, with ws = w if the vertex is anchored to the node, else 0,
			//   jt += ws dv,   jr += -ws (dv x R (v - g) + dn x R n)
			// i.e. the reference's dv [-w R (v - g)]_x + dn [-w R n]_x (PixelVertexAnchorJacobiansImpl.h:179-363,
			// WarpedSurfaceJacobiansImpl.h:117-156) with -w factored out of the cross products and every product-sum an
			// FMA (the build is -ffp-contract=off), as nvcc's default contraction of the reference's CUDA path also
			// does: 43 VALU per face vertex instead of 78, the terms within a few float ulps of the unfused rows (the
			// unfused, oracle-bit-identical form: -DNNRT_JAC_FMA=0). A vertex not anchored to the node adds ws = 0
			// products, i.e. +-0, which leave the +0-started sums unchanged bit for bit (finite inputs: the vertex's own
			// canonical position / normal, the pixel's record and the node's state, never the padding row's data).
			{
				float R[9];
				f3 g = make3(0.f, 0.f, 0.f);
				if (MODE != NNRT_ITERATION_TRANSLATION_ONLY) {
					g = make3(ns4[0].x, ns4[0].y, ns4[0].z);
					if (a.state_identity) {
#pragma unroll
						for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0) ? 1.f : 0.f;
					} else {
						const float Rl[9] = {ns4[1].z, ns4[1].w, ns4[2].x, ns4[2].y, ns4[2].z, ns4[2].w, ns4[3].x, ns4[3].y, ns4[3].z};
#pragma unroll
						for (int i = 0; i < 9; i++) R[i] = Rl[i];
					}
				}
#pragma unroll
				for (int fv = 0; fv < 3; fv++) {
					const float ws = rows[fv] >= 0 ? jv[fv].w : 0.f;
					const f3 dv = make3(dr_dV[3 * fv], dr_dV[3 * fv + 1], dr_dV[3 * fv + 2]);
					if (MODE != NNRT_ITERATION_ROTATION_ONLY) {
						jt[0] = fmaf(dv.x, ws, jt[0]);
						jt[1] = fmaf(dv.y, ws, jt[1]);
						jt[2] = fmaf(dv.z, ws, jt[2]);
					}
					if (MODE != NNRT_ITERATION_TRANSLATION_ONLY) {
						const f3 d3 = sub3(make3(cp4[fv].x, cp4[fv].y, cp4[fv].z), g);
						const f3 n3 = make3(cn4[fv].x, cn4[fv].y, cn4[fv].z);
						const f3 p = make3(fmaf(R[0], d3.x, fmaf(R[1], d3.y, R[2] * d3.z)), fmaf(R[3], d3.x, fmaf(R[4], d3.y, R[5] * d3.z)),
						                   fmaf(R[6], d3.x, fmaf(R[7], d3.y, R[8] * d3.z)));
						const f3 q = make3(fmaf(R[0], n3.x, fmaf(R[1], n3.y, R[2] * n3.z)), fmaf(R[3], n3.x, fmaf(R[4], n3.y, R[5] * n3.z)),
						                   fmaf(R[6], n3.x, fmaf(R[7], n3.y, R[8] * n3.z)));
						const f3 dn = make3(rn[0] * rho[fv], rn[1] * rho[fv], rn[2] * rho[fv]);
						// dv x p + dn x q
						const float cx = fmaf(dv.y, p.z, fmaf(-dv.z, p.y, fmaf(dn.y, q.z, -dn.z * q.y)));
						const float cy = fmaf(dv.z, p.x, fmaf(-dv.x, p.z, fmaf(dn.z, q.x, -dn.x * q.z)));
						const float cz = fmaf(dv.x, p.y, fmaf(-dv.y, p.x, fmaf(dn.x, q.y, -dn.y * q.x)));
						jr[0] = fmaf(-ws, cx, jr[0]);
						jr[1] = fmaf(-ws, cy, jr[1]);
						jr[2] = fmaf(-ws, cz, jr[2]);
					}
				}
			}
#else
#if !NNRT_GATHER_ROWS
			if (MODE != NNRT_ITERATION_TRANSLATION_ONLY) {
				// (-w R (v - g), -w R n) per face vertex: warp_slot's expressions (kernels.hpp), bit-identical to its rows
				const f3 g = make3(ns4[0].x, ns4[0].y, ns4[0].z);
				float R[9];
				if (a.state_identity) {
#pragma unroll
					for (int i = 0; i < 9; i++) R[i] = (i % 4 == 0) ? 1.f : 0.f;
				} else {
					const float Rl[9] = {ns4[1].z, ns4[1].w, ns4[2].x, ns4[2].y, ns4[2].z, ns4[2].w, ns4[3].x, ns4[3].y, ns4[3].z};
#pragma unroll
					for (int i = 0; i < 9; i++) R[i] = Rl[i];
				}
#pragma unroll
				for (int fv = 0; fv < 3; fv++) {
					const float w = jv[fv].w;
					const f3 Rj = matvec3(R, sub3(make3(cp4[fv].x, cp4[fv].y, cp4[fv].z), g));
					const f3 Rnj = matvec3(R, make3(cn4[fv].x, cn4[fv].y, cn4[fv].z));
					jv[fv] = make_float4(-w * Rj.x, -w * Rj.y, -w * Rj.z, w);
					jn[fv] = make_float4(-w * Rnj.x, -w * Rnj.y, -w * Rnj.z, 0.f);
				}
			}
#endif
			// branch-free over the face vertices: a vertex not anchored to the node adds an exact +0 (selected, so the
			// row it loaded in its place -- row 0 -- never reaches the sums, NaN or not)
#pragma unroll
			for (int fv = 0; fv < 3; fv++) {
				const bool on = rows[fv] >= 0;
				const f3 dv = make3(dr_dV[3 * fv], dr_dV[3 * fv + 1], dr_dV[3 * fv + 2]);
				if (MODE != NNRT_ITERATION_ROTATION_ONLY) {
					jt[0] += on ? dv.x * jv[fv].w : 0.f;
					jt[1] += on ? dv.y * jv[fv].w : 0.f;
					jt[2] += on ? dv.z * jv[fv].w : 0.f;
				}
				if (MODE != NNRT_ITERATION_TRANSLATION_ONLY) {
					const f3 dn = make3(rn[0] * rho[fv], rn[1] * rho[fv], rn[2] * rho[fv]);
					const f3 t1 = row_times_skew(dv, make3(jv[fv].x, jv[fv].y, jv[fv].z));
					const f3 t2 = row_times_skew(dn, make3(jn[fv].x, jn[fv].y, jn[fv].z));
					jr[0] += on ? t1.x + t2.x : 0.f;
					jr[1] += on ? t1.y + t2.y : 0.f;
					jr[2] += on ? t1.z + t2.z : 0.f;
				}
			}
#endif
			float J[8];
			if (MODE == NNRT_ITERATION_ALL) {
				J[0] = jr[0];
				J[1] = jr[1];
				J[2] = jr[2];
				J[3] = jt[0];
				J[4] = jt[1];
				J[5] = jt[2];
			} else if (MODE == NNRT_ITERATION_TRANSLATION_ONLY) {
				J[0] = jt[0];
				J[1] = jt[1];
				J[2] = jt[2];
			} else {
				J[0] = jr[0];
				J[1] = jr[1];
				J[2] = jr[2];
			}
			J[S] = q[15];
#pragma unroll
			for (int c = 0; c <= S; c++) slots[c * NG_STRIDE + lane] = J[c];
		}
	};
	// (3) exact sums of the chunk's products per node
	auto sums = [&](const float* slots, int count) {
		(void)count;
#pragma unroll
		for (int j = 0; j < SEG; j += NG_BATCH) {
			// every LDS read of the batch is issued before the dependent double adds
			const float* base = slots + grp * SEG + j;
			// the products two slots at a time (v_pk_mul_f32: the same correctly rounded float products)
			float prod[NG_BATCH];
#pragma unroll
			for (int q = 0; q < NG_BATCH; q += 2) {
				const f32x2 x = {base[c0 * NG_STRIDE + q], base[c0 * NG_STRIDE + q + 1]};
				const f32x2 y = {base[c1 * NG_STRIDE + q], base[c1 * NG_STRIDE + q + 1]};
				const f32x2 pr = x * y;
				prod[q] = pr.x;
				prod[q + 1] = pr.y;
			}
			// every node of a chunk forms ONE contiguous run (grouping files all of a node's pending associations at once;
			// only a chunk's capacity splits it, into the next chunk), so a batch is a single node iff its first and last
			// slots are: two node reads instead of one per slot. A single-node batch whose node differs from `cur` (a
			// run starting on the batch boundary, e.g. a group's first batch of a chunk) flushes `cur` first.
			const int n_first = __builtin_bit_cast(int, base[7 * NG_STRIDE]), n_last = __builtin_bit_cast(int, base[7 * NG_STRIDE + NG_BATCH - 1]);
			if (__all(n_first == n_last)) {
				if (n_first != cur) {
					if (cur >= 0 && e_valid) ng_flush(a.acc + static_cast<int64_t>(cur) * ACC_STRIDE + e, acc);
					acc = 0.0;
					cur = n_first;
				}
				// independent partial sums: the double adds of a batch do not wait on one another. Each partial starts at
				// its first product (not 0.0 + product: that differs only for -0.0, which the +0.0-started accumulator
				// absorbs either way)
				double part[4];
#pragma unroll
				for (int q = 0; q < 4; q++) part[q] = static_cast<double>(prod[q]);
#pragma unroll
				for (int q = 4; q < NG_BATCH; q++) part[q & 3] += static_cast<double>(prod[q]);
				acc += (part[0] + part[1]) + (part[2] + part[3]);
			} else {
#ifdef NNRT_FIT_STAMPS
				n_serial++;
#endif
				int nodes[NG_BATCH];
#pragma unroll
				for (int q = 0; q < NG_BATCH; q++) nodes[q] = __builtin_bit_cast(int, base[7 * NG_STRIDE + q]);
#pragma unroll
				for (int q = 0; q < NG_BATCH; q++) {
					if (nodes[q] != cur) {
						if (cur >= 0 && e_valid) ng_flush(a.acc + static_cast<int64_t>(cur) * ACC_STRIDE + e, acc);
						acc = 0.0;
						cur = nodes[q];
					}
					acc += static_cast<double>(prod[q]);
				}
			}
		}
	};
	auto wave_sync = [&]() {
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
		__builtin_amdgcn_wave_barrier();
		__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
	};

	// chunk c: its row gathers are issued first and land while chunk c + 1 is grouped (LDS / scalar work); the loads
	// are consumed in the same iteration, so no loaded register is carried across the loop (a loop-carried load
	// destination gets copied into the phi register right after the load, i.e. waited for)
	int cb = 0;
#ifdef NNRT_FIT_STAMPS
	unsigned long long ph[4] = {0, 0, 0, 0}, t0 = PHASE_CLOCK(), t1;
#define PHASE_ADD(i) (t1 = PHASE_CLOCK(), ph[i] += t1 - t0, t0 = t1)
#else
#define PHASE_ADD(i) ((void)0)
#endif
	int count = group(slots0);
	PHASE_ADD(0);
	while (count > 0) {
		float* cur_slots = cb ? slots1 : slots0;
		float* nxt = cb ? slots0 : slots1;
		wave_sync();
		gather(cur_slots, count);
		const int next = group(nxt);
		wave_sync();
		PHASE_ADD(0);
		jacobians(cur_slots, count);
		wave_sync();
		PHASE_ADD(1);
		sums(cur_slots, count);
		wave_sync();
		PHASE_ADD(2);
#ifdef NNRT_FIT_STAMPS
		ph[3]++;
#endif
		cb ^= 1;
		count = next;
	}
	if (cur >= 0 && e_valid) ng_flush(a.acc + static_cast<int64_t>(cur) * ACC_STRIDE + e, acc);
#ifdef NNRT_FIT_STAMPS
	{
		const int wid_ = static_cast<int>(blockIdx.x) * (PIX_BLOCK / 64) + static_cast<int>(threadIdx.x >> 6);
		if (lane == 0 && wid_ < 16384)
			for (int i = 0; i < 4; i++) g_fit_phases[wid_][i] = ph[i];
		if (lane == 0 && wid_ < 16384) {
			g_fit_phases[wid_][4] = n_serial;
			g_fit_phases[wid_][5] = n_steps;
		}
	}
#endif
#undef PHASE_ADD
}

// ---- both passes in one launch ------------------------------------------------------------------------------------
// Each wave runs pass 1 over its 8 x 8 pixels, then pass 2 over the same pixels (the two passes map tiles and waves
// identically). One LDS region per wave serves pass 1's parked terms and then pass 2's chunk buffers and face-table
// rows; the records and keys go through global memory and are re-read by the same wave (L1 / L2 hits). Fusing removes a
// launch boundary and lets one wave's pass-2 memory phases overlap other waves' pass-1 arithmetic: C2 17.5 + 25.2 us
// as two launches -> one launch ~6 us shorter.
// development timing build only (-DNNRT_FIT_STAMPS, tools/dev/stamps_build.sh): per wave of the fused launch, the
// constant-rate clock (100 MHz) at its start, after pass 1 and at its end, and its hardware id (CU / SIMD placement)
#ifdef NNRT_FIT_STAMPS
__device__ unsigned long long g_fit_stamps[16384][4];
#define FIT_STAMP(i, v)                                                                                                  \
	do {                                                                                                                 \
		const int wid_ = static_cast<int>(blockIdx.x) * (PIX_BLOCK / 64) + static_cast<int>(threadIdx.x >> 6);         \
		if ((threadIdx.x & 63) == 0 && wid_ < 16384) g_fit_stamps[wid_][i] = (v);                                      \
	} while (0)
#else
#define FIT_STAMP(i, v) \
	do {                \
	} while (0)
#endif

// WPE: the waves per SIMD the launch is compiled for. 5 (96 VGPRs, one dword spilled; the LDS allows 5 workgroups per
// CU): single-round launches (C2: 40.4 us; 47.2 at 4). 4 (108 VGPRs, no spill): launches of several residency rounds,
// whose pass-2 gathers miss L2 and congest the memory pipeline (C3: 198.6 -> 188 us) -- FitPixelArgs::low_occupancy.
#ifndef NNRT_PIX_KEEP_RECORDS
#define NNRT_PIX_KEEP_RECORDS 1
#endif
template <int MODE, int MAXK, int WPE>
__global__ __launch_bounds__(PIX_BLOCK) __attribute__((amdgpu_waves_per_eu(WPE))) void k_fit_pixels_fused(FitPixelArgs a) {
	constexpr int NODE_WORDS = 2 * 8 * NG_STRIDE + 3 * MAXK * 64;
	constexpr int WORDS = NODE_WORDS > 27 * 64 ? NODE_WORDS : 27 * 64;
#ifdef NNRT_DEV_PIX_LDS_WORDS   // timing build only: per-wave LDS region padded to this many words (occupancy probe)
	__shared__ float s_u[PIX_BLOCK / 64][NNRT_DEV_PIX_LDS_WORDS > WORDS ? NNRT_DEV_PIX_LDS_WORDS : WORDS];
#else
	__shared__ float s_u[PIX_BLOCK / 64][WORDS];
#endif
	// ARAP path: the launch's last arap_blocks workgroups compute the edge terms (independent of the data term: they read
	// the node state only), in the SIMD slots the pixel waves leave free
	if (a.arap_blocks > 0) {
		const int first = static_cast<int>(gridDim.x) - a.arap_blocks;
		if (static_cast<int>(blockIdx.x) >= first) {
			const int e = (static_cast<int>(blockIdx.x) - first) * PIX_BLOCK + static_cast<int>(threadIdx.x);
			if (e < a.arap.E) arap_edge(a.arap, e);
			return;
		}
	}
	const int wave = static_cast<int>(threadIdx.x >> 6), lane = static_cast<int>(threadIdx.x & 63);
	FIT_STAMP(0, __builtin_amdgcn_s_memrealtime());
	FIT_STAMP(3, static_cast<unsigned long long>(__builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11))) |
	                 (static_cast<unsigned long long>(__builtin_amdgcn_s_getreg((20) | (0 << 6) | (31 << 11))) << 32));
	float* w = s_u[wave];
	int face = -1, vid[3] = {0, 0, 0}, nodes = 3 * MAXK;
	constexpr bool RK = WPE == 4 && NNRT_PIX_KEEP_RECORDS;
	float rk[16];
#pragma unroll
	for (int i = 0; i < 16; i++) rk[i] = 0.f;
	pixel_body<MODE, RK>(a, w + lane, 64, face, vid, rk, nodes);
	FIT_STAMP(1, __builtin_amdgcn_s_memrealtime());
	// the node pass reads the records / keys this wave just stored (other lanes' pixels; same CU, same L1): workgroup-scope
	// release + acquire (an agent-scope release writes back L2 on gfx950: 10x slower); the LDS region is reused in program
	// order by the same wave
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
#ifdef NNRT_DEV_PASS1_ONLY   // timing build only: pass 1 alone (instruction counts per pass by difference)
	if (face != -2) return;
#endif
	node_body<MODE, MAXK, RK>(a, w, w + 8 * NG_STRIDE, reinterpret_cast<uint32_t*>(w + 2 * 8 * NG_STRIDE), face, vid, rk, nodes);
	FIT_STAMP(2, __builtin_amdgcn_s_memrealtime());
}

#define NNRT_EV(call)                                                                                                   \
	do {                                                                                                                \
		if ((call) != hipSuccess) {                                                                                     \
			set_error("event record/wait failed");                                                                      \
			return NNRT_ERROR_HIP;                                                                                      \
		}                                                                                                               \
	} while (0)

#ifdef NNRT_FIT_STAMPS
extern "C" int nnrt_dev_fit_phases(unsigned long long* out) {   // [16384][8] of the last fused launch
	return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fit_phases), sizeof(unsigned long long) * 16384 * 8) == hipSuccess ? 0 : 1;
}
extern "C" int nnrt_dev_fit_stamps(unsigned long long* out) {   // [16384][4] of the last fused launch
	return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fit_stamps), sizeof(unsigned long long) * 16384 * 4) == hipSuccess ? 0 : 1;
}
#endif

// the pixel-node Jacobian arithmetic of this build (NNRT_JAC_FMA), for the test checker's matching mode
extern "C" int nnrt_build_jacobian_fma() { return NNRT_JAC_FMA && !NNRT_GATHER_ROWS; }
extern "C" float nnrt_build_refine_floor() { return NNRT_REFINE_PIVOT_FLOOR; }

int fit_pixels_arap_blocks(int E) { return static_cast<int>(ceil_div(E, PIX_BLOCK)); }
// the per-frame tile table maps one 16 x 16 tile per 4-wave workgroup; other NNRT_PIX_WAVES builds use the arithmetic
// mapping, whose grid the table's would not cover
bool fit_pixels_tile_order_supported() { return PIX_WAVES == 4; }

// ---- per-frame tile order of the pixel launch (launch_tile_order) ----
__host__ __device__ inline int tiles_per_band(int tiles) { return (tiles + 7) / 8 + 1; }   // ceil(w / 8) + ceil(i / 8) <= this
int tile_order_blocks(int tiles) { return 8 * tiles_per_band(tiles); }

// per 16 x 16 tile (one wave): does any pixel hold a valid reference point
__global__ __launch_bounds__(64) void k_tile_flags(const float4* __restrict__ ref, int H, int W, int tiles_x, int* __restrict__ flags) {
	const int tile = static_cast<int>(blockIdx.x), lane = static_cast<int>(threadIdx.x);
	const int tu = tile % tiles_x, tv = tile / tiles_x;
	bool any = false;
#pragma unroll
	for (int k = 0; k < 4; k++) {
		const int q = lane + 64 * k, u = tu * PIX_TILE + (q & 15), v = tv * PIX_TILE + (q >> 4);
		if (u < W && v < H) any |= ref[static_cast<int64_t>(v) * W + u].w != 0.f;
	}
	const unsigned long long b = __ballot(any);
	if (lane == 0) flags[tile] = b != 0ull;
}

// one workgroup: ranks of the working / idle tiles in raster order (chunked block scan), then each XCD band x (the
// workgroups b = x + 8 k, k = 0, 1, ... of the launch, dispatched in k order) gets its eighth of the working tiles at
// k = 0.. and its eighth of the idle tiles after them; unused entries hold `tiles` (a workgroup with no pixels)
constexpr int ORDER_THREADS = 1024;
__global__ __launch_bounds__(ORDER_THREADS) void k_tile_order(const int* __restrict__ flags, int tiles, int* __restrict__ order) {
	__shared__ int s_w[ORDER_THREADS], s_i[ORDER_THREADS];
	const int t = static_cast<int>(threadIdx.x);
	const int per_band = tiles_per_band(tiles);
	for (int i = t; i < 8 * per_band; i += ORDER_THREADS) order[i] = tiles;
	const int c = (tiles + ORDER_THREADS - 1) / ORDER_THREADS, t0 = t * c, t1 = t0 + c < tiles ? t0 + c : tiles;
	int nw = 0, ni = 0;
	for (int q = t0; q < t1; q++) (flags[q] ? nw : ni)++;
	s_w[t] = nw;
	s_i[t] = ni;
	__syncthreads();
	for (int d = 1; d < ORDER_THREADS; d <<= 1) {   // inclusive scan (Hillis-Steele)
		const int aw = t >= d ? s_w[t - d] : 0, ai = t >= d ? s_i[t - d] : 0;
		__syncthreads();
		s_w[t] += aw;
		s_i[t] += ai;
		__syncthreads();
	}
	const int W = s_w[ORDER_THREADS - 1], I = s_i[ORDER_THREADS - 1];
	int m = s_w[t] - nw, n = s_i[t] - ni;   // ranks of this chunk's first working / idle tile
	__syncthreads();   // (the pad fill above is ordered before the entries below by the scan's barriers)
	for (int q = t0; q < t1; q++) {
		if (flags[q]) {
			int x = 7;
			while (x > 0 && (static_cast<int64_t>(x) * W) / 8 > m) x--;
			order[x * per_band + (m - static_cast<int>((static_cast<int64_t>(x) * W) / 8))] = q;
			m++;
		} else {
			int x = 7;
			while (x > 0 && (static_cast<int64_t>(x) * I) / 8 > n) x--;
			const int wx = static_cast<int>((static_cast<int64_t>(x + 1) * W) / 8 - (static_cast<int64_t>(x) * W) / 8);
			order[x * per_band + wx + (n - static_cast<int>((static_cast<int64_t>(x) * I) / 8))] = q;
			n++;
		}
	}
}

nnrt_status launch_tile_order(const float4* ref_points, int H, int W, int tiles_x, int tiles_y, int* flags, int* order, hipStream_t stream) {
	const int tiles = tiles_x * tiles_y;
	if (tiles == 0) return NNRT_OK;
	k_tile_flags<<<static_cast<unsigned>(tiles), 64, 0, stream>>>(ref_points, H, W, tiles_x, flags);
	NNRT_LAUNCH_CHECK();
	k_tile_order<<<1, ORDER_THREADS, 0, stream>>>(flags, tiles, order);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

nnrt_status launch_fit_pixels(int mode, const FitPixelArgs& args, hipStream_t stream, hipEvent_t between) {
	// `between` (stage timing) is recorded before the fused launch: the pixel-pass stage reads 0, the node-pass stage
	// times both passes
	if (between) NNRT_EV(hipEventRecord(between, stream));
	const unsigned grid = static_cast<unsigned>((args.tile_order ? args.order_blocks : ((4 * args.tiles_x * args.tiles_y + PIX_WAVES - 1) / PIX_WAVES + 7) / 8 * 8) +
	                                            args.arap_blocks);
	// anchor slots per vertex: the common 4-anchor configuration gets its own instantiation (half the slot logic)
	const bool k4 = args.anchor_count <= 4;
	const bool low = args.low_occupancy != 0;
	switch (mode) {
		case NNRT_ITERATION_ALL:
			if (k4 && low) k_fit_pixels_fused<NNRT_ITERATION_ALL, 4, 4><<<grid, PIX_BLOCK, 0, stream>>>(args);
			else if (k4) k_fit_pixels_fused<NNRT_ITERATION_ALL, 4, 5><<<grid, PIX_BLOCK, 0, stream>>>(args);
			else k_fit_pixels_fused<NNRT_ITERATION_ALL, MAX_ANCHORS, 5><<<grid, PIX_BLOCK, 0, stream>>>(args);
			break;
		case NNRT_ITERATION_TRANSLATION_ONLY:
			if (k4 && low) k_fit_pixels_fused<NNRT_ITERATION_TRANSLATION_ONLY, 4, 4><<<grid, PIX_BLOCK, 0, stream>>>(args);
			else if (k4) k_fit_pixels_fused<NNRT_ITERATION_TRANSLATION_ONLY, 4, 5><<<grid, PIX_BLOCK, 0, stream>>>(args);
			else k_fit_pixels_fused<NNRT_ITERATION_TRANSLATION_ONLY, MAX_ANCHORS, 5><<<grid, PIX_BLOCK, 0, stream>>>(args);
			break;
		case NNRT_ITERATION_ROTATION_ONLY:
			if (k4 && low) k_fit_pixels_fused<NNRT_ITERATION_ROTATION_ONLY, 4, 4><<<grid, PIX_BLOCK, 0, stream>>>(args);
			else if (k4) k_fit_pixels_fused<NNRT_ITERATION_ROTATION_ONLY, 4, 5><<<grid, PIX_BLOCK, 0, stream>>>(args);
			else k_fit_pixels_fused<NNRT_ITERATION_ROTATION_ONLY, MAX_ANCHORS, 5><<<grid, PIX_BLOCK, 0, stream>>>(args);
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
// old = the node's (t, R) as loaded at kernel start (stride-15 state row, entries 3..14)
template <int MODE>
__device__ inline void apply_update(float* ns, const float* old, const float* x) {
	if (MODE == NNRT_ITERATION_ALL) {
		ns[3] = old[0] + x[3];
		ns[4] = old[1] + x[4];
		ns[5] = old[2] + x[5];
	} else if (MODE == NNRT_ITERATION_TRANSLATION_ONLY) {
		ns[3] = old[0] + x[0];
		ns[4] = old[1] + x[1];
		ns[5] = old[2] + x[2];
	} else {
		ns[3] = old[0];
		ns[4] = old[1];
		ns[5] = old[2];
	}
	if (MODE != NNRT_ITERATION_TRANSLATION_ONLY) {
		float dR[9], R[9], o[9];
		rodrigues_device(x[0], x[1], x[2], dR);
#pragma unroll
		for (int i = 0; i < 9; i++) R[i] = old[3 + i];
#pragma unroll
		for (int r = 0; r < 3; r++)
#pragma unroll
			for (int c = 0; c < 3; c++) o[3 * r + c] = (R[3 * r] * dR[c] + R[3 * r + 1] * dR[3 + c]) + R[3 * r + 2] * dR[6 + c];
#pragma unroll
		for (int i = 0; i < 9; i++) ns[6 + i] = o[i];
	} else {
#pragma unroll
		for (int i = 0; i < 9; i++) ns[6 + i] = old[3 + i];
	}
}

// IDENTITY: the node's motion before the update is R = I, t = 0 (iterate-from-identity) and is not read. Otherwise the
// (t, R) row is loaded up front so its latency overlaps the accumulator loads.
template <int MODE, bool IDENTITY>
__global__ __launch_bounds__(64) void k_solve_update(SolveArgs a) {
	using T = ModeTraits<MODE>;
	constexpr int S = T::S;
	const int n = blockIdx.x * blockDim.x + threadIdx.x;
#if NNRT_SOLVE_ACC_LDS
	// the wave's 64 accumulator rows are one contiguous block: read and re-zeroed with coalesced 16-B accesses
	__shared__ __attribute__((aligned(16))) double s_acc[64 * ACC_STRIDE];
	{
		const int64_t base = static_cast<int64_t>(blockIdx.x) * 64 * ACC_STRIDE;
		const int64_t lim = static_cast<int64_t>(a.N) * ACC_STRIDE - base;   // doubles of this wave's rows
		double2* g2 = reinterpret_cast<double2*>(a.acc + base);
#pragma unroll
		for (int i = 0; i < ACC_STRIDE / 2; i++) {
			const int q = i * 64 + static_cast<int>(threadIdx.x);
			if (2 * q < lim) {
				reinterpret_cast<double2*>(s_acc)[q] = g2[q];
				g2[q] = make_double2(0.0, 0.0);
			}
		}
		__syncthreads();
	}
#endif
	if (n >= a.N) return;
	float* ns = a.node_state + static_cast<int64_t>(n) * NODE_STRIDE;
	const float* ns_in = a.state_in + static_cast<int64_t>(n) * NODE_STRIDE;
	float old[12];
	if constexpr (IDENTITY) {
#pragma unroll
		for (int i = 0; i < 12; i++) old[i] = (i == 3 || i == 7 || i == 11) ? 1.f : 0.f;
	} else {
#pragma unroll
		for (int i = 0; i < 12; i++) old[i] = __builtin_nontemporal_load(ns_in + 3 + i);
	}
#if NNRT_SOLVE_ACC_LDS
	const double* acc = s_acc + threadIdx.x * ACC_STRIDE;
#else
	double* acc = a.acc + static_cast<int64_t>(n) * ACC_STRIDE;
#endif
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
#if !NNRT_SOLVE_ACC_LDS
#pragma unroll
	for (int k = 0; k < T::NACC; k++) acc[k] = 0.0;
#endif
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
	apply_update<MODE>(ns, old, x);
}

// Eight lanes per node (lane r of the node's group owns row r of H and of its factor L): the same operations as
// k_solve_update, element for element, in fewer instructions per wave and over 8x the waves.
//   Factor: column j of L in one step over the group -- lane i forms H_ij - sum_k<j L_ik L_jk (k ascending, row j
//   broadcast from lane j), lane j's value is the pivot, sqrt on lane j, broadcast, L_ij = t / L_jj on the lanes below.
//   Solves, Rodrigues and the rotation product: every lane runs cholesky_solve_small / apply_update's operations on
//   the factor read back from LDS (replicated: one instruction serves all groups), and lane r stores entries r, r + 8.
// Bit-identical to the one-lane-per-node kernel (the same float operations in the same order).
constexpr int SOLVE_GL = 8;   // lanes per node
// lane s of each quad (DPP quad_perm [s, s, s, s]); s is a constant after unrolling
__device__ __forceinline__ int quad_bcast(int v, int s) {
	switch (s) {
		case 0: return __builtin_amdgcn_update_dpp(0, v, 0x00, 0xf, 0xf, false);
		case 1: return __builtin_amdgcn_update_dpp(0, v, 0x55, 0xf, 0xf, false);
		case 2: return __builtin_amdgcn_update_dpp(0, v, 0xAA, 0xf, 0xf, false);
		default: return __builtin_amdgcn_update_dpp(0, v, 0xFF, 0xf, 0xf, false);
	}
}
// lane j of each 8-lane group in VALU DPP moves, no LDS round trip (a ds_swizzle broadcast waited ~100 cycles on the
// factor's critical chain; 0.8 us of the launch at C2): the quad holding lane j reads it by quad_perm, the other quad
// reads the half-row mirror image (lane i <- lane 7 - i), where lane j sits at quad position 3 - (j & 3)
__device__ __forceinline__ float group_bcast(float v, int j) {
	const int iv = __builtin_bit_cast(int, v);
	const int same = quad_bcast(iv, j & 3);
	const int mirrored = __builtin_amdgcn_update_dpp(0, iv, 0x141, 0xf, 0xf, false);   // row_half_mirror
	const int other = quad_bcast(mirrored, 3 - (j & 3));
	const bool in_quad = static_cast<int>((threadIdx.x >> 2) & 1) == (j >> 2);
	return __builtin_bit_cast(float, in_quad ? same : other);
}

template <int MODE, bool IDENTITY>
__global__ __launch_bounds__(64) void k_solve_update_lanes(SolveArgs a) {
	using T = ModeTraits<MODE>;
	constexpr int S = T::S;
	constexpr int NPW = 64 / SOLVE_GL;   // nodes per wave
	__shared__ __attribute__((aligned(16))) double s_acc[NPW * ACC_STRIDE];
	__shared__ float s_l[NPW][S * S];
	const int lane = static_cast<int>(threadIdx.x), gl = lane & (SOLVE_GL - 1), grp = lane / SOLVE_GL;
	const int n = static_cast<int>(blockIdx.x) * NPW + grp;
	// the node's motion before the update, loaded together with the accumulator rows (one memory round trip for both)
	float old[12];
	if constexpr (IDENTITY) {
#pragma unroll
		for (int i = 0; i < 12; i++) old[i] = (i == 3 || i == 7 || i == 11) ? 1.f : 0.f;
	} else {
		const float* ns_in = a.state_in + static_cast<int64_t>(n < a.N ? n : 0) * NODE_STRIDE;
#pragma unroll
		for (int i = 0; i < 12; i++) old[i] = ns_in[3 + i];
	}
	{   // the wave's 8 accumulator rows: one contiguous block, read and re-zeroed with coalesced 16-B accesses
		const int64_t base = static_cast<int64_t>(blockIdx.x) * NPW * ACC_STRIDE;
		const int64_t lim = static_cast<int64_t>(a.N) * ACC_STRIDE - base;
		double2* g2 = reinterpret_cast<double2*>(a.acc + base);
#pragma unroll
		for (int q = lane; q < NPW * ACC_STRIDE / 2; q += 64)
			if (2 * q < lim) {
				reinterpret_cast<double2*>(s_acc)[q] = g2[q];
				g2[q] = make_double2(0.0, 0.0);
			}
		// one wave per workgroup: its own LDS writes ordered before its reads, no workgroup barrier
		__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
		__builtin_amdgcn_wave_barrier();
		__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
	}
	if (n >= a.N) return;   // whole groups: the group_bcast sources stay in the active set
	const double* acc = s_acc + grp * ACC_STRIDE;
	const int r = gl < S ? gl : S - 1;   // lanes S..7 shadow row S - 1 (their results are never stored)
	// row r of H (packed upper triangle: entry (c0, c1), c0 <= c1, at c0 S - c0 (c0 - 1) / 2 + c1 - c0)
	float h[S];
#pragma unroll
	for (int c = 0; c < S; c++) {
		const int c0 = c < r ? c : r, c1 = c < r ? r : c;
		h[c] = static_cast<float>(acc[c0 * S - (c0 * (c0 - 1)) / 2 + (c1 - c0)]);
	}
	const float gr = 0.f - static_cast<float>(acc[T::NH + r]);
	if (gl < S) {
		if (a.hessian_out) {
#pragma unroll
			for (int c = 0; c < S; c++) a.hessian_out[static_cast<int64_t>(n) * S * S + r * S + c] = h[c];
		}
		a.gradient_out[static_cast<int64_t>(n) * S + r] = gr;
	}
	if (a.lm > 0.f) {
#pragma unroll
		for (int c = 0; c < S; c++)
			if (c == r) h[c] += a.lm;
	}
	// factor: lane r holds L_r0 .. L_rr in h[0 .. r]
	bool bad = false;
#pragma unroll
	for (int j = 0; j < S; j++) {
		float t = h[j];
#pragma unroll
		for (int k = 0; k < j; k++) {
			const float ljk = group_bcast(h[k], j);   // L_jk
			t -= h[k] * ljk;
		}
		// the pivot test on lane j's t through its square root (t > 0 iff sqrt(t) > 0, NaN included): one broadcast
		const float l = group_bcast(sqrtf(t), j);
		bad |= !(l > 0.f);
		if (r == j) h[j] = l;
		else if (r > j) h[j] = t / l;
	}
	float* Lm = s_l[grp];
	if (gl < S) {
#pragma unroll
		for (int c = 0; c < S; c++) Lm[r * S + c] = c <= r ? h[c] : 0.f;
	}
	__builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
	__builtin_amdgcn_wave_barrier();
	__builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
	float L[S][S], x[S];
#pragma unroll
	for (int i = 0; i < S; i++)
#pragma unroll
		for (int c = 0; c < S; c++) L[i][c] = Lm[i * S + c];
#pragma unroll
	for (int c = 0; c < S; c++) x[c] = group_bcast(gr, c);   // g
	if (bad) {
		if (gl == 0) atomicOr(a.error_flag, 1);
#pragma unroll
		for (int c = 0; c < S; c++) x[c] = NAN;
	} else {
		cholesky_solve_small<S>(L, x);
	}
	float xr = x[0];
#pragma unroll
	for (int c = 1; c < S; c++) xr = r == c ? x[c] : xr;
	if (gl < S) a.updates_out[static_cast<int64_t>(n) * S + r] = xr;
	float o[15];
	apply_update<MODE>(o, old, x);   // o[3 .. 14]: the node's new (t, R)
	float* ns = a.node_state + static_cast<int64_t>(n) * NODE_STRIDE;
	float v0 = o[3], v1 = o[11];
#pragma unroll
	for (int c = 1; c < 8; c++) v0 = gl == c ? o[3 + c] : v0;
#pragma unroll
	for (int c = 1; c < 4; c++) v1 = gl == c ? o[11 + c] : v1;
	ns[3 + gl] = v0;
	if (gl < 4) ns[11 + gl] = v1;
}

template <bool IDENTITY>
static nnrt_status solve_update_mode(int mode, const SolveArgs& args, hipStream_t stream) {
#if NNRT_SOLVE_LANES
	const unsigned grid = static_cast<unsigned>(ceil_div(args.N, 64 / SOLVE_GL));   // one wave per workgroup, 8 nodes per wave
	switch (mode) {
		case NNRT_ITERATION_ALL: k_solve_update_lanes<NNRT_ITERATION_ALL, IDENTITY><<<grid, 64, 0, stream>>>(args); break;
		case NNRT_ITERATION_TRANSLATION_ONLY: k_solve_update_lanes<NNRT_ITERATION_TRANSLATION_ONLY, IDENTITY><<<grid, 64, 0, stream>>>(args); break;
		case NNRT_ITERATION_ROTATION_ONLY: k_solve_update_lanes<NNRT_ITERATION_ROTATION_ONLY, IDENTITY><<<grid, 64, 0, stream>>>(args); break;
		default: set_error("unknown iteration mode"); return NNRT_ERROR_ARGUMENT;
	}
#else
	const unsigned grid = static_cast<unsigned>(ceil_div(args.N, 64));   // one wave per workgroup: more CUs take part
	switch (mode) {
		case NNRT_ITERATION_ALL: k_solve_update<NNRT_ITERATION_ALL, IDENTITY><<<grid, 64, 0, stream>>>(args); break;
		case NNRT_ITERATION_TRANSLATION_ONLY: k_solve_update<NNRT_ITERATION_TRANSLATION_ONLY, IDENTITY><<<grid, 64, 0, stream>>>(args); break;
		case NNRT_ITERATION_ROTATION_ONLY: k_solve_update<NNRT_ITERATION_ROTATION_ONLY, IDENTITY><<<grid, 64, 0, stream>>>(args); break;
		default: set_error("unknown iteration mode"); return NNRT_ERROR_ARGUMENT;
	}
#endif
	return NNRT_OK;
}

nnrt_status launch_solve_update(int mode, const SolveArgs& args, hipStream_t stream, bool from_identity) {
	const nnrt_status st = from_identity ? solve_update_mode<true>(mode, args, stream) : solve_update_mode<false>(mode, args, stream);
	if (st) return st;
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

// block-wise SPD inverse (API stage entry point; the same device functions as the arrowhead stem's D^-1)
template <int S>
__global__ void k_invert_psd_blocks(const float* __restrict__ blocks, int count, float* __restrict__ out, int* error_flag) {
	const int n = blockIdx.x * blockDim.x + threadIdx.x;
	if (n >= count) return;
	float L[S][S], Ai[S][S];
#pragma unroll
	for (int r = 0; r < S; r++)
#pragma unroll
		for (int c = 0; c < S; c++) L[r][c] = blocks[static_cast<int64_t>(n) * S * S + r * S + c];
	if (!cholesky_small<S>(L)) {
		atomicOr(error_flag, 1);
#pragma unroll
		for (int r = 0; r < S; r++)
#pragma unroll
			for (int c = 0; c < S; c++) Ai[r][c] = NAN;
	} else {
		invert_from_cholesky_small<S>(L, Ai);
	}
#pragma unroll
	for (int r = 0; r < S; r++)
#pragma unroll
		for (int c = 0; c < S; c++) out[static_cast<int64_t>(n) * S * S + r * S + c] = Ai[r][c];
}

nnrt_status launch_invert_psd_blocks(const float* blocks, int count, int s, float* out, int* error_flag, hipStream_t stream) {
	if (count == 0) return NNRT_OK;
	const unsigned grid = static_cast<unsigned>(ceil_div(count, 256));
	if (s == 6) k_invert_psd_blocks<6><<<grid, 256, 0, stream>>>(blocks, count, out, error_flag);
	else if (s == 3) k_invert_psd_blocks<3><<<grid, 256, 0, stream>>>(blocks, count, out, error_flag);
	else {
		set_error("block size must be 3 or 6");
		return NNRT_ERROR_ARGUMENT;
	}
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

} // namespace nnrt
