// ARAP regularization + block-sparse arrowhead solve (regularized path of DeformableMeshToImageFitter.cpp:223-247).
//
//   edge residuals   ComputeArapResiduals_* (DeformableMeshToImageFitterImpl.h:644-784; fixed-coverage weight indexed by
//                    node_j as written: A3) + Huber (DeformableMeshToImageFitter.cpp:434-444)
//   edge Jacobians   ArapJacobianImpl.h:35-209 (condensed: -lw R_i (g_i - g_j), lw, -lw)
//   arrowhead H      ArapHessianImpl.h:44-195: wing blocks dEi^T dEj, diagonal sums dE^T dE (+ data blocks, + LM)
//   solve            SolveBlockSparseArrowheadCholesky.cpp:30-95 / SchurComplement.cpp:44-79, uncapped (A1):
//                    x_C = chol(C - B^T D^-1 B) \ (b_C - B^T D^-1 b_D),  x_D = D^-1 (b_D - B x_C).
//                    Corner off-diagonal blocks (edges whose source lies outside the stem, >= 3 layers) are included
//                    (the reference drops them: A3) as in sparse_block_cholesky_scripts.py:106-160.
#include <algorithm>


#include "fitter_kernels.hpp"

namespace nnrt {

// dE^T dE for dE = [skew(a) | s I] (i side) ; returns the 21 upper-triangle entries
__device__ inline void edge_block_i(const float* j5, float (&dE)[3][6]) {
	const float a0 = j5[0], a1 = j5[1], a2 = j5[2];
	const float sk[3][3] = {{0.f, -a2, a1}, {a2, 0.f, -a0}, {-a1, a0, 0.f}};
#pragma unroll
	for (int r = 0; r < 3; r++) {
#pragma unroll
		for (int c = 0; c < 3; c++) dE[r][c] = sk[r][c];
#pragma unroll
		for (int c = 0; c < 3; c++) dE[r][3 + c] = (r == c) ? j5[3] : 0.f;
	}
}

__global__ void k_arap_edges(ArapArgs a) {
	const int e = blockIdx.x * blockDim.x + threadIdx.x;
	if (e >= a.E) return;
	const int i = a.edges[2 * e], j = a.edges[2 * e + 1];
	const float* si = a.node_state + static_cast<int64_t>(i) * NODE_STRIDE;
	const float* sj = a.node_state + static_cast<int64_t>(j) * NODE_STRIDE;
	const f3 gi = make3(si[0], si[1], si[2]), gj = make3(sj[0], sj[1], sj[2]);
	const f3 ti = make3(si[3], si[4], si[5]), tj = make3(sj[3], sj[4], sj[5]);
	const f3 Rd = matvec3(si + 6, sub3(gi, gj));
	float w_res, w_jac;
	if (a.coverage_variable) {
		w_res = w_jac = fmaxf(a.node_weights[i], a.node_weights[j]);
	} else {
		if (j >= a.E) {   // reference indexes edge_layer_indices[node_j] (A3); out of bounds there
			atomicOr(a.error_flag, 2);
			for (int q = 0; q < EDGE_TERMS; q++) a.edge_jr[static_cast<int64_t>(e) * EDGE_TERMS + q] = 0.f;
			return;
		}
		w_res = a.radii[a.edge_layers[j]];
		w_jac = a.radii[a.edge_layers[e]];
	}
	const float lw = a.lambda * w_res;
	float r[3] = {lw * (((gi.x + ti.x) - (gj.x + tj.x)) - Rd.x), lw * (((gi.y + ti.y) - (gj.y + tj.y)) - Rd.y),
	              lw * (((gi.z + ti.z) - (gj.z + tj.z)) - Rd.z)};
	if (a.use_huber) {
		const float half = 0.5f * a.huber_delta * a.huber_delta;
#pragma unroll
		for (int c = 0; c < 3; c++) r[c] = (r[c] >= a.huber_delta) ? fabsf(r[c]) - half : 0.5f * r[c] * r[c];
	}
#pragma unroll
	for (int c = 0; c < 3; c++) a.edge_residuals[3 * e + c] = r[c];
	const float s = -a.lambda * w_jac;
	const float j5[5] = {s * Rd.x, s * Rd.y, s * Rd.z, a.lambda * w_jac, -a.lambda * w_jac};
	float dEi[3][6];
	edge_block_i(j5, dEi);
	// wing block dEi^T dEj: dEj = [0 | b I]
	float* wb = a.wing + static_cast<int64_t>(e) * 36;
#pragma unroll
	for (int r0 = 0; r0 < 6; r0++)
#pragma unroll
		for (int c0 = 0; c0 < 6; c0++) {
			float v = 0.f;
			if (c0 >= 3) {
				const float dej[3] = {(c0 - 3 == 0) ? j5[4] : 0.f, (c0 - 3 == 1) ? j5[4] : 0.f, (c0 - 3 == 2) ? j5[4] : 0.f};
				v = (dEi[0][r0] * dej[0] + dEi[1][r0] * dej[1]) + dEi[2][r0] * dej[2];
			}
			wb[6 * r0 + c0] = v;
		}
	// the edge's contributions to its two nodes' diagonal blocks and gradients, summed per node by k_arrow_prepare (no
	// atomics; every node sums its incident edges in ascending edge order): source i: dEi^T dEi (21 upper-triangle
	// entries, ComputeBlockSums) + J_i^T e (6); target j: b^2 on the translation diagonal + b e (3)
	float* src = a.edge_jr + static_cast<int64_t>(e) * EDGE_TERMS;
	int q = 0;
#pragma unroll
	for (int r0 = 0; r0 < 6; r0++)
#pragma unroll
		for (int c0 = r0; c0 < 6; c0++) src[q++] = (dEi[0][r0] * dEi[0][c0] + dEi[1][r0] * dEi[1][c0]) + dEi[2][r0] * dEi[2][c0];
	const float skT[3][3] = {{0.f, j5[2], -j5[1]}, {-j5[2], 0.f, j5[0]}, {j5[1], -j5[0], 0.f}};
#pragma unroll
	for (int c = 0; c < 3; c++) {
		src[21 + c] = (skT[c][0] * r[0] + skT[c][1] * r[1]) + skT[c][2] * r[2];
		src[24 + c] = j5[3] * r[c];
	}
	src[27] = (j5[4] * j5[4] + 0.f * 0.f) + 0.f * 0.f;   // target j: dEj = [0 | b I]
#pragma unroll
	for (int c = 0; c < 3; c++) src[28 + c] = j5[4] * r[c];
	src[31] = 0.f;
}

nnrt_status launch_arap_edges(const ArapArgs& args, hipStream_t stream) {
	if (args.E == 0) return NNRT_OK;
	k_arap_edges<<<static_cast<unsigned>(ceil_div(args.E, 256)), 256, 0, stream>>>(args);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

// ---- data acc + ARAP edge terms -> full diagonal blocks (+LM) and rhs = negative gradient ----
// 32 lanes per node: lane q < 21 owns upper-triangle entry q of the 6x6 block, lanes 21..26 the gradient. The ARAP
// terms (ComputeBlockSums of dEi^T dEi / dEj^T dEj and J^T e, ArapHessianImpl.h / DeformableMeshToImageFitterImpl.h)
// are gathered from the node's incident edges (CSR, ascending edge order; entry = 2 e + (node is the edge's target)).
__global__ __launch_bounds__(256) void k_arrow_prepare(int N, float lm, double* __restrict__ acc, const int* __restrict__ inc_off,
                                                       const int* __restrict__ inc_list, const float* __restrict__ edge_terms, float* __restrict__ diag,
                                                       float* __restrict__ rhs, float* __restrict__ gradient_out, float* __restrict__ hessian_out) {
	const int n = static_cast<int>((static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 5);
	const int q = static_cast<int>(threadIdx.x & 31);
	if (n >= N) return;   // uniform per 32-lane node group
	// the term this lane sums from a source incidence / a target incidence (-1: none)
	const int q_src = q < 27 ? q : -1;
	const int q_tgt = (q == 15 || q == 18 || q == 20) ? 27 : (q >= 24 && q < 27) ? 28 + (q - 24) : -1;
	float arap = 0.f;
	const int beg = inc_off[n], end = inc_off[n + 1];
	for (int u0 = beg; u0 < end; u0 += 32) {
		const int nu = end - u0 < 32 ? end - u0 : 32;
		const int mine = q < nu ? inc_list[u0 + q] : 0;   // one incidence per lane, broadcast below
		float v[32];
#pragma unroll
		for (int u = 0; u < 32; u++) {
			const int code = __shfl(mine, u, 32);
			const int col = (code & 1) ? q_tgt : q_src;
			v[u] = (u < nu && col >= 0) ? edge_terms[static_cast<int64_t>(code >> 1) * EDGE_TERMS + col] : 0.f;
		}
#pragma unroll
		for (int u = 0; u < 32; u++)
			if (u < nu) arap += v[u];
	}
	if (q >= 27) return;
	int r0 = 0, c0 = 0;   // upper-triangle enumeration of entry q (q < 21)
	{
		int qq = q;
		while (r0 < 6 && qq >= 6 - r0) {
			qq -= 6 - r0;
			r0++;
		}
		c0 = r0 + qq;
	}
	double* ad = acc + static_cast<int64_t>(n) * ACC_STRIDE;
	const double hq = ad[q];
	ad[q] = 0.0;
	if (q < 21) {
		const float hd = static_cast<float>(hq);
		float v = arap + hd;
		if (r0 == c0 && lm > 0.f) v += lm;
		float* d = diag + static_cast<int64_t>(n) * 36;
		d[6 * r0 + c0] = v;
		d[6 * c0 + r0] = v;
		if (hessian_out) {
			hessian_out[static_cast<int64_t>(n) * 36 + 6 * r0 + c0] = hd;
			hessian_out[static_cast<int64_t>(n) * 36 + 6 * c0 + r0] = hd;
		}
	} else {
		const float g = (0.f - static_cast<float>(hq)) - arap;
		rhs[6 * static_cast<int64_t>(n) + q - 21] = g;
		gradient_out[6 * static_cast<int64_t>(n) + q - 21] = g;
	}
}

// ---- corner init: S = C (diagonal corner blocks + corner off-diagonal blocks), identity on the padding; cb = b_C ----
// One thread per 4 consecutive entries of a row (one 16-B store; 32-bit index arithmetic: ld <= 32768). Strictly-upper
// 64 x 64 tiles are left unwritten: the factorization and both substitutions touch tiles I >= J only (k_chol_step,
// k_chol_back_group), so half the corner's bytes need no initialisation.
__global__ void k_arrow_corner_init(int n0, int m, int ld, const float* __restrict__ diag, float* __restrict__ S, const float* __restrict__ rhs,
                                    float* __restrict__ cb) {
	const int q = ld >> 2;
	const int idx = static_cast<int>(blockIdx.x) * static_cast<int>(blockDim.x) + static_cast<int>(threadIdx.x);
	if (idx >= ld * q) return;
	const int r = idx / q, c0 = (idx - r * q) * 4;
	if (c0 == 0) cb[r] = r < m ? rhs[6 * static_cast<int64_t>(n0) + r] : 0.f;
	if ((c0 / CORNER_NB) > (r / CORNER_NB)) return;
	float v[4];
#pragma unroll
	for (int j = 0; j < 4; j++) {
		const int c = c0 + j;
		v[j] = 0.f;
		if (r < m && c < m) {
			if (r / 6 == c / 6) v[j] = diag[static_cast<int64_t>(n0 + r / 6) * 36 + 6 * (r % 6) + (c % 6)];
		} else if (r == c) {
			v[j] = 1.f;
		}
	}
	*reinterpret_cast<float4*>(S + static_cast<int64_t>(r) * ld + c0) = make_float4(v[0], v[1], v[2], v[3]);
}

__global__ void k_arrow_corner_offdiag(int E, int n0, int ld, const int32_t* __restrict__ edges, const float* __restrict__ wing,
                                       float* __restrict__ S) {
	const int e = blockIdx.x;
	const int i = edges[2 * e], j = edges[2 * e + 1];
	if (i < n0) return;
	const int t = threadIdx.x;
	if (t >= 36) return;
	const int r = t / 6, c = t % 6;
	const float v = wing[static_cast<int64_t>(e) * 36 + t];
	const int ai = i - n0, bj = j - n0;
	atomicAdd(S + static_cast<int64_t>(6 * ai + r) * ld + 6 * bj + c, v);
	atomicAdd(S + static_cast<int64_t>(6 * bj + c) * ld + 6 * ai + r, v);
	(void) E;
}

// ---- stem: D^-1 and D^-1 B per stem node (one thread per stem node) ----
__global__ __launch_bounds__(64) void k_arrow_stem(int n0, const float* __restrict__ diag, const int* __restrict__ edge_offsets, const int* __restrict__ edge_list,
                             const float* __restrict__ wing, float* __restrict__ dinv, float* __restrict__ dinv_b, int* error_flag) {
	const int i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n0) return;
	// 6 x 6 blocks are 144 B = nine 16-B words: loaded and stored as float4
	float L[6][6];
	{
		const float4* d4 = reinterpret_cast<const float4*>(diag + static_cast<int64_t>(i) * 36);
		float f[36];
#pragma unroll
		for (int q = 0; q < 9; q++) {
			const float4 v = d4[q];
			f[4 * q] = v.x;
			f[4 * q + 1] = v.y;
			f[4 * q + 2] = v.z;
			f[4 * q + 3] = v.w;
		}
#pragma unroll
		for (int k = 0; k < 36; k++) L[k / 6][k % 6] = f[k];
	}
	if (!cholesky_small<6>(L)) {
		atomicOr(error_flag, 1);
		return;
	}
	float Di[6][6];
	invert_from_cholesky_small<6>(L, Di);
	float4* o4 = reinterpret_cast<float4*>(dinv + static_cast<int64_t>(i) * 36);
#pragma unroll
	for (int q = 0; q < 9; q++)
		o4[q] = make_float4(Di[(4 * q) / 6][(4 * q) % 6], Di[(4 * q + 1) / 6][(4 * q + 1) % 6], Di[(4 * q + 2) / 6][(4 * q + 2) % 6],
		                    Di[(4 * q + 3) / 6][(4 * q + 3) % 6]);
	for (int ei = edge_offsets[i]; ei < edge_offsets[i + 1]; ei++) {
		const int e = edge_list[ei];
		const float4* B4 = reinterpret_cast<const float4*>(wing + static_cast<int64_t>(e) * 36);
		float B[36];
#pragma unroll
		for (int q = 0; q < 9; q++) {
			const float4 v = B4[q];
			B[4 * q] = v.x;
			B[4 * q + 1] = v.y;
			B[4 * q + 2] = v.z;
			B[4 * q + 3] = v.w;
		}
		float Y[36];
#pragma unroll
		for (int r = 0; r < 6; r++)
#pragma unroll
			for (int c = 0; c < 6; c++) {
				float acc = 0.f;
#pragma unroll
				for (int k = 0; k < 6; k++) acc += Di[r][k] * B[6 * k + c];
				Y[6 * r + c] = acc;
			}
		float4* Y4 = reinterpret_cast<float4*>(dinv_b + static_cast<int64_t>(e) * 36);
#pragma unroll
		for (int q = 0; q < 9; q++) Y4[q] = make_float4(Y[4 * q], Y[4 * q + 1], Y[4 * q + 2], Y[4 * q + 3]);
	}
}

// ---- Schur update S_ab -= sum over stem nodes i adjacent to a and b of B_ia^T D_i^-1 B_ib (one wave per target) ----
// Lane (r, c) < 36 owns entry (r, c) of the 6x6 target block. The target's pair list is loaded once, one pair per lane,
// and broadcast by shuffle, so the wing / D^-1 B loads of eight pairs are in flight together (no dependent index load
// per pair). Pairs are summed in list order.
__global__ __launch_bounds__(256) void k_stem_schur(int targets, int ld, const int* __restrict__ tgt_off, const int2* __restrict__ tgt_ab,
                                                    const int2* __restrict__ pairs, const float* __restrict__ wing, const float* __restrict__ dinv_b,
                                                    float* __restrict__ S) {
	const int w = static_cast<int>((static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6);
	const int lane = static_cast<int>(threadIdx.x & 63);
	if (w >= targets) return;
	const int r = lane < 36 ? lane / 6 : 0, c = lane < 36 ? lane % 6 : 0;
	const int beg = tgt_off[w], end = tgt_off[w + 1];
	float acc = 0.f;
	for (int p0 = beg; p0 < end; p0 += 64) {
		const int np = end - p0 < 64 ? end - p0 : 64;
		const int2 mine = lane < np ? pairs[p0 + lane] : make_int2(0, 0);
		for (int u0 = 0; u0 < np; u0 += 8) {
			float b1[8][6], y2[8][6];
#pragma unroll
			for (int u = 0; u < 8; u++) {
				const int e1 = __shfl(mine.x, u0 + u), e2 = __shfl(mine.y, u0 + u);
				const bool live = u0 + u < np;
				const float* B1 = wing + static_cast<int64_t>(live ? e1 : 0) * 36;
				const float* Y2 = dinv_b + static_cast<int64_t>(live ? e2 : 0) * 36;
#pragma unroll
				for (int k = 0; k < 6; k++) {
					b1[u][k] = live ? B1[6 * k + r] : 0.f;
					y2[u][k] = live ? Y2[6 * k + c] : 0.f;
				}
			}
#pragma unroll
			for (int u = 0; u < 8; u++) {
				if (u0 + u < np) {
					float sum = 0.f;
#pragma unroll
					for (int k = 0; k < 6; k++) sum += b1[u][k] * y2[u][k];
					acc += sum;
				}
			}
		}
	}
	if (lane < 36) {
		const int2 ab = tgt_ab[w];
		S[static_cast<int64_t>(6 * ab.x + r) * ld + 6 * ab.y + c] -= acc;
	}
}

// ---- fitter form of the Schur update: the ARAP wing blocks dEi^T dEj (dEj = [0 | b I]) are zero outside their last
// three columns, so B_ia^T D_i^-1 B_ib is zero outside its lower-right 3x3 block and only those 9 entries change
// (the others would subtract exact zeros). 7 pair slots x 9 entries per wave; slots reduced in order at the end.
__global__ __launch_bounds__(256) void k_stem_schur_t3(int targets, int ld, const int* __restrict__ tgt_off, const int2* __restrict__ tgt_ab,
                                                       const int2* __restrict__ pairs, const float* __restrict__ wing,
                                                       const float* __restrict__ dinv_b, float* __restrict__ S) {
	__shared__ float s_part[4][7][9];
	const int w = static_cast<int>((static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6);
	const int lane = static_cast<int>(threadIdx.x & 63), wl = static_cast<int>(threadIdx.x >> 6);
	if (w >= targets) return;
	const int slot = lane < 63 ? lane / 9 : 6, ent = lane < 63 ? lane % 9 : 0;
	const int r = 3 + ent / 3, c = 3 + ent % 3;
	const int beg = tgt_off[w], end = tgt_off[w + 1];
	float acc = 0.f;
	for (int p0 = beg; p0 < end; p0 += 14) {
		float b1[2][6], y2[2][6];
		bool live[2];
#pragma unroll
		for (int h = 0; h < 2; h++) {
			const int p = p0 + 7 * h + slot;
			live[h] = lane < 63 && p < end;
			const int2 e = live[h] ? pairs[p] : make_int2(0, 0);
			const float* B1 = wing + static_cast<int64_t>(e.x) * 36;
			const float* Y2 = dinv_b + static_cast<int64_t>(e.y) * 36;
#pragma unroll
			for (int k = 0; k < 6; k++) {
				b1[h][k] = live[h] ? B1[6 * k + r] : 0.f;
				y2[h][k] = live[h] ? Y2[6 * k + c] : 0.f;
			}
		}
#pragma unroll
		for (int h = 0; h < 2; h++)
			if (live[h]) {
				float sum = 0.f;
#pragma unroll
				for (int k = 0; k < 6; k++) sum += b1[h][k] * y2[h][k];
				acc += sum;
			}
	}
	if (lane < 63) s_part[wl][slot][ent] = acc;
	__builtin_amdgcn_wave_barrier();   // LDS is in order within the wave; keep the compiler from moving the reads up
	if (lane < 9) {
		float t = 0.f;
#pragma unroll
		for (int sl = 0; sl < 7; sl++) t += s_part[wl][sl][lane];
		const int2 ab = tgt_ab[w];
		S[static_cast<int64_t>(6 * ab.x + 3 + lane / 3) * ld + 6 * ab.y + 3 + lane % 3] -= t;
	}
}

// ---- b_C -= sum over stem edges i->a of (D_i^-1 B_ia)^T b_i (one wave per corner node; lanes over its edges) ----
__global__ __launch_bounds__(256) void k_stem_rhs(int nc, const int* __restrict__ rhs_off, const int* __restrict__ rhs_edges,
                                                  const int32_t* __restrict__ edges, const float* __restrict__ dinv_b, const float* __restrict__ rhs,
                                                  float* __restrict__ cb) {
	const int a = static_cast<int>((static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6);
	const int lane = static_cast<int>(threadIdx.x & 63);
	if (a >= nc) return;
	float s[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
	for (int q = rhs_off[a] + lane; q < rhs_off[a + 1]; q += 64) {
		const int e = rhs_edges[q];
		const int i = edges[2 * e];
		const float* Y = dinv_b + static_cast<int64_t>(e) * 36;
		const float* g = rhs + 6 * static_cast<int64_t>(i);
		float gk[6];
#pragma unroll
		for (int k = 0; k < 6; k++) gk[k] = g[k];
#pragma unroll
		for (int c = 0; c < 6; c++) {
			float t = 0.f;
#pragma unroll
			for (int k = 0; k < 6; k++) t += Y[6 * k + c] * gk[k];
			s[c] += t;
		}
	}
#pragma unroll
	for (int c = 0; c < 6; c++) {
#pragma unroll
		for (int off = 32; off > 0; off >>= 1) s[c] += __shfl_xor(s[c], off);
	}
	if (lane < 6) {
		float v = s[0];
#pragma unroll
		for (int c = 1; c < 6; c++) v = lane == c ? s[c] : v;
		cb[6 * static_cast<int64_t>(a) + lane] -= v;
	}
}

StemSchurLists build_stem_schur_lists(const int32_t* edges, int E, int n0, int N) {
	StemSchurLists L;
	const int nc = N - n0;
	std::vector<std::vector<int>> out(static_cast<size_t>(n0));
	std::vector<int> rhs_count(static_cast<size_t>(nc) + 1, 0);
	for (int e = 0; e < E; e++) {
		const int i = edges[2 * e], j = edges[2 * e + 1];
		if (i < n0 && j >= n0) {
			out[static_cast<size_t>(i)].push_back(e);
			rhs_count[static_cast<size_t>(j - n0) + 1]++;
		}
	}
	L.rhs_off.assign(rhs_count.begin(), rhs_count.end());
	for (int a = 0; a < nc; a++) L.rhs_off[static_cast<size_t>(a) + 1] += L.rhs_off[static_cast<size_t>(a)];
	L.rhs_edges.assign(static_cast<size_t>(L.rhs_off.back()), 0);
	std::vector<int> fill(L.rhs_off.begin(), L.rhs_off.end() - 1);
	struct Q {
		int a, b, e1, e2;
	};
	std::vector<Q> q;
	for (int i = 0; i < n0; i++) {
		const auto& es = out[static_cast<size_t>(i)];
		for (int e1 : es) {
			L.rhs_edges[static_cast<size_t>(fill[static_cast<size_t>(edges[2 * e1 + 1] - n0)]++)] = e1;
			for (int e2 : es) {
				const int a = edges[2 * e1 + 1] - n0, b = edges[2 * e2 + 1] - n0;
				if (a >= b) q.push_back({a, b, e1, e2});
			}
		}
	}
	std::stable_sort(q.begin(), q.end(), [](const Q& x, const Q& y) { return x.a != y.a ? x.a < y.a : x.b < y.b; });
	L.tgt_off.push_back(0);
	for (size_t k = 0; k < q.size(); k++) {
		if (k == 0 || q[k].a != q[k - 1].a || q[k].b != q[k - 1].b) {
			if (k > 0) L.tgt_off.push_back(static_cast<int>(k));
			L.tgt_ab.push_back(make_int2(q[k].a, q[k].b));
		}
		L.pairs.push_back(make_int2(q[k].e1, q[k].e2));
	}
	if (!q.empty()) L.tgt_off.push_back(static_cast<int>(q.size()));
	return L;
}

// ---- dense corner: blocked right-looking Cholesky of S (ld x ld, row-major, lower triangle) and S x = b -------------
// SolveBlockSparseArrowheadCholesky.cpp:30-95 factors the Schur complement with a dense potrf. Here ONE launch per
// 64-column block k (k_chol_step), whose workgroups play two roles:
//   panel   (block rows I >= k, dealt first): apply the previous block's update to the two tiles this row needs,
//           A_kk -= L_k,k-1 L_k,k-1^T and A_Ik -= L_I,k-1 L_k,k-1^T (f32 MFMA, v_mfma_f32_32x32x2_f32, one 32 x 32
//           quadrant per wave, into LDS); then one wave holds both tiles (lane = row) in registers and runs the 64
//           column eliminations of A_kk, applying each to its panel row as it goes (one packed FMA per column pair):
//           L_kk and L_Ik = A_Ik L_kk^-T come out of one pass with no inverse. The right-hand side rides along as the
//           panel row of the diagonal workgroup (lane 0): y_k = L_kk^-1 b_k.
//   trailing (tiles k < J <= I): A_IJ -= L_I,k-1 L_J,k-1^T on the MFMA, and b_J -= L_J,k-1 y_k-1 by the diagonal tiles.
// Every operand of launch k was finished by launch k - 1, so consecutive launches are the only synchronisation.
// The block back substitution L^T x = y then runs BACK_G block rows per launch (k_chol_back_group).
constexpr int CT = 256;   // threads per workgroup of the corner kernels
constexpr int CORNER_LAZY = 4;   // trailing columns are updated every CORNER_LAZY-th launch (k_chol_step; C5: 2 / 3 / 4 / 5 / 6
                                 // / 8 -> 769 / 743 / 737 / 749 / 814 / 950 us solve stage)
constexpr int CS4 = CORNER_NB + 4;   // LDS row stride of the staged tiles (16-B aligned rows for ds_read_b128)

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ inline float lane_bcast(float v, int src) {
	return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), src));
}

// 32 x 32 quadrant (qr, qc) of X Y^T for X, Y 64 x 64 row-major tiles at row stride ld (lane l feeds
// A[i = l & 31][k'] = X[32 qr + i][32 (l >> 5) + s] and B[k'][j] = Y[32 qc + j][32 (l >> 5) + s] to MFMA step s, so the 32
// steps x 2 lane halves cover the 64-wide k range; each lane reads 32 contiguous floats). C/D map: column l & 31, row
// (v & 3) + 8 (v >> 2) + 4 (l >> 5).
__device__ inline f32x16 quadrant_xyt(const float* X, const float* Y, int64_t ld, int qr, int qc, int lane, f32x16 acc = {}) {
	const int half = lane >> 5, l32 = lane & 31;
	const float4* x4 = reinterpret_cast<const float4*>(X + (32 * qr + l32) * ld + 32 * half);
	const float4* y4 = reinterpret_cast<const float4*>(Y + (32 * qc + l32) * ld + 32 * half);
	float4 vx[8], vy[8];
#pragma unroll
	for (int q = 0; q < 8; q++) {
		vx[q] = x4[q];
		vy[q] = y4[q];
	}
#pragma unroll
	for (int q = 0; q < 8; q++) {
		acc = __builtin_amdgcn_mfma_f32_32x32x2f32(vx[q].x, vy[q].x, acc, 0, 0, 0);
		acc = __builtin_amdgcn_mfma_f32_32x32x2f32(vx[q].y, vy[q].y, acc, 0, 0, 0);
		acc = __builtin_amdgcn_mfma_f32_32x32x2f32(vx[q].z, vy[q].z, acc, 0, 0, 0);
		acc = __builtin_amdgcn_mfma_f32_32x32x2f32(vx[q].w, vy[q].w, acc, 0, 0, 0);
	}
	return acc;
}

__device__ inline int quad_row(int v, int lane) { return (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5); }

// s_t[r][c] = T[r][c] - (X Y^T)[r][c] for the workgroup's quadrant of a 64 x 64 tile T (global, row stride ld)
__device__ inline void stage_updated_tile(const float* T, const float* X, const float* Y, int64_t ld, int wave, int lane, float* s_t) {
	const int qr = wave >> 1, qc = wave & 1;
	float tv[16];
#pragma unroll
	for (int v = 0; v < 16; v++) tv[v] = T[(32 * qr + quad_row(v, lane)) * ld + 32 * qc + (lane & 31)];
	const f32x16 acc = quadrant_xyt(X, Y, ld, qr, qc, lane);
#pragma unroll
	for (int v = 0; v < 16; v++) s_t[(32 * qr + quad_row(v, lane)) * CS4 + 32 * qc + (lane & 31)] = tv[v] - acc[v];
}

// b_J -= L_J y for a 64 x 64 tile L (row stride ld) and the 64-vector y: 4 threads per row, 16 columns each
__device__ inline float rhs_row_update(const float* L, int64_t ld, const float* y, int t) {
	const int r = t >> 2, q4 = t & 3;
	const float* Lr = L + r * ld + 16 * q4;
	const float* yq = y + 16 * q4;
	float s0 = 0.f, s1 = 0.f;
#pragma unroll
	for (int c = 0; c < 16; c += 2) {
		s0 += Lr[c] * yq[c];
		s1 += Lr[c + 1] * yq[c + 1];
	}
	float s = s0 + s1;
	s += __shfl_xor(s, 1);
	s += __shfl_xor(s, 2);
	return s;
}


// Column eliminations J0 <= j < J1 of the row pairs ap (lane = row), applied to the columns c < J1 only, in blocks of
// four: the four columns are factored among themselves, then applied to every later column c with four packed FMAs
// whose multipliers L_c,jb..jb+3 are read from lane c by readlane (scalar operands: nothing on the elimination path
// waits on LDS). Every element sees its updates in ascending column order.
template <int J0, int J1>
__device__ inline void eliminate_columns(f32x2 (&ap)[CORNER_NB], int lane, int& bad) {
	__shared__ float4 s_l4[2][CORNER_NB];   // s_l4[.][c] = (L_c,jb .. L_c,jb+3)
#pragma clang loop unroll(full)
	for (int jb = J0; jb < J1; jb += 4) {
		// The 4 x 4 diagonal sub-block is read once (10 independent readlanes) and factored wave-uniformly; every lane
		// then runs the same operations on its own row with the uniform multipliers. The uniform values are exactly
		// the ones lanes jb..jb+3 compute (same operations, same order), so the pivot chain has no readlane round trip
		// per column.
		float M[4][4], Lu[4][4], rsv[4];
#pragma unroll
		for (int q = 0; q < 4; q++)
#pragma unroll
			for (int i = q; i < 4; i++) M[i][q] = lane_bcast(ap[jb + q].x, jb + i);
#pragma unroll
		for (int q = 0; q < 4; q++) {
			float piv = M[q][q];   // A_jj after the first j eliminations
			bad |= !(piv > 0.f);
			piv = piv > 0.f ? piv : 1.f;
			rsv[q] = __builtin_amdgcn_rsqf(piv);
#pragma unroll
			for (int i = q; i < 4; i++) Lu[i][q] = M[i][q] * rsv[q];
#pragma unroll
			for (int q2 = q + 1; q2 < 4; q2++)
#pragma unroll
				for (int i = q2; i < 4; i++) M[i][q2] = __builtin_fmaf(-Lu[i][q], Lu[q2][q], M[i][q2]);
		}
		float lx[4];
		f32x2 nl[4];
#pragma unroll
		for (int q = 0; q < 4; q++) {
			const f32x2 l = ap[jb + q] * rsv[q];   // (L_rj for rows r >= j of the diagonal block, panel / rhs entry)
			ap[jb + q] = l;
			lx[q] = l.x;
			nl[q] = -l;
#pragma unroll
			for (int q2 = q + 1; q2 < 4; q2++) {
				const float lc = Lu[q2][q];
				ap[jb + q2] = __builtin_elementwise_fma(nl[q], f32x2{lc, lc}, ap[jb + q2]);
			}
		}
		// next block's columns first (readlane: on the pivot chain), the rest from a wave-uniform 16-B LDS broadcast
		// whose latency hides behind them
		float4* row = &s_l4[(jb >> 2) & 1][0];
		if (jb + 8 < J1) row[lane] = make_float4(lx[0], lx[1], lx[2], lx[3]);
#pragma unroll
		for (int q = 0; q < 4; q++)   // q outer: consecutive FMAs are independent
#pragma unroll
			for (int c = jb + 4; c < J1 && c < jb + 8; c++) {
				const float lc = lane_bcast(lx[q], c);   // L_c,jb+q, c > jb + 3
				ap[c] = __builtin_elementwise_fma(nl[q], f32x2{lc, lc}, ap[c]);
			}
#pragma unroll
		for (int c0 = jb + 8; c0 < J1; c0 += 8) {   // chunks of 8 columns: 8 broadcasts in flight
			float4 L4[8];
#pragma unroll
			for (int u = 0; u < 8; u++)
				if (c0 + u < J1) L4[u] = row[c0 + u];
#pragma unroll
			for (int u = 0; u < 8; u++)
				if (c0 + u < J1) ap[c0 + u] = __builtin_elementwise_fma(nl[0], f32x2{L4[u].x, L4[u].x}, ap[c0 + u]);
#pragma unroll
			for (int u = 0; u < 8; u++)
				if (c0 + u < J1) ap[c0 + u] = __builtin_elementwise_fma(nl[1], f32x2{L4[u].y, L4[u].y}, ap[c0 + u]);
#pragma unroll
			for (int u = 0; u < 8; u++)
				if (c0 + u < J1) ap[c0 + u] = __builtin_elementwise_fma(nl[2], f32x2{L4[u].z, L4[u].z}, ap[c0 + u]);
#pragma unroll
			for (int u = 0; u < 8; u++)
				if (c0 + u < J1) ap[c0 + u] = __builtin_elementwise_fma(nl[3], f32x2{L4[u].w, L4[u].w}, ap[c0 + u]);
		}
	}
}

__global__ __launch_bounds__(CT) void k_chol_step(float* __restrict__ A, int ld, int k, int T, float* __restrict__ b, int* error_flag) {
	__shared__ float s_d[CORNER_NB * CS4];   // A_kk after the previous block's update
	__shared__ float s_p[CORNER_NB * CS4];   // A_Ik after the previous block's update (panel workgroups below the diagonal)
	__shared__ float s_b[CORNER_NB];         // b_k after the previous block's update (diagonal workgroup)
	const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
	const int64_t LD = ld;
	const int npanel = T - k;
	const int64_t ok0 = static_cast<int64_t>(k) * CORNER_NB, op = ok0 - CORNER_NB;   // column offsets of blocks k and k - 1
	if (static_cast<int>(blockIdx.x) >= npanel) {
		// ---- trailing tile (I, J), k < J <= I: lazy updates. Launch k updates the columns J = k + 1, k + 1 + LAZY, ..
		// (every tile I >= J of them) with their pending blocks max(0, k - LAZY) .. k - 1: each column takes LAZY blocks
		// every LAZY-th launch (1 / LAZY of the tile passes of one update per block) and is complete up to block J - 2
		// when its panel launch stages block J - 1.
		int r = static_cast<int>(blockIdx.x) - npanel, m = 0, cnt = T - (k + 1);
		while (r >= cnt) {   // column k + 1 + LAZY m holds T - (k + 1 + LAZY m) tiles
			r -= cnt;
			m++;
			cnt -= CORNER_LAZY;
		}
		const int jj = CORNER_LAZY * m, ii = jj + r;   // J = k + 1 + jj, I = k + 1 + ii
		const int b0 = k >= CORNER_LAZY ? k - CORNER_LAZY : 0;
		const int64_t rI = static_cast<int64_t>(k + 1 + ii) * CORNER_NB, rJ = static_cast<int64_t>(k + 1 + jj) * CORNER_NB;
		const int qr = wave >> 1, qc = wave & 1;
		float* C = A + rI * LD + rJ + 32 * qc + (lane & 31);
		float cv[16];
#pragma unroll
		for (int v = 0; v < 16; v++) cv[v] = C[(32 * qr + quad_row(v, lane)) * LD];
		// one product per pending block, subtracted in block order: the same float operations as one update per launch
		for (int pb = b0; pb < k; pb++) {
			const int64_t ob = static_cast<int64_t>(pb) * CORNER_NB;
			const f32x16 acc = quadrant_xyt(A + rI * LD + ob, A + rJ * LD + ob, LD, qr, qc, lane);
#pragma unroll
			for (int v = 0; v < 16; v++) cv[v] -= acc[v];
		}
#pragma unroll
		for (int v = 0; v < 16; v++) C[(32 * qr + quad_row(v, lane)) * LD] = cv[v];
		if (rI == rJ) {
			float bj = (t & 3) == 0 ? b[rJ + (t >> 2)] : 0.f;
			for (int pb = b0; pb < k; pb++) {
				const int64_t ob = static_cast<int64_t>(pb) * CORNER_NB;
				bj -= rhs_row_update(A + rJ * LD + ob, LD, b + ob, t);
			}
			if ((t & 3) == 0) b[rJ + (t >> 2)] = bj;
		}
		return;
	}
	// ---- panel row I = k + blockIdx.x ----
	const bool diag = blockIdx.x == 0;
	const int64_t rI = ok0 + static_cast<int64_t>(blockIdx.x) * CORNER_NB;
	if (k > 0) {
		stage_updated_tile(A + ok0 * LD + ok0, A + ok0 * LD + op, A + ok0 * LD + op, LD, wave, lane, s_d);
		if (!diag) {
			stage_updated_tile(A + rI * LD + ok0, A + rI * LD + op, A + ok0 * LD + op, LD, wave, lane, s_p);
		} else {
			const float s = rhs_row_update(A + ok0 * LD + op, LD, b + op, t);
			if ((t & 3) == 0) s_b[t >> 2] = b[ok0 + (t >> 2)] - s;
		}
	} else {
		for (int e = t; e < CORNER_NB * CORNER_NB; e += CT) {
			const int rr = e / CORNER_NB, cc = e % CORNER_NB;
			s_d[rr * CS4 + cc] = A[(ok0 + rr) * LD + ok0 + cc];
			if (!diag) s_p[rr * CS4 + cc] = A[(rI + rr) * LD + ok0 + cc];
		}
		if (diag && t < CORNER_NB) s_b[t] = b[ok0 + t];
	}
	__syncthreads();
	// ap[c] = (A_kk[lane][c], A_Ik[lane][c]): both rows see the same column operations, so one packed FMA
	// (v_pk_fma_f32) updates the pair. Wave 0 holds them; the other waves join for the rank-32 update between the halves.
	f32x2 ap[CORNER_NB];
	int bad = 0;
	if (wave == 0) {
#pragma unroll
		for (int q = 0; q < CORNER_NB / 4; q++) {
			const float4 va = *reinterpret_cast<const float4*>(s_d + lane * CS4 + 4 * q);
			float4 vp;
			if (diag)   // the augmented row: b_k on lane 0, zero elsewhere
				vp = lane == 0 ? *reinterpret_cast<const float4*>(s_b + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
			else
				vp = *reinterpret_cast<const float4*>(s_p + lane * CS4 + 4 * q);
			ap[4 * q] = f32x2{va.x, vp.x};
			ap[4 * q + 1] = f32x2{va.y, vp.y};
			ap[4 * q + 2] = f32x2{va.z, vp.z};
			ap[4 * q + 3] = f32x2{va.w, vp.w};
		}
		eliminate_columns<0, CORNER_NB / 2>(ap, lane, bad);
		// L[:, 0:32] of the A_kk rows and of the panel rows -> LDS (s_d / s_p are free once loaded)
#pragma unroll
		for (int q = 0; q < CORNER_NB / 8; q++) {
			*reinterpret_cast<float4*>(s_d + lane * CS4 + 4 * q) = make_float4(ap[4 * q].x, ap[4 * q + 1].x, ap[4 * q + 2].x, ap[4 * q + 3].x);
			*reinterpret_cast<float4*>(s_p + lane * CS4 + 4 * q) = make_float4(ap[4 * q].y, ap[4 * q + 1].y, ap[4 * q + 2].y, ap[4 * q + 3].y);
		}
	}
	__syncthreads();
	// rank-32 update of columns 32..63: C = L[rows, 0:32] L_kk[32:64, 0:32]^T on the MFMA, one 32-row block per wave
	// (wave 1: A_kk rows 32..63; waves 2, 3: panel rows 0..31, 32..63; A_kk rows 0..31 lie above the diagonal there)
	f32x16 cacc = {};
	if (wave > 0) {
		const float* X = wave == 1 ? s_d + 32 * CS4 : s_p + 32 * (wave - 2) * CS4;
		const int half = lane >> 5, l32 = lane & 31;
		const float4* x4 = reinterpret_cast<const float4*>(X + l32 * CS4 + 16 * half);
		const float4* y4 = reinterpret_cast<const float4*>(s_d + (32 + l32) * CS4 + 16 * half);
#pragma unroll
		for (int q = 0; q < 4; q++) {
			const float4 vx = x4[q], vy = y4[q];
			cacc = __builtin_amdgcn_mfma_f32_32x32x2f32(vx.x, vy.x, cacc, 0, 0, 0);
			cacc = __builtin_amdgcn_mfma_f32_32x32x2f32(vx.y, vy.y, cacc, 0, 0, 0);
			cacc = __builtin_amdgcn_mfma_f32_32x32x2f32(vx.z, vy.z, cacc, 0, 0, 0);
			cacc = __builtin_amdgcn_mfma_f32_32x32x2f32(vx.w, vy.w, cacc, 0, 0, 0);
		}
	}
	__syncthreads();   // every wave is done reading L before the products overwrite it
	if (wave > 0) {
		float* Cb = wave == 1 ? s_d + 32 * CS4 : s_p + 32 * (wave - 2) * CS4;
#pragma unroll
		for (int v = 0; v < 16; v++) Cb[quad_row(v, lane) * CS4 + 32 + (lane & 31)] = cacc[v];
	}
	__syncthreads();
	if (wave != 0) return;
#pragma unroll
	for (int q = CORNER_NB / 8; q < CORNER_NB / 4; q++) {
		const float4 ca = lane >= 32 ? *reinterpret_cast<const float4*>(s_d + lane * CS4 + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
		const float4 cp = *reinterpret_cast<const float4*>(s_p + lane * CS4 + 4 * q);
		ap[4 * q] -= f32x2{ca.x, cp.x};
		ap[4 * q + 1] -= f32x2{ca.y, cp.y};
		ap[4 * q + 2] -= f32x2{ca.z, cp.z};
		ap[4 * q + 3] -= f32x2{ca.w, cp.w};
	}
	eliminate_columns<CORNER_NB / 2, CORNER_NB>(ap, lane, bad);
	const bool ok = !bad;
	if (diag) {
		float4* wa = reinterpret_cast<float4*>(A + (ok0 + lane) * LD + ok0);
#pragma unroll
		for (int q = 0; q < CORNER_NB / 4; q++)
			wa[q] = make_float4(4 * q <= lane ? ap[4 * q].x : 0.f, 4 * q + 1 <= lane ? ap[4 * q + 1].x : 0.f,
			                    4 * q + 2 <= lane ? ap[4 * q + 2].x : 0.f, 4 * q + 3 <= lane ? ap[4 * q + 3].x : 0.f);
		if (lane == 0) {
			float4* wb = reinterpret_cast<float4*>(b + ok0);
#pragma unroll
			for (int q = 0; q < CORNER_NB / 4; q++) wb[q] = make_float4(ap[4 * q].y, ap[4 * q + 1].y, ap[4 * q + 2].y, ap[4 * q + 3].y);
			if (!ok) atomicOr(error_flag, 1);
		}
	} else {
		float4* wp = reinterpret_cast<float4*>(A + (rI + lane) * LD + ok0);
#pragma unroll
		for (int q = 0; q < CORNER_NB / 4; q++) wp[q] = make_float4(ap[4 * q].y, ap[4 * q + 1].y, ap[4 * q + 2].y, ap[4 * q + 3].y);
	}
}

// ---- block back substitution L^T x = y, BACK_G block rows per launch (from the last block up) ----------------------
// Launch for blocks k0, k0 - 1, .., kl (g = k0 - block): wave g holds L_{k0-g,k0-g} by columns in registers; as soon as
// x_{k0-g2} is known every later wave subtracts L_{k0-g2,k0-g}^T x_{k0-g2} from its z (coupling tiles staged in LDS by
// the whole workgroup), and wave g, once its z is complete, solves L^T x = z by column-oriented substitution (x_i broadcast by readlane; lane = column, so column i of L^T is the lanes'
// register i). Every workgroup forms the group's x redundantly; workgroup i < kl then applies y_i -= sum L_ki^T x_k
// (its tiles prefetched meanwhile) and the group's own workgroups store x (into xout, not over y).
constexpr int BACK_G = 4;

__global__ __launch_bounds__(CT) void k_chol_back_group(const float* __restrict__ A, int ld, int k0, int kl, float* __restrict__ b, int m,
                                                       float* __restrict__ xout) {
	__shared__ float s_cpl[BACK_G * (BACK_G - 1) / 2][CORNER_NB][CORNER_NB + 1];   // [g(g-1)/2 + g2][r][c] = L_{k0-g2,k0-g}[r][c]
	__shared__ __attribute__((aligned(16))) float s_x[BACK_G][CORNER_NB];
	__shared__ float s_part[4][CORNER_NB];
	const int t = threadIdx.x, c = t % CORNER_NB, seg = t / CORNER_NB, wave = t >> 6, lane = t & 63;
	const int i = static_cast<int>(blockIdx.x);   // target block (i >= kl: a block of the group, store its x)
	const int64_t LD = ld, ci = static_cast<int64_t>(i) * CORNER_NB;
	const int G = k0 - kl + 1;
	float lk[BACK_G][16];
	if (i < kl) {   // L_ki (rows of block k, columns of block i) for the target update
#pragma unroll
		for (int g = 0; g < BACK_G; g++)
			if (g < G) {
				const int64_t ck = static_cast<int64_t>(k0 - g) * CORNER_NB;
#pragma unroll
				for (int q = 0; q < 16; q++) lk[g][q] = A[(ck + seg * 16 + q) * LD + ci + c];
			}
	}
	for (int g = 1; g < G; g++)
		for (int g2 = 0; g2 < g; g2++) {
			const int64_t rr = static_cast<int64_t>(k0 - g2) * CORNER_NB, cc = static_cast<int64_t>(k0 - g) * CORNER_NB;
			float(*dst)[CORNER_NB + 1] = s_cpl[g * (g - 1) / 2 + g2];
#pragma unroll
			for (int q = 0; q < 16; q++) dst[seg * 16 + q][c] = A[(rr + seg * 16 + q) * LD + cc + c];
		}
	float col[CORNER_NB];   // wave g: col[r] = L_kk[r][lane], k = k0 - g
	float inv_d = 1.f, z = 0.f;
	if (wave < G) {
		const int64_t ok = static_cast<int64_t>(k0 - wave) * CORNER_NB;
#pragma unroll
		for (int r = 0; r < CORNER_NB; r++) col[r] = A[(ok + r) * LD + ok + lane];
		inv_d = 1.f / A[(ok + lane) * LD + ok + lane];
		z = b[ok + lane];
	}
	for (int g = 0; g < G; g++) {
		__syncthreads();   // x_{g-1} and the staged coupling tiles are visible
		if (g > 0 && wave >= g && wave < G) {   // every later block applies the newest x at once (off the chain)
			const float(*cp)[CORNER_NB + 1] = s_cpl[wave * (wave - 1) / 2 + g - 1];
			const float4* xv = reinterpret_cast<const float4*>(s_x[g - 1]);
			float s0 = 0.f, s1 = 0.f;
#pragma unroll
			for (int r4 = 0; r4 < CORNER_NB / 4; r4++) {
				const float4 x4 = xv[r4];
				s0 += cp[4 * r4][lane] * x4.x;
				s1 += cp[4 * r4 + 1][lane] * x4.y;
				s0 += cp[4 * r4 + 2][lane] * x4.z;
				s1 += cp[4 * r4 + 3][lane] * x4.w;
			}
			z -= s0 + s1;
		}
		if (wave == g) {
			float x = 0.f;
#pragma unroll
			for (int r = CORNER_NB - 1; r >= 0; r--) {
				const float xr = lane_bcast(z, r) * lane_bcast(inv_d, r);   // x_r = z_r / L_rr
				x = lane == r ? xr : x;
				z -= col[r] * xr;   // z_c -= L_rc x_r (only c < r matter)
			}
			s_x[g][lane] = x;
		}
	}
	__syncthreads();
	if (i >= kl) {   // x goes to its own array: the group's y, which b holds, may still be read by a workgroup starting late
		if (t < CORNER_NB && ci + t < m) xout[ci + t] = s_x[k0 - i][t];
		return;
	}
	float acc = 0.f;
#pragma unroll
	for (int g = 0; g < BACK_G; g++)
		if (g < G) {
#pragma unroll
			for (int q = 0; q < 16; q++) acc += lk[g][q] * s_x[g][seg * 16 + q];
		}
	s_part[seg][c] = acc;
	__syncthreads();
	if (t < CORNER_NB) b[ci + t] -= (s_part[0][t] + s_part[1][t]) + (s_part[2][t] + s_part[3][t]);
}

// x (the first m corner unknowns) -> xout
nnrt_status corner_cholesky_solve(float* A, int ld, float* cb, int m, float* xout, int* error_flag, hipStream_t stream) {
	const int T = ld / CORNER_NB;
	// k_chol_step's panel workgroups read A_kk while the diagonal one overwrites it with L_kk: they must all be resident
	// before any finishes, which the dispatch order (panels first) guarantees while T fits the chip's 512 workgroup
	// slots at two per CU (a 32768-unknown corner, 5461 coarse nodes)
	NNRT_CHECK_ARG(T <= 512, "arrowhead corner larger than 32768 unknowns");
	for (int k = 0; k < T; k++) {   // factor [S | b]: the forward substitution rides along as an augmented row
		const int panel = T - k;
		int trailing = 0;   // lazy trailing updates on every CORNER_LAZY-th column (k_chol_step)
		if (k > 0)
			for (int J = k + 1; J < T; J += CORNER_LAZY) trailing += T - J;
		k_chol_step<<<panel + trailing, CT, 0, stream>>>(A, ld, k, T, cb, error_flag);
		NNRT_LAUNCH_CHECK();
	}
	for (int k0 = T - 1; k0 >= 0; k0 -= BACK_G) {
		const int kl = k0 - BACK_G + 1 > 0 ? k0 - BACK_G + 1 : 0;
		k_chol_back_group<<<k0 + 1, CT, 0, stream>>>(A, ld, k0, kl, cb, m, xout);
		NNRT_LAUNCH_CHECK();
	}
	return NNRT_OK;
}

// ---- stem back-substitution: x_D = D^-1 (b_D - B x_C) ----
__global__ void k_arrow_back(int n0, const float* __restrict__ dinv, const int* __restrict__ edge_offsets, const int* __restrict__ edge_list,
                             const int32_t* __restrict__ edges, const float* __restrict__ wing, const float* __restrict__ rhs,
                             float* __restrict__ x) {
	const int i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n0) return;
	float r6[6];
	for (int c = 0; c < 6; c++) r6[c] = rhs[6 * static_cast<int64_t>(i) + c];
	// 6 x 6 blocks as nine float4, 6-vectors as three float2 (the same products and sums as element-wise loads)
	auto load36 = [](const float* src, float (&dst)[36]) {
		const float4* s4 = reinterpret_cast<const float4*>(src);
#pragma unroll
		for (int q = 0; q < 9; q++) {
			const float4 v = s4[q];
			dst[4 * q] = v.x;
			dst[4 * q + 1] = v.y;
			dst[4 * q + 2] = v.z;
			dst[4 * q + 3] = v.w;
		}
	};
	for (int ei = edge_offsets[i]; ei < edge_offsets[i + 1]; ei++) {
		const int e = edge_list[ei];
		const int j = edges[2 * e + 1];
		float B[36], xj[6];
		load36(wing + static_cast<int64_t>(e) * 36, B);
		const float2* x2 = reinterpret_cast<const float2*>(x + 6 * static_cast<int64_t>(j));
#pragma unroll
		for (int q = 0; q < 3; q++) {
			const float2 v = x2[q];
			xj[2 * q] = v.x;
			xj[2 * q + 1] = v.y;
		}
#pragma unroll
		for (int r = 0; r < 6; r++) {
			float acc = 0.f;
#pragma unroll
			for (int k = 0; k < 6; k++) acc += B[6 * r + k] * xj[k];
			r6[r] -= acc;
		}
	}
	float D[36];
	load36(dinv + static_cast<int64_t>(i) * 36, D);
	float o[6];
#pragma unroll
	for (int r = 0; r < 6; r++) {
		float acc = 0.f;
#pragma unroll
		for (int k = 0; k < 6; k++) acc += D[6 * r + k] * r6[k];
		o[r] = acc;
	}
	float2* xo = reinterpret_cast<float2*>(x + 6 * static_cast<int64_t>(i));
#pragma unroll
	for (int q = 0; q < 3; q++) xo[q] = make_float2(o[2 * q], o[2 * q + 1]);
}

__global__ void k_arrow_update(int N, const float* __restrict__ x, float* __restrict__ node_state, float* __restrict__ updates_out) {
	const int n = blockIdx.x * blockDim.x + threadIdx.x;
	if (n >= N) return;
	float xl[6];
	for (int c = 0; c < 6; c++) {
		xl[c] = x[6 * static_cast<int64_t>(n) + c];
		updates_out[6 * static_cast<int64_t>(n) + c] = xl[c];
	}
	float* ns = node_state + static_cast<int64_t>(n) * NODE_STRIDE;
	ns[3] += xl[3];
	ns[4] += xl[4];
	ns[5] += xl[5];
	float dR[9], R[9];
	rodrigues_device(xl[0], xl[1], xl[2], dR);
	for (int i = 0; i < 9; i++) R[i] = ns[6 + i];
	for (int r = 0; r < 3; r++)
		for (int c = 0; c < 3; c++) ns[6 + 3 * r + c] = (R[3 * r] * dR[c] + R[3 * r + 1] * dR[3 + c]) + R[3 * r + 2] * dR[6 + c];
}

nnrt_status arrowhead_solve_core(const ArrowheadWorkspace& ws, const int32_t* edges, const float* wing, int* error_flag, hipStream_t stream,
                                 bool arap_wings) {
	const int m = ws.m, ld = ws.ld;
	if (m > 0) {
		NNRT_CHECK_ARG(ld <= 32768, "arrowhead corner larger than 32768 unknowns");
		k_arrow_corner_init<<<static_cast<unsigned>(ceil_div(static_cast<int64_t>(ld) * (ld / 4), 256)), 256, 0, stream>>>(ws.n0, m, ld, ws.diag,
		                                                                                                                    ws.schur, ws.rhs, ws.cb);
		NNRT_LAUNCH_CHECK();
		if (ws.E > 0) {
			k_arrow_corner_offdiag<<<ws.E, 64, 0, stream>>>(ws.E, ws.n0, ld, edges, wing, ws.schur);
			NNRT_LAUNCH_CHECK();
		}
	}
	if (ws.n0 > 0) {
		k_arrow_stem<<<static_cast<unsigned>(ceil_div(ws.n0, 64)), 64, 0, stream>>>(ws.n0, ws.diag, ws.edge_offsets, ws.edge_list, wing, ws.dinv,
		                                                                           ws.dinv_b, error_flag);
		NNRT_LAUNCH_CHECK();
		if (m > 0 && ws.targets > 0) {
			if (arap_wings)
				k_stem_schur_t3<<<static_cast<unsigned>(ceil_div(static_cast<int64_t>(ws.targets) * 64, 256)), 256, 0, stream>>>(
				    ws.targets, ld, ws.tgt_off, ws.tgt_ab, ws.pairs, wing, ws.dinv_b, ws.schur);
			else
				k_stem_schur<<<static_cast<unsigned>(ceil_div(static_cast<int64_t>(ws.targets) * 64, 256)), 256, 0, stream>>>(
				    ws.targets, ld, ws.tgt_off, ws.tgt_ab, ws.pairs, wing, ws.dinv_b, ws.schur);
			NNRT_LAUNCH_CHECK();
			k_stem_rhs<<<static_cast<unsigned>(ceil_div(static_cast<int64_t>(m / 6) * 64, 256)), 256, 0, stream>>>(m / 6, ws.rhs_off, ws.rhs_edges,
			                                                                                                         edges, ws.dinv_b, ws.rhs, ws.cb);
			NNRT_LAUNCH_CHECK();
		}
	}
	if (m > 0) {
		nnrt_status st = corner_cholesky_solve(ws.schur, ld, ws.cb, m, ws.x + 6 * static_cast<int64_t>(ws.n0), error_flag, stream);
		if (st) return st;
	}
	if (ws.n0 > 0) {
		k_arrow_back<<<static_cast<unsigned>(ceil_div(ws.n0, 64)), 64, 0, stream>>>(ws.n0, ws.dinv, ws.edge_offsets, ws.edge_list, edges, wing,
		                                                                           ws.rhs, ws.x);
		NNRT_LAUNCH_CHECK();
	}
	return NNRT_OK;
}

nnrt_status launch_arrowhead_iteration(const ArrowheadWorkspace& ws, const double* acc, float lm, const int32_t* edges, const float* wing,
                                       float* node_state, const float* edge_jr, float* updates_out, float* gradient_out, float* hessian_out,
                                       int* error_flag, hipStream_t stream) {
	k_arrow_prepare<<<static_cast<unsigned>(ceil_div(static_cast<int64_t>(ws.N) * 32, 256)), 256, 0, stream>>>(
	    ws.N, lm, const_cast<double*>(acc), ws.inc_off, ws.inc_list, edge_jr, ws.diag, ws.rhs, gradient_out, hessian_out);
	NNRT_LAUNCH_CHECK();
	nnrt_status st = arrowhead_solve_core(ws, edges, wing, error_flag, stream, true);
	if (st) return st;
	k_arrow_update<<<static_cast<unsigned>(ceil_div(ws.N, 256)), 256, 0, stream>>>(ws.N, ws.x, node_state, updates_out);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

} // namespace nnrt
