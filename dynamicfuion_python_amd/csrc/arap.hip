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

#ifndef NNRT_FIT_VARIANT
#define NNRT_FIT_VARIANT 0   // development timing builds only (Makefile `variants`): 0 = product
#endif

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
	// diagonal contributions (ComputeBlockSums of dEi^T dEi / dEj^T dEj)
	float* acc_i = a.acc + static_cast<int64_t>(i) * ACC_STRIDE;
	float* acc_j = a.acc + static_cast<int64_t>(j) * ACC_STRIDE;
	int q = 0;
#pragma unroll
	for (int r0 = 0; r0 < 6; r0++)
#pragma unroll
		for (int c0 = r0; c0 < 6; c0++) {
			const float v = (dEi[0][r0] * dEi[0][c0] + dEi[1][r0] * dEi[1][c0]) + dEi[2][r0] * dEi[2][c0];
			atomicAdd(acc_i + q, v);
			q++;
		}
	const float bb = (j5[4] * j5[4] + 0.f * 0.f) + 0.f * 0.f;
	atomicAdd(acc_j + 15, bb);   // (3,3) in the upper-triangle enumeration
	atomicAdd(acc_j + 18, bb);   // (4,4)
	atomicAdd(acc_j + 20, bb);   // (5,5)
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
	// J^T e (the accumulator stores +J^T r; the solve negates)
	const float skT[3][3] = {{0.f, j5[2], -j5[1]}, {-j5[2], 0.f, j5[0]}, {j5[1], -j5[0], 0.f}};
#pragma unroll
	for (int c = 0; c < 3; c++) {
		atomicAdd(acc_i + 21 + c, (skT[c][0] * r[0] + skT[c][1] * r[1]) + skT[c][2] * r[2]);
		atomicAdd(acc_i + 24 + c, j5[3] * r[c]);
		atomicAdd(acc_j + 24 + c, j5[4] * r[c]);
	}
}

nnrt_status launch_arap_edges(const ArapArgs& args, hipStream_t stream) {
	if (args.E == 0) return NNRT_OK;
	k_arap_edges<<<static_cast<unsigned>(ceil_div(args.E, 256)), 256, 0, stream>>>(args);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

// ---- acc (data) + arap_acc -> full diagonal blocks (+LM) and rhs = negative gradient ----
__global__ void k_arrow_prepare(int N, float lm, double* __restrict__ acc, float* __restrict__ arap_acc, float* __restrict__ diag,
                                float* __restrict__ rhs, float* __restrict__ gradient_out, float* __restrict__ hessian_out) {
	const int n = blockIdx.x * blockDim.x + threadIdx.x;
	if (n >= N) return;
	double* ad = acc + static_cast<int64_t>(n) * ACC_STRIDE;
	float* aa = arap_acc + static_cast<int64_t>(n) * ACC_STRIDE;
	float* d = diag + static_cast<int64_t>(n) * 36;
	int q = 0;
	for (int r = 0; r < 6; r++)
		for (int c = r; c < 6; c++) {
			const float hd = static_cast<float>(ad[q]);
			const float v = aa[q] + hd;
			if (hessian_out) {
				hessian_out[static_cast<int64_t>(n) * 36 + 6 * r + c] = hd;
				hessian_out[static_cast<int64_t>(n) * 36 + 6 * c + r] = hd;
			}
			d[6 * r + c] = v;
			d[6 * c + r] = v;
			q++;
		}
	if (lm > 0.f)
		for (int i = 0; i < 6; i++) d[7 * i] += lm;
	for (int c = 0; c < 6; c++) {
		const float g = (0.f - static_cast<float>(ad[21 + c])) - aa[21 + c];
		rhs[6 * n + c] = g;
		gradient_out[6 * n + c] = g;
	}
	for (int k = 0; k < 27; k++) {
		ad[k] = 0.0;
		aa[k] = 0.f;
	}
}

// ---- corner init: S = C (diagonal corner blocks + corner off-diagonal blocks), identity on the padding; cb = b_C ----
__global__ void k_arrow_corner_init(int n0, int m, int ld, const float* __restrict__ diag, float* __restrict__ S, const float* __restrict__ rhs,
                                    float* __restrict__ cb) {
	const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (idx >= static_cast<int64_t>(ld) * ld) return;
	const int r = static_cast<int>(idx / ld), c = static_cast<int>(idx % ld);
	float v = 0.f;
	if (r < m && c < m) {
		if (r / 6 == c / 6) v = diag[static_cast<int64_t>(n0 + r / 6) * 36 + 6 * (r % 6) + (c % 6)];
	} else if (r == c) {
		v = 1.f;
	}
	S[idx] = v;
	if (c == 0) cb[r] = r < m ? rhs[6 * static_cast<int64_t>(n0) + r] : 0.f;
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
	float L[6][6];
#pragma unroll
	for (int r = 0; r < 6; r++)
#pragma unroll
		for (int c = 0; c < 6; c++) L[r][c] = diag[static_cast<int64_t>(i) * 36 + 6 * r + c];
	if (!cholesky_small<6>(L)) {
		atomicOr(error_flag, 1);
		return;
	}
	float Di[6][6];
#pragma unroll
	for (int c = 0; c < 6; c++) {
		float col[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
		col[c] = 1.f;
		cholesky_solve_small<6>(L, col);
#pragma unroll
		for (int r = 0; r < 6; r++) Di[r][c] = col[r];
	}
#pragma unroll
	for (int k = 0; k < 36; k++) dinv[static_cast<int64_t>(i) * 36 + k] = Di[k / 6][k % 6];
	for (int ei = edge_offsets[i]; ei < edge_offsets[i + 1]; ei++) {
		const int e = edge_list[ei];
		const float* B = wing + static_cast<int64_t>(e) * 36;
		float* Y = dinv_b + static_cast<int64_t>(e) * 36;
#pragma unroll
		for (int r = 0; r < 6; r++)
#pragma unroll
			for (int c = 0; c < 6; c++) {
				float acc = 0.f;
#pragma unroll
				for (int k = 0; k < 6; k++) acc += Di[r][k] * B[6 * k + c];
				Y[6 * r + c] = acc;
			}
	}
}

// ---- Schur update S_ab -= sum over stem nodes i adjacent to a and b of B_ia^T D_i^-1 B_ib (one wave per target) ----
__global__ void k_stem_schur(int targets, int ld, const int* __restrict__ tgt_off, const int2* __restrict__ tgt_ab, const int2* __restrict__ pairs,
                             const float* __restrict__ wing, const float* __restrict__ dinv_b, float* __restrict__ S) {
	const int w = static_cast<int>((static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6);
	const int lane = static_cast<int>(threadIdx.x & 63);
	if (w >= targets || lane >= 36) return;
	const int r = lane / 6, c = lane % 6;
	float acc = 0.f;
	for (int p = tgt_off[w]; p < tgt_off[w + 1]; p++) {
		const int2 e = pairs[p];
		const float* B1 = wing + static_cast<int64_t>(e.x) * 36;
		const float* Y2 = dinv_b + static_cast<int64_t>(e.y) * 36;
		float s = 0.f;
		for (int k = 0; k < 6; k++) s += B1[6 * k + r] * Y2[6 * k + c];
		acc += s;
	}
	const int2 ab = tgt_ab[w];
	S[static_cast<int64_t>(6 * ab.x + r) * ld + 6 * ab.y + c] -= acc;
}

// ---- b_C -= sum over stem edges i->a of (D_i^-1 B_ia)^T b_i (one thread per corner entry) ----
__global__ void k_stem_rhs(int m, const int* __restrict__ rhs_off, const int* __restrict__ rhs_edges, const int32_t* __restrict__ edges,
                           const float* __restrict__ dinv_b, const float* __restrict__ rhs, float* __restrict__ cb) {
	const int idx = blockIdx.x * blockDim.x + threadIdx.x;
	if (idx >= m) return;
	const int a = idx / 6, c = idx % 6;
	float acc = 0.f;
	for (int q = rhs_off[a]; q < rhs_off[a + 1]; q++) {
		const int e = rhs_edges[q];
		const int i = edges[2 * e];
		const float* Y = dinv_b + static_cast<int64_t>(e) * 36;
		const float* g = rhs + 6 * static_cast<int64_t>(i);
		float s = 0.f;
		for (int k = 0; k < 6; k++) s += Y[6 * k + c] * g[k];
		acc += s;
	}
	cb[idx] -= acc;
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
// SolveBlockSparseArrowheadCholesky.cpp:30-95 factors the Schur complement with a dense potrf. Here, per 64-column
// block k: k_chol_diag factors the diagonal block in LDS and inverts it (L_kk^-1 kept for the panel and the
// substitutions), k_chol_panel forms L_Ik = A_Ik L_kk^-T for every block row below (one workgroup per block row), and
// k_chol_update applies A_IJ -= L_Ik L_Jk^T to every lower tile of the trailing matrix (one workgroup per tile). The
// substitutions are block-parallel matrix-vector products with the stored inverses.
constexpr int CT = 256;   // threads per workgroup of the corner kernels (64 x 64 tiles: 4 x 4 outputs per thread)
#if NNRT_FIT_VARIANT == 30
__device__ unsigned long long g_chol_stamps[64][8];
#define CSTAMP(i) \
	do { \
		if (threadIdx.x == 0 && k < 64) g_chol_stamps[k][i] = __builtin_amdgcn_s_memrealtime(); \
	} while (0)
extern "C" int nnrt_dev_chol_stamps(unsigned long long* host) {
	return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_chol_stamps), sizeof(g_chol_stamps)) == hipSuccess ? 0 : 1;
}
#else
#define CSTAMP(i) do {} while (0)
#endif

// The 64 x 64 diagonal block is factored in four 16-column steps inside one workgroup: wave 0 factors the 16 x 16
// diagonal sub-block in registers (lane = row, static register indices, pivots and columns broadcast with readlane) and
// inverts it; the rows below are solved against that inverse and the trailing lower triangle updated by all threads.
// L^-1 of the whole block is then assembled block row by block row from the four 16 x 16 inverses.
constexpr int CS = CORNER_NB + 1;   // LDS row stride

// 16 x 16 lower Cholesky + inverse of the sub-block at (o, o) of s (row stride CS), lanes 0..15 of one wave
__device__ inline float lane_bcast(float v, int src) {
	return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), src));
}

// 16 x 16 lower Cholesky + inverse of the sub-block at (o, o) of s (row stride CS), lanes 0..15 of one wave. The
// column chain is latency-bound (one wave): hardware square root / reciprocal, independent partial sums.
__device__ inline bool potrf16_inv16(float* s, int o, float* x16, int lane) {
	float a[16];
	const int r = lane & 15;
#pragma unroll
	for (int c = 0; c < 16; c++) a[c] = s[(o + r) * CS + o + c];
	bool ok = true;
	float inv_diag[16];
#pragma unroll
	for (int j = 0; j < 16; j++) {
		float d = lane_bcast(a[j], j);
		if (!(d > 0.f)) {
			ok = false;
			d = 1.f;
		}
		const float ip = __builtin_amdgcn_rsqf(d);   // 1 / sqrt(d)
		inv_diag[j] = ip;
		const float l = r > j ? a[j] * ip : (r == j ? d * ip : 0.f);
		a[j] = l;
#pragma unroll
		for (int c = j + 1; c < 16; c++) a[c] -= l * lane_bcast(l, c);
	}
	// inverse, lane = column: x_i = (delta_ir - sum_{k<i} L_ik x_k) / L_ii with L_ik broadcast from lane i
	float x[16];
#pragma unroll
	for (int i = 0; i < 16; i++) {
		float s0 = 0.f, s1 = 0.f;
#pragma unroll
		for (int q = 0; q < i; q++) {
			if (q & 1) s1 += lane_bcast(a[q], i) * x[q];
			else s0 += lane_bcast(a[q], i) * x[q];
		}
		x[i] = ((r == i ? 1.f : 0.f) - (s0 + s1)) * inv_diag[i];
	}
	if (lane < 16) {
#pragma unroll
		for (int c = 0; c < 16; c++) {
			s[(o + r) * CS + o + c] = c <= r ? a[c] : 0.f;
			x16[c * 17 + r] = x[c];   // x16[i][col]
		}
	}
	return ok;
}

__global__ __launch_bounds__(CT) void k_chol_diag(float* __restrict__ A, int ld, int k, float* __restrict__ linv, float* __restrict__ b,
                                                  int* error_flag) {
	__shared__ float s_a[CORNER_NB * CS];          // the block, then L
	__shared__ float s_x[CORNER_NB * CS];          // L^-1 (and scratch)
	__shared__ float s_x16[4][16 * 17];            // inverses of the 16 x 16 diagonal sub-blocks
	__shared__ float s_b[CORNER_NB];
	__shared__ int s_fail;
	const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
	const int64_t o = static_cast<int64_t>(k) * CORNER_NB;
	CSTAMP(0);
	for (int e = t; e < CORNER_NB * CORNER_NB; e += CT) s_a[(e / CORNER_NB) * CS + e % CORNER_NB] = A[(o + e / CORNER_NB) * ld + o + e % CORNER_NB];
	if (t < CORNER_NB) s_b[t] = b[o + t];
	if (t == 0) s_fail = 0;
	__syncthreads();
	CSTAMP(1);
	for (int p = 0; p < 4; p++) {
		const int o16 = 16 * p;
		if (wave == 0) {
			if (!potrf16_inv16(s_a, o16, s_x16[p], lane) && lane == 0) s_fail = 1;
		}
		__syncthreads();
		if (p == 0) CSTAMP(5);
		const int rows = CORNER_NB - o16 - 16;
		if (rows > 0) {
			// panel rows below: L_r = A_r X16^T (X16 lower) into scratch, then back into s_a
			for (int e = t; e < rows * 16; e += CT) {
				const int rr = o16 + 16 + e / 16, c = e % 16;
				float acc = 0.f;
#pragma unroll
				for (int q = 0; q < 16; q++) acc += s_a[rr * CS + o16 + q] * s_x16[p][c * 17 + q];
				s_x[rr * CS + c] = acc;
			}
			__syncthreads();
			for (int e = t; e < rows * 16; e += CT) {
				const int rr = o16 + 16 + e / 16, c = e % 16;
				s_a[rr * CS + o16 + c] = s_x[rr * CS + c];
			}
			__syncthreads();
			if (p == 0) CSTAMP(6);
			// trailing lower triangle: A_rc -= sum_q L_rq L_cq
			for (int e = t; e < rows * rows; e += CT) {
				const int rr = o16 + 16 + e / rows, cc = o16 + 16 + e % rows;
				if (cc > rr) continue;
				float acc = 0.f;
#pragma unroll
				for (int q = 0; q < 16; q++) acc += s_a[rr * CS + o16 + q] * s_a[cc * CS + o16 + q];
				s_a[rr * CS + cc] -= acc;
			}
			__syncthreads();
			if (p == 0) CSTAMP(7);
		}
	}
	CSTAMP(2);
	// L^-1: diagonal blocks X_II = inverse of L_II; block row I: X_IJ = -X_II (sum_{J<=K<I} L_IK X_KJ), J < I
	for (int e = t; e < CORNER_NB * CORNER_NB; e += CT) {
		const int r = e / CORNER_NB, c = e % CORNER_NB;
		s_x[r * CS + c] = (r / 16 == c / 16) ? s_x16[r / 16][(r % 16) * 17 + c % 16] : 0.f;
	}
	__syncthreads();
	for (int I = 1; I < 4; I++) {
		// tmp_IJ = sum_{K=J}^{I-1} L_IK X_KJ for every J < I (16 x 16 I values; at most 3 per thread, static slots)
		const int n = 16 * 16 * I;
		float tmp[3];
#pragma unroll
		for (int it = 0; it < 3; it++) {
			const int e = t + it * CT;
			tmp[it] = 0.f;
			if (e < n) {
				const int r = e / (16 * I), cg = e % (16 * I);
				const int J = cg / 16;
				float acc = 0.f;
				for (int q = 16 * J; q < 16 * I; q++) acc += s_a[(16 * I + r) * CS + q] * s_x[q * CS + cg];
				tmp[it] = acc;
			}
		}
		__syncthreads();
#pragma unroll
		for (int it = 0; it < 3; it++) {
			const int e = t + it * CT;
			if (e < n) s_x[(16 * I + e / (16 * I)) * CS + e % (16 * I)] = tmp[it];   // staged: block row I, columns < 16 I
		}
		__syncthreads();
#pragma unroll
		for (int it = 0; it < 3; it++) {
			const int e = t + it * CT;
			if (e < n) {
				const int r = e / (16 * I), cg = e % (16 * I);
				float acc = 0.f;
#pragma unroll
				for (int q = 0; q < 16; q++) acc += s_x16[I][r * 17 + q] * s_x[(16 * I + q) * CS + cg];
				tmp[it] = -acc;
			}
		}
		__syncthreads();
#pragma unroll
		for (int it = 0; it < 3; it++) {
			const int e = t + it * CT;
			if (e < n) s_x[(16 * I + e / (16 * I)) * CS + e % (16 * I)] = tmp[it];
		}
		__syncthreads();
	}
	CSTAMP(3);
	float* Li = linv + static_cast<int64_t>(k) * CORNER_NB * CORNER_NB;
	for (int e = t; e < CORNER_NB * CORNER_NB; e += CT) {
		const int r = e / CORNER_NB, c = e % CORNER_NB;
		A[(o + r) * ld + o + c] = c <= r ? s_a[r * CS + c] : 0.f;
		Li[e] = s_x[r * CS + c];
	}
	// forward substitution of the augmented column: y_k = L_kk^-1 b_k (b_k already carries every earlier block's update)
	if (t < CORNER_NB) {
		float y = 0.f;
		for (int c = 0; c <= t; c++) y += s_x[t * CS + c] * s_b[c];
		b[o + t] = y;
	}
	__syncthreads();
	CSTAMP(4);
	if (s_fail && t == 0) atomicOr(error_flag, 1);
}

// 64 x 64 x 64 tile product in LDS: thread (ty, tx) owns rows 4 ty.., columns 4 tx.. of C = X Y^T
__device__ inline void tile_xyt(const float (*X)[CORNER_NB + 1], const float (*Y)[CORNER_NB + 1], int ty, int tx, float (&c)[4][4]) {
#pragma unroll
	for (int r = 0; r < 4; r++)
#pragma unroll
		for (int q = 0; q < 4; q++) c[r][q] = 0.f;
	for (int kk = 0; kk < CORNER_NB; kk++) {
		float x[4], y[4];
#pragma unroll
		for (int r = 0; r < 4; r++) x[r] = X[4 * ty + r][kk];
#pragma unroll
		for (int q = 0; q < 4; q++) y[q] = Y[4 * tx + q][kk];
#pragma unroll
		for (int r = 0; r < 4; r++)
#pragma unroll
			for (int q = 0; q < 4; q++) c[r][q] += x[r] * y[q];
	}
}

// L_Ik = A_Ik L_kk^-T for block rows I = k + 1 + blockIdx.x
__global__ __launch_bounds__(CT) void k_chol_panel(float* __restrict__ A, int ld, int k, const float* __restrict__ linv, float* __restrict__ b) {
	__shared__ float s_x[CORNER_NB][CORNER_NB + 1];
	__shared__ float s_y[CORNER_NB][CORNER_NB + 1];
	const int t = threadIdx.x;
	const int64_t rI = static_cast<int64_t>(k + 1 + blockIdx.x) * CORNER_NB, ck = static_cast<int64_t>(k) * CORNER_NB;
	const float* Li = linv + static_cast<int64_t>(k) * CORNER_NB * CORNER_NB;
	for (int e = t; e < CORNER_NB * CORNER_NB; e += CT) {
		s_x[e / CORNER_NB][e % CORNER_NB] = A[(rI + e / CORNER_NB) * ld + ck + e % CORNER_NB];
		s_y[e / CORNER_NB][e % CORNER_NB] = Li[e];
	}
	__syncthreads();
	const int ty = t / 16, tx = t % 16;
	float c[4][4];
	tile_xyt(s_x, s_y, ty, tx, c);
#pragma unroll
	for (int r = 0; r < 4; r++)
#pragma unroll
		for (int q = 0; q < 4; q++) A[(rI + 4 * ty + r) * ld + ck + 4 * tx + q] = c[r][q];
	// augmented column: b_I -= L_Ik y_k (rows 4 ty + r; the 16 threads of a row group share the sum through LDS)
	__syncthreads();
	float* s_part = &s_x[0][0];   // [64][16]
#pragma unroll
	for (int r = 0; r < 4; r++) {
		float acc = 0.f;
#pragma unroll
		for (int q = 0; q < 4; q++) acc += c[r][q] * b[ck + 4 * tx + q];
		s_part[(4 * ty + r) * 16 + tx] = acc;
	}
	__syncthreads();
	if (t < CORNER_NB) {
		float acc = 0.f;
		for (int q = 0; q < 16; q++) acc += s_part[t * 16 + q];
		b[rI + t] -= acc;
	}
}

// A_IJ -= L_Ik L_Jk^T for the lower tiles k < J <= I of the trailing matrix (blockIdx.x enumerates them row by row)
__global__ __launch_bounds__(CT) void k_chol_update(float* __restrict__ A, int ld, int k) {
	__shared__ float s_x[CORNER_NB][CORNER_NB + 1];
	__shared__ float s_y[CORNER_NB][CORNER_NB + 1];
	int b = static_cast<int>(blockIdx.x), ii = 0;
	while (b > ii) {   // row ii holds ii + 1 tiles
		b -= ii + 1;
		ii++;
	}
	const int I = k + 1 + ii, J = k + 1 + b;
	const int t = threadIdx.x;
	const int64_t ck = static_cast<int64_t>(k) * CORNER_NB, rI = static_cast<int64_t>(I) * CORNER_NB, rJ = static_cast<int64_t>(J) * CORNER_NB;
	for (int e = t; e < CORNER_NB * CORNER_NB; e += CT) {
		s_x[e / CORNER_NB][e % CORNER_NB] = A[(rI + e / CORNER_NB) * ld + ck + e % CORNER_NB];
		s_y[e / CORNER_NB][e % CORNER_NB] = A[(rJ + e / CORNER_NB) * ld + ck + e % CORNER_NB];
	}
	__syncthreads();
	const int ty = t / 16, tx = t % 16;
	float c[4][4];
	tile_xyt(s_x, s_y, ty, tx, c);
#pragma unroll
	for (int r = 0; r < 4; r++)
#pragma unroll
		for (int q = 0; q < 4; q++) A[(rI + 4 * ty + r) * ld + rJ + 4 * tx + q] -= c[r][q];
}

// back substitution L^T x = y in place, right-looking over block rows: launch k (from the last block) has
// workgroup i < k form x_k = L_kk^-T y_k (each workgroup redundantly, 64 x 64) and apply y_i -= L_ki^T x_k; workgroup
// k itself stores x_k. Block rows are read coalesced (L_ki is row block k).
__global__ __launch_bounds__(CT) void k_chol_back_step(const float* __restrict__ A, int ld, int k, const float* __restrict__ linv,
                                                       float* __restrict__ b) {
	__shared__ float s_y[CORNER_NB], s_x[CORNER_NB];
	__shared__ float s_part[4][CORNER_NB];
	const int t = threadIdx.x, c = t % CORNER_NB, seg = t / CORNER_NB;
	const int i = static_cast<int>(blockIdx.x);   // target block (i == k: store x_k)
	const int64_t ck = static_cast<int64_t>(k) * CORNER_NB, ci = static_cast<int64_t>(i) * CORNER_NB;
	if (t < CORNER_NB) s_y[t] = b[ck + t];
	__syncthreads();
	// x_k[c] = sum_q Linv[q][c] y_q
	const float* Li = linv + static_cast<int64_t>(k) * CORNER_NB * CORNER_NB;
	float acc = 0.f;
#pragma unroll
	for (int q = seg * 16; q < seg * 16 + 16; q++) acc += Li[q * CORNER_NB + c] * s_y[q];
	s_part[seg][c] = acc;
	__syncthreads();
	if (t < CORNER_NB) s_x[t] = (s_part[0][t] + s_part[1][t]) + (s_part[2][t] + s_part[3][t]);
	__syncthreads();
	if (i == k) {
		if (t < CORNER_NB) b[ck + t] = s_x[t];
		return;
	}
	// y_i[c] -= sum_r L[k-block row r][i-block col c] x_k[r]
	acc = 0.f;
#pragma unroll
	for (int r = seg * 16; r < seg * 16 + 16; r++) acc += A[(ck + r) * ld + ci + c] * s_x[r];
	__syncthreads();
	s_part[seg][c] = acc;
	__syncthreads();
	if (t < CORNER_NB) b[ci + t] -= (s_part[0][t] + s_part[1][t]) + (s_part[2][t] + s_part[3][t]);
}

__global__ void k_corner_out(int m, const float* __restrict__ cb, float* __restrict__ x) {
	const int i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i < m) x[i] = cb[i];
}

nnrt_status corner_cholesky_solve(float* A, int ld, float* linv, float* cb, int* error_flag, hipStream_t stream) {
	const int T = ld / CORNER_NB;
	for (int k = 0; k < T; k++) {   // factor [S | b]: the forward substitution rides along as an augmented column
		k_chol_diag<<<1, CT, 0, stream>>>(A, ld, k, linv, cb, error_flag);
		NNRT_LAUNCH_CHECK();
		const int below = T - 1 - k;
		if (below > 0) {
			k_chol_panel<<<below, CT, 0, stream>>>(A, ld, k, linv, cb);
			NNRT_LAUNCH_CHECK();
			k_chol_update<<<below * (below + 1) / 2, CT, 0, stream>>>(A, ld, k);
			NNRT_LAUNCH_CHECK();
		}
	}
	for (int k = T - 1; k >= 0; k--) {
		k_chol_back_step<<<k + 1, CT, 0, stream>>>(A, ld, k, linv, cb);
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
	for (int ei = edge_offsets[i]; ei < edge_offsets[i + 1]; ei++) {
		const int e = edge_list[ei];
		const int j = edges[2 * e + 1];
		const float* B = wing + static_cast<int64_t>(e) * 36;
		for (int r = 0; r < 6; r++) {
			float acc = 0.f;
			for (int k = 0; k < 6; k++) acc += B[6 * r + k] * x[6 * static_cast<int64_t>(j) + k];
			r6[r] -= acc;
		}
	}
	const float* D = dinv + static_cast<int64_t>(i) * 36;
	for (int r = 0; r < 6; r++) {
		float acc = 0.f;
		for (int k = 0; k < 6; k++) acc += D[6 * r + k] * r6[k];
		x[6 * static_cast<int64_t>(i) + r] = acc;
	}
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

nnrt_status arrowhead_solve_core(const ArrowheadWorkspace& ws, const int32_t* edges, const float* wing, int* error_flag, hipStream_t stream) {
	const int m = ws.m, ld = ws.ld;
	if (m > 0) {
		k_arrow_corner_init<<<static_cast<unsigned>(ceil_div(static_cast<int64_t>(ld) * ld, 256)), 256, 0, stream>>>(ws.n0, m, ld, ws.diag,
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
			k_stem_schur<<<static_cast<unsigned>(ceil_div(static_cast<int64_t>(ws.targets) * 64, 256)), 256, 0, stream>>>(
			    ws.targets, ld, ws.tgt_off, ws.tgt_ab, ws.pairs, wing, ws.dinv_b, ws.schur);
			NNRT_LAUNCH_CHECK();
			k_stem_rhs<<<static_cast<unsigned>(ceil_div(m, 256)), 256, 0, stream>>>(m, ws.rhs_off, ws.rhs_edges, edges, ws.dinv_b, ws.rhs, ws.cb);
			NNRT_LAUNCH_CHECK();
		}
	}
	if (m > 0) {
		nnrt_status st = corner_cholesky_solve(ws.schur, ld, ws.linv, ws.cb, error_flag, stream);
		if (st) return st;
		k_corner_out<<<static_cast<unsigned>(ceil_div(m, 256)), 256, 0, stream>>>(m, ws.cb, ws.x + 6 * static_cast<int64_t>(ws.n0));
		NNRT_LAUNCH_CHECK();
	}
	if (ws.n0 > 0) {
		k_arrow_back<<<static_cast<unsigned>(ceil_div(ws.n0, 64)), 64, 0, stream>>>(ws.n0, ws.dinv, ws.edge_offsets, ws.edge_list, edges, wing,
		                                                                           ws.rhs, ws.x);
		NNRT_LAUNCH_CHECK();
	}
	return NNRT_OK;
}

nnrt_status launch_arrowhead_iteration(const ArrowheadWorkspace& ws, const double* acc, float lm, const int32_t* edges, const float* wing,
                                       float* node_state, float* arap_acc, float* updates_out, float* gradient_out, float* hessian_out,
                                       int* error_flag, hipStream_t stream) {
	k_arrow_prepare<<<static_cast<unsigned>(ceil_div(ws.N, 256)), 256, 0, stream>>>(ws.N, lm, const_cast<double*>(acc), arap_acc, ws.diag,
	                                                                               ws.rhs, gradient_out, hessian_out);
	NNRT_LAUNCH_CHECK();
	nnrt_status st = arrowhead_solve_core(ws, edges, wing, error_flag, stream);
	if (st) return st;
	k_arrow_update<<<static_cast<unsigned>(ceil_div(ws.N, 256)), 256, 0, stream>>>(ws.N, ws.x, node_state, updates_out);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

} // namespace nnrt
