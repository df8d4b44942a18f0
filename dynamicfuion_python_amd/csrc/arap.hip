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

// ---- corner init: S = C (diagonal corner blocks + corner off-diagonal blocks) ----
__global__ void k_arrow_corner_init(int N, int n0, int m, const float* __restrict__ diag, float* __restrict__ S) {
	const int64_t idx = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (idx >= static_cast<int64_t>(m) * m) return;
	const int r = static_cast<int>(idx / m), c = static_cast<int>(idx % m);
	float v = 0.f;
	if (r / 6 == c / 6) v = diag[static_cast<int64_t>(n0 + r / 6) * 36 + 6 * (r % 6) + (c % 6)];
	S[idx] = v;
	(void) N;
}

__global__ void k_arrow_corner_offdiag(int E, int n0, int m, const int32_t* __restrict__ edges, const float* __restrict__ wing,
                                       float* __restrict__ S) {
	const int e = blockIdx.x;
	const int i = edges[2 * e], j = edges[2 * e + 1];
	if (i < n0) return;
	const int t = threadIdx.x;
	if (t >= 36) return;
	const int r = t / 6, c = t % 6;
	const float v = wing[static_cast<int64_t>(e) * 36 + t];
	const int ai = i - n0, bj = j - n0;
	atomicAdd(S + static_cast<int64_t>(6 * ai + r) * m + 6 * bj + c, v);
	atomicAdd(S + static_cast<int64_t>(6 * bj + c) * m + 6 * ai + r, v);
	(void) E;
}

// ---- stem: D^-1, D^-1 B, Schur update S -= B^T D^-1 B, b_C -= B^T D^-1 b_D. One thread per stem node. ----
__global__ void k_arrow_stem(int n0, int m, const float* __restrict__ diag, const int* __restrict__ edge_offsets,
                             const int* __restrict__ edge_list, const int32_t* __restrict__ edges, const float* __restrict__ wing,
                             float* __restrict__ dinv, float* __restrict__ dinv_b, float* __restrict__ S, const float* __restrict__ rhs,
                             float* __restrict__ bc, int* error_flag) {
	const int i = blockIdx.x * blockDim.x + threadIdx.x;
	if (i >= n0) return;
	float L[6][6];
	for (int r = 0; r < 6; r++)
		for (int c = 0; c < 6; c++) L[r][c] = diag[static_cast<int64_t>(i) * 36 + 6 * r + c];
	if (!cholesky_small<6>(L)) {
		atomicOr(error_flag, 1);
		return;
	}
	float Di[6][6];
	for (int c = 0; c < 6; c++) {
		float col[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
		col[c] = 1.f;
		cholesky_solve_small<6>(L, col);
		for (int r = 0; r < 6; r++) Di[r][c] = col[r];
	}
	for (int k = 0; k < 36; k++) dinv[static_cast<int64_t>(i) * 36 + k] = Di[k / 6][k % 6];
	const int e0 = edge_offsets[i], e1 = edge_offsets[i + 1];
	for (int ei = e0; ei < e1; ei++) {
		const int e = edge_list[ei];
		const float* B = wing + static_cast<int64_t>(e) * 36;
		float* Y = dinv_b + static_cast<int64_t>(e) * 36;
		for (int r = 0; r < 6; r++)
			for (int c = 0; c < 6; c++) {
				float acc = 0.f;
				for (int k = 0; k < 6; k++) acc += Di[r][k] * B[6 * k + c];
				Y[6 * r + c] = acc;
			}
	}
	const float* g = rhs + 6 * static_cast<int64_t>(i);
	for (int ea = e0; ea < e1; ea++) {
		const int e_1 = edge_list[ea];
		const int a_ = edges[2 * e_1 + 1] - n0;
		const float* B1 = wing + static_cast<int64_t>(e_1) * 36;
		const float* Y1 = dinv_b + static_cast<int64_t>(e_1) * 36;
		for (int c = 0; c < 6; c++) {
			float acc = 0.f;
			for (int k = 0; k < 6; k++) acc += Y1[6 * k + c] * g[k];
			atomicAdd(bc + 6 * a_ + c, -acc);
		}
		for (int eb = e0; eb < e1; eb++) {
			const int e_2 = edge_list[eb];
			const int b_ = edges[2 * e_2 + 1] - n0;
			const float* Y2 = dinv_b + static_cast<int64_t>(e_2) * 36;
			for (int r = 0; r < 6; r++)
				for (int c = 0; c < 6; c++) {
					float acc = 0.f;
					for (int k = 0; k < 6; k++) acc += B1[6 * k + r] * Y2[6 * k + c];
					atomicAdd(S + static_cast<int64_t>(6 * a_ + r) * m + 6 * b_ + c, -acc);
				}
		}
	}
}

// ---- dense corner: in-place lower Cholesky of S (m x m, row-major) and solve S x = b, single workgroup ----
// Right-looking, 16-column panels: the diagonal block is factored in LDS by one wave, the panel below is solved
// row-parallel, the panel is staged in LDS, and the trailing lower triangle is updated by all 1024 threads.
constexpr int DC_NB = 16;
constexpr int DC_THREADS = 1024;

__global__ __launch_bounds__(DC_THREADS) void k_dense_cholesky_solve(float* __restrict__ A, int m, float* __restrict__ b, int* error_flag,
                                                                    int panel_in_lds) {
	extern __shared__ float s_panel[];   // [m][DC_NB] when panel_in_lds
	__shared__ float s_diag[DC_NB][DC_NB + 1];
	__shared__ int s_fail;
	const int tid = threadIdx.x;
	if (tid == 0) s_fail = 0;
	__syncthreads();
	for (int k0 = 0; k0 < m; k0 += DC_NB) {
		const int nb = min(DC_NB, m - k0);
		for (int t = tid; t < nb * nb; t += DC_THREADS) s_diag[t / nb][t % nb] = A[static_cast<int64_t>(k0 + t / nb) * m + k0 + t % nb];
		__syncthreads();
		if (tid == 0) {   // tiny unblocked factorization of the diagonal block
			for (int j = 0; j < nb; j++) {
				float s = s_diag[j][j];
				for (int k = 0; k < j; k++) s -= s_diag[j][k] * s_diag[j][k];
				if (!(s > 0.f)) {
					s_fail = 1;
					s = 1.f;
				}
				const float l = sqrtf(s);
				s_diag[j][j] = l;
				for (int i = j + 1; i < nb; i++) {
					float t = s_diag[i][j];
					for (int k = 0; k < j; k++) t -= s_diag[i][k] * s_diag[j][k];
					s_diag[i][j] = t / l;
				}
			}
		}
		__syncthreads();
		for (int t = tid; t < nb * nb; t += DC_THREADS) {
			const int r = t / nb, c = t % nb;
			A[static_cast<int64_t>(k0 + r) * m + k0 + c] = (c <= r) ? s_diag[r][c] : 0.f;
		}
		// panel solve: L21 = A21 L11^-T (one thread per row)
		for (int i = k0 + nb + tid; i < m; i += DC_THREADS) {
			float row[DC_NB];
			for (int c = 0; c < nb; c++) {
				float t = A[static_cast<int64_t>(i) * m + k0 + c];
				for (int q = 0; q < c; q++) t -= row[q] * s_diag[c][q];
				row[c] = t / s_diag[c][c];
			}
			for (int c = 0; c < nb; c++) {
				A[static_cast<int64_t>(i) * m + k0 + c] = row[c];
				if (panel_in_lds) s_panel[static_cast<int64_t>(i) * DC_NB + c] = row[c];
			}
		}
		__syncthreads();
		// trailing update of the lower triangle: A[i][j] -= sum_q L21[i][q] L21[j][q], k0+nb <= j <= i < m
		const int base = k0 + nb;
		const int64_t rows = m - base;
		const int64_t total = rows * (rows + 1) / 2;
		for (int64_t t = tid; t < total; t += DC_THREADS) {
			// map t -> (i, j) in the lower triangle, row-major
			int64_t ii = static_cast<int64_t>((sqrt(8.0 * static_cast<double>(t) + 1.0) - 1.0) / 2.0);
			while ((ii + 1) * (ii + 2) / 2 <= t) ii++;
			while (ii * (ii + 1) / 2 > t) ii--;
			const int64_t jj = t - ii * (ii + 1) / 2;
			const int i = base + static_cast<int>(ii), j = base + static_cast<int>(jj);
			float acc = 0.f;
			if (panel_in_lds) {
				for (int q = 0; q < nb; q++) acc += s_panel[static_cast<int64_t>(i) * DC_NB + q] * s_panel[static_cast<int64_t>(j) * DC_NB + q];
			} else {
				for (int q = 0; q < nb; q++) acc += A[static_cast<int64_t>(i) * m + k0 + q] * A[static_cast<int64_t>(j) * m + k0 + q];
			}
			A[static_cast<int64_t>(i) * m + j] -= acc;
		}
		__syncthreads();
	}
	// zero the strict upper triangle, then solve L y = b, L^T x = y (blocked: one wave per diagonal block)
	for (int64_t t = tid; t < static_cast<int64_t>(m) * m; t += DC_THREADS) {
		const int r = static_cast<int>(t / m), c = static_cast<int>(t % m);
		if (c > r) A[t] = 0.f;
	}
	__syncthreads();
	for (int k0 = 0; k0 < m; k0 += DC_NB) {
		const int nb = min(DC_NB, m - k0);
		if (tid == 0) {
			for (int r = 0; r < nb; r++) {
				float s = b[k0 + r];
				for (int q = 0; q < r; q++) s -= A[static_cast<int64_t>(k0 + r) * m + k0 + q] * b[k0 + q];
				b[k0 + r] = s / A[static_cast<int64_t>(k0 + r) * m + k0 + r];
			}
		}
		__syncthreads();
		for (int i = k0 + nb + tid; i < m; i += DC_THREADS) {
			float s = 0.f;
			for (int q = 0; q < nb; q++) s += A[static_cast<int64_t>(i) * m + k0 + q] * b[k0 + q];
			b[i] -= s;
		}
		__syncthreads();
	}
	for (int k1 = m; k1 > 0; k1 -= DC_NB) {
		const int k0 = max(0, k1 - DC_NB);
		const int nb = k1 - k0;
		if (tid == 0) {
			for (int r = nb - 1; r >= 0; r--) {
				float s = b[k0 + r];
				for (int q = r + 1; q < nb; q++) s -= A[static_cast<int64_t>(k0 + q) * m + k0 + r] * b[k0 + q];
				b[k0 + r] = s / A[static_cast<int64_t>(k0 + r) * m + k0 + r];
			}
		}
		__syncthreads();
		for (int i = tid; i < k0; i += DC_THREADS) {
			float s = 0.f;
			for (int q = 0; q < nb; q++) s += A[static_cast<int64_t>(k0 + q) * m + i] * b[k0 + q];
			b[i] -= s;
		}
		__syncthreads();
	}
	if (tid == 0 && s_fail) atomicOr(error_flag, 1);
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
	const int m = ws.m;
	if (m > 0) {
		k_arrow_corner_init<<<static_cast<unsigned>(ceil_div(static_cast<int64_t>(m) * m, 256)), 256, 0, stream>>>(ws.N, ws.n0, m, ws.diag,
		                                                                                                             ws.schur);
		NNRT_LAUNCH_CHECK();
		if (ws.E > 0) {
			k_arrow_corner_offdiag<<<ws.E, 64, 0, stream>>>(ws.E, ws.n0, m, edges, wing, ws.schur);
			NNRT_LAUNCH_CHECK();
		}
		NNRT_HIP(hipMemcpyAsync(ws.x + 6 * static_cast<int64_t>(ws.n0), ws.rhs + 6 * static_cast<int64_t>(ws.n0), sizeof(float) * m,
		                        hipMemcpyDeviceToDevice, stream));
	}
	if (ws.n0 > 0) {
		k_arrow_stem<<<static_cast<unsigned>(ceil_div(ws.n0, 64)), 64, 0, stream>>>(ws.n0, m, ws.diag, ws.edge_offsets, ws.edge_list, edges, wing,
		                                                                           ws.dinv, ws.dinv_b, ws.schur, ws.rhs,
		                                                                           ws.x + 6 * static_cast<int64_t>(ws.n0), error_flag);
		NNRT_LAUNCH_CHECK();
	}
	if (m > 0) {
		const size_t panel_bytes = sizeof(float) * static_cast<size_t>(m) * DC_NB;
		const int in_lds = panel_bytes <= 120 * 1024 ? 1 : 0;
		k_dense_cholesky_solve<<<1, DC_THREADS, in_lds ? panel_bytes : 0, stream>>>(ws.schur, m, ws.x + 6 * static_cast<int64_t>(ws.n0),
		                                                                           error_flag, in_lds);
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
