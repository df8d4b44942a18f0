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


#include "arrow_device.hpp"

namespace nnrt {

// ---- data acc + ARAP edge terms -> full diagonal blocks (+LM) and rhs = negative gradient ----
// 32 lanes per node: lane q < 21 owns upper-triangle entry q of the 6x6 block, lanes 21..26 the gradient. The ARAP
// terms (ComputeBlockSums of dEi^T dEi / dEj^T dEj and J^T e, ArapHessianImpl.h / DeformableMeshToImageFitterImpl.h)
// come from the node's incidence slots (edge_terms: node-major, ascending edge order per node; the ARAP edge kernel
// wrote each edge's terms for its two nodes there, laid out as the prepared row), lane q summing entry q.
// lane q of node n's 32-lane group: the node's prepared entry (q < 21: diagonal-block entry (r0, c0), r0 <= c0, with LM
// -> *dv; 21 <= q < 27: right-hand side entry q - 21 -> *dv), its global outputs written; false for lanes q >= 27
__device__ __forceinline__ bool prepare_node(int n, int q, float lm, double* __restrict__ acc, const int* __restrict__ inc_off,
                                             const float* __restrict__ edge_terms, float* __restrict__ diag, float* __restrict__ rhs,
                                             float* __restrict__ gradient_out, float* __restrict__ hessian_out, int& r0, int& c0, float& dv) {
	// the accumulator entry first: its load (memory-side atomics' target) overlaps the slot loads below
	double* ad = acc + static_cast<int64_t>(n) * ACC_STRIDE;
	const double hq = q < 27 ? ad[q] : 0.0;
	float arap = 0.f;
	const int beg = inc_off[n], end = inc_off[n + 1];
	for (int u0 = beg; u0 < end; u0 += 32) {
		const int nu = end - u0 < 32 ? end - u0 : 32;
		float v[32];
#pragma unroll
		for (int u = 0; u < 32; u++) v[u] = (u < nu && q < 27) ? edge_terms[static_cast<int64_t>(u0 + u) * EDGE_TERMS + q] : 0.f;
#pragma unroll
		for (int u = 0; u < 32; u++)
			if (u < nu) arap += v[u];
	}
	if (q >= 27) return false;
	r0 = 0;   // upper-triangle enumeration of entry q (q < 21)
	{
		int qq = q;
		while (r0 < 6 && qq >= 6 - r0) {
			qq -= 6 - r0;
			r0++;
		}
		c0 = r0 + qq;
	}
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
		dv = v;
	} else {
		const float g = (0.f - static_cast<float>(hq)) - arap;
		rhs[6 * static_cast<int64_t>(n) + q - 21] = g;
		gradient_out[6 * static_cast<int64_t>(n) + q - 21] = g;
		dv = g;
	}
	return true;
}

// ---- data acc + ARAP edge terms -> full diagonal blocks (+LM) and rhs = negative gradient (every node) ----
__global__ __launch_bounds__(256) void k_arrow_prepare(int N, float lm, double* __restrict__ acc, const int* __restrict__ inc_off,
                                                       const float* __restrict__ edge_terms, float* __restrict__ diag, float* __restrict__ rhs,
                                                       float* __restrict__ gradient_out, float* __restrict__ hessian_out) {
	const int n = static_cast<int>((static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 5);
	const int q = static_cast<int>(threadIdx.x & 31);
	if (n >= N) return;   // uniform per 32-lane node group
	int r0, c0;
	float dv;
	prepare_node(n, q, lm, acc, inc_off, edge_terms, diag, rhs, gradient_out, hessian_out, r0, c0, dv);
}

// ---- stem: D^-1 and D^-1 B per stem node, four lanes per node (each forms D^-1 with the same arithmetic and the products
// of every fourth of the node's edges), in one launch with the corner init (the last init_blocks blocks: corner.hip's
// corner_init_thread; both read the prepared diagonal blocks and write disjoint outputs) ----
constexpr int STEM_LANES = 4;
// lane s of each quad (DPP quad_perm [s, s, s, s]); s is a constant after unrolling
__device__ __forceinline__ float stem_quad_bcast(float v, int s) {
	const int x = __builtin_bit_cast(int, v);
	switch (s) {
		case 0: return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, x, 0x00, 0xf, 0xf, false));
		case 1: return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, x, 0x55, 0xf, 0xf, false));
		case 2: return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, x, 0xAA, 0xf, 0xf, false));
		default: return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, x, 0xFF, 0xf, 0xf, false));
	}
}
// stem node i, lane sub of its STEM_LANES: Cholesky of the prepared block f (potrf semantics: a failure sets the error
// flag), D_i^-1 (lane 0 stores it) and D_i^-1 B_e for every STEM_LANES-th of its edges
__device__ __forceinline__ void stem_factor(int i, int sub, const float (&f)[36], const int* __restrict__ edge_offsets, const int* __restrict__ edge_list,
                                            const float* __restrict__ wing, float* __restrict__ dinv, float* __restrict__ dinv_b, int* error_flag) {
	float L[6][6];
#pragma unroll
	for (int k = 0; k < 36; k++) L[k / 6][k % 6] = f[k];
	if (!cholesky_small<6>(L)) {
		if (sub == 0) atomicOr(error_flag, 1);
		return;
	}
	// D_i^-1 one potrs per identity column (invert_from_cholesky_small's operations), the columns dealt over the node's
	// four lanes (columns sub and sub + 4) and broadcast within the quad by DPP: a third of the dependent divisions per
	// lane, bit-identical
	static_assert(STEM_LANES == 4, "quad broadcasts");
	float cv[2][6];
#pragma unroll
	for (int k = 0; k < 2; k++) {
		const int c = sub + 4 * k;   // (6, 7: an all-zero column, never broadcast)
#pragma unroll
		for (int r = 0; r < 6; r++) cv[k][r] = r == c ? 1.f : 0.f;
		cholesky_solve_small<6>(L, cv[k]);
	}
	float Di[6][6];
#pragma unroll
	for (int c = 0; c < 6; c++)
#pragma unroll
		for (int r = 0; r < 6; r++) Di[r][c] = stem_quad_bcast(cv[c / 4][r], c % 4);
	if (sub == 0) {
		float4* o4 = reinterpret_cast<float4*>(dinv + static_cast<int64_t>(i) * 36);
#pragma unroll
		for (int q = 0; q < 9; q++)
			o4[q] = make_float4(Di[(4 * q) / 6][(4 * q) % 6], Di[(4 * q + 1) / 6][(4 * q + 1) % 6], Di[(4 * q + 2) / 6][(4 * q + 2) % 6],
			                    Di[(4 * q + 3) / 6][(4 * q + 3) % 6]);
	}
	for (int ei = edge_offsets[i] + sub; ei < edge_offsets[i + 1]; ei += STEM_LANES) {
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

__global__ __launch_bounds__(256) void k_init_stem(CornerInitArgs ia, int init_blocks, const float* __restrict__ rhs, int n0,
                                                   const float* __restrict__ diag, const int* __restrict__ edge_offsets,
                                                   const int* __restrict__ edge_list, const float* __restrict__ wing, float* __restrict__ dinv,
                                                   float* __restrict__ dinv_b, int* error_flag) {
	// the stem's blocks come first: their dependent chains (Cholesky, inverse, D^-1 B) start with the launch while the
	// corner-init blocks (independent stores) fill the rest of the machine behind them
	const int stem_blocks = static_cast<int>(gridDim.x) - init_blocks;
	if (static_cast<int>(blockIdx.x) >= stem_blocks) {
		corner_init_thread(static_cast<int64_t>(blockIdx.x - stem_blocks) * blockDim.x + threadIdx.x, ia, diag, rhs);
		return;
	}
	const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	const int i = static_cast<int>(t / STEM_LANES), sub = static_cast<int>(t % STEM_LANES);
	if (i >= n0) return;
	// 6 x 6 blocks are 144 B = nine 16-B words: loaded and stored as float4
	float f[36];
	{
		const float4* d4 = reinterpret_cast<const float4*>(diag + static_cast<int64_t>(i) * 36);
#pragma unroll
		for (int q = 0; q < 9; q++) {
			const float4 v = d4[q];
			f[4 * q] = v.x;
			f[4 * q + 1] = v.y;
			f[4 * q + 2] = v.z;
			f[4 * q + 3] = v.w;
		}
	}
	stem_factor(i, sub, f, edge_offsets, edge_list, wing, dinv, dinv_b, error_flag);
}

// ---- Schur update S_ab -= sum over stem nodes i adjacent to a and b of B_ia^T D_i^-1 B_ib (one wave per target) ----
// Lane (r, c) < 36 owns entry (r, c) of the 6x6 target block. The target's pair list is loaded once, one pair per lane,
// and broadcast by shuffle, so the wing / D^-1 B loads of eight pairs are in flight together (no dependent index load
// per pair). Pairs are summed in list order.
__device__ __forceinline__ void stem_schur_wave(int w, int lane, const CornerMap& S, const int* __restrict__ tgt_off, const int2* __restrict__ tgt_ab,
                                                const int2* __restrict__ pairs, const float* __restrict__ wing, const float* __restrict__ dinv_b) {
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
		float* dst = corner_block_entry(S, ab.x, ab.y, r, c);
		if (dst) {
			const float v = *dst - acc;
			*dst = v;
			if (S.sdiag && ab.x == ab.y && r == c) S.sdiag[S.node_row[ab.x] + r] = v;   // diag(S): the refinement gate's reference
		}
	}
}

// ---- fitter form of the Schur update: the ARAP wing blocks dEi^T dEj (dEj = [0 | b I]) are zero outside their last
// three columns, so B_ia^T D_i^-1 B_ib is zero outside its lower-right 3x3 block and only those 9 entries change
// (the others would subtract exact zeros). 7 pair slots x 9 entries per wave; slots reduced in order at the end.
// s_part: this wave's [7][9] LDS partials
__device__ __forceinline__ void stem_schur_t3_wave(int w, int lane, float (*s_part)[9], const CornerMap& S, const int* __restrict__ tgt_off,
                                                   const int2* __restrict__ tgt_ab, const int2* __restrict__ pairs, const float* __restrict__ wing,
                                                   const float* __restrict__ dinv_b) {
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
	if (lane < 63) s_part[slot][ent] = acc;
	__builtin_amdgcn_wave_barrier();   // LDS is in order within the wave; keep the compiler from moving the reads up
	if (lane < 9) {
		float t = 0.f;
#pragma unroll
		for (int sl = 0; sl < 7; sl++) t += s_part[sl][lane];
		const int2 ab = tgt_ab[w];
		float* dst = corner_block_entry(S, ab.x, ab.y, 3 + lane / 3, 3 + lane % 3);
		if (dst) {
			const float v = *dst - t;
			*dst = v;
			if (S.sdiag && ab.x == ab.y && lane % 4 == 0) S.sdiag[S.node_row[ab.x] + 3 + lane / 3] = v;   // diag(S) (lanes 0, 4, 8)
		}
	}
}

// ---- b_C -= sum over stem edges i->a of (D_i^-1 B_ia)^T b_i (one wave per corner node; lanes over its edges) ----
__device__ __forceinline__ void stem_rhs_wave(int a, int lane, const int* __restrict__ rhs_off, const int* __restrict__ rhs_edges,
                                              const int32_t* __restrict__ edges, const float* __restrict__ dinv_b, const float* __restrict__ rhs,
                                              const int* __restrict__ node_row, float* __restrict__ cb) {
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
		cb[node_row[a] + lane] -= v;   // the corner's permuted order
	}
}

// Both stem-side corner updates in one launch (they read the same D^-1 B and write disjoint outputs): waves
// [0, targets) update the Schur targets, waves [targets, targets + nc) the corner right-hand side.
template <bool T3>
__global__ __launch_bounds__(256) void k_stem_schur_rhs(int targets, int nc, CornerMap S, const int* __restrict__ tgt_off,
                                                        const int2* __restrict__ tgt_ab, const int2* __restrict__ pairs, const float* __restrict__ wing,
                                                        const float* __restrict__ dinv_b, const int* __restrict__ rhs_off, const int* __restrict__ rhs_edges,
                                                        const int32_t* __restrict__ edges, const float* __restrict__ rhs, float* __restrict__ cb) {
	__shared__ float s_part[4][7][9];
	const int w = static_cast<int>((static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6);
	const int lane = static_cast<int>(threadIdx.x & 63), wl = static_cast<int>(threadIdx.x >> 6);
	if (w < targets) {
		if constexpr (T3) stem_schur_t3_wave(w, lane, s_part[wl], S, tgt_off, tgt_ab, pairs, wing, dinv_b);
		else stem_schur_wave(w, lane, S, tgt_off, tgt_ab, pairs, wing, dinv_b);
	} else if (w - targets < nc) {
		stem_rhs_wave(w - targets, lane, rhs_off, rhs_edges, edges, dinv_b, rhs, S.node_row, cb);
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

// ---- stem back-substitution: x_D = D^-1 (b_D - B x_C) (arrow_device.hpp: arrow_back_node) ----
// gate (refinement; nullable): mode 1 = the first pass of a gated refinement: x_i always, the update only when the
// refinement does not run, else the stem residual r_i -> res; mode 2 = the refinement's last pass: runs only when it does.
__global__ void k_arrow_back(int n0, int n_update, const float* __restrict__ dinv, const int* __restrict__ edge_offsets, const int* __restrict__ edge_list,
                             const int32_t* __restrict__ edges, const float* __restrict__ wing, const float* __restrict__ rhs,
                             float* __restrict__ x, const float* state_in, float* node_state, float* __restrict__ updates_out,
                             float* __restrict__ x_base, const unsigned* gate = nullptr, float ratio = 0.f, int mode = 0,
                             const float* __restrict__ diag = nullptr, float* __restrict__ res = nullptr) {
	const int i = blockIdx.x * blockDim.x + threadIdx.x;
	bool refining = false;
	if (gate && mode == 2) {
		refining = refine_gate_on(gate, ratio);
		if (!refining) return;
	}
	if (gate && mode == 1) refining = refine_gate_on(gate, ratio);
	if (i >= n_update && i >= n0) return;
	arrow_back_node<false>(i, n0, n_update, dinv, edge_offsets, edge_list, edges, wing, XPlain{rhs}, x, XPlain{x}, state_in, node_state,
	                       updates_out, x_base, XPlain{x_base}, gate ? mode : 0, refining, diag, res);
}

// ---- iterative refinement: the correction's corner right-hand side (one wave per corner node a; runs only when the gate
// is on; arrow_device.hpp: refine_rhs_node) ----
__global__ __launch_bounds__(256) void k_refine_corner_rhs(int n0, int nc, const float* __restrict__ dinv_b, const float* __restrict__ diag,
                                                           const int* __restrict__ inc_off, const int* __restrict__ inc_list,
                                                           const int32_t* __restrict__ edges, const float* __restrict__ wing,
                                                           const float* __restrict__ rhs, const float* __restrict__ x, const float* __restrict__ res,
                                                           const int* __restrict__ node_row, float* __restrict__ rhs2, const unsigned* gate, float ratio) {
	if (!refine_gate_on(gate, ratio)) return;
	const int a = static_cast<int>((static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6);
	const int lane = static_cast<int>(threadIdx.x & 63);
	if (a >= nc) return;
	const float v = refine_rhs_node(a, lane, n0, dinv_b, diag, inc_off, inc_list, edges, wing, rhs, XPlain{x}, XPlain{res});
	if (lane < 6) rhs2[node_row[a] + lane] = v;
}

// ---- the refinement's safeguarded last step (arrow_device.hpp), per-stage form: run only when the gate is on ----
__global__ __launch_bounds__(64) void k_refine_correction(int n0, int N, const float* __restrict__ dinv, const int* __restrict__ edge_offsets,
                                                          const int* __restrict__ edge_list, const int32_t* __restrict__ edges,
                                                          const float* __restrict__ wing, const float* __restrict__ res, float* __restrict__ dx,
                                                          const float* __restrict__ x, const unsigned* gate, float ratio, unsigned* guard) {
	if (!refine_gate_on(gate, ratio)) return;
	refine_correction_node<false>(static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x), n0, N, dinv, edge_offsets, edge_list, edges, wing,
	                              XPlain{res}, dx, XPlain{dx}, XPlain{x}, guard);
}
__global__ __launch_bounds__(64) void k_refine_apply(int N, const float* __restrict__ dx, float* __restrict__ x, const float* state_in, float* node_state,
                                                     float* __restrict__ updates_out, const unsigned* gate, float ratio, const unsigned* guard) {
	if (!refine_gate_on(gate, ratio)) return;
	refine_apply_node(static_cast<int>(blockIdx.x * blockDim.x + threadIdx.x), N, refine_guard_accepts(guard), XPlain{dx}, XPlain{x}, x, state_in,
	                  node_state, updates_out);
}

nnrt_status arrowhead_solve_core(const ArrowheadWorkspace& ws, const int32_t* edges, const float* wing, int* error_flag, hipStream_t stream,
                                 bool arap_wings, float* node_state, float* updates_out, const float* state_in) {
	const int m = ws.m;
	if (!state_in) state_in = node_state;
	NNRT_CHECK_ARG(m == 0 || ws.corner, "arrowhead workspace without a corner plan");
	if (ws.n0 > 0 || m > 0) {   // corner init and stem in one launch
		const CornerInitArgs ia = m > 0 ? ws.corner->init_args(ws.n0) : CornerInitArgs{0, 0, 0, nullptr, nullptr, nullptr, nullptr};
		const int init_blocks = m > 0 ? static_cast<int>(ceil_div(ia.threads(), 256)) : 0;
		const int stem_blocks = static_cast<int>(ceil_div(static_cast<int64_t>(ws.n0) * STEM_LANES, 256));
		k_init_stem<<<static_cast<unsigned>(init_blocks + stem_blocks), 256, 0, stream>>>(ia, init_blocks, ws.rhs, ws.n0, ws.diag, ws.edge_offsets,
		                                                                                  ws.edge_list, wing, ws.dinv, ws.dinv_b, error_flag);
		NNRT_LAUNCH_CHECK();
		if (m > 0) {
			nnrt_status st = ws.corner->launch_offdiag(ws.n0, edges, wing, stream);   // >= 3 layers: after the init
			if (st) return st;
		}
	}
	if (ws.n0 > 0) {
		if (m > 0 && ws.targets > 0) {
			const CornerMap cm = ws.corner->map();
			const unsigned grid = static_cast<unsigned>(ceil_div((static_cast<int64_t>(ws.targets) + m / 6) * 64, 256));
			if (arap_wings)
				k_stem_schur_rhs<true><<<grid, 256, 0, stream>>>(ws.targets, m / 6, cm, ws.tgt_off, ws.tgt_ab, ws.pairs, wing, ws.dinv_b, ws.rhs_off,
				                                                 ws.rhs_edges, edges, ws.rhs, ws.corner->rhs_perm());
			else
				k_stem_schur_rhs<false><<<grid, 256, 0, stream>>>(ws.targets, m / 6, cm, ws.tgt_off, ws.tgt_ab, ws.pairs, wing, ws.dinv_b, ws.rhs_off,
				                                                  ws.rhs_edges, edges, ws.rhs, ws.corner->rhs_perm());
			NNRT_LAUNCH_CHECK();
		}
	}
	const bool refine = ws.refine && ws.inc_off && ws.res && ws.dx && m > 0;
	if (m > 0 && ws.corner->flow_ok()) {
		// the corner's factorization, then one dataflow launch (corner.hip k_corner_flow): the back substitution chains
		// with the stem pass (x, the update or, when the refinement gate opens, the stem residual), then the gated
		// refinement step's roles (they return at once when the gate is shut)
		nnrt_status st = ws.corner->launch_factor(error_flag, stream);
		if (st) return st;
		FlowStem fs;
		fs.n0 = ws.n0;
		fs.N = ws.N;
		fs.n_update = node_state ? ws.N : ws.n0;
		fs.mode = refine ? 1 : 0;
		fs.dinv = ws.dinv;
		fs.wing = wing;
		fs.diag = ws.diag;
		fs.dinv_b = ws.dinv_b;
		fs.edge_offsets = ws.edge_offsets;
		fs.edge_list = ws.edge_list;
		fs.inc_off = ws.inc_off;
		fs.inc_list = ws.inc_list;
		fs.edges = edges;
		fs.rhs = ws.rhs;
		fs.x = ws.x;
		fs.dx = ws.dx;
		fs.state_in = state_in;
		fs.node_state = node_state;
		fs.updates_out = updates_out;
		fs.res = ws.res;
		fs.gate = refine ? ws.corner->pivot_ratio() : nullptr;
		fs.guard = refine ? ws.corner->refine_guard() : nullptr;
		fs.ratio = ws.refine_ratio;
		fs.error_flag = error_flag;
		return ws.corner->launch_flow(fs, stream);
	}
	if (m > 0) {
		nnrt_status st = ws.corner->launch_solve(ws.x + 6 * static_cast<int64_t>(ws.n0), error_flag, stream);
		if (st) return st;
	}
	if (!refine) {
		// with node_state, the node updates ride along (all N nodes) in the back-substitution launch
		const int threads = node_state ? ws.N : ws.n0;
		if (threads > 0) {
			k_arrow_back<<<static_cast<unsigned>(ceil_div(threads, 64)), 64, 0, stream>>>(ws.n0, threads, ws.dinv, ws.edge_offsets, ws.edge_list, edges,
			                                                                             wing, ws.rhs, ws.x, state_in, node_state, updates_out, nullptr);
			NNRT_LAUNCH_CHECK();
		}
		return NNRT_OK;
	}
	// gated iterative refinement (one step): the corner factorization left its smallest pivot / diag(S) ratio on the
	// device; below ws.refine_ratio the next launches form res = rhs - H x (double sums) and solve H d = res with the
	// same factors, x += d; otherwise the first pass applies the update and the others return at once
	const unsigned* gate = ws.corner->pivot_ratio();
	const float ratio = ws.refine_ratio;
	k_arrow_back<<<static_cast<unsigned>(ceil_div(ws.N, 64)), 64, 0, stream>>>(ws.n0, ws.N, ws.dinv, ws.edge_offsets, ws.edge_list, edges, wing,
	                                                                          ws.rhs, ws.x, state_in, node_state, updates_out, nullptr, gate, ratio, 1,
	                                                                          ws.diag, ws.res);
	NNRT_LAUNCH_CHECK();
	k_refine_corner_rhs<<<static_cast<unsigned>(ceil_div(static_cast<int64_t>(m / 6) * 64, 256)), 256, 0, stream>>>(
	    ws.n0, m / 6, ws.dinv_b, ws.diag, ws.inc_off, ws.inc_list, edges, wing, ws.rhs, ws.x, ws.res, ws.corner->map().node_row,
	    ws.corner->refine_rhs(), gate, ratio);
	NNRT_LAUNCH_CHECK();
	nnrt_status st = ws.corner->launch_resolve(ws.dx + 6 * static_cast<int64_t>(ws.n0), stream, gate, ratio);
	if (st) return st;
	// the safeguarded step: correction pass (the stem rows of d, max |d| / max |x|), then the apply pass
	k_refine_correction<<<static_cast<unsigned>(ceil_div(ws.N, 64)), 64, 0, stream>>>(ws.n0, ws.N, ws.dinv, ws.edge_offsets, ws.edge_list, edges, wing,
	                                                                                 ws.res, ws.dx, ws.x, gate, ratio, ws.corner->refine_guard());
	NNRT_LAUNCH_CHECK();
	k_refine_apply<<<static_cast<unsigned>(ceil_div(ws.N, 64)), 64, 0, stream>>>(ws.N, ws.dx, ws.x, state_in, node_state, updates_out, gate, ratio,
	                                                                            ws.corner->refine_guard());
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

nnrt_status launch_arrowhead_iteration(const ArrowheadWorkspace& ws, const double* acc, float lm, const int32_t* edges, const float* wing,
                                       float* node_state, const float* edge_jr, float* updates_out, float* gradient_out, float* hessian_out,
                                       int* error_flag, hipStream_t stream, const float* state_in) {
	// (one launch of prepare + stem + corner init, every node's block kept in its workgroup, measured 22.4 µs at C5 against
	// 11.6 + 9.1 µs as two launches: the stem phase then ran on 4 of every 32 lanes; round 4, not kept)
	k_arrow_prepare<<<static_cast<unsigned>(ceil_div(static_cast<int64_t>(ws.N) * 32, 256)), 256, 0, stream>>>(
	    ws.N, lm, const_cast<double*>(acc), ws.inc_off, edge_jr, ws.diag, ws.rhs, gradient_out, hessian_out);
	NNRT_LAUNCH_CHECK();
	return arrowhead_solve_core(ws, edges, wing, error_flag, stream, true, node_state, updates_out, state_in);
}

} // namespace nnrt
