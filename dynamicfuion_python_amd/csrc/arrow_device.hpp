// Device helpers of the arrowhead solve's stem side, shared by the per-stage kernels (arap.hip) and the corner's dataflow
// substitution launches (corner.hip k_corner_flow): the stem back substitution x_D = D^-1 (b_D - B x_C)
// (SolveBlockSparseArrowheadCholesky.cpp:84-90), the fp64 residual rows of the gated refinement,
// the corner right-hand side of the refinement's correction, and the node update R <- R Rodrigues(w), t += dt
// (HierarchicalGraphWarpField.cpp:261-282, A10).
//
// Vectors that another workgroup of the same launch writes are read through a loader (XSc1: sc1 loads that bypass this
// CU's L1, the hand-off form of MI355X_MICROARCH.md "inter-workgroup visibility"); vectors from earlier launches through
// XPlain. Both give the same values and the same arithmetic.
#pragma once

#include "fitter_kernels.hpp"

namespace nnrt {

typedef int flow_v2i __attribute__((ext_vector_type(2)));
typedef int flow_v4i __attribute__((ext_vector_type(4)));

// buffer descriptor over n bytes at p (p, n wave-uniform: kernel arguments)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t flow_rsrc(const void* p, int64_t bytes) {
	return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, static_cast<int>(bytes), 0x00020000);
}
// sc1 (L1-bypassing) loads through a descriptor, byte offsets
__device__ __forceinline__ float4 ld_sc1_f4(__amdgpu_buffer_rsrc_t r, int off) {
	return __builtin_bit_cast(float4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 16));
}
__device__ __forceinline__ float2 ld_sc1_f2(__amdgpu_buffer_rsrc_t r, int off) {
	return __builtin_bit_cast(float2, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 16));
}
__device__ __forceinline__ float ld_sc1_f(__amdgpu_buffer_rsrc_t r, int off) {
	return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 16));
}
// sc1 (write-through) store of one float
__device__ __forceinline__ void st_sc1(float* p, float v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

// 6 x 6 blocks as nine float4, 6-vectors as three float2 (the same products and sums as element-wise loads)
__device__ __forceinline__ void load36(const float* src, float (&dst)[36]) {
	const float4* s4 = reinterpret_cast<const float4*>(src);
#pragma unroll
	for (int q = 0; q < 9; q++) {
		const float4 v = s4[q];
		dst[4 * q] = v.x;
		dst[4 * q + 1] = v.y;
		dst[4 * q + 2] = v.z;
		dst[4 * q + 3] = v.w;
	}
}
__device__ __forceinline__ void load6(const float* src, float (&dst)[6]) {
	const float2* x2 = reinterpret_cast<const float2*>(src);
#pragma unroll
	for (int q = 0; q < 3; q++) {
		const float2 v = x2[q];
		dst[2 * q] = v.x;
		dst[2 * q + 1] = v.y;
	}
}

// 6-float node rows of a vector: from an earlier launch (plain loads) ...
struct XPlain {
	const float* p;
	__device__ __forceinline__ void ld6(int64_t node, float (&o)[6]) const { load6(p + 6 * node, o); }
};
// ... or written by other workgroups of this launch (sc1 loads; base = the vector's first float, bytes = its size)
struct XSc1 {
	__amdgpu_buffer_rsrc_t r;
	__device__ __forceinline__ void ld6(int64_t node, float (&o)[6]) const {
#pragma unroll
		for (int q = 0; q < 3; q++) {
			const float2 v = ld_sc1_f2(r, static_cast<int>(24 * node + 8 * q));
			o[2 * q] = v.x;
			o[2 * q + 1] = v.y;
		}
	}
};

// where the stem pass's per-node outputs go: plain stores (read by later launches) or sc1 stores (read by other
// workgroups of the same dataflow launch), 8 B at a time
template <bool SC1>
__device__ __forceinline__ void store6(float* dst, const float (&v)[6]) {
	if constexpr (SC1) {
#pragma unroll
		for (int q = 0; q < 3; q++)
			__hip_atomic_store(reinterpret_cast<unsigned long long*>(dst) + q,
			                   static_cast<unsigned long long>(__float_as_uint(v[2 * q])) |
			                       (static_cast<unsigned long long>(__float_as_uint(v[2 * q + 1])) << 32),
			                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	} else {
		float2* d2 = reinterpret_cast<float2*>(dst);
#pragma unroll
		for (int q = 0; q < 3; q++) d2[q] = make_float2(v[2 * q], v[2 * q + 1]);
	}
}

// node update (R <- R Rodrigues(omega), t += dt) from the node's solved increment x6; updates_out gets x6. The motion
// the iteration started from is read from state_in (the warp field's state, or a snapshot the iteration restarts from)
// and the result written to node_state (g is never changed by an update)
// (state_in may equal node_state: no __restrict__ on either)
__device__ __forceinline__ void arrow_update_node(int n, const float (&xl)[6], const float* state_in, float* node_state, float* __restrict__ updates_out) {
	for (int c = 0; c < 6; c++) updates_out[6 * static_cast<int64_t>(n) + c] = xl[c];
	const float* os = state_in + static_cast<int64_t>(n) * NODE_STRIDE;
	float* ns = node_state + static_cast<int64_t>(n) * NODE_STRIDE;
	float old[12];
	for (int i = 0; i < 12; i++) old[i] = os[3 + i];
	ns[3] = old[0] + xl[3];
	ns[4] = old[1] + xl[4];
	ns[5] = old[2] + xl[5];
	float dR[9];
	rodrigues_device(xl[0], xl[1], xl[2], dR);
	const float* R = old + 3;
	for (int r = 0; r < 3; r++)
		for (int c = 0; c < 3; c++) ns[6 + 3 * r + c] = (R[3 * r] * dR[c] + R[3 * r + 1] * dR[3 + c]) + R[3 * r + 2] * dR[6 + c];
}

// stem row i of the back substitution: x_i = D_i^-1 (b_i - sum over its edges e = (i, j) of B_e x_j) in float, edges in
// CSR order (the one arithmetic every caller shares, so a recomputation is bit-identical)
template <class RL, class XL>
__device__ __forceinline__ void stem_solve(int i, const float* __restrict__ dinv, const int* __restrict__ edge_offsets, const int* __restrict__ edge_list,
                                           const int32_t* __restrict__ edges, const float* __restrict__ wing, const RL& rhs, const XL& x,
                                           float (&o)[6]) {
	float r6[6];
	rhs.ld6(i, r6);
	for (int ei = edge_offsets[i]; ei < edge_offsets[i + 1]; ei++) {
		const int e = edge_list[ei];
		const int j = edges[2 * e + 1];
		float B[36], xj[6];
		load36(wing + static_cast<int64_t>(e) * 36, B);
		x.ld6(j, xj);
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
#pragma unroll
	for (int r = 0; r < 6; r++) {
		float acc = 0.f;
#pragma unroll
		for (int k = 0; k < 6; k++) acc += D[6 * r + k] * r6[k];
		o[r] = acc;
	}
}

// The part of a stem row's back substitution that does not depend on the corner solution, done while a dataflow stem
// worker waits for the corner (k_corner_flow): the row's edge and corner-node indices into registers, and one load
// from every 64-B line the row reads after the wait (wing blocks, D_i^-1, b_i, the node state) so those lines are in
// L2 by then. n = -1: more than STEM_PRE_EDGES edges (the caller takes stem_solve).
constexpr int STEM_PRE_EDGES = 8;
struct StemPre {
	int n;
	int e[STEM_PRE_EDGES], j[STEM_PRE_EDGES];
};
__device__ __forceinline__ void touch_lines(const float* p, int floats) {   // one load per 64-B line, kept by an empty asm
	for (int q = 0; q < floats; q += 16) {
		const float v = p[q];
		asm volatile("" ::"v"(v));
	}
}
__device__ __forceinline__ StemPre stem_prefetch(int i, const float* __restrict__ dinv, const int* __restrict__ edge_offsets,
                                                 const int* __restrict__ edge_list, const int32_t* __restrict__ edges,
                                                 const float* __restrict__ wing, const float* rhs, const float* state_in) {
	StemPre pre;
	const int beg = edge_offsets[i], end = edge_offsets[i + 1];
	pre.n = end - beg <= STEM_PRE_EDGES ? end - beg : -1;
#pragma unroll
	for (int q = 0; q < STEM_PRE_EDGES; q++) {
		const bool ok = q < pre.n;
		const int e = ok ? edge_list[beg + q] : 0;
		pre.e[q] = e;
		pre.j[q] = ok ? edges[2 * e + 1] : 0;
		if (ok) touch_lines(wing + static_cast<int64_t>(e) * 36, 36);
	}
	touch_lines(dinv + static_cast<int64_t>(i) * 36, 36);
	touch_lines(rhs + 6 * static_cast<int64_t>(i), 6);
	if (state_in) touch_lines(state_in + static_cast<int64_t>(i) * NODE_STRIDE, NODE_STRIDE);
	return pre;
}
// stem_solve with the row's indices from stem_prefetch: the same arithmetic in the same order (bit-identical)
template <class RL, class XL>
__device__ __forceinline__ void stem_solve_pre(int i, const StemPre& pre, const float* __restrict__ dinv, const float* __restrict__ wing,
                                               const RL& rhs, const XL& x, float (&o)[6]) {
	float r6[6];
	rhs.ld6(i, r6);
#pragma unroll
	for (int q = 0; q < STEM_PRE_EDGES; q++) {   // constant indices: pre stays in registers
		if (q >= pre.n) break;
		float B[36], xj[6];
		load36(wing + static_cast<int64_t>(pre.e[q]) * 36, B);
		x.ld6(pre.j[q], xj);
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
#pragma unroll
	for (int r = 0; r < 6; r++) {
		float acc = 0.f;
#pragma unroll
		for (int k = 0; k < 6; k++) acc += D[6 * r + k] * r6[k];
		o[r] = acc;
	}
}

// residual of stem row i, rhs_i - D_i x_i - sum over its edges of B_e x_j, the products and sums in double, rounded once
// (D_i: the prepared diagonal block with LM; stem nodes couple to corner nodes only)
template <class RL, class XL>
__device__ __forceinline__ void stem_residual(int i, const float (&xi)[6], const float* __restrict__ diag, const int* __restrict__ edge_offsets,
                                              const int* __restrict__ edge_list, const int32_t* __restrict__ edges, const float* __restrict__ wing,
                                              const RL& rhs, const XL& x, float (&res)[6]) {
	double r[6];
	float D[36];
	load36(diag + static_cast<int64_t>(i) * 36, D);
	float b6[6];
	rhs.ld6(i, b6);
#pragma unroll
	for (int c = 0; c < 6; c++) {
		double s = static_cast<double>(b6[c]);
#pragma unroll
		for (int k = 0; k < 6; k++) s -= static_cast<double>(D[6 * c + k]) * static_cast<double>(xi[k]);
		r[c] = s;
	}
	for (int ei = edge_offsets[i]; ei < edge_offsets[i + 1]; ei++) {
		const int e = edge_list[ei];
		float B[36], xj[6];
		load36(wing + static_cast<int64_t>(e) * 36, B);
		x.ld6(edges[2 * e + 1], xj);
#pragma unroll
		for (int c = 0; c < 6; c++)
#pragma unroll
			for (int k = 0; k < 6; k++) r[c] -= static_cast<double>(B[6 * c + k]) * static_cast<double>(xj[k]);
	}
#pragma unroll
	for (int c = 0; c < 6; c++) res[c] = static_cast<float>(r[c]);
}

// The stem side of one arrowhead back-substitution pass for node i (one thread per node):
// i < n0: stem back substitution (and, with node_state, that node's update from the x it just formed);
// n0 <= i < n_update: the corner node's update from the corner solve's x (node_state non-null only).
// x_base (refinement pass): x holds the correction d (rhs = the residual); the solution is x_base + d, written to x_base
// and applied (x_base is read and written by its own thread only; x is read across threads and only written by stem
// threads at their own rows, which no thread of the pass reads).
// mode 1 = the first pass of a gated refinement (refining: the gate's decision): x_i always, the update only when the
// refinement does not run, else the stem residual r_i -> res; mode 2 = the refinement's last pass.
// Loaders: rl the right-hand side's rows, xc x's corner rows (written by the corner substitution), bl x_base's rows;
// SC1OUT: x's stem rows and res are read by other workgroups of the same launch (sc1 stores).
template <bool SC1OUT, class RL, class XL, class BL>
__device__ __forceinline__ void arrow_back_node(int i, int n0, int n_update, const float* __restrict__ dinv, const int* __restrict__ edge_offsets,
                                                const int* __restrict__ edge_list, const int32_t* __restrict__ edges, const float* __restrict__ wing,
                                                const RL& rl, float* __restrict__ x, const XL& xc, const float* state_in, float* node_state,
                                                float* __restrict__ updates_out, float* __restrict__ x_base, const BL& bl, int mode, bool refining,
                                                const float* __restrict__ diag, float* __restrict__ res) {
	if (mode == 1 && refining) node_state = nullptr;   // the refinement's last pass applies the update
	if (i >= n0) {
		if (i < n_update && (node_state || x_base)) {
			float xl[6];
			xc.ld6(i, xl);
			if (x_base) {
				float xb[6];
				bl.ld6(i, xb);
				for (int c = 0; c < 6; c++) {
					xl[c] = xb[c] + xl[c];
					x_base[6 * static_cast<int64_t>(i) + c] = xl[c];
				}
			}
			if (node_state) arrow_update_node(i, xl, state_in, node_state, updates_out);
		}
		return;
	}
	float o[6];
	stem_solve(i, dinv, edge_offsets, edge_list, edges, wing, rl, xc, o);
	store6<SC1OUT>(x + 6 * static_cast<int64_t>(i), o);
	if (mode == 1 && refining) {   // the stem row's residual (reads only corner x: no thread of this pass writes those)
		float ri[6];
		stem_residual(i, o, diag, edge_offsets, edge_list, edges, wing, rl, xc, ri);
		store6<SC1OUT>(res + 6 * static_cast<int64_t>(i), ri);
	}
	if (x_base) {
		float xb[6];
		bl.ld6(i, xb);
#pragma unroll
		for (int c = 0; c < 6; c++) {
			o[c] = xb[c] + o[c];
			x_base[6 * static_cast<int64_t>(i) + c] = o[c];
		}
	}
	if (node_state) arrow_update_node(i, o, state_in, node_state, updates_out);
}

// ---- the refinement's last passes (round 6: a safeguarded step) ----
// correction pass, node i (one thread per node): d_i -- stem rows solved from the residual (the stem back substitution
// of H d = r, rl = r, xc = the corner rows of d), stored into dx; corner rows already in dx (the corner substitution) --
// and its max |d_i| / max |x_i| (x from bl) folded into the guard words (one atomic max per wave); a non-finite d
// counts as +inf, so the step is rejected
template <bool SC1OUT, class RL, class XL, class BL>
__device__ __forceinline__ void refine_correction_node(int i, int n0, int n_update, const float* __restrict__ dinv, const int* __restrict__ edge_offsets,
                                                       const int* __restrict__ edge_list, const int32_t* __restrict__ edges,
                                                       const float* __restrict__ wing, const RL& rl, float* __restrict__ dx, const XL& xc, const BL& bl,
                                                       unsigned* guard) {
	float dm = 0.f, xm = 0.f;
	if (i < n0 || i < n_update) {
		float d[6], xb[6];
		if (i < n0) {
			stem_solve(i, dinv, edge_offsets, edge_list, edges, wing, rl, xc, d);
			store6<SC1OUT>(dx + 6 * static_cast<int64_t>(i), d);
		} else {
			xc.ld6(i, d);
		}
		bl.ld6(i, xb);
		bool finite = true;
#pragma unroll
		for (int c = 0; c < 6; c++) {
			finite &= __builtin_isfinite(d[c]);
			dm = fmaxf(dm, fabsf(d[c]));
			xm = fmaxf(xm, fabsf(xb[c]));
		}
		if (!finite) dm = __builtin_inff();
	}
#pragma unroll
	for (int off = 32; off > 0; off >>= 1) {
		dm = fmaxf(dm, __shfl_xor(dm, off));
		xm = fmaxf(xm, __shfl_xor(xm, off));
	}
	if ((threadIdx.x & 63) == 0) {
		__hip_atomic_fetch_max(guard + REFINE_GUARD_D, __float_as_uint(dm), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		__hip_atomic_fetch_max(guard + REFINE_GUARD_X, __float_as_uint(xm), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	}
}
// whether the guard words (every correction pass done) accept the step
__device__ __forceinline__ bool refine_guard_accepts(const unsigned* guard) {
	const float dm = __uint_as_float(__hip_atomic_load(guard + REFINE_GUARD_D, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
	const float xm = __uint_as_float(__hip_atomic_load(guard + REFINE_GUARD_X, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
	return refine_accept(dm, xm);
}
// apply pass, node i < n_update: x = x_base + d when the step is accepted (the same addition as before the safeguard),
// else x_base; x_base <- x and the node's update (the solve's own pass skipped it while refining)
template <class DL, class BL>
__device__ __forceinline__ void refine_apply_node(int i, int n_update, bool accept, const DL& dl, const BL& bl, float* __restrict__ x_base,
                                                  const float* state_in, float* node_state, float* __restrict__ updates_out) {
	if (i >= n_update) return;
	float o[6];
	bl.ld6(i, o);
	if (accept) {
		float d[6];
		dl.ld6(i, d);
#pragma unroll
		for (int c = 0; c < 6; c++) {
			o[c] = o[c] + d[c];
			x_base[6 * static_cast<int64_t>(i) + c] = o[c];
		}
	}
	if (node_state) arrow_update_node(i, o, state_in, node_state, updates_out);
}

// ---- iterative refinement: the correction's corner right-hand side of corner node a (one wave; lane < 6 returns entry
// `lane`, others 0): r_a - sum over stem edges i -> a of (D_i^-1 B_ia)^T r_i, with r_a = b_a - D_a x_a - sum over a's
// incidences of the wing blocks times x (B^T x_i for stem edges, B x_b / B^T x_b for corner edges), products and sums in
// double, rounded once; x (all rows) and r_i of the stem rows from the first back-substitution pass (earlier launches) ----
template <class XL, class RSL>
__device__ __forceinline__ float refine_rhs_node(int a, int lane, int n0, const float* __restrict__ dinv_b, const float* __restrict__ diag,
                                                 const int* __restrict__ inc_off, const int* __restrict__ inc_list, const int32_t* __restrict__ edges,
                                                 const float* __restrict__ wing, const float* __restrict__ rhs, const XL& x, const RSL& res) {
	const int n = n0 + a;
	double ra[6] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0};   // this lane's share of sum H_an x_n over a's incidences
	float s2[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};    // this lane's share of sum (D_i^-1 B_ia)^T r_i
	for (int u = inc_off[n] + lane; u < inc_off[n + 1]; u += 64) {
		const int code = inc_list[u];
		const int e = code >> 1;
		const bool tgt = code & 1;
		const int other = edges[2 * e + (tgt ? 0 : 1)];
		float B[36], xo[6];
		load36(wing + static_cast<int64_t>(e) * 36, B);
		x.ld6(other, xo);
		if (other < n0) {   // stem edge other -> n
			float ri[6], Y[36];
			res.ld6(other, ri);
			load36(dinv_b + static_cast<int64_t>(e) * 36, Y);
#pragma unroll
			for (int c = 0; c < 6; c++) {
				float t = 0.f;
#pragma unroll
				for (int k = 0; k < 6; k++) t += Y[6 * k + c] * ri[k];
				s2[c] += t;
			}
		}
#pragma unroll
		for (int c = 0; c < 6; c++)
#pragma unroll
			for (int k = 0; k < 6; k++) ra[c] += static_cast<double>(tgt ? B[6 * k + c] : B[6 * c + k]) * static_cast<double>(xo[k]);
	}
#pragma unroll
	for (int c = 0; c < 6; c++)
#pragma unroll
		for (int off = 32; off > 0; off >>= 1) {
			ra[c] += __shfl_xor(ra[c], off);
			s2[c] += __shfl_xor(s2[c], off);
		}
	float out = 0.f;
	if (lane < 6) {
		double t = 0.0;
		float u = 0.f;
#pragma unroll
		for (int c = 0; c < 6; c++)
			if (lane == c) {
				t = ra[c];
				u = s2[c];
			}
		float xa[6];
		x.ld6(n, xa);
		double r = static_cast<double>(rhs[6 * static_cast<int64_t>(n) + lane]);
#pragma unroll
		for (int k = 0; k < 6; k++) r -= static_cast<double>(diag[static_cast<int64_t>(n) * 36 + 6 * lane + k]) * static_cast<double>(xa[k]);
		out = static_cast<float>(r - t) - u;
	}
	return out;
}

} // namespace nnrt
