// Argument blocks of the GN-iteration kernels (passed by value; stable pointers so iterations can be hipGraph-captured).
#pragma once

#include <algorithm>
#include <vector>

#include "kernels.hpp"

namespace nnrt {

#ifndef NNRT_SOLVE_LANES
#define NNRT_SOLVE_LANES 1   // block-diagonal solve + update with 8 lanes per node (k_solve_update_lanes)
#endif
#ifndef NNRT_SOLVE_ACC_LDS
#define NNRT_SOLVE_ACC_LDS 1   // k_solve_update stages the wave's accumulator rows through LDS (coalesced read + zero)
#endif
constexpr int ACC_STRIDE = 28;   // per node: 21 JtJ upper-triangle entries + 6 Jt r (+1 pad); 3-dof modes use 6 + 3

// ARAP (regularized, mode ALL) path
struct ArapArgs {
	int E, N, n0;
	float lambda;
	int use_huber;
	float huber_delta;
	int coverage_variable;          // 1: edge weight = max(c2_i, c2_j)
	const int32_t* edges;           // [E,2] virtual
	const int8_t* edge_layers;      // [E]
	const float* radii;             // [layers]
	const float* node_weights;      // [N] (variable coverage)
	const float* node_state;        // [N,16]
	float* edge_jr;                 // [2E,EDGE_TERMS]: per node incidence (inc_slot order), the edge's diagonal-block /
	                                // gradient terms for that node (node-major: a node's incidences are contiguous)
	const int* inc_slot;            // [2E]: slot of incidence 2 e (source) / 2 e + 1 (target) in the node-ordered list
	float* wing;                    // [E,36]: dEi^T dEj
	float* edge_residuals;          // [3E]
	int* error_flag;
};
// per node incidence: the 27 entries of the node's prepared row (21 diagonal-block upper-triangle entries, 6 gradient)
// the edge adds there -- a source incidence all 27, a target incidence b^2 at the translation diagonal (15, 18, 20) and
// b e at 24..26 -- zeros elsewhere, 5 pad
constexpr int EDGE_TERMS = 32;

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

// one ARAP edge: residual, Jacobian terms and wing block, run by the extra workgroups of the fused pixel launch
// (k_fit_pixels_fused's arap_blocks), beside the data term
__device__ inline void arap_edge(const ArapArgs& a, int e) {
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
			for (int h = 0; h < 2; h++)
				for (int q = 0; q < EDGE_TERMS; q++) a.edge_jr[static_cast<int64_t>(a.inc_slot[2 * e + h]) * EDGE_TERMS + q] = 0.f;
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
	// entries, ComputeBlockSums) + J_i^T e (6); target j: b^2 on the translation diagonal + b e (3). Each goes to its
	// incidence's slot, laid out as the node's prepared row (zeros where the edge adds nothing)
	float s27[EDGE_TERMS];
	int q = 0;
#pragma unroll
	for (int r0 = 0; r0 < 6; r0++)
#pragma unroll
		for (int c0 = r0; c0 < 6; c0++) s27[q++] = (dEi[0][r0] * dEi[0][c0] + dEi[1][r0] * dEi[1][c0]) + dEi[2][r0] * dEi[2][c0];
	const float skT[3][3] = {{0.f, j5[2], -j5[1]}, {-j5[2], 0.f, j5[0]}, {j5[1], -j5[0], 0.f}};
#pragma unroll
	for (int c = 0; c < 3; c++) {
		s27[21 + c] = (skT[c][0] * r[0] + skT[c][1] * r[1]) + skT[c][2] * r[2];
		s27[24 + c] = j5[3] * r[c];
	}
#pragma unroll
	for (int k = 27; k < EDGE_TERMS; k++) s27[k] = 0.f;
	const float b2 = (j5[4] * j5[4] + 0.f * 0.f) + 0.f * 0.f;   // target j: dEj = [0 | b I]
	float t27[EDGE_TERMS];
#pragma unroll
	for (int k = 0; k < EDGE_TERMS; k++) t27[k] = 0.f;
	t27[15] = b2;
	t27[18] = b2;
	t27[20] = b2;
#pragma unroll
	for (int c = 0; c < 3; c++) t27[24 + c] = j5[4] * r[c];
	float4* so = reinterpret_cast<float4*>(a.edge_jr + static_cast<int64_t>(a.inc_slot[2 * e]) * EDGE_TERMS);
	float4* to = reinterpret_cast<float4*>(a.edge_jr + static_cast<int64_t>(a.inc_slot[2 * e + 1]) * EDGE_TERMS);
#pragma unroll
	for (int k = 0; k < EDGE_TERMS / 4; k++) {
		so[k] = make_float4(s27[4 * k], s27[4 * k + 1], s27[4 * k + 2], s27[4 * k + 3]);
		to[k] = make_float4(t27[4 * k], t27[4 * k + 1], t27[4 * k + 2], t27[4 * k + 3]);
	}
}

// warped-surface Jacobian rows (-w R (v - g), -w R n): 0 = formed per association in pass 2 from the node state and the
// canonical vertex (the warp stores positions and normals only); 1 = materialised by the warp kernel and gathered
#ifndef NNRT_GATHER_ROWS
#define NNRT_GATHER_ROWS 0
#endif
// pass 2 forms the pixel-node Jacobians as the reference CPU path's unfused products (0, the product: bit-identical to
// the oracle's default arithmetic) or with fused multiply-adds (1, a development build: 2.2 us faster at C2, but on
// ill-conditioned ARAP systems the per-term rounding moves the solution past north_star's 1e-4 from the reference
// arithmetic -- DESIGN.md section 6)
#ifndef NNRT_JAC_FMA
#define NNRT_JAC_FMA 0
#endif

struct FitPixelArgs {
	int H, W, tiles_x, tiles_y;   // tiles of 16 x 16 pixels; this launch covers tile rows [tile_row0, tile_row0 + tiles_y)
	int tile_row0;
	Camera pix;             // pixel-space intrinsics (float)
	NdcSetup ndc;
	float blur;             // NDC units
	PixelAxis ax, ay;       // pixel-centre NDC constants (make_pixel_axis)
	int perspective;
	float max_depth;
	int use_tukey;
	float tukey_c;
	int anchor_count;
	uint64_t* keys;         // [P] raster keys (consumed and reset)
	const int4* faces4;     // [F]
	const float4* wpos;     // [V] warped positions
	const float4* wnrm;     // [V] warped normals
	const int32_t* anchors; // [V,K]
	const uint32_t* face_nodes; // [F, face_node_slots(K)] per face: its unique anchor nodes, ascending (face_node_entry)
	const float2* jrows;    // [V,K,3] (-w R (v-g), -w R n) as 24 B (store_jacobian_row; NNRT_GATHER_ROWS builds only)
	const float4* state_in; // [N,4] node motion the iteration started from (g, t, R: the warp's input)
	int state_identity;     // the iteration starts from R = I, t = 0 (the state is not read, as in the warp)
	const float4* cmesh_p;  // [V] canonical vertex positions (x, y, z, 0)
	const float4* cmesh_n;  // [V] canonical vertex normals
	const float* weights;   // [V,K] anchor weights w
	const float4* ref_points; // [P] reference point (x, y, z, valid)
	float* residuals;       // [P]
	uint8_t* residual_mask; // [P]
	int32_t* pixel_face;    // [P]
	double* acc;            // [N, ACC_STRIDE] fp64 data-term accumulator (21 JtJ + 6 J r)
	float4* records;        // [P, 4] per-pixel Jacobian record (pass 1 -> pass 2)
	int low_occupancy;      // the 4-waves-per-SIMD build of the launch (several residency rounds; k_fit_pixels_fused)
	ArapArgs arap;          // ARAP edge terms, computed by the launch's last arap_blocks workgroups (0: none)
	int arap_blocks;
	const int* tile_order;  // [order_blocks] workgroup -> tile (launch_tile_order; nullable: the arithmetic XCD bands)
	int order_blocks;
};

struct SolveArgs {
	int N;
	float lm;
	double* acc;
	const float* state_in;  // [N,16] the motion the iteration started from (read)
	float* node_state;      // [N,16] updated motion (written; may equal state_in)
	float* updates_out;     // [N*s]
	float* gradient_out;    // [N*s]
	float* hessian_out;     // [N*s*s] (nullable)
	int* error_flag;
};

// Per face (once per frame, after the anchors): the face's distinct anchor nodes in ascending order, each with, per face
// vertex, the LAST anchor slot holding it (AssociateFacesWithAnchorsImpl.h:34-107): entry = node << 12 | k2 << 8 | k1 << 4 | k0
// (k = 0xF: the vertex does not anchor to the node), padded with FACE_NODE_NONE. Nodes must be < 2^20 - 1.
constexpr uint32_t FACE_NODE_NONE = 0xFFFFFFFFu;
constexpr int FACE_NODE_SHIFT = 12;
constexpr int FACE_NODE_MAX_NODES = (1 << 20) - 1;
inline int face_node_slots(int K) { return K <= 4 ? 12 : 3 * MAX_ANCHORS; }
nnrt_status launch_face_node_table(int4* faces4, int64_t F, const int32_t* anchors, int K, uint32_t* out, hipStream_t stream);

// pass 1 then pass 2 in one launch (k_fit_pixels_fused); `between` (optional, stage timing) is recorded before it.
// args.arap_blocks extra workgroups (fit_pixels_arap_blocks(E), 0 without ARAP) compute the ARAP edge terms.
nnrt_status launch_fit_pixels(int mode, const FitPixelArgs& args, hipStream_t stream, hipEvent_t between = nullptr);
int fit_pixels_arap_blocks(int E);
// once per frame: the pixel launch's workgroup -> tile table. Tiles with a valid reference pixel (the only ones the data
// term can use) fill the front of each XCD's band in raster order, the others its end: the workgroups dispatched last --
// the fifth per CU -- get the tiles with nothing to sum. flags: [tiles] scratch; order: [tile_order_blocks(tiles)]
int tile_order_blocks(int tiles);
bool fit_pixels_tile_order_supported();   // false in NNRT_PIX_WAVES != 4 builds: the launch then ignores the table
nnrt_status launch_tile_order(const float4* ref_points, int H, int W, int tiles_x, int tiles_y, int* flags, int* order, hipStream_t stream);
nnrt_status launch_solve_update(int mode, const SolveArgs& args, hipStream_t stream, bool from_identity = false);


constexpr int CORNER_NB = 64;   // Schur-corner tile size (tile columns are padded to a multiple with identity)
inline int corner_ld(int m) { return (m + CORNER_NB - 1) / CORNER_NB * CORNER_NB; }

// ---- Schur corner: tile-sparse supernodal Cholesky (corner.hip) ----
struct CornerTask {   // one workgroup of a factor launch
	int I, J;           // tile (I, J), I >= J
	int slot_t, slot_d; // slots of tile (I, J) and of the diagonal tile (J, J) (-1 for trailing tasks)
	int src, nd, np;    // update terms in `srcs`: nd for the diagonal tile (trailing: the tile's), then np for the panel tile
	int nreal;          // panel tasks: real (non-padding) rows of column J, a prefix of its 64; the elimination stops there
};
struct CornerMap {      // device view: permuted (row, column) -> stored entry
	int T;
	const int* tile_slot;   // [T, T]
	const int* node_row;    // [nc] first permuted unknown of each corner node
	float* tiles;           // [slots, 64, 64]
	float* sdiag;           // [ld] diagonal of S before the factorization (the refinement gate's reference; nullable)
};
// stored position of corner entry (R, C), R >= C (permuted unknowns)
__device__ inline float* corner_entry(const CornerMap& m, int R, int C) {
	const int slot = m.tile_slot[static_cast<int64_t>(R / CORNER_NB) * m.T + C / CORNER_NB];
	return m.tiles + static_cast<int64_t>(slot) * (CORNER_NB * CORNER_NB) + (R % CORNER_NB) * CORNER_NB + (C % CORNER_NB);
}
// entry (r, c) of the 6 x 6 corner block of nodes (a, b), a >= b, at its lower-triangle position (S is symmetric: an
// entry above the diagonal is its transpose partner's); nullptr for the upper half of a diagonal block (a == b), which the
// block's lower half already carries
__device__ inline float* corner_block_entry(const CornerMap& m, int a, int b, int r, int c) {
	const int R = m.node_row[a] + r, C = m.node_row[b] + c;
	if (R >= C) return corner_entry(m, R, C);
	return a == b ? nullptr : corner_entry(m, C, R);
}
// corner init (corner.hip): every stored tile gets its entries of C (the corner nodes' diagonal blocks) and the identity
// on the padding; cb = b_C in the permuted order. Thread idx < threads(): 4 consecutive entries of a tile row (one 16-B
// store) and, for idx < ld, one entry of cb. Exposed so the arrowhead launch can run it beside the stem (arap.hip).
struct CornerInitArgs {
	int n0, ld, slots;
	const int2* slot_ij;
	const int* row_node;
	float* tiles;
	float* cb;
	float* sdiag;              // [ld] diag(C) (the Schur update lowers it to diag(S)); nullable
	unsigned* pivot_word;      // reset to +inf: the factorization's minimum pivot / diag(S) ratio; nullable
	int64_t threads() const { return std::max<int64_t>(static_cast<int64_t>(slots) * (CORNER_NB * CORNER_NB / 4), ld); }
};
__device__ inline void corner_init_thread(int64_t idx, const CornerInitArgs& a, const float* __restrict__ diag, const float* __restrict__ rhs) {
	constexpr int TL = CORNER_NB, TE = CORNER_NB * CORNER_NB;
	if (idx < a.ld) {
		const int rn = a.row_node[idx];
		a.cb[idx] = rn >= 0 ? rhs[6 * static_cast<int64_t>(a.n0 + (rn >> 3)) + (rn & 7)] : 0.f;
		if (a.sdiag) a.sdiag[idx] = rn >= 0 ? diag[static_cast<int64_t>(a.n0 + (rn >> 3)) * 36 + 7 * (rn & 7)] : 1.f;
		if (idx == 0 && a.pivot_word) {   // the gate word, then the refinement safeguard's words (REFINE_GUARD_*)
			a.pivot_word[0] = 0x7f800000u;
			a.pivot_word[1] = 0u;
			a.pivot_word[2] = 0u;
			a.pivot_word[3] = 0u;
		}
	}
	if (idx >= static_cast<int64_t>(a.slots) * (TE / 4)) return;
	const int s = static_cast<int>(idx / (TE / 4)), w = static_cast<int>(idx % (TE / 4));
	const int r = w / (TL / 4), c0 = (w % (TL / 4)) * 4;
	const int2 ij = a.slot_ij[s];
	const int R = ij.x * TL + r;
	const int rn = a.row_node[R];
	float v[4];
#pragma unroll
	for (int j = 0; j < 4; j++) {
		const int C = ij.y * TL + c0 + j;
		const int cn = a.row_node[C];
		v[j] = 0.f;
		if (rn >= 0 && cn >= 0) {
			if ((rn >> 3) == (cn >> 3)) v[j] = diag[static_cast<int64_t>(a.n0 + (rn >> 3)) * 36 + 6 * (rn & 7) + (cn & 7)];
		} else if (R == C) {
			v[j] = 1.f;
		}
	}
	*reinterpret_cast<float4*>(a.tiles + static_cast<int64_t>(s) * TE + r * TL + c0) = make_float4(v[0], v[1], v[2], v[3]);
}

struct WalkElem;   // corner.hip: one tile of a single-workgroup substitution walk

// the stem side of a dataflow substitution launch (CornerSolver::launch_flow; arap.hip fills it)
struct FlowStem {
	int n0 = 0, N = 0, n_update = 0, mode = 0;   // mode: 0 plain, 1 the solve's pass of a gated refinement (the refinement follows)
	const float *dinv = nullptr, *wing = nullptr, *diag = nullptr, *dinv_b = nullptr;
	const int *edge_offsets = nullptr, *edge_list = nullptr, *inc_off = nullptr, *inc_list = nullptr;
	const int32_t* edges = nullptr;
	const float* rhs = nullptr;   // b
	float* x = nullptr;           // [6N] the solve's x (its corner rows: the corner substitution's output); x + d after a refinement
	float* dx = nullptr;          // [6N] the refinement's correction d (mode 1)
	const float* state_in = nullptr;
	float* node_state = nullptr;
	float* updates_out = nullptr;
	float* res = nullptr;         // [6N] mode 1: the stem residual (the refinement's right-hand side)
	const unsigned* gate = nullptr;
	unsigned* guard = nullptr;    // the refinement safeguard's words (the gate word's block: REFINE_GUARD_*)
	float ratio = 0.f;
	int* error_flag = nullptr;
};
__host__ __device__ inline int flow_ctl_words(int nB) { return 4 + 3 * nB; }

class CornerSolver {
public:
	~CornerSolver();
	// host, once per hierarchy (edges [E,2] host, virtual order; corner = nodes >= n0; corner_pos [N - n0, 3] host or
	// nullptr): ordering (coordinate bisection with positions, graph separators without), symbolic factorisation, launch
	// plan, device buffers. A repeated call with the same inputs keeps everything (stable pointers for graphs).
	nnrt_status prepare(const int32_t* edges, int E, int n0, int N, const float* corner_pos = nullptr);
	// S = C (+ corner off-diagonal blocks) in the stored tiles, cb = b_C (permuted); diag [N,36], rhs [6N], edges / wing device
	nnrt_status launch_init(int n0, const float* diag, const float* rhs, const int32_t* edges, const float* wing, hipStream_t s) const;
	// the two halves of launch_init, for callers that run the init threads inside a launch of their own
	CornerInitArgs init_args(int n0) const { return CornerInitArgs{n0, ld, slots, d_slot_ij, d_row_node, tiles, cb, sdiag, pivot_word}; }
	nnrt_status launch_offdiag(int n0, const int32_t* edges, const float* wing, hipStream_t s) const;   // >= 3 layers
	// factor S (after the stem's Schur update), solve S x = cb; x -> xout[6 nc] in corner-node order
	nnrt_status launch_solve(float* xout, int* error_flag, hipStream_t s) const;
	// iterative refinement: solve S d = rhs2 with the factor of the last launch_solve (rhs2 = refine_rhs(), permuted,
	// written by the caller); d -> xout[6 nc] in corner-node order
	// gate (nullable, device): skip unless the factorization's minimum pivot / diag(S) ratio is below refine_ratio
	nnrt_status launch_resolve(float* xout, hipStream_t s, const unsigned* gate = nullptr, float refine_ratio = 0.f) const;
	nnrt_status launch_back(const float* y, float* xout, hipStream_t s, const unsigned* gate, float refine_ratio) const;
	// dataflow substitution (k_corner_flow), one launch: the back substitution of the last launch_factor + the stem pass
	// (st.x + 6 n0 receives the corner's solution) and, with st.mode 1, the gated refinement step after them
	nnrt_status launch_flow(const FlowStem& st, hipStream_t s) const;
	// factor S and form the diagonal inverses (the first half of launch_solve; the flow launches do the rest)
	nnrt_status launch_factor(int* error_flag, hipStream_t s) const;
	bool flow_ok() const { return use_flow; }
	float* refine_rhs() const { return cb2; }
	// the factorization's minimum pivot / diag(S) ratio of the last solve (device word, float bits)
	const unsigned* pivot_ratio() const { return pivot_word; }
	unsigned* refine_guard() const { return pivot_word; }   // [REFINE_WORDS]: the gate word, then the safeguard's
	CornerMap map() const;
	float* rhs_perm() const { return cb; }
	int levels() const { return H; }
	int tile_columns() const { return T; }
	int back_launches() const { return walk_ok ? 1 : back_off.empty() ? 0 : static_cast<int>(back_off.size()) - 1; }
	int64_t stored_tiles() const { return fill_tiles; }
	int64_t dense_lower_tiles() const { return dense_tiles; }
	// executed factorization work: MFMA flops (update terms + rank-32 products), update terms, eliminated columns
	int64_t mfma_flops() const { return exec_mfma_flops; }
	int64_t update_terms() const { return n_terms; }
	int64_t eliminated_columns() const { return elim_cols; }
	uint64_t generation = 0;    // bumped whenever the plan (and its buffers) change

private:
	void release();
	std::vector<int32_t> key;
	int nc = 0, ld = 0, T = 0, H = 0, slots = 0, n_corner_edges = 0;
	int64_t fill_tiles = 0, dense_tiles = 0, exec_mfma_flops = 0, n_terms = 0, elim_cols = 0;
	float *tiles = nullptr, *ldiag = nullptr, *minv = nullptr, *cb = nullptr, *cb2 = nullptr, *xp = nullptr, *sdiag = nullptr;
	float* xp2 = nullptr;   // the refinement's back substitution in a dataflow launch (its own lines: no L1 copy of xp's)
	float* zx = nullptr;   // [ld] substitution pre-sums (NNRT_SUBST_PRESUM)
	int2 *d_back_pre = nullptr, *d_fwd_pre = nullptr;
	std::vector<int> back_pre_off, fwd_pre_off;
	unsigned* pivot_word = nullptr;
	int2 *d_fwd_chains = nullptr, *d_fwd_ent = nullptr;
	int4* d_fwd_cols = nullptr;
	// single-workgroup substitution walks (corner.hip k_corner_walk), when the permuted vector and the descriptors fit in LDS
	bool walk_ok = false;
	// dataflow substitution plan (k_corner_flow): per chain (back column first, count, forward column first, parent)
	bool use_flow = false;
	int n_chains = 0, n_flow_ctl = 0;
	int4* d_flow_chains = nullptr;
	int *d_flow_need = nullptr, *d_col_chain = nullptr;
	unsigned* flow_ctl = nullptr;
	bool fold_invert = false;   // the diagonal inverses in the last factor launch (no k_corner_invert launch)
	int n_inv_cols = 0;         // tile columns inverted by that launch's extra workgroups
	int* d_inv_cols = nullptr;
	int walk_ring = 0, walk_lds = 0, n_walk_back = 0, n_walk_fwd = 0;
	WalkElem* d_walk_back = nullptr;
	WalkElem* d_walk_fwd = nullptr;
	int *d_tile_slot = nullptr, *d_row_node = nullptr, *d_node_row = nullptr, *d_corner_edges = nullptr;
	int2 *d_slot_ij = nullptr, *d_back_ent = nullptr, *d_back_chains = nullptr;
	CornerTask* d_tasks = nullptr;
	int4 *d_srcs = nullptr, *d_back_cols = nullptr;
	std::vector<int> level_off, level_panel, back_off, fwd_off;
};

// one step of iterative refinement after the fitter's arrowhead solve; 0: the float solve alone.
// It runs only when the corner factorization's smallest pivot / diag(S) ratio (the cancellation a float32 Cholesky loses
// digits to) falls below NNRT_REFINE_PIVOT_RATIO; otherwise its launches return at once.
// Substitution pre-sums: before each chain launch of the corner's forward / back substitution, a launch of one workgroup
// per column sums the column's entries whose vector segments come from earlier launches (in parallel over CUs); the
// chains then walk only the entries inside themselves. 0 (default): the chains sum every entry -- at C5 the extra
// launches cost more than the parallel pre-sums save (solve stage 322 vs 342 µs, round 4).
#ifndef NNRT_SUBST_PRESUM
#define NNRT_SUBST_PRESUM 0
#endif
#ifndef NNRT_ARAP_REFINE
#define NNRT_ARAP_REFINE 1
#endif
// upper end of the refinement window. Round 4 put it at 1e-3 (the plain float32 solve within 3.3e-5 of fp64 at every
// ratio >= 1.7e-3 on the C1_ARAP / C2_ARAP / C5 trajectories); against the exact float system (round 6) the plain solve
// missed 1e-4 at ratios 0.0054 (4-layer S1, fp64 pivot ratio 1.0e-7: 1.09e-4) and 0.0011 (the DeepDeform frame pair:
// 8.2e-5, its rotations 2.6e-4 of max |R - I|), so the window now reaches 1e-2. The bench states sit at 0.18 - 0.28
// (C1_ARAP, C5): shut, free; a refinement step costs a second substitution (C5: solve stage 210 -> 351 us)
#ifndef NNRT_REFINE_PIVOT_RATIO
#define NNRT_REFINE_PIVOT_RATIO 1e-2f
#endif
// below this ratio one refinement step with the float32 factors is not relied on: measured against the fp64 solution of
// exactly the float system the fitter solved (nnrt_fitter_get_arrowhead_system; round 6), one step reaches 2e-8 .. 2e-6
// at ratios 1.2e-5 .. 7.7e-5 (C2_ARAP iteration 5, C5 iterations 3-4) and 1.7e-5 at 1.3e-5 (C5 iteration 5), but 3e-3 ..
// 4e-3 at ratios near 1e-6 (degenerate systems, fp64 pivot ratio < 1e-13); such a solve is left as the float
// factorization gives it, as the reference's is. (Rounds 4-5 held the floor at 1e-4, judged against a re-assembled
// system whose own rounding moved the fp64 solution by up to 2.6e-4.)
#ifndef NNRT_REFINE_PIVOT_FLOOR
#define NNRT_REFINE_PIVOT_FLOOR 1e-5f
#endif
// The refinement's safeguard (round 6): one step x + d with float32 factors converges only while the factorization's
// error operator contracts; on degenerate systems (fp64 pivot ratio ~1e-12, after A7 NaN rotations) it was measured to
// move the solution AWAY from the exact one (C2_ARAP trajectory iteration 7: 0.0068 -> 0.089). Since the plain solve's
// relative error is ~ the contraction factor and the correction d ~ that error, the step is accepted only when
// max |d| <= NNRT_REFINE_ACCEPT * max |x| (d finite); otherwise the plain solve stands, as the reference's would.
#ifndef NNRT_REFINE_ACCEPT
#define NNRT_REFINE_ACCEPT 1e-2f
#endif
// the four words at the corner's pivot_word: the gate (min pivot / diag(S), reset to +inf by the corner init), max |d|,
// max |x| (float bits: non-negative floats order as their bits; reset to 0), the correction workgroups done (flow)
constexpr int REFINE_GUARD_D = 1, REFINE_GUARD_X = 2, REFINE_GUARD_COUNT = 3, REFINE_WORDS = 4;
__host__ __device__ inline bool refine_accept(float dmax, float xmax) { return dmax <= NNRT_REFINE_ACCEPT * xmax; }
__host__ __device__ inline bool refine_window(float r, float ratio) { return r < ratio && r >= NNRT_REFINE_PIVOT_FLOOR; }
__device__ inline bool refine_gate_on(const unsigned* gate, float ratio) {
	return gate && refine_window(__uint_as_float(*gate), ratio);
}

struct ArrowheadWorkspace {
	int N = 0, n0 = 0, E = 0, m = 0;
	const CornerSolver* corner = nullptr;   // Schur corner (m = 6 (N - n0) > 0)
	float* diag = nullptr;      // [N,36] full diagonal blocks (with LM)
	float* dinv = nullptr;      // [n0,36]
	float* dinv_b = nullptr;    // [E,36]
	float* rhs = nullptr;       // [6N] negative gradient
	float* x = nullptr;         // [6N]
	// iterative refinement (refine: one step after the first solve): res [6N] = rhs - H x (fp64 sums, rounded), dx [6N]
	// the correction; the update is x + dx
	bool refine = false;
	float refine_ratio = NNRT_REFINE_PIVOT_RATIO;   // gate threshold on the corner's min pivot / diag(S)
	float* res = nullptr;
	float* dx = nullptr;
	int* edge_offsets = nullptr;// [n0+1] CSR of stem edges by source node (edges grouped by source)
	int* edge_list = nullptr;   // [E]
	int* inc_off = nullptr;     // [N+1] CSR of edge incidences by node (fitter only: k_arrow_prepare)
	int* inc_list = nullptr;    // [2E] 2 e + (node is the edge's target), ascending e per node
	// Schur update S -= B^T D^-1 B grouped by target block (lower block triangle), and b_C -= B^T D^-1 b_D by corner
	// node: each target is written by one owner, no atomics (build_stem_schur_lists)
	int targets = 0;
	int* tgt_off = nullptr;     // [targets+1] CSR into `pairs`
	int2* tgt_ab = nullptr;     // [targets] (a, b) corner node coordinates, a >= b
	int2* pairs = nullptr;      // (e1, e2): stem edges i->a, i->b of one stem node i
	int* rhs_off = nullptr;     // [N - n0 + 1] CSR into `rhs_edges` by corner node
	int* rhs_edges = nullptr;   // stem edges into each corner node
};
struct StemSchurLists {
	std::vector<int> tgt_off, rhs_off, rhs_edges;
	std::vector<int2> tgt_ab, pairs;
};
// host: group the stem's edge pairs by Schur target block (edges [E,2] host, virtual order; stem = first n0 nodes)
StemSchurLists build_stem_schur_lists(const int32_t* edges, int E, int n0, int N);
// acc -> diagonal blocks (+lm) + rhs ; arrowhead solve ; update node state
nnrt_status launch_arrowhead_iteration(const ArrowheadWorkspace& ws, const double* acc, float lm, const int32_t* edges, const float* wing,
                                       float* node_state, const float* edge_jr, float* updates_out, float* gradient_out, float* hessian_out,
                                       int* error_flag, hipStream_t stream, const float* state_in = nullptr);
// arap_wings: the wing blocks have the ARAP structure dEi^T [0 | b I] (zero outside their last three columns);
// node_state / updates_out (fitter): apply the solved increments to the node motion in the back-substitution launch;
// state_in (default: node_state): the motion the iteration started from (a snapshot the iteration restarts from)
nnrt_status arrowhead_solve_core(const ArrowheadWorkspace& ws, const int32_t* edges, const float* wing, int* error_flag, hipStream_t stream,
                                 bool arap_wings = false, float* node_state = nullptr, float* updates_out = nullptr, const float* state_in = nullptr);

} // namespace nnrt
