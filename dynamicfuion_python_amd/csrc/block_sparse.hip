// Block-sparse linear-algebra stages of the arrowhead solve as standalone API entry points (nnrt.core.linalg):
// the reference's SolveBlockSparseArrowheadCholesky (SolveBlockSparseArrowheadCholesky.cpp:30-95) and its dense stem
// Schur complement (SchurComplement.cpp:43-78) are composed of these operations, which the fitter's arrowhead path runs
// fused (k_stem_schur / k_stem_rhs / k_arrow_back in arap.hip). Here each one is its own kernel with the reference's
// argument meaning, so the reference's own KATs (test_linalg_matmul_block_sparse.cpp, test_linalg_block_routines.cpp)
// can pin them.
//
// Float order: every block product entry is a serial sum over the inner index in ascending order (no FMA contraction,
// -ffp-contract=off), and products of several block pairs are summed in ascending inner-block order -- the oracle's
// restatement (oracle/nnrt_oracle.cpp, orc_matmul_block_sparse*) does the same, so the two agree bit for bit. The
// reference leaves both orders to cuBLAS / its atomic block sums. BlockSparseAndVectorProduct keeps the reference's
// atomic row sums (MatmulBlockSparseImpl.h:569-570), so it agrees with the oracle to rounding only.
//
// Coordinates that fall outside the matrix or vector are rejected with an error (the reference does not check them and
// reads or writes out of bounds).
#include "common.hpp"
#include "kernels.hpp"

namespace nnrt {

namespace {

constexpr int kThreads = 256;

// MatmulBlockSparseImpl.h:94-142: c_i = a[row(b_i)] b_i; rows without an A block give a zero block, mask 0
__global__ __launch_bounds__(kThreads) void k_matmul_row_wise(const float* __restrict__ a, int a_count, const float* __restrict__ b,
                                                              const int32_t* __restrict__ b_coords, int64_t count, int s,
                                                              float* __restrict__ c, uint8_t* __restrict__ mask, int* error_flag) {
	const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	const int64_t ss = static_cast<int64_t>(s) * s;
	if (t >= count * ss) return;
	const int64_t blk = t / ss;
	const int e = static_cast<int>(t - blk * ss), r = e / s, col = e % s;
	const int row = b_coords[2 * blk];
	if (row < 0) atomicOr(error_flag, 1);
	float acc = 0.f;
	if (row >= 0 && row < a_count) {
		const float* ab = a + row * ss + static_cast<int64_t>(r) * s;
		const float* bb = b + blk * ss + col;
		for (int l = 0; l < s; l++) acc += ab[l] * bb[static_cast<int64_t>(l) * s];
	}
	c[t] = acc;
	if (e == 0) mask[blk] = row >= 0 && row < a_count;
}

// MatmulBlockSparseImpl.h:160-391: output block (i, j) = sum over inner k of op(A)(i, k) op(B)(k, j) over the block pairs
// both breadboards hold (-1 = empty); mask 1 where at least one pair exists. Output blocks are dense [out_rows * out_cols]
// in row-major block order, the reference's meshgrid order before its mask selection.
template <bool TA, bool TB>
__global__ __launch_bounds__(kThreads) void k_matmul_generic(const float* __restrict__ a, int a_count, const int16_t* __restrict__ a_board,
                                                             int a_cols, const float* __restrict__ b, int b_count,
                                                             const int16_t* __restrict__ b_board, int b_cols, int out_cols,
                                                             int inner, int64_t out_blocks, int s, float* __restrict__ c,
                                                             uint8_t* __restrict__ mask, int* error_flag) {
	const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	const int64_t ss = static_cast<int64_t>(s) * s;
	if (t >= out_blocks * ss) return;
	const int64_t ob = t / ss;
	const int e = static_cast<int>(t - ob * ss), r = e / s, col = e % s;
	const int oi = static_cast<int>(ob / out_cols), oj = static_cast<int>(ob % out_cols);
	float acc = 0.f;
	bool any = false;
	for (int k = 0; k < inner; k++) {
		const int ia = TA ? a_board[static_cast<int64_t>(k) * a_cols + oi] : a_board[static_cast<int64_t>(oi) * a_cols + k];
		if (ia == -1) continue;
		const int ib = TB ? b_board[static_cast<int64_t>(oj) * b_cols + k] : b_board[static_cast<int64_t>(k) * b_cols + oj];
		if (ib == -1) continue;
		if (ia < 0 || ia >= a_count || ib < 0 || ib >= b_count) {
			atomicOr(error_flag, 1);
			continue;
		}
		const float* ab = a + ia * ss;
		const float* bb = b + ib * ss;
		float p = 0.f;
		for (int l = 0; l < s; l++) {
			const float av = TA ? ab[static_cast<int64_t>(l) * s + r] : ab[static_cast<int64_t>(r) * s + l];
			const float bv = TB ? bb[static_cast<int64_t>(col) * s + l] : bb[static_cast<int64_t>(l) * s + col];
			p += av * bv;
		}
		acc = any ? acc + p : p;
		any = true;
	}
	c[t] = acc;
	if (e == 0) mask[ob] = any;
}

// MatmulBlockSparseImpl.h:441-582: out[row(i)] += op(A_i) v[column(i)], atomic row sums as in ComputeBlockSums
template <bool TA>
__global__ __launch_bounds__(kThreads) void k_block_vector(const float* __restrict__ blocks, const int32_t* __restrict__ coords, int64_t count,
                                                           int s, int row_off, int col_off, const float* __restrict__ v, int64_t n_v,
                                                           float* __restrict__ out, int64_t m, int* error_flag) {
	const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (t >= count * s) return;
	const int64_t blk = t / s;
	const int r = static_cast<int>(t - blk * s);
	const int64_t brow = static_cast<int64_t>(TA ? coords[2 * blk + 1] + col_off : coords[2 * blk] + row_off);
	const int64_t bcol = static_cast<int64_t>(TA ? coords[2 * blk] + row_off : coords[2 * blk + 1] + col_off);
	if (brow < 0 || (brow + 1) * s > m || bcol < 0 || (bcol + 1) * s > n_v) {
		atomicOr(error_flag, 1);
		return;
	}
	const int64_t ss = static_cast<int64_t>(s) * s;
	const float* bb = blocks + blk * ss;
	const float* vv = v + bcol * s;
	float p = 0.f;
	for (int l = 0; l < s; l++) p += (TA ? bb[static_cast<int64_t>(l) * s + r] : bb[static_cast<int64_t>(r) * s + l]) * vv[l];
	atomicAdd(out + brow * s + r, p);
}

// MatmulBlockSparseImpl.h:604-690: out_i = D_i v_i
__global__ __launch_bounds__(kThreads) void k_diag_block_vector(const float* __restrict__ blocks, int64_t count, int s, const float* __restrict__ v,
                                                                float* __restrict__ out) {
	const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (t >= count * s) return;
	const int64_t blk = t / s;
	const int r = static_cast<int>(t - blk * s);
	const float* bb = blocks + blk * s * s + static_cast<int64_t>(r) * s;
	const float* vv = v + blk * s;
	float p = 0.f;
	for (int l = 0; l < s; l++) p += bb[l] * vv[l];
	out[t] = p;
}

// SparseBlocksImpl.h:30-190 (Fill / Add / SubtractSparseBlocks; DiagonalBlocksImpl.h FillInDiagonalBlocks when coords is
// null): transpose places block (i, j) at (j, i) transposed, the offset added after the flip
template <int OP>
__global__ __launch_bounds__(kThreads) void k_sparse_blocks_op(float* __restrict__ matrix, int64_t rows, int64_t cols, const float* __restrict__ blocks,
                                                               const int32_t* __restrict__ coords, int64_t count, int s, int64_t row_off,
                                                               int64_t col_off, int transpose, int* error_flag) {
	const int64_t ss = static_cast<int64_t>(s) * s;
	const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (t >= count * ss) return;
	const int64_t blk = t / ss;
	const int e = static_cast<int>(t - blk * ss);
	const int64_t ci = coords ? coords[2 * blk] : blk, cj = coords ? coords[2 * blk + 1] : blk;
	const int64_t br = (transpose ? cj : ci) + row_off, bc = (transpose ? ci : cj) + col_off;
	const int64_t i = br * s + (transpose ? e % s : e / s), j = bc * s + (transpose ? e / s : e % s);
	if (br < 0 || bc < 0 || i >= rows || j >= cols) {
		atomicOr(error_flag, 1);
		return;
	}
	float* dst = matrix + i * cols + j;
	if (OP == 0) *dst = blocks[t];
	else if (OP == 1) atomicAdd(dst, blocks[t]);
	else atomicAdd(dst, -blocks[t]);
}

// SparseBlocksImpl.h:192-230 (GetSparseBlocks; GetDiagonalBlocks when coords is null)
__global__ __launch_bounds__(kThreads) void k_get_sparse_blocks(const float* __restrict__ matrix, int64_t rows, int64_t cols, int s,
                                                                const int32_t* __restrict__ coords, int64_t count, float* __restrict__ blocks,
                                                                int* error_flag) {
	const int64_t ss = static_cast<int64_t>(s) * s;
	const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (t >= count * ss) return;
	const int64_t blk = t / ss;
	const int e = static_cast<int>(t - blk * ss);
	const int64_t br = coords ? coords[2 * blk] : blk, bc = coords ? coords[2 * blk + 1] : blk;
	const int64_t i = br * s + e / s, j = bc * s + e % s;
	if (br < 0 || bc < 0 || i >= rows || j >= cols) {
		atomicOr(error_flag, 1);
		blocks[t] = NAN;
		return;
	}
	blocks[t] = matrix[i * cols + j];
}

// TransposeBlocksCUDA.cu: every block transposed in place (one thread per strictly-lower entry swaps it with its mirror)
__global__ __launch_bounds__(kThreads) void k_transpose_blocks(float* __restrict__ blocks, int64_t count, int s) {
	const int64_t ss = static_cast<int64_t>(s) * s;
	const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (t >= count * ss) return;
	const int64_t blk = t / ss;
	const int e = static_cast<int>(t - blk * ss), r = e / s, c = e % s;
	if (c >= r) return;
	float* bb = blocks + blk * ss;
	const float lo = bb[r * s + c], up = bb[c * s + r];
	bb[r * s + c] = up;
	bb[c * s + r] = lo;
}

// InvertBlocksCPU.cpp / InvertBlocksCUDA.cu (trtri per block): one thread per (block, column j) of the inverse; lower:
// forward substitution x_j = 1 / L_jj, x_i = -(sum_{k=j}^{i-1} L_ik x_k) / L_ii; upper: the mirror image upwards. The
// column is formed in the output block itself; entries off the triangle are 0. A zero diagonal raises (trtri info > 0).
__global__ __launch_bounds__(kThreads) void k_invert_triangular(const float* __restrict__ blocks, int64_t count, int s, int upper,
                                                                float* __restrict__ out, int* error_flag) {
	const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (t >= count * s) return;
	const int64_t blk = t / s;
	const int j = static_cast<int>(t - blk * s);
	const int64_t ss = static_cast<int64_t>(s) * s;
	const float* A = blocks + blk * ss;
	float* X = out + blk * ss;
	bool singular = false;
	if (!upper) {
		for (int i = 0; i < j; i++) X[i * s + j] = 0.f;
		for (int i = j; i < s; i++) {
			float acc = 0.f;
			for (int k = j; k < i; k++) acc += A[i * s + k] * X[k * s + j];
			const float d = A[i * s + i];
			singular |= d == 0.f;
			X[i * s + j] = i == j ? 1.f / d : -acc / d;
		}
	} else {
		for (int i = j + 1; i < s; i++) X[i * s + j] = 0.f;
		for (int i = j; i >= 0; i--) {
			float acc = 0.f;
			for (int k = i + 1; k <= j; k++) acc += A[i * s + k] * X[k * s + j];
			const float d = A[i * s + i];
			singular |= d == 0.f;
			X[i * s + j] = i == j ? 1.f / d : -acc / d;
		}
	}
	if (singular) atomicOr(error_flag, 1);
}

unsigned grid_for(int64_t n) { return static_cast<unsigned>(ceil_div(n, kThreads)); }

} // namespace

nnrt_status launch_matmul_block_sparse_row_wise(const float* a, int a_count, const float* b, const int32_t* b_coords, int64_t count, int s,
                                                float* c, uint8_t* mask, int* error_flag, hipStream_t stream) {
	if (count == 0) return NNRT_OK;
	k_matmul_row_wise<<<grid_for(count * s * s), kThreads, 0, stream>>>(a, a_count, b, b_coords, count, s, c, mask, error_flag);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

nnrt_status launch_matmul_block_sparse(const float* a, int a_count, const int16_t* a_board, int a_rows, int a_cols, bool ta, const float* b,
                                       int b_count, const int16_t* b_board, int b_rows, int b_cols, bool tb, int s, float* c, uint8_t* mask,
                                       int* error_flag, hipStream_t stream) {
	const int out_rows = ta ? a_cols : a_rows, out_cols = tb ? b_rows : b_cols, inner = ta ? a_rows : a_cols;
	const int64_t out_blocks = static_cast<int64_t>(out_rows) * out_cols;
	if (out_blocks == 0) return NNRT_OK;
	const unsigned g = grid_for(out_blocks * s * s);
#define NNRT_MBS(TA_, TB_)                                                                                                             \
	k_matmul_generic<TA_, TB_><<<g, kThreads, 0, stream>>>(a, a_count, a_board, a_cols, b, b_count, b_board, b_cols, out_cols, inner, \
	                                                       out_blocks, s, c, mask, error_flag)
	if (ta) {
		if (tb) NNRT_MBS(true, true);
		else NNRT_MBS(true, false);
	} else {
		if (tb) NNRT_MBS(false, true);
		else NNRT_MBS(false, false);
	}
#undef NNRT_MBS
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

nnrt_status launch_block_sparse_vector(const float* blocks, const int32_t* coords, int64_t count, int s, int row_off, int col_off, bool ta,
                                       const float* v, int64_t n_v, float* out, int64_t m, int* error_flag, hipStream_t stream) {
	if (m > 0) NNRT_HIP(hipMemsetAsync(out, 0, sizeof(float) * m, stream));
	if (count == 0) return NNRT_OK;
	if (ta) k_block_vector<true><<<grid_for(count * s), kThreads, 0, stream>>>(blocks, coords, count, s, row_off, col_off, v, n_v, out, m, error_flag);
	else k_block_vector<false><<<grid_for(count * s), kThreads, 0, stream>>>(blocks, coords, count, s, row_off, col_off, v, n_v, out, m, error_flag);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

nnrt_status launch_diagonal_block_vector(const float* blocks, int64_t count, int s, const float* v, float* out, hipStream_t stream) {
	if (count == 0) return NNRT_OK;
	k_diag_block_vector<<<grid_for(count * s), kThreads, 0, stream>>>(blocks, count, s, v, out);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

nnrt_status launch_sparse_blocks_op(float* matrix, int64_t rows, int64_t cols, const float* blocks, const int32_t* coords, int64_t count, int s,
                                    int64_t row_off, int64_t col_off, bool transpose, int op, int* error_flag, hipStream_t stream) {
	if (count == 0) return NNRT_OK;
	const unsigned g = grid_for(count * s * s);
	if (op == 0) k_sparse_blocks_op<0><<<g, kThreads, 0, stream>>>(matrix, rows, cols, blocks, coords, count, s, row_off, col_off, transpose, error_flag);
	else if (op == 1) k_sparse_blocks_op<1><<<g, kThreads, 0, stream>>>(matrix, rows, cols, blocks, coords, count, s, row_off, col_off, transpose, error_flag);
	else k_sparse_blocks_op<2><<<g, kThreads, 0, stream>>>(matrix, rows, cols, blocks, coords, count, s, row_off, col_off, transpose, error_flag);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

nnrt_status launch_get_sparse_blocks(const float* matrix, int64_t rows, int64_t cols, int s, const int32_t* coords, int64_t count, float* blocks,
                                     int* error_flag, hipStream_t stream) {
	if (count == 0) return NNRT_OK;
	k_get_sparse_blocks<<<grid_for(count * s * s), kThreads, 0, stream>>>(matrix, rows, cols, s, coords, count, blocks, error_flag);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

nnrt_status launch_transpose_blocks(float* blocks, int64_t count, int s, hipStream_t stream) {
	if (count == 0) return NNRT_OK;
	k_transpose_blocks<<<grid_for(count * s * s), kThreads, 0, stream>>>(blocks, count, s);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

nnrt_status launch_invert_triangular_blocks(const float* blocks, int64_t count, int s, bool upper, float* out, int* error_flag,
                                            hipStream_t stream) {
	if (count == 0) return NNRT_OK;
	k_invert_triangular<<<grid_for(count * s), kThreads, 0, stream>>>(blocks, count, s, upper ? 1 : 0, out, error_flag);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

} // namespace nnrt
