// TSDF voxel block grid on gfx950: the canonical-mesh source and sink either side of the fitter in a DynamicFusion loop
// (SURVEY.md 8(f) row 2). Reference: nnrt.geometry.NonRigidSurfaceVoxelBlockGrid (cpp/geometry/NonRigidSurfaceVoxelBlockGrid.cpp,
// cpp/geometry/kernel/NonRigidSurfaceVoxelBlockGridImpl.h) over NNRT's VoxelBlockGrid (cpp/geometry/VoxelBlockGrid.cpp), whose
// hash map, depth touch, rigid integration and mesh extraction are Open3D 0.17 kernels (third-party, not in the
// reference tree; restated from Open3D's published t::geometry::kernel::voxel_grid algorithms).
//
// Layout in HBM (one grid):
//   block keys   int32 [capacity, 3]; buffer index = activation order (dense: blocks are never erased)
//   hash table   open addressing, linear probing: uint64 packed key [T] + int32 buffer index [T], T = pow2 >= 2 capacity
//   voxels       tsdf f32 [capacity, res^3], weight (f32 | u16) [capacity, res^3], color (f32 | u16 | u8) [capacity, res^3, 3];
//                voxel (x, y, z) of a block at x + res (y + res z) (Open3D ArrayIndexer order)
// Activation is deterministic: every key takes the lowest input index that carries it (atomicMin), new keys get buffer
// indices by a prefix sum in input order -- so block order, and everything derived from it, is reproducible.
#include <hipcub/hipcub.hpp>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstring>
#include <memory>
#include <type_traits>
#include <vector>

#include "kernels.hpp"
#include "mc_table.hpp"

namespace nnrt {
namespace {

constexpr uint64_t HASH_EMPTY = ~0ull;
constexpr int KEY_BIAS = 1 << 20;   // block coordinates in [-2^20, 2^20)
constexpr int TSDF_MAX_ANCHORS = 8;

enum StoreType : int { ST_NONE = 0, ST_F32 = 1, ST_U16 = 2, ST_U8 = 3 };

__host__ __device__ inline bool key_in_range(int x, int y, int z) {
	return x >= -KEY_BIAS && x < KEY_BIAS && y >= -KEY_BIAS && y < KEY_BIAS && z >= -KEY_BIAS && z < KEY_BIAS;
}
__host__ __device__ inline uint64_t pack_key(int x, int y, int z) {
	return static_cast<uint64_t>(static_cast<uint32_t>(x + KEY_BIAS)) | (static_cast<uint64_t>(static_cast<uint32_t>(y + KEY_BIAS)) << 21) |
	       (static_cast<uint64_t>(static_cast<uint32_t>(z + KEY_BIAS)) << 42);
}
__device__ inline uint64_t hash_mix(uint64_t k) {
	k ^= k >> 33;
	k *= 0xff51afd7ed558ccdull;
	k ^= k >> 33;
	k *= 0xc4ceb9fe1a85ec53ull;
	k ^= k >> 33;
	return k;
}

struct HashView {
	uint64_t* keys;
	int* block;     // buffer index per slot (-1: none yet)
	int* first;     // scratch: lowest input index per slot during one activation / dedupe
	uint64_t mask;
};

// the slot holding `key`, inserting it if absent (never fails: the table is kept at most half full)
__device__ inline uint64_t hash_insert(const HashView& h, uint64_t key) {
	uint64_t s = hash_mix(key) & h.mask;
	while (true) {
		const uint64_t prev = atomicCAS(reinterpret_cast<unsigned long long*>(h.keys + s), HASH_EMPTY, key);
		if (prev == HASH_EMPTY || prev == key) return s;
		s = (s + 1) & h.mask;
	}
}
__device__ inline int hash_find(const HashView& h, uint64_t key) {
	uint64_t s = hash_mix(key) & h.mask;
	while (true) {
		const uint64_t k = h.keys[s];
		if (k == key) return h.block[s];
		if (k == HASH_EMPTY) return -1;
		s = (s + 1) & h.mask;
	}
}
__device__ inline int find_block(const HashView& h, int x, int y, int z) {
	return key_in_range(x, y, z) ? hash_find(h, pack_key(x, y, z)) : -1;
}

// Open3D TransformIndexer (float rows of the 3x4 extrinsic, float intrinsics)
struct Xform {
	float m[12];
	float fx, fy, cx, cy;
	__device__ __host__ void rigid(float x, float y, float z, float& ox, float& oy, float& oz) const {
		ox = ((x * m[0] + y * m[1]) + z * m[2]) + m[3];
		oy = ((x * m[4] + y * m[5]) + z * m[6]) + m[7];
		oz = ((x * m[8] + y * m[9]) + z * m[10]) + m[11];
	}
	__device__ __host__ void project(float x, float y, float z, float& u, float& v) const {
		const float inv_z = 1.0f / z;
		u = (fx * x) * inv_z + cx;
		v = (fy * y) * inv_z + cy;
	}
	__device__ __host__ void unproject(float u, float v, float d, float& x, float& y, float& z) const {
		x = ((u - cx) * d) / fx;
		y = ((v - cy) * d) / fy;
		z = d;
	}
};
Xform make_xform(const double* K, const double* E) {
	Xform t{};
	for (int r = 0; r < 3; r++)
		for (int c = 0; c < 4; c++) t.m[4 * r + c] = E ? static_cast<float>(E[4 * r + c]) : (r == c ? 1.f : 0.f);
	if (K) {
		t.fx = static_cast<float>(K[0]);
		t.fy = static_cast<float>(K[4]);
		t.cx = static_cast<float>(K[2]);
		t.cy = static_cast<float>(K[5]);
	} else {
		t.fx = t.fy = 1.f;
		t.cx = t.cy = 0.f;
	}
	return t;
}
// inverse of a 4x4 (double, Gauss-Jordan with partial pivoting; Open3D inverts the extrinsic in double on the host)
bool invert4(const double* a, double* out) {
	double m[4][8];
	for (int r = 0; r < 4; r++)
		for (int c = 0; c < 8; c++) m[r][c] = c < 4 ? a[4 * r + c] : (c - 4 == r ? 1.0 : 0.0);
	for (int c = 0; c < 4; c++) {
		int p = c;
		for (int r = c + 1; r < 4; r++)
			if (std::fabs(m[r][c]) > std::fabs(m[p][c])) p = r;
		if (m[p][c] == 0.0) return false;
		if (p != c)
			for (int k = 0; k < 8; k++) std::swap(m[p][k], m[c][k]);
		const double d = m[c][c];
		for (int k = 0; k < 8; k++) m[c][k] /= d;
		for (int r = 0; r < 4; r++)
			if (r != c) {
				const double f = m[r][c];
				for (int k = 0; k < 8; k++) m[r][k] -= f * m[c][k];
			}
	}
	for (int r = 0; r < 4; r++)
		for (int c = 0; c < 4; c++) out[4 * r + c] = m[r][c + 4];
	return true;
}

// Open3D ArrayIndexer::InBoundary for float pixel coordinates of an H x W image
__device__ inline bool in_image(float u, float v, int H, int W) {
	return u >= 0.f && v >= 0.f && u <= static_cast<float>(W) - 1.0f && v <= static_cast<float>(H) - 1.0f;
}

template <typename T>
__device__ inline float load_f(const void* base, int64_t i) {
	return static_cast<float>(static_cast<const T*>(base)[i]);
}
// storage element read / write by runtime store type
__device__ inline float read_store(const void* base, int type, int64_t i) {
	switch (type) {
		case ST_F32: return static_cast<const float*>(base)[i];
		case ST_U16: return static_cast<float>(static_cast<const uint16_t*>(base)[i]);
		case ST_U8: return static_cast<float>(static_cast<const uint8_t*>(base)[i]);
		default: return 0.f;
	}
}
// C++ float -> integer conversion truncates toward zero (as the reference's typed stores)
__device__ inline void write_store(void* base, int type, int64_t i, float v) {
	switch (type) {
		case ST_F32: static_cast<float*>(base)[i] = v; break;
		case ST_U16: static_cast<uint16_t*>(base)[i] = static_cast<uint16_t>(static_cast<uint32_t>(v)); break;
		case ST_U8: static_cast<uint8_t*>(base)[i] = static_cast<uint8_t>(static_cast<uint32_t>(v)); break;
		default: break;
	}
}

struct GridView {
	float voxel_size;
	int res, res3;
	const int32_t* keys;   // [cap,3]
	float* tsdf;
	void* weight;
	int weight_type;
	void* color;
	int color_type;
	HashView hash;
};

struct ImageView {
	const void* depth;
	int depth_type;   // ST_F32 | ST_U16
	int H, W;
	const void* color;   // [Hc, Wc, 3]: f32 when depth is f32, else u8 (Open3D input_color_t)
	int Hc, Wc;
	float depth_scale, depth_max;
};

__device__ inline float read_depth(const ImageView& im, int u, int v) {
	const int64_t i = static_cast<int64_t>(v) * im.W + u;
	return im.depth_type == ST_U16 ? static_cast<float>(static_cast<const uint16_t*>(im.depth)[i]) : static_cast<const float*>(im.depth)[i];
}
__device__ inline float read_color(const ImageView& im, int u, int v, int c) {
	const int64_t i = (static_cast<int64_t>(v) * im.Wc + u) * 3 + c;
	return im.depth_type == ST_U16 ? static_cast<float>(static_cast<const uint8_t*>(im.color)[i]) : static_cast<const float*>(im.color)[i];
}

__device__ inline void voxel_local(int idx, int res, int& x, int& y, int& z) {
	x = idx % res;
	y = (idx / res) % res;
	z = idx / (res * res);
}

// ---------------------------------------------------------------------------------------------------------------------
// hash activation / dedupe
// ---------------------------------------------------------------------------------------------------------------------
__global__ void k_insert_min(HashView h, const int32_t* __restrict__ coords, const uint64_t* __restrict__ packed, int64_t n,
                             uint64_t* __restrict__ in_slot, int* error_flag) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= n) return;
	uint64_t key;
	if (coords) {
		const int x = coords[3 * i], y = coords[3 * i + 1], z = coords[3 * i + 2];
		if (!key_in_range(x, y, z)) {
			atomicOr(error_flag, 1);
			in_slot[i] = HASH_EMPTY;
			return;
		}
		key = pack_key(x, y, z);
	} else {
		key = packed[i];
		if (key == HASH_EMPTY) {
			in_slot[i] = HASH_EMPTY;
			return;
		}
	}
	const uint64_t s = hash_insert(h, key);
	atomicMin(h.first + s, static_cast<int>(i));
	in_slot[i] = s;
}

// new[i] = input i is the first carrier of a key not yet holding a block
__global__ void k_mark_new(HashView h, const uint64_t* __restrict__ in_slot, int64_t n, int* __restrict__ is_new) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= n) return;
	const uint64_t s = in_slot[i];
	is_new[i] = (s != HASH_EMPTY && h.first[s] == static_cast<int>(i) && h.block[s] < 0) ? 1 : 0;
}

__global__ void k_assign_blocks(HashView h, const uint64_t* __restrict__ in_slot, const int* __restrict__ is_new, const int* __restrict__ rank,
                                int64_t n, int64_t base, int32_t* __restrict__ keys_out) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= n || !is_new[i]) return;
	const uint64_t s = in_slot[i];
	const int64_t b = base + rank[i];
	h.block[s] = static_cast<int>(b);
	const uint64_t k = h.keys[s];
	keys_out[3 * b] = static_cast<int32_t>(k & 0x1fffff) - KEY_BIAS;
	keys_out[3 * b + 1] = static_cast<int32_t>((k >> 21) & 0x1fffff) - KEY_BIAS;
	keys_out[3 * b + 2] = static_cast<int32_t>((k >> 42) & 0x1fffff) - KEY_BIAS;
}

__global__ void k_fill_i32(int* p, int64_t n, int v) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i < n) p[i] = v;
}
__global__ void k_fill_u64(uint64_t* p, int64_t n, uint64_t v) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i < n) p[i] = v;
}
// rehash: every existing block key back into a fresh table
__global__ void k_rehash(HashView h, const int32_t* __restrict__ keys, int64_t n) {
	const int64_t b = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (b >= n) return;
	const uint64_t s = hash_insert(h, pack_key(keys[3 * b], keys[3 * b + 1], keys[3 * b + 2]));
	h.block[s] = static_cast<int>(b);
}
// buffer index of each coordinate (-1: inactive)
__global__ void k_find_blocks(HashView h, const int32_t* __restrict__ coords, int64_t n, int* __restrict__ out) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= n) return;
	out[i] = find_block(h, coords[3 * i], coords[3 * i + 1], coords[3 * i + 2]);
}

// ---------------------------------------------------------------------------------------------------------------------
// Open3D DepthTouch (GetUniqueBlockCoordinates, VoxelBlockGrid.cpp:237-270, down factor 4): every 4th pixel (both axes)
// with 0 < d < depth_max samples 4 points t_min + i (t_max - t_min) / 3 along its camera ray (t in [max(d - trunc, 0),
// min(d + trunc, depth_max)]) and touches the blocks that contain them. Keys are written at fixed positions
// (pixel-major, then sample) and deduplicated in that order.
// ---------------------------------------------------------------------------------------------------------------------
constexpr int TOUCH_STEPS = 3;
__global__ void k_touch_depth(ImageView im, int stride, Xform cam_to_world, float sdf_trunc, float block_size, uint64_t* __restrict__ out) {
	const int rows = im.H / stride, cols = im.W / stride;
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= static_cast<int64_t>(rows) * cols) return;
	const int y = static_cast<int>(i / cols) * stride, x = static_cast<int>(i % cols) * stride;
	const float d = read_depth(im, x, y) / im.depth_scale;
	uint64_t* o = out + (TOUCH_STEPS + 1) * i;
	if (!(d > 0.f && d < im.depth_max)) {
		for (int s = 0; s <= TOUCH_STEPS; s++) o[s] = HASH_EMPTY;
		return;
	}
	float xc, yc, zc, xg, yg, zg;
	cam_to_world.unproject(static_cast<float>(x), static_cast<float>(y), 1.0f, xc, yc, zc);
	cam_to_world.rigid(xc, yc, zc, xg, yg, zg);
	const float xo = cam_to_world.m[3], yo = cam_to_world.m[7], zo = cam_to_world.m[11];
	const float xd = xg - xo, yd = yg - yo, zd = zg - zo;
	const float t_min = fmaxf(d - sdf_trunc, 0.0f);
	const float t_max = fminf(d + sdf_trunc, im.depth_max);
	const float t_step = (t_max - t_min) / static_cast<float>(TOUCH_STEPS);
	float t = t_min;
	for (int s = 0; s <= TOUCH_STEPS; s++) {
		const int xb = static_cast<int>(floorf((xo + t * xd) / block_size));
		const int yb = static_cast<int>(floorf((yo + t * yd) / block_size));
		const int zb = static_cast<int>(floorf((zo + t * zd) / block_size));
		o[s] = key_in_range(xb, yb, zb) ? pack_key(xb, yb, zb) : HASH_EMPTY;
		t += t_step;
	}
}

__global__ void k_unique_compact(HashView h, const uint64_t* __restrict__ packed, const uint64_t* __restrict__ in_slot, const int* __restrict__ first,
                                 const int* __restrict__ rank, int64_t n, int32_t* __restrict__ out) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= n || !first[i]) return;
	const uint64_t k = packed[i];
	const int64_t r = rank[i];
	out[3 * r] = static_cast<int32_t>(k & 0x1fffff) - KEY_BIAS;
	out[3 * r + 1] = static_cast<int32_t>((k >> 21) & 0x1fffff) - KEY_BIAS;
	out[3 * r + 2] = static_cast<int32_t>((k >> 42) & 0x1fffff) - KEY_BIAS;
	(void) h;
	(void) in_slot;
}
__global__ void k_mark_first(HashView h, const uint64_t* __restrict__ in_slot, int64_t n, int* __restrict__ first) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= n) return;
	const uint64_t s = in_slot[i];
	first[i] = (s != HASH_EMPTY && h.first[s] == static_cast<int>(i)) ? 1 : 0;
}

// ---------------------------------------------------------------------------------------------------------------------
// Open3D Integrate (VoxelBlockGrid.cpp:317-350 -> voxel_grid::Integrate): one lane per voxel of the listed blocks.
// ---------------------------------------------------------------------------------------------------------------------
__global__ void k_integrate_rigid(GridView g, const int* __restrict__ blocks, int64_t nb, ImageView im, Xform depth_x, Xform color_x,
                                  float sdf_trunc, float color_multiplier) {
	const int64_t w = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (w >= nb * g.res3) return;
	const int b = blocks[w / g.res3];
	if (b < 0) return;
	const int vi = static_cast<int>(w % g.res3);
	int xv, yv, zv;
	voxel_local(vi, g.res, xv, yv, zv);
	const float x = static_cast<float>(g.keys[3 * b] * g.res + xv) * g.voxel_size;
	const float y = static_cast<float>(g.keys[3 * b + 1] * g.res + yv) * g.voxel_size;
	const float z = static_cast<float>(g.keys[3 * b + 2] * g.res + zv) * g.voxel_size;
	float xc, yc, zc, u, v;
	depth_x.rigid(x, y, z, xc, yc, zc);
	depth_x.project(xc, yc, zc, u, v);
	if (!in_image(u, v, im.H, im.W)) return;
	int ui = static_cast<int>(roundf(u)), vi2 = static_cast<int>(roundf(v));
	const float depth = read_depth(im, ui, vi2) / im.depth_scale;
	float sdf = depth - zc;
	if (depth <= 0.0f || depth > im.depth_max || zc <= 0.0f || sdf < -sdf_trunc) return;
	sdf = sdf < sdf_trunc ? sdf : sdf_trunc;
	sdf /= sdf_trunc;
	const int64_t lin = static_cast<int64_t>(b) * g.res3 + vi;
	const float weight = read_store(g.weight, g.weight_type, lin);
	const float inv_wsum = 1.0f / (weight + 1);
	g.tsdf[lin] = (weight * g.tsdf[lin] + sdf) * inv_wsum;
	if (g.color && im.color) {
		float xu, yu, zu, uc, vc;
		depth_x.unproject(static_cast<float>(ui), static_cast<float>(vi2), 1.0f, xu, yu, zu);
		color_x.project(xu, yu, zu, uc, vc);
		if (in_image(uc, vc, im.Hc, im.Wc)) {
			ui = static_cast<int>(roundf(uc));
			vi2 = static_cast<int>(roundf(vc));
			for (int c = 0; c < 3; c++) {
				const float old = read_store(g.color, g.color_type, 3 * lin + c);
				write_store(g.color, g.color_type, 3 * lin + c, (weight * old + read_color(im, ui, vi2, c) * color_multiplier) * inv_wsum);
			}
		}
	}
	write_store(g.weight, g.weight_type, lin, weight + 1);
}

// ---------------------------------------------------------------------------------------------------------------------
// Anchors of a point with the node-distance threshold (WarpUtilities.h:131-153, :319-341; KnnUtilities.h:146-220): the
// K nearest nodes by Euclidean norm with replace-the-current-maximum insertion, squared norms above 4 c^2 dropped (-1),
// Gaussian weights exp(-d^2 / 2c^2) normalized over the valid ones. Only nodes within 2 c (the largest coverage for
// variable coverage) can be valid, so the search runs over those candidates in ascending node order; the valid set
// equals the reference KD-tree's (its slot order, and thus the blend's float summation order, may differ).
// Nodes farther than that range never enter the search (per voxel), so the slot order is a function of the in-range
// nodes alone. Returns the valid count; weights are normalized only when valid >= minimum (the reference returns false otherwise
// and, where the return value is ignored, blends the unnormalized weights).
// ---------------------------------------------------------------------------------------------------------------------
template <int KT>
struct Anchors {
	int idx[KT];
	float w[KT];
	int valid;
	bool ok;
	__device__ void reset() {
#pragma unroll
		for (int k = 0; k < KT; k++) {
			idx[k] = -1;
			w[k] = INFINITY;
		}
	}
};

// replace-the-maximum insertion with static register indices (the slot to overwrite is selected, not indexed)
template <int KT>
__device__ inline void knn_insert(Anchors<KT>& a, float d, int node, float& maxd, int& max_at) {
	if (maxd > d) {
#pragma unroll
		for (int k = 0; k < KT; k++)
			if (k == max_at) {
				a.w[k] = d;   // distances held in the weight slots (WarpUtilities.h:325)
				a.idx[k] = node;
			}
		max_at = 0;
		maxd = a.w[0];
#pragma unroll
		for (int k = 1; k < KT; k++)
			if (a.w[k] > maxd) {
				max_at = k;
				maxd = a.w[k];
			}
	}
}
template <int KT>
__device__ inline void anchors_finish(Anchors<KT>& a, const WarpFieldView& wf) {
	const float c2_fixed = wf.coverage * wf.coverage;
	float sum = 0.f;
	a.valid = 0;
#pragma unroll
	for (int k = 0; k < KT; k++) {
		if (a.idx[k] < 0) continue;
		float sq = a.w[k];
		sq = sq * sq;
		const float c2 = wf.fixed_coverage ? c2_fixed : wf.node_weights[a.idx[k]];
		if (sq > 4 * c2) {
			a.idx[k] = -1;
			continue;
		}
		const float wt = exp_cr(-sq / (2 * c2));
		sum += wt;
		a.w[k] = wt;
		a.valid++;
	}
	a.ok = a.valid >= wf.minimum_valid;
	if (a.ok) {   // NormalizeAnchorWeights (WarpUtilities.h:36-46)
		if (sum > 0.0f) {
#pragma unroll
			for (int k = 0; k < KT; k++) a.w[k] /= sum;
		} else if (a.valid > 0) {
#pragma unroll
			for (int k = 0; k < KT; k++) a.w[k] = 1.0f / static_cast<float>(a.valid);
		}
	}
}
// BlendWarp (WarpUtilities.h:429-445): sum_k w_k (g_k + R_k (p - g_k) + t_k) over valid anchors
template <int KT>
__device__ inline void blend_warp(const Anchors<KT>& a, const WarpFieldView& wf, float px, float py, float pz, float& ox, float& oy, float& oz) {
	ox = oy = oz = 0.f;
#pragma unroll
	for (int k = 0; k < KT; k++) {
		const int n = a.idx[k];
		if (n < 0) continue;
		const float* s = wf.state + static_cast<int64_t>(n) * NODE_STRIDE;
		const float gx = s[0], gy = s[1], gz = s[2];
		const float dx = px - gx, dy = py - gy, dz = pz - gz;
		const float rx = (s[6] * dx + s[7] * dy) + s[8] * dz;
		const float ry = (s[9] * dx + s[10] * dy) + s[11] * dz;
		const float rz = (s[12] * dx + s[13] * dy) + s[14] * dz;
		const float w = a.w[k];
		ox += w * ((gx + rx) + s[3]);
		oy += w * ((gy + ry) + s[4]);
		oz += w * ((gz + rz) + s[5]);
	}
}
__device__ inline float node_dist(const float* s, float px, float py, float pz) {
	const float dx = s[0] - px, dy = s[1] - py, dz = s[2] - pz;
	return sqrtf((dx * dx + dy * dy) + dz * dz);
}

// ---------------------------------------------------------------------------------------------------------------------
// IntegrateNonRigid (NonRigidSurfaceVoxelBlockGridImpl.h:52-229): one workgroup per active block. The block's nodes
// within anchor range (2 c of its camera-space bounding box) are compacted into LDS in ascending node order; each
// voxel searches only those. Reproduced as written: the weight is read but never incremented, oblique views
// (cos(view, normal) > 0.5) and psdf <= -trunc are skipped, the cosine map is written before those tests.
// ---------------------------------------------------------------------------------------------------------------------
constexpr int NR_BLOCK = 256;
constexpr int NR_CAND = 2048;
template <int KT>
__global__ __launch_bounds__(NR_BLOCK) void k_integrate_non_rigid(GridView g, int64_t nb, WarpFieldView wf, ImageView im, const float* __restrict__ normals,
                                                                  Xform depth_x, Xform color_x, float sdf_trunc, float color_multiplier,
                                                                  float range, uint64_t* __restrict__ cos_key) {
	__shared__ int s_cand[NR_CAND];
	__shared__ int s_count;
	__shared__ int s_wave_counts[NR_BLOCK / 64];
	const int b = blockIdx.x;
	if (b >= nb) return;
	const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
	// camera-space bounding box of the block (its 8 corners, as voxel centres span [0, res - 1])
	float bmin[3] = {INFINITY, INFINITY, INFINITY}, bmax[3] = {-INFINITY, -INFINITY, -INFINITY};
	for (int c = 0; c < 8; c++) {
		const float x = static_cast<float>(g.keys[3 * b] * g.res + ((c & 1) ? g.res - 1 : 0)) * g.voxel_size;
		const float y = static_cast<float>(g.keys[3 * b + 1] * g.res + ((c & 2) ? g.res - 1 : 0)) * g.voxel_size;
		const float z = static_cast<float>(g.keys[3 * b + 2] * g.res + ((c & 4) ? g.res - 1 : 0)) * g.voxel_size;
		float o[3];
		depth_x.rigid(x, y, z, o[0], o[1], o[2]);
		for (int k = 0; k < 3; k++) {
			bmin[k] = fminf(bmin[k], o[k]);
			bmax[k] = fmaxf(bmax[k], o[k]);
		}
	}
	if (t == 0) s_count = 0;
	__syncthreads();
	bool overflow = false;
	for (int base = 0; base < wf.N; base += NR_BLOCK) {   // ordered compaction of the candidates
		const int n = base + t;
		bool near = false;
		if (n < wf.N) {
			const float* s = wf.state + static_cast<int64_t>(n) * NODE_STRIDE;
			float d2 = 0.f;
			for (int k = 0; k < 3; k++) {
				const float e = fmaxf(fmaxf(bmin[k] - s[k], s[k] - bmax[k]), 0.f);
				d2 += e * e;
			}
			near = d2 <= range * range * 1.0001f + 1e-12f;
		}
		const uint64_t m = __ballot(near);
		if (lane == 0) s_wave_counts[wave] = __popcll(m);
		__syncthreads();
		int before = s_count;
		for (int w = 0; w < wave; w++) before += s_wave_counts[w];
		const int pos = before + __popcll(m & ((1ull << lane) - 1ull));
		if (near && pos < NR_CAND) s_cand[pos] = n;
		__syncthreads();
		if (t == 0) {
			int tot = s_count;
			for (int w = 0; w < NR_BLOCK / 64; w++) tot += s_wave_counts[w];
			s_count = tot;
		}
		__syncthreads();
	}
	const int ncand = s_count;
	overflow = ncand > NR_CAND;
	for (int vi = t; vi < g.res3; vi += NR_BLOCK) {
		int xv, yv, zv;
		voxel_local(vi, g.res, xv, yv, zv);
		const float x = static_cast<float>(g.keys[3 * b] * g.res + xv) * g.voxel_size;
		const float y = static_cast<float>(g.keys[3 * b + 1] * g.res + yv) * g.voxel_size;
		const float z = static_cast<float>(g.keys[3 * b + 2] * g.res + zv) * g.voxel_size;
		float xc, yc, zc;
		depth_x.rigid(x, y, z, xc, yc, zc);
		Anchors<KT> a;
		a.reset();
		float maxd = INFINITY;
		int max_at = 0;
		if (!overflow) {
			for (int q = 0; q < ncand; q++) {
				const int n = s_cand[q];
				const float d = node_dist(wf.state + static_cast<int64_t>(n) * NODE_STRIDE, xc, yc, zc);
				if (d <= range) knn_insert<KT>(a, d, n, maxd, max_at);
			}
		} else {
			for (int n = 0; n < wf.N; n++) {
				const float d = node_dist(wf.state + static_cast<int64_t>(n) * NODE_STRIDE, xc, yc, zc);
				if (d <= range) knn_insert<KT>(a, d, n, maxd, max_at);
			}
		}
		anchors_finish<KT>(a, wf);
		if (!a.ok) continue;
		float wx, wy, wz;
		blend_warp<KT>(a, wf, xc, yc, zc, wx, wy, wz);
		if (wz < 0) continue;
		float u, v;
		depth_x.project(wx, wy, wz, u, v);
		if (!in_image(u, v, im.H, im.W)) continue;
		int ui = static_cast<int>(roundf(u)), vr = static_cast<int>(roundf(v));
		const float depth = read_depth(im, ui, vr) / im.depth_scale;
		if (depth <= 0.0f || depth > im.depth_max) continue;
		const float psdf = depth - wz;
		float vx = -wx, vy = -wy, vz = -wz;   // view direction, Eigen normalize()
		const float vn2 = (vx * vx + vy * vy) + vz * vz;
		if (vn2 > 0.f) {
			const float vn = sqrtf(vn2);
			vx /= vn;
			vy /= vn;
			vz /= vn;
		}
		const int64_t pix = static_cast<int64_t>(vr) * im.W + ui;
		const float cosine = (vx * normals[3 * pix] + vy * normals[3 * pix + 1]) + vz * normals[3 * pix + 2];
		const int64_t lin = static_cast<int64_t>(b) * g.res3 + vi;
		// the reference's plain store races between voxels that project to one pixel; here the voxel with the highest
		// linear index wins (the serial loop's last writer)
		atomicMax(reinterpret_cast<unsigned long long*>(cos_key + pix),
		          (static_cast<unsigned long long>(lin + 1) << 32) | __builtin_bit_cast(uint32_t, cosine));
		if (psdf <= -sdf_trunc || cosine > 0.5f) continue;
		const float tsdf_n = (psdf < sdf_trunc ? psdf : sdf_trunc) / sdf_trunc;
		const float weight = read_store(g.weight, g.weight_type, lin);
		const float inv_wsum = 1.0f / (weight + 1);
		g.tsdf[lin] = (weight * g.tsdf[lin] + tsdf_n) * inv_wsum;
		if (g.color && im.color) {
			float xu, yu, zu, uc, vc;
			depth_x.unproject(static_cast<float>(ui), static_cast<float>(vr), 1.0f, xu, yu, zu);
			color_x.project(xu, yu, zu, uc, vc);
			if (in_image(uc, vc, im.Hc, im.Wc)) {
				ui = static_cast<int>(roundf(uc));
				vr = static_cast<int>(roundf(vc));
				for (int c = 0; c < 3; c++) {
					const float old = read_store(g.color, g.color_type, 3 * lin + c);
					write_store(g.color, g.color_type, 3 * lin + c, (weight * old + read_color(im, ui, vr, c) * color_multiplier) * inv_wsum);
				}
			}
		}
	}
}

__global__ void k_cos_resolve(const uint64_t* __restrict__ key, int64_t n, float* __restrict__ cos_out) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= n) return;
	const uint64_t k = key[i];
	cos_out[i] = k ? __builtin_bit_cast(float, static_cast<uint32_t>(k & 0xffffffffu)) : 0.f;
}

// ---------------------------------------------------------------------------------------------------------------------
// ExtractVoxelValuesAndCoordinates / ExtractVoxelValuesAt (NonRigidSurfaceVoxelBlockGridImpl.h:446-652)
// rows: x, y, z (metres), tsdf, weight, (r, g, b)
// ---------------------------------------------------------------------------------------------------------------------
__global__ void k_values_all(GridView g, int64_t nb, int C, float* __restrict__ out) {
	const int64_t w = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (w >= nb * g.res3) return;
	const int b = static_cast<int>(w / g.res3), vi = static_cast<int>(w % g.res3);
	int xv, yv, zv;
	voxel_local(vi, g.res, xv, yv, zv);
	float* o = out + w * C;
	o[0] = static_cast<float>(g.keys[3 * b] * g.res + xv) * g.voxel_size;
	o[1] = static_cast<float>(g.keys[3 * b + 1] * g.res + yv) * g.voxel_size;
	o[2] = static_cast<float>(g.keys[3 * b + 2] * g.res + zv) * g.voxel_size;
	const int64_t lin = static_cast<int64_t>(b) * g.res3 + vi;
	o[3] = g.tsdf[lin];
	o[4] = read_store(g.weight, g.weight_type, lin);
	if (C > 5)
		for (int c = 0; c < 3; c++) o[5 + c] = read_store(g.color, g.color_type, 3 * lin + c);
}

// The reference indexes the voxel inside its block with the GLOBAL coordinate (CoordToWorkload of x, y, z, :619-620),
// which is the local index only for block (0, 0, 0); reproduced, rows whose index leaves the voxel storage keep -2.
// Query blocks are x / res with C++ integer division (toward zero), as the tensor division at :239.
__global__ void k_values_at(GridView g, int64_t capacity, const int32_t* __restrict__ q, int64_t n, int C, float* __restrict__ out) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= n) return;
	float* o = out + i * C;
	for (int c = 0; c < C; c++) o[c] = -2.f;
	const int x = q[3 * i], y = q[3 * i + 1], z = q[3 * i + 2];
	const int b = find_block(g.hash, x / g.res, y / g.res, z / g.res);
	if (b < 0) return;
	const int64_t vib = static_cast<int64_t>(x) + static_cast<int64_t>(g.res) * (y + static_cast<int64_t>(g.res) * z);
	const int64_t lin = static_cast<int64_t>(b) * g.res3 + vib;
	if (lin < 0 || lin >= capacity * g.res3) return;
	o[0] = static_cast<float>(x) * g.voxel_size;
	o[1] = static_cast<float>(y) * g.voxel_size;
	o[2] = static_cast<float>(z) * g.voxel_size;
	o[3] = g.tsdf[lin];
	o[4] = read_store(g.weight, g.weight_type, lin);
	if (C > 5)
		for (int c = 0; c < 3; c++) o[5 + c] = read_store(g.color, g.color_type, 3 * lin + c);
}
// rows of found queries only (the reference drops queries whose block is inactive, :241-243)
__global__ void k_found_mask(GridView g, const int32_t* __restrict__ q, int64_t n, int* __restrict__ found) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= n) return;
	found[i] = find_block(g.hash, q[3 * i] / g.res, q[3 * i + 1] / g.res, q[3 * i + 2] / g.res) >= 0 ? 1 : 0;
}
__global__ void k_compact_rows(const float* __restrict__ rows, const int* __restrict__ found, const int* __restrict__ rank, int64_t n, int C,
                               float* __restrict__ out) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= n || !found[i]) return;
	for (int c = 0; c < C; c++) out[rank[i] * C + c] = rows[i * C + c];
}

// ---------------------------------------------------------------------------------------------------------------------
// GetBoundingBoxesOfWarpedBlocks (NonRigidSurfaceVoxelBlockGridImpl.h:289-356), reproduced as written: the block corner
// is the integer block key itself plus the block side length (metric only when the side is 1), the anchors' return
// value is ignored, and the min / max updates are an if / else-if pair.
// ---------------------------------------------------------------------------------------------------------------------
// One lane per (block, corner): 8 consecutive lanes hold one block's corners (the corner order of the reference's
// block_corners array); node positions are staged in LDS and only nodes within 2 c of the corner enter the K-NN
// (nodes farther away are never valid anchors; the oracle applies the same rule). Lane 0 of each octet then folds the
// 8 warped corners in order with the reference's if / else-if min-max.
constexpr int BOX_BLOCK = 256;
constexpr int BOX_LDS_NODES = 4096;
template <int KT>
__global__ __launch_bounds__(BOX_BLOCK) void k_warped_block_boxes(const int32_t* __restrict__ keys, int64_t n, float side, WarpFieldView wf,
                                                                  Xform ex, float range, float* __restrict__ boxes) {
	__shared__ float s_nodes[BOX_LDS_NODES * 3];
	const bool staged = wf.N <= BOX_LDS_NODES;
	if (staged)
		for (int i = threadIdx.x; i < wf.N; i += BOX_BLOCK)
			for (int k = 0; k < 3; k++) s_nodes[3 * i + k] = wf.state[static_cast<int64_t>(i) * NODE_STRIDE + k];
	__syncthreads();
	const int64_t gid = static_cast<int64_t>(blockIdx.x) * BOX_BLOCK + threadIdx.x;
	const int64_t i = gid >> 3;
	const int c = static_cast<int>(gid & 7);
	float w[3] = {0.f, 0.f, 0.f};
	if (i < n) {
		const float x0 = static_cast<float>(keys[3 * i]), y0 = static_cast<float>(keys[3 * i + 1]), z0 = static_cast<float>(keys[3 * i + 2]);
		const float x1 = x0 + side, y1 = y0 + side, z1 = z0 + side;
		// block_corners order (:322-331): 000, 001, 010, 100, 011, 101, 110, 111 (bit pattern x y z)
		const int pat[8] = {0, 1, 2, 4, 3, 5, 6, 7};
		const int m = pat[c];
		float p[3];
		ex.rigid((m & 4) ? x1 : x0, (m & 2) ? y1 : y0, (m & 1) ? z1 : z0, p[0], p[1], p[2]);
		Anchors<KT> a;
		a.reset();
		float maxd = INFINITY;
		int max_at = 0;
		for (int nn = 0; nn < wf.N; nn++) {
			const float* q = staged ? s_nodes + 3 * nn : wf.state + static_cast<int64_t>(nn) * NODE_STRIDE;
			const float dx = q[0] - p[0], dy = q[1] - p[1], dz = q[2] - p[2];
			const float d = sqrtf((dx * dx + dy * dy) + dz * dz);
			if (d <= range) knn_insert<KT>(a, d, nn, maxd, max_at);
		}
		WarpFieldView fixed = wf;
		fixed.fixed_coverage = 1;   // ComputeAnchorsForPoint<.., true, true>: fixed node coverage
		anchors_finish<KT>(a, fixed);
		blend_warp<KT>(a, wf, p[0], p[1], p[2], w[0], w[1], w[2]);
	}
	float all[8][3];
#pragma unroll
	for (int q = 0; q < 8; q++)
#pragma unroll
		for (int k = 0; k < 3; k++) all[q][k] = __shfl(w[k], (threadIdx.x & ~7) + q);
	if (i < n && c == 0) {
		float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
		for (int q = 0; q < 8; q++)
			for (int k = 0; k < 3; k++) {
				if (mn[k] > all[q][k]) mn[k] = all[q][k];
				else if (mx[k] < all[q][k]) mx[k] = all[q][k];
			}
		for (int k = 0; k < 3; k++) {
			boxes[6 * i + k] = mn[k];
			boxes[6 * i + 3 + k] = mx[k];
		}
	}
}

// GetAxisAlignedBoxesInterceptingSurfaceMask (:359-437): a segment [d - trunc, d + trunc] along the ray of every
// stride-th pixel, slab test (Segment.h IntersectsAxisAlignedBox) against every box. Segments at fixed positions
// (invalid pixels: none), one lane per box walking them.
struct Seg {
	float o[3], inv[3];
	int sign[3];
	int valid;
};
__global__ void k_make_segments(ImageView im, int stride, Xform K, float trunc, Seg* __restrict__ segs) {
	const int rows = im.H / stride, cols = im.W / stride;
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= static_cast<int64_t>(rows) * cols) return;
	const int v = static_cast<int>(i / cols) * stride, u = static_cast<int>(i % cols) * stride;
	const float d = read_depth(im, u, v) / im.depth_scale;
	Seg s{};
	s.valid = d > 0 && d < im.depth_max;
	if (s.valid) {
		float a[3], e[3];
		K.unproject(static_cast<float>(u), static_cast<float>(v), d - trunc, a[0], a[1], a[2]);
		K.unproject(static_cast<float>(u), static_cast<float>(v), d + trunc, e[0], e[1], e[2]);
		for (int k = 0; k < 3; k++) {
			s.o[k] = a[k];
			s.inv[k] = 1.f / (e[k] - a[k]);
			s.sign[k] = s.inv[k] < 0;
		}
	}
	segs[i] = s;
}
__device__ inline bool seg_hits_box(const Seg& s, const float* bmin, const float* bmax) {
	const float* bounds[2] = {bmin, bmax};
	float t_min = (bounds[s.sign[0]][0] - s.o[0]) * s.inv[0];
	float t_max = (bounds[1 - s.sign[0]][0] - s.o[0]) * s.inv[0];
	const float ty_min = (bounds[s.sign[1]][1] - s.o[1]) * s.inv[1];
	const float ty_max = (bounds[1 - s.sign[1]][1] - s.o[1]) * s.inv[1];
	if ((t_min > ty_max) || (ty_min > t_max)) return false;
	if (ty_min > t_min) t_min = ty_min;
	if (ty_max < t_max) t_max = ty_max;
	const float tz_min = (bounds[s.sign[2]][2] - s.o[2]) * s.inv[2];
	const float tz_max = (bounds[1 - s.sign[2]][2] - s.o[2]) * s.inv[2];
	if ((t_min > tz_max) || (tz_min > t_max)) return false;
	if (tz_min > t_min) t_min = tz_min;
	if (tz_max < t_max) t_max = tz_max;
	return !(t_max < 0.0f || t_min > 1.0f);
}
__global__ void k_boxes_mask(const float* __restrict__ boxes, int64_t nbox, const Seg* __restrict__ segs, int64_t nseg, uint8_t* __restrict__ mask) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= nbox) return;
	const float* bmin = boxes + 6 * i;
	const float* bmax = bmin + 3;
	uint8_t hit = 0;
	for (int64_t s = 0; s < nseg && !hit; s++)
		if (segs[s].valid && seg_hits_box(segs[s], bmin, bmax)) hit = 1;
	mask[i] = hit;
}

// BufferCoordinatesOfInactiveNeighborBlocks (NonRigidSurfaceVoxelBlockGrid.cpp:68-96): the 27 neighbours of every
// active block, neighbour-major ([27][count]), kept when inactive (duplicates kept, as the reference)
__global__ void k_inactive_neighbors(GridView g, int64_t nb, int32_t* __restrict__ coords, int* __restrict__ inactive) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= 27 * nb) return;
	const int nbr = static_cast<int>(i / nb);
	const int64_t b = i % nb;
	const int dz = nbr / 9, dy = (nbr % 9) / 3, dx = nbr % 3;
	const int x = g.keys[3 * b] + dx - 1, y = g.keys[3 * b + 1] + dy - 1, z = g.keys[3 * b + 2] + dz - 1;
	coords[3 * i] = x;
	coords[3 * i + 1] = y;
	coords[3 * i + 2] = z;
	inactive[i] = key_in_range(x, y, z) && find_block(g.hash, x, y, z) < 0 ? 1 : 0;
}
__global__ void k_compact_coords(const int32_t* __restrict__ coords, const int* __restrict__ keep, const int* __restrict__ rank, int64_t n,
                                 int32_t* __restrict__ out) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= n || !keep[i]) return;
	for (int c = 0; c < 3; c++) out[3 * rank[i] + c] = coords[3 * i + c];
}
__global__ void k_and_mask(int* __restrict__ keep, const uint8_t* __restrict__ m, int64_t n) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i < n) keep[i] = m[i] ? 1 : 0;
}

// ---------------------------------------------------------------------------------------------------------------------
// Marching cubes (the Open3D ExtractTriangleMesh algorithm, VoxelBlockGrid.cpp:461-497 -> voxel_grid::ExtractTriangleMesh,
// restated): corner i of the cube at voxel v is v + (i & 1, (i >> 1) & 1, i >> 2) in Bourke numbering (v0 (0,0,0),
// v1 (1,0,0), v2 (1,1,0), v3 (0,1,0), v4..v7 the same at z + 1); bit i of the cube index is tsdf < 0. A cube counts
// only if all 8 corners exist with weight > threshold. Every cube edge is owned by its lower voxel and axis (the
// reference's edge_shifts): a vertex lives on each owned edge of some valid surface cube, at the zero crossing of the
// linear interpolation, with the normal interpolated from central-difference tsdf gradients and the color likewise.
// The triangle table is the published one Open3D indexes (csrc/mc_table.hpp: Lorensen-Cline / Bourke), each triangle
// emitted in Open3D's vertex order (normals towards positive tsdf).
// Vertex and triangle order: blocks in buffer order, voxels in block order, owned edges x, y, z -- deterministic.
// ---------------------------------------------------------------------------------------------------------------------
constexpr int MC_MAX_TRI = 10;
struct McTables {
	uint16_t edge_mask[256];
	int8_t tri[256][3 * MC_MAX_TRI + 1];   // edge triples, -1 terminated
	int8_t ntri[256];
};
__constant__ McTables c_mc;
__constant__ int8_t c_edge_owner[12][4] = {{0, 0, 0, 0}, {1, 0, 0, 1}, {0, 1, 0, 0}, {0, 0, 0, 1}, {0, 0, 1, 0}, {1, 0, 1, 1},
                                           {0, 1, 1, 0}, {0, 0, 1, 1}, {0, 0, 0, 2}, {1, 0, 0, 2}, {1, 1, 0, 2}, {0, 1, 0, 2}};

McTables build_mc_tables() {
	static const int edge_v[12][2] = {{0, 1}, {1, 2}, {2, 3}, {3, 0}, {4, 5}, {5, 6}, {6, 7}, {7, 4}, {0, 4}, {1, 5}, {2, 6}, {3, 7}};
	McTables t{};
	for (int cfg = 0; cfg < 256; cfg++) {
		uint16_t mask = 0;
		for (int e = 0; e < 12; e++)
			if (((cfg >> edge_v[e][0]) & 1) != ((cfg >> edge_v[e][1]) & 1)) mask |= static_cast<uint16_t>(1u << e);
		t.edge_mask[cfg] = mask;
		int nt = 0;
		// (a, b, c) -> (c, b, a): Open3D's ExtractTriangleMesh stores table vertex v at triangle slot 2 - v (third-party,
		// absent here: restated from its published source; same winding as (a, c, b), parity unpinned)
		for (int i = 0; i < 16 && MC_TRI_TABLE[cfg][i] >= 0; i += 3, nt++) {
			t.tri[cfg][3 * nt] = MC_TRI_TABLE[cfg][i + 2];
			t.tri[cfg][3 * nt + 1] = MC_TRI_TABLE[cfg][i + 1];
			t.tri[cfg][3 * nt + 2] = MC_TRI_TABLE[cfg][i];
		}
		t.tri[cfg][3 * nt] = -1;
		t.ntri[cfg] = static_cast<int8_t>(nt);
	}
	return t;
}

struct MeshGridView {
	GridView g;
	const int* nbr;   // [nb, 27] buffer index of neighbour (dx, dy, dz) in {-1,0,1}^3 at (dx+1) + 3 (dy+1) + 9 (dz+1); -1: none
	float weight_threshold;
};
// the voxel at local (x, y, z) of block b, which may lie in a neighbouring block (-1: none)
__device__ inline int64_t voxel_at(const MeshGridView& m, int b, int x, int y, int z) {
	const int R = m.g.res;
	const int dx = x < 0 ? -1 : (x >= R ? 1 : 0), dy = y < 0 ? -1 : (y >= R ? 1 : 0), dz = z < 0 ? -1 : (z >= R ? 1 : 0);
	const int nb = m.nbr[27 * static_cast<int64_t>(b) + (dx + 1) + 3 * (dy + 1) + 9 * (dz + 1)];
	if (nb < 0) return -1;
	const int lx = x - dx * R, ly = y - dy * R, lz = z - dz * R;
	return static_cast<int64_t>(nb) * m.g.res3 + lx + R * (ly + R * lz);
}

__global__ void k_block_neighbors(GridView g, int64_t nb, int* __restrict__ nbr) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= 27 * nb) return;
	const int64_t b = i / 27;
	const int k = static_cast<int>(i % 27);
	nbr[i] = find_block(g.hash, g.keys[3 * b] + k % 3 - 1, g.keys[3 * b + 1] + (k / 3) % 3 - 1, g.keys[3 * b + 2] + k / 9 - 1);
}

// pass 1: cube index per voxel (0 = no surface) and its triangle count
__global__ void k_mc_cubes(MeshGridView m, int64_t nb, uint8_t* __restrict__ cube, int* __restrict__ ntri, int* __restrict__ edge_flag) {
	const int64_t w = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (w >= nb * m.g.res3) return;
	const int b = static_cast<int>(w / m.g.res3), vi = static_cast<int>(w % m.g.res3);
	int x, y, z;
	voxel_local(vi, m.g.res, x, y, z);
	int idx = 0;
	bool valid = true;
	// Bourke corner offsets
	const int off[8][3] = {{0, 0, 0}, {1, 0, 0}, {1, 1, 0}, {0, 1, 0}, {0, 0, 1}, {1, 0, 1}, {1, 1, 1}, {0, 1, 1}};
	for (int c = 0; c < 8; c++) {
		const int64_t v = voxel_at(m, b, x + off[c][0], y + off[c][1], z + off[c][2]);
		if (v < 0 || !(read_store(m.g.weight, m.g.weight_type, v) > m.weight_threshold)) {
			valid = false;
			break;
		}
		if (m.g.tsdf[v] < 0) idx |= 1 << c;
	}
	if (!valid || idx == 0 || idx == 255) {
		cube[w] = 0;
		ntri[w] = 0;
		return;
	}
	cube[w] = static_cast<uint8_t>(idx);
	ntri[w] = c_mc.ntri[idx];
	const uint16_t mask = c_mc.edge_mask[idx];
	for (int e = 0; e < 12; e++) {
		if (!(mask & (1u << e))) continue;
		const int64_t ov = voxel_at(m, b, x + c_edge_owner[e][0], y + c_edge_owner[e][1], z + c_edge_owner[e][2]);
		edge_flag[3 * ov + c_edge_owner[e][3]] = 1;   // benign race: every writer stores 1
	}
}

__device__ inline float tsdf_or(const MeshGridView& m, int b, int x, int y, int z, float fallback) {
	const int64_t v = voxel_at(m, b, x, y, z);
	return v < 0 ? fallback : m.g.tsdf[v];
}
// central-difference tsdf gradient (a missing neighbour contributes the centre value)
__device__ inline void grad_at(const MeshGridView& m, int b, int x, int y, int z, float c, float* n) {
	n[0] = tsdf_or(m, b, x + 1, y, z, c) - tsdf_or(m, b, x - 1, y, z, c);
	n[1] = tsdf_or(m, b, x, y + 1, z, c) - tsdf_or(m, b, x, y - 1, z, c);
	n[2] = tsdf_or(m, b, x, y, z + 1, c) - tsdf_or(m, b, x, y, z - 1, c);
}

// pass 2: vertices on the flagged owned edges (index = exclusive scan of the flags)
__global__ void k_mc_vertices(MeshGridView m, int64_t nb, const int* __restrict__ edge_flag, const int* __restrict__ vidx, float* __restrict__ vpos,
                              float* __restrict__ vnrm, float* __restrict__ vcol) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= 3 * nb * m.g.res3 || !edge_flag[i]) return;
	const int64_t w = i / 3;
	const int d = static_cast<int>(i % 3);
	const int b = static_cast<int>(w / m.g.res3), vi = static_cast<int>(w % m.g.res3);
	int x, y, z;
	voxel_local(vi, m.g.res, x, y, z);
	const int ex = d == 0, ey = d == 1, ez = d == 2;
	const int64_t vo = w, ve = voxel_at(m, b, x + ex, y + ey, z + ez);
	const float to = m.g.tsdf[vo], te = m.g.tsdf[ve];
	const float ratio = (0.0f - to) / (te - to);
	const int64_t o = vidx[i];
	const int R = m.g.res;
	vpos[3 * o] = (static_cast<float>(m.g.keys[3 * b] * R + x) + ratio * ex) * m.g.voxel_size;
	vpos[3 * o + 1] = (static_cast<float>(m.g.keys[3 * b + 1] * R + y) + ratio * ey) * m.g.voxel_size;
	vpos[3 * o + 2] = (static_cast<float>(m.g.keys[3 * b + 2] * R + z) + ratio * ez) * m.g.voxel_size;
	float no[3], ne[3], n[3];
	grad_at(m, b, x, y, z, to, no);
	grad_at(m, b, x + ex, y + ey, z + ez, te, ne);
	for (int k = 0; k < 3; k++) n[k] = (1 - ratio) * no[k] + ratio * ne[k];
	const float nn = sqrtf((n[0] * n[0] + n[1] * n[1]) + n[2] * n[2]);
	for (int k = 0; k < 3; k++) vnrm[3 * o + k] = nn > 0.f ? n[k] / nn : 0.f;
	if (vcol) {
		for (int k = 0; k < 3; k++) {
			const float co = read_store(m.g.color, m.g.color_type, 3 * vo + k), ce = read_store(m.g.color, m.g.color_type, 3 * ve + k);
			vcol[3 * o + k] = ((1 - ratio) * co + ratio * ce) / 255.0f;
		}
	}
}

// pass 3: triangles (offset = exclusive scan of the per-cube counts)
__global__ void k_mc_triangles(MeshGridView m, int64_t nb, const uint8_t* __restrict__ cube, const int* __restrict__ toff, const int* __restrict__ vidx,
                               int64_t* __restrict__ tris) {
	const int64_t w = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (w >= nb * m.g.res3 || cube[w] == 0) return;
	const int idx = cube[w];
	const int b = static_cast<int>(w / m.g.res3), vi = static_cast<int>(w % m.g.res3);
	int x, y, z;
	voxel_local(vi, m.g.res, x, y, z);
	int64_t o = toff[w];
	for (int t = 0; t < c_mc.ntri[idx]; t++, o++) {
		for (int k = 0; k < 3; k++) {
			const int e = c_mc.tri[idx][3 * t + k];
			const int64_t ov = voxel_at(m, b, x + c_edge_owner[e][0], y + c_edge_owner[e][1], z + c_edge_owner[e][2]);
			tris[3 * o + k] = vidx[3 * ov + c_edge_owner[e][3]];
		}
	}
}

} // namespace
} // namespace nnrt

// =====================================================================================================================
// host side: the grid handle and the C-ABI (include/nnrt_mi355x.h, "TSDF voxel block grid")
// =====================================================================================================================
namespace nnrt {
namespace {
template <typename T>
struct DevBuf {
	T* ptr = nullptr;
	size_t count = 0;
	nnrt_status ensure(size_t n) {
		if (n <= count && ptr) return NNRT_OK;
		if (ptr) hipFree(ptr);
		ptr = nullptr;
		count = 0;
		if (hipMalloc(reinterpret_cast<void**>(&ptr), sizeof(T) * std::max<size_t>(n, 1)) != hipSuccess) {
			ptr = nullptr;
			set_error("hipMalloc failed (voxel block grid)");
			return NNRT_ERROR_HIP;
		}
		count = std::max<size_t>(n, 1);
		return NNRT_OK;
	}
	void release() {
		if (ptr) hipFree(ptr);
		ptr = nullptr;
		count = 0;
	}
	~DevBuf() { release(); }
};
inline unsigned grid_of(int64_t n, int block = 256) { return static_cast<unsigned>((n + block - 1) / block); }
size_t store_bytes(int type) { return type == ST_F32 ? 4 : type == ST_U16 ? 2 : type == ST_U8 ? 1 : 0; }
} // namespace
} // namespace nnrt

using namespace nnrt;

struct nnrt_voxel_grid {
	int device = 0;
	float voxel_size = 0.f;
	int res = 8, res3 = 512;
	int64_t capacity = 0, active = 0;
	int weight_type = ST_F32, color_type = ST_NONE;
	uint64_t table_size = 0;
	DevBuf<float> tsdf;
	DevBuf<uint8_t> weight, color;
	DevBuf<int32_t> keys;
	DevBuf<uint64_t> hkeys;
	DevBuf<int> hblock, hfirst;
	// scratch
	DevBuf<uint64_t> s_slot, s_packed;
	DevBuf<int> s_flag, s_rank, s_nbr, s_ntri, s_toff, s_vidx, s_eflag, s_found, s_blocks;
	DevBuf<uint8_t> s_cube, s_mask;
	DevBuf<unsigned char> s_cub;
	DevBuf<int32_t> s_coords;
	DevBuf<float> s_boxes, s_rows_all;
	DevBuf<Seg> s_segs;
	// results awaiting a copy-out
	DevBuf<int32_t> r_coords;
	int64_t r_coord_count = 0;
	DevBuf<float> r_rows;
	int64_t r_row_count = 0;
	int r_row_channels = 0;
	DevBuf<float> r_vpos, r_vnrm, r_vcol;
	DevBuf<int64_t> r_tris;
	int64_t r_nv = 0, r_nt = 0;

	GridView view() {
		GridView g{};
		g.voxel_size = voxel_size;
		g.res = res;
		g.res3 = res3;
		g.keys = keys.ptr;
		g.tsdf = tsdf.ptr;
		g.weight = weight.ptr;
		g.weight_type = weight_type;
		g.color = color_type != ST_NONE ? color.ptr : nullptr;
		g.color_type = color_type;
		g.hash = HashView{hkeys.ptr, hblock.ptr, hfirst.ptr, table_size - 1};
		return g;
	}
	int channels() const { return color_type != ST_NONE ? 8 : 5; }
};

namespace {
struct GridGuard {
	int prev = 0;
	explicit GridGuard(int dev) {
		hipGetDevice(&prev);
		if (prev != dev) hipSetDevice(dev);
	}
	~GridGuard() { hipSetDevice(prev); }
};

// exclusive prefix sum of n ints; returns the total on the host (synchronizes the stream)
nnrt_status scan_total(nnrt_voxel_grid* vg, const int* in, int* out, int64_t n, hipStream_t s, int64_t* total) {
	*total = 0;
	if (n == 0) return NNRT_OK;
	size_t bytes = 0;
	NNRT_HIP(hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, in, out, static_cast<int>(n), s));
	nnrt_status st = vg->s_cub.ensure(bytes);
	if (st) return st;
	NNRT_HIP(hipcub::DeviceScan::ExclusiveSum(vg->s_cub.ptr, bytes, in, out, static_cast<int>(n), s));
	int last[2] = {0, 0};
	NNRT_HIP(hipMemcpyAsync(&last[0], out + n - 1, sizeof(int), hipMemcpyDeviceToHost, s));
	NNRT_HIP(hipMemcpyAsync(&last[1], in + n - 1, sizeof(int), hipMemcpyDeviceToHost, s));
	NNRT_HIP(hipStreamSynchronize(s));
	*total = static_cast<int64_t>(last[0]) + last[1];
	return NNRT_OK;
}

nnrt_status rebuild_table(nnrt_voxel_grid* vg, uint64_t size, hipStream_t s) {
	nnrt_status st;
	if ((st = vg->hkeys.ensure(size)) || (st = vg->hblock.ensure(size)) || (st = vg->hfirst.ensure(size))) return st;
	vg->table_size = size;
	k_fill_u64<<<grid_of(static_cast<int64_t>(size)), 256, 0, s>>>(vg->hkeys.ptr, static_cast<int64_t>(size), HASH_EMPTY);
	k_fill_i32<<<grid_of(static_cast<int64_t>(size)), 256, 0, s>>>(vg->hblock.ptr, static_cast<int64_t>(size), -1);
	k_fill_i32<<<grid_of(static_cast<int64_t>(size)), 256, 0, s>>>(vg->hfirst.ptr, static_cast<int64_t>(size), 0x7fffffff);
	if (vg->active > 0) k_rehash<<<grid_of(vg->active), 256, 0, s>>>(vg->view().hash, vg->keys.ptr, vg->active);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

// grow block storage to hold `need` blocks (x2 steps), keeping contents; the table is rebuilt at >= 2x capacity
nnrt_status ensure_capacity(nnrt_voxel_grid* vg, int64_t need, hipStream_t s) {
	if (need <= vg->capacity) return NNRT_OK;
	int64_t cap = std::max<int64_t>(vg->capacity, 1);
	while (cap < need) cap *= 2;
	const size_t vox_old = static_cast<size_t>(vg->capacity) * vg->res3, vox_new = static_cast<size_t>(cap) * vg->res3;
	auto grow = [&](auto& buf, size_t elem_old, size_t elem_new) -> nnrt_status {
		using T = std::remove_pointer_t<decltype(buf.ptr)>;
		T* fresh = nullptr;
		if (hipMalloc(reinterpret_cast<void**>(&fresh), sizeof(T) * std::max<size_t>(elem_new, 1)) != hipSuccess) {
			set_error("hipMalloc failed growing the voxel block grid");
			return NNRT_ERROR_HIP;
		}
		NNRT_HIP(hipMemsetAsync(fresh, 0, sizeof(T) * elem_new, s));
		if (buf.ptr && elem_old) NNRT_HIP(hipMemcpyAsync(fresh, buf.ptr, sizeof(T) * elem_old, hipMemcpyDeviceToDevice, s));
		NNRT_HIP(hipStreamSynchronize(s));
		buf.release();
		buf.ptr = fresh;
		buf.count = std::max<size_t>(elem_new, 1);
		return NNRT_OK;
	};
	nnrt_status st;
	if ((st = grow(vg->tsdf, vox_old, vox_new)) || (st = grow(vg->weight, vox_old * store_bytes(vg->weight_type), vox_new * store_bytes(vg->weight_type))) ||
	    (st = grow(vg->color, vox_old * 3 * store_bytes(vg->color_type), vox_new * 3 * store_bytes(vg->color_type))) ||
	    (st = grow(vg->keys, static_cast<size_t>(vg->capacity) * 3, static_cast<size_t>(cap) * 3)))
		return st;
	vg->capacity = cap;
	uint64_t tsize = 16;
	while (tsize < static_cast<uint64_t>(2 * cap)) tsize <<= 1;
	if (tsize != vg->table_size) return rebuild_table(vg, tsize, s);
	return NNRT_OK;
}

// Activate (Open3D HashMap::Activate): coordinates [n,3] (or packed keys, HASH_EMPTY entries skipped) -> blocks;
// `n_new` receives the number of blocks created
nnrt_status activate_keys(nnrt_voxel_grid* vg, const int32_t* coords, const uint64_t* packed, int64_t n, hipStream_t s, int64_t* n_new,
                          int* d_error) {
	*n_new = 0;
	if (n == 0) return NNRT_OK;
	nnrt_status st;
	// worst case: every input new -> keep the table at most half full before inserting
	if ((st = ensure_capacity(vg, vg->active + n, s))) return st;
	if ((st = vg->s_slot.ensure(n)) || (st = vg->s_flag.ensure(n)) || (st = vg->s_rank.ensure(n))) return st;
	const GridView g = vg->view();
	k_fill_i32<<<grid_of(static_cast<int64_t>(vg->table_size)), 256, 0, s>>>(vg->hfirst.ptr, static_cast<int64_t>(vg->table_size), 0x7fffffff);
	k_insert_min<<<grid_of(n), 256, 0, s>>>(g.hash, coords, packed, n, vg->s_slot.ptr, d_error);
	k_mark_new<<<grid_of(n), 256, 0, s>>>(g.hash, vg->s_slot.ptr, n, vg->s_flag.ptr);
	NNRT_LAUNCH_CHECK();
	int64_t total = 0;
	if ((st = scan_total(vg, vg->s_flag.ptr, vg->s_rank.ptr, n, s, &total))) return st;
	if (total > 0) {
		k_assign_blocks<<<grid_of(n), 256, 0, s>>>(g.hash, vg->s_slot.ptr, vg->s_flag.ptr, vg->s_rank.ptr, n, vg->active, vg->keys.ptr);
		NNRT_LAUNCH_CHECK();
		// new blocks start at zero (tsdf, weight, color)
		const size_t v0 = static_cast<size_t>(vg->active) * vg->res3, nv = static_cast<size_t>(total) * vg->res3;
		NNRT_HIP(hipMemsetAsync(vg->tsdf.ptr + v0, 0, sizeof(float) * nv, s));
		NNRT_HIP(hipMemsetAsync(vg->weight.ptr + v0 * store_bytes(vg->weight_type), 0, nv * store_bytes(vg->weight_type), s));
		if (vg->color_type != ST_NONE) NNRT_HIP(hipMemsetAsync(vg->color.ptr + v0 * 3 * store_bytes(vg->color_type), 0, nv * 3 * store_bytes(vg->color_type), s));
	}
	vg->active += total;
	*n_new = total;
	return NNRT_OK;
}

// unique coordinates of packed keys (HASH_EMPTY skipped), in first-occurrence order, into vg->r_coords, via a scratch
// table (the grid's own table is not touched)
nnrt_status unique_packed(nnrt_voxel_grid* vg, const uint64_t* packed, int64_t n, hipStream_t s) {
	vg->r_coord_count = 0;
	if (n == 0) return NNRT_OK;
	uint64_t tsize = 16;
	while (tsize < static_cast<uint64_t>(2 * n)) tsize <<= 1;
	DevBuf<uint64_t> tk;
	DevBuf<int> tb, tf;
	nnrt_status st;
	if ((st = tk.ensure(tsize)) || (st = tb.ensure(tsize)) || (st = tf.ensure(tsize)) || (st = vg->s_slot.ensure(n)) || (st = vg->s_flag.ensure(n)) ||
	    (st = vg->s_rank.ensure(n)))
		return st;
	k_fill_u64<<<grid_of(static_cast<int64_t>(tsize)), 256, 0, s>>>(tk.ptr, static_cast<int64_t>(tsize), HASH_EMPTY);
	k_fill_i32<<<grid_of(static_cast<int64_t>(tsize)), 256, 0, s>>>(tb.ptr, static_cast<int64_t>(tsize), -1);
	k_fill_i32<<<grid_of(static_cast<int64_t>(tsize)), 256, 0, s>>>(tf.ptr, static_cast<int64_t>(tsize), 0x7fffffff);
	const HashView h{tk.ptr, tb.ptr, tf.ptr, tsize - 1};
	k_insert_min<<<grid_of(n), 256, 0, s>>>(h, nullptr, packed, n, vg->s_slot.ptr, nullptr);
	k_mark_first<<<grid_of(n), 256, 0, s>>>(h, vg->s_slot.ptr, n, vg->s_flag.ptr);
	NNRT_LAUNCH_CHECK();
	int64_t total = 0;
	if ((st = scan_total(vg, vg->s_flag.ptr, vg->s_rank.ptr, n, s, &total))) return st;
	if ((st = vg->r_coords.ensure(3 * static_cast<size_t>(std::max<int64_t>(total, 1))))) return st;
	k_unique_compact<<<grid_of(n), 256, 0, s>>>(h, packed, vg->s_slot.ptr, vg->s_flag.ptr, vg->s_rank.ptr, n, vg->r_coords.ptr);
	NNRT_LAUNCH_CHECK();
	NNRT_HIP(hipStreamSynchronize(s));
	vg->r_coord_count = total;
	return NNRT_OK;
}

ImageView make_image(const void* depth, int depth_dtype, int H, int W, const void* color, int Hc, int Wc, float scale, float dmax) {
	ImageView im{};
	im.depth = depth;
	im.depth_type = depth_dtype == NNRT_DTYPE_UINT16 ? ST_U16 : ST_F32;
	im.H = H;
	im.W = W;
	im.color = color;
	im.Hc = Hc;
	im.Wc = Wc;
	im.depth_scale = scale;
	im.depth_max = dmax;
	return im;
}
int store_type_of(int dtype) {
	switch (dtype) {
		case NNRT_DTYPE_FLOAT32: return ST_F32;
		case NNRT_DTYPE_UINT16: return ST_U16;
		case NNRT_DTYPE_UINT8: return ST_U8;
		default: return ST_NONE;
	}
}

// check + clear the device error word used by activation (out-of-range block coordinates)
nnrt_status take_error(int* d_error, hipStream_t s) {
	int h = 0;
	NNRT_HIP(hipMemcpyAsync(&h, d_error, sizeof(int), hipMemcpyDeviceToHost, s));
	NNRT_HIP(hipStreamSynchronize(s));
	if (h) {
		set_error("block coordinate out of range (|coordinate| must stay below 2^20)");
		return NNRT_ERROR_ARGUMENT;
	}
	return NNRT_OK;
}

nnrt_status activate_coords(nnrt_voxel_grid* vg, const int32_t* d_coords, int64_t n, hipStream_t s) {
	if (n == 0) return NNRT_OK;
	DevBuf<int> err;
	nnrt_status st;
	if ((st = err.ensure(1))) return st;
	NNRT_HIP(hipMemsetAsync(err.ptr, 0, sizeof(int), s));
	int64_t created = 0;
	if ((st = activate_keys(vg, d_coords, nullptr, n, s, &created, err.ptr))) return st;
	return take_error(err.ptr, s);
}

// inactive neighbours of every active block (neighbour-major, duplicates kept) -> s_coords [27 active, 3] + keep flags
nnrt_status inactive_neighbors(nnrt_voxel_grid* vg, hipStream_t s, int64_t* n_all) {
	const int64_t n = 27 * vg->active;
	*n_all = n;
	nnrt_status st;
	if ((st = vg->s_coords.ensure(3 * static_cast<size_t>(std::max<int64_t>(n, 1)))) || (st = vg->s_found.ensure(std::max<int64_t>(n, 1))) ||
	    (st = vg->s_rank.ensure(std::max<int64_t>(n, 1))))
		return st;
	if (n > 0) k_inactive_neighbors<<<grid_of(n), 256, 0, s>>>(vg->view(), vg->active, vg->s_coords.ptr, vg->s_found.ptr);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}
// compact s_coords by s_found into r_coords
nnrt_status compact_found_coords(nnrt_voxel_grid* vg, int64_t n, hipStream_t s) {
	int64_t total = 0;
	nnrt_status st;
	if ((st = scan_total(vg, vg->s_found.ptr, vg->s_rank.ptr, n, s, &total))) return st;
	if ((st = vg->r_coords.ensure(3 * static_cast<size_t>(std::max<int64_t>(total, 1))))) return st;
	if (n > 0) k_compact_coords<<<grid_of(n), 256, 0, s>>>(vg->s_coords.ptr, vg->s_found.ptr, vg->s_rank.ptr, n, vg->r_coords.ptr);
	NNRT_LAUNCH_CHECK();
	NNRT_HIP(hipStreamSynchronize(s));
	vg->r_coord_count = total;
	return NNRT_OK;
}

float color_multiplier(int depth_dtype) { return depth_dtype == NNRT_DTYPE_FLOAT32 ? 255.0f : 1.0f; }

nnrt_status upload_mc_tables() {
	static bool done_for[64] = {false};
	int dev = 0;
	hipGetDevice(&dev);
	if (dev >= 0 && dev < 64 && done_for[dev]) return NNRT_OK;
	const McTables t = build_mc_tables();
	NNRT_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_mc), &t, sizeof(t)));
	if (dev >= 0 && dev < 64) done_for[dev] = true;
	return NNRT_OK;
}
} // namespace

extern "C" {

nnrt_status nnrt_voxel_grid_create(float voxel_size, int32_t block_resolution, int64_t block_count, int32_t weight_dtype, int32_t color_dtype,
                                   int32_t device, nnrt_voxel_grid** out) {
	NNRT_CHECK_ARG(out, "null output");
	*out = nullptr;
	NNRT_CHECK_ARG(voxel_size > 0.f && block_resolution >= 2 && block_resolution <= 32 && block_count >= 1, "invalid grid geometry");
	NNRT_CHECK_ARG(weight_dtype == NNRT_DTYPE_FLOAT32 || weight_dtype == NNRT_DTYPE_UINT16, "weight dtype must be float32 or uint16");
	NNRT_CHECK_ARG(color_dtype == NNRT_DTYPE_NONE || color_dtype == NNRT_DTYPE_FLOAT32 || color_dtype == NNRT_DTYPE_UINT16 ||
	                   color_dtype == NNRT_DTYPE_UINT8,
	               "color dtype must be none, float32, uint16 or uint8");
	GridGuard guard(device);
	std::unique_ptr<nnrt_voxel_grid> vg(new nnrt_voxel_grid());
	vg->device = device;
	vg->voxel_size = voxel_size;
	vg->res = block_resolution;
	vg->res3 = block_resolution * block_resolution * block_resolution;
	vg->weight_type = store_type_of(weight_dtype);
	vg->color_type = store_type_of(color_dtype);
	nnrt_status st = ensure_capacity(vg.get(), block_count, nullptr);
	if (st) return st;
	if (!vg->table_size && (st = rebuild_table(vg.get(), 16, nullptr))) return st;
	NNRT_HIP(hipDeviceSynchronize());
	*out = vg.release();
	return NNRT_OK;
}

void nnrt_voxel_grid_destroy(nnrt_voxel_grid* vg) {
	if (!vg) return;
	GridGuard guard(vg->device);
	hipDeviceSynchronize();
	delete vg;
}

nnrt_status nnrt_voxel_grid_get_info(const nnrt_voxel_grid* vg, int64_t* h_active_blocks, int64_t* h_capacity, float* h_voxel_size,
                                     int32_t* h_block_resolution) {
	NNRT_CHECK_ARG(vg, "null grid");
	if (h_active_blocks) *h_active_blocks = vg->active;
	if (h_capacity) *h_capacity = vg->capacity;
	if (h_voxel_size) *h_voxel_size = vg->voxel_size;
	if (h_block_resolution) *h_block_resolution = vg->res;
	return NNRT_OK;
}

nnrt_status nnrt_voxel_grid_activate(nnrt_voxel_grid* vg, const int32_t* d_block_coords, int64_t count, void* stream) {
	NNRT_CHECK_ARG(vg && (count == 0 || d_block_coords) && count >= 0, "invalid arguments");
	GridGuard guard(vg->device);
	return activate_coords(vg, d_block_coords, count, static_cast<hipStream_t>(stream));
}

nnrt_status nnrt_voxel_grid_get_block_coordinates(const nnrt_voxel_grid* vg, int32_t* d_out, void* stream) {
	NNRT_CHECK_ARG(vg && d_out, "invalid arguments");
	GridGuard guard(vg->device);
	if (vg->active) NNRT_HIP(hipMemcpyAsync(d_out, vg->keys.ptr, sizeof(int32_t) * 3 * vg->active, hipMemcpyDeviceToDevice, static_cast<hipStream_t>(stream)));
	return NNRT_OK;
}

nnrt_status nnrt_voxel_grid_unique_block_coordinates(nnrt_voxel_grid* vg, const void* d_depth, int32_t depth_dtype, int32_t height, int32_t width,
                                                     const double* h_K, const double* h_E, float depth_scale, float depth_max,
                                                     float trunc_voxel_multiplier, int64_t* h_count, void* stream) {
	NNRT_CHECK_ARG(vg && d_depth && h_K && h_count && height > 0 && width > 0, "invalid arguments");
	NNRT_CHECK_ARG(depth_dtype == NNRT_DTYPE_UINT16 || depth_dtype == NNRT_DTYPE_FLOAT32, "depth must be uint16 or float32");
	GridGuard guard(vg->device);
	hipStream_t s = static_cast<hipStream_t>(stream);
	double Einv[16];
	static const double I4[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
	if (!invert4(h_E ? h_E : I4, Einv)) {
		set_error("extrinsic matrix is singular");
		return NNRT_ERROR_ARGUMENT;
	}
	constexpr int STRIDE = 4;   // VoxelBlockGrid.cpp:250 down_factor
	const int64_t n = static_cast<int64_t>(height / STRIDE) * (width / STRIDE) * (TOUCH_STEPS + 1);
	nnrt_status st;
	if ((st = vg->s_packed.ensure(std::max<int64_t>(n, 1)))) return st;
	const ImageView im = make_image(d_depth, depth_dtype, height, width, nullptr, 0, 0, depth_scale, depth_max);
	if (n > 0) k_touch_depth<<<grid_of(n / (TOUCH_STEPS + 1)), 256, 0, s>>>(im, STRIDE, make_xform(h_K, Einv), vg->voxel_size * trunc_voxel_multiplier,
	                                                                      vg->voxel_size * static_cast<float>(vg->res), vg->s_packed.ptr);
	NNRT_LAUNCH_CHECK();
	if ((st = unique_packed(vg, vg->s_packed.ptr, n, s))) return st;
	*h_count = vg->r_coord_count;
	return NNRT_OK;
}

nnrt_status nnrt_voxel_grid_copy_result_coordinates(const nnrt_voxel_grid* vg, int32_t* d_out, void* stream) {
	NNRT_CHECK_ARG(vg && (d_out || vg->r_coord_count == 0), "invalid arguments");
	GridGuard guard(vg->device);
	if (vg->r_coord_count)
		NNRT_HIP(hipMemcpyAsync(d_out, vg->r_coords.ptr, sizeof(int32_t) * 3 * vg->r_coord_count, hipMemcpyDeviceToDevice, static_cast<hipStream_t>(stream)));
	return NNRT_OK;
}

nnrt_status nnrt_voxel_grid_integrate(nnrt_voxel_grid* vg, const int32_t* d_block_coords, int64_t count, const void* d_depth, int32_t depth_dtype,
                                      int32_t height, int32_t width, const void* d_color, int32_t color_height, int32_t color_width,
                                      const double* h_depth_K, const double* h_color_K, const double* h_E, float depth_scale, float depth_max,
                                      float trunc_voxel_multiplier, void* stream) {
	NNRT_CHECK_ARG(vg && d_depth && h_depth_K && height > 0 && width > 0 && count >= 0 && (count == 0 || d_block_coords), "invalid arguments");
	NNRT_CHECK_ARG(depth_dtype == NNRT_DTYPE_UINT16 || depth_dtype == NNRT_DTYPE_FLOAT32, "depth must be uint16 or float32");
	GridGuard guard(vg->device);
	hipStream_t s = static_cast<hipStream_t>(stream);
	nnrt_status st;
	if ((st = activate_coords(vg, d_block_coords, count, s))) return st;
	if (count == 0) return NNRT_OK;
	if ((st = vg->s_blocks.ensure(count))) return st;
	const GridView g = vg->view();
	k_find_blocks<<<grid_of(count), 256, 0, s>>>(g.hash, d_block_coords, count, vg->s_blocks.ptr);
	const ImageView im = make_image(d_depth, depth_dtype, height, width, d_color, color_height, color_width, depth_scale, depth_max);
	k_integrate_rigid<<<grid_of(count * vg->res3), 256, 0, s>>>(g, vg->s_blocks.ptr, count, im, make_xform(h_depth_K, h_E),
	                                                           make_xform(h_color_K ? h_color_K : h_depth_K, nullptr),
	                                                           vg->voxel_size * trunc_voxel_multiplier, color_multiplier(depth_dtype));
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

nnrt_status nnrt_voxel_grid_integrate_non_rigid(nnrt_voxel_grid* vg, const int32_t* d_block_coords, int64_t count, const nnrt_warp_field* wf,
                                                const void* d_depth, int32_t depth_dtype, int32_t height, int32_t width, const void* d_color,
                                                int32_t color_height, int32_t color_width, const float* d_depth_normals, const double* h_depth_K,
                                                const double* h_color_K, const double* h_E, float depth_scale, float depth_max,
                                                float trunc_voxel_multiplier, float* d_cos_out, void* stream) {
	NNRT_CHECK_ARG(vg && wf && d_depth && d_depth_normals && h_depth_K && d_cos_out && height > 0 && width > 0 && count >= 0 &&
	                   (count == 0 || d_block_coords),
	               "invalid arguments");
	NNRT_CHECK_ARG(depth_dtype == NNRT_DTYPE_UINT16 || depth_dtype == NNRT_DTYPE_FLOAT32, "depth must be uint16 or float32");
	GridGuard guard(vg->device);
	hipStream_t s = static_cast<hipStream_t>(stream);
	nnrt_status st;
	if ((st = activate_coords(vg, d_block_coords, count, s))) return st;
	const WarpFieldView wv = warp_field_view(wf);
	NNRT_CHECK_ARG(wv.anchor_count >= 1 && wv.anchor_count <= TSDF_MAX_ANCHORS, "anchor_count must be in [1, 8]");
	const int64_t P = static_cast<int64_t>(height) * width;
	NNRT_HIP(hipMemsetAsync(d_cos_out, 0, sizeof(float) * P, s));   // Tensor::Zeros (:72)
	if (vg->active == 0) return NNRT_OK;
	if ((st = vg->s_packed.ensure(P))) return st;
	NNRT_HIP(hipMemsetAsync(vg->s_packed.ptr, 0, sizeof(uint64_t) * P, s));
	float range = 2.f * wv.coverage;   // nodes farther than 2 c are never valid anchors
	if (!wv.fixed_coverage) {
		std::vector<float> w(static_cast<size_t>(wv.N));
		NNRT_HIP(hipMemcpy(w.data(), wv.node_weights, sizeof(float) * w.size(), hipMemcpyDeviceToHost));
		float mx = 0.f;
		for (float v : w) mx = std::max(mx, v);
		range = 2.f * std::sqrt(mx);
	}
	const ImageView im = make_image(d_depth, depth_dtype, height, width, d_color, color_height, color_width, depth_scale, depth_max);
	const GridView gv = vg->view();
	const Xform xd = make_xform(h_depth_K, h_E), xc = make_xform(h_color_K ? h_color_K : h_depth_K, nullptr);
	const float trunc = vg->voxel_size * trunc_voxel_multiplier, cm = color_multiplier(depth_dtype);
	switch (wv.anchor_count) {
#define NNRT_NR_CASE(KK)                                                                                                          \
	case KK:                                                                                                                      \
		k_integrate_non_rigid<KK><<<static_cast<unsigned>(vg->active), NR_BLOCK, 0, s>>>(gv, vg->active, wv, im, d_depth_normals, xd, xc, \
		                                                                               trunc, cm, range, vg->s_packed.ptr);        \
		break;
		NNRT_NR_CASE(1) NNRT_NR_CASE(2) NNRT_NR_CASE(3) NNRT_NR_CASE(4) NNRT_NR_CASE(5) NNRT_NR_CASE(6) NNRT_NR_CASE(7) NNRT_NR_CASE(8)
#undef NNRT_NR_CASE
	}
	k_cos_resolve<<<grid_of(P), 256, 0, s>>>(vg->s_packed.ptr, P, d_cos_out);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

nnrt_status nnrt_voxel_grid_extract_voxel_values_and_coordinates(const nnrt_voxel_grid* vg, float* d_out, int32_t* h_channels, void* stream) {
	NNRT_CHECK_ARG(vg && (d_out || vg->active == 0), "invalid arguments");
	GridGuard guard(vg->device);
	if (h_channels) *h_channels = vg->channels();
	const int64_t n = vg->active * vg->res3;
	if (n > 0)
		k_values_all<<<grid_of(n), 256, 0, static_cast<hipStream_t>(stream)>>>(const_cast<nnrt_voxel_grid*>(vg)->view(), vg->active, vg->channels(), d_out);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

nnrt_status nnrt_voxel_grid_extract_voxel_values_at(nnrt_voxel_grid* vg, const int32_t* d_query, int64_t count, int64_t* h_rows, int32_t* h_channels,
                                                    void* stream) {
	NNRT_CHECK_ARG(vg && h_rows && (count == 0 || d_query) && count >= 0, "invalid arguments");
	GridGuard guard(vg->device);
	hipStream_t s = static_cast<hipStream_t>(stream);
	const int C = vg->channels();
	if (h_channels) *h_channels = C;
	vg->r_row_channels = C;
	vg->r_row_count = 0;
	*h_rows = 0;
	if (count == 0) return NNRT_OK;
	nnrt_status st;
	if ((st = vg->s_rows_all.ensure(static_cast<size_t>(count) * C)) || (st = vg->s_found.ensure(count)) || (st = vg->s_rank.ensure(count))) return st;
	const GridView g = vg->view();
	k_values_at<<<grid_of(count), 256, 0, s>>>(g, vg->capacity, d_query, count, C, vg->s_rows_all.ptr);
	k_found_mask<<<grid_of(count), 256, 0, s>>>(g, d_query, count, vg->s_found.ptr);
	NNRT_LAUNCH_CHECK();
	int64_t total = 0;
	if ((st = scan_total(vg, vg->s_found.ptr, vg->s_rank.ptr, count, s, &total))) return st;
	if ((st = vg->r_rows.ensure(static_cast<size_t>(std::max<int64_t>(total, 1)) * C))) return st;
	k_compact_rows<<<grid_of(count), 256, 0, s>>>(vg->s_rows_all.ptr, vg->s_found.ptr, vg->s_rank.ptr, count, C, vg->r_rows.ptr);
	NNRT_LAUNCH_CHECK();
	NNRT_HIP(hipStreamSynchronize(s));
	vg->r_row_count = total;
	*h_rows = total;
	return NNRT_OK;
}

nnrt_status nnrt_voxel_grid_copy_result_rows(const nnrt_voxel_grid* vg, float* d_out, void* stream) {
	NNRT_CHECK_ARG(vg && (d_out || vg->r_row_count == 0), "invalid arguments");
	GridGuard guard(vg->device);
	if (vg->r_row_count)
		NNRT_HIP(hipMemcpyAsync(d_out, vg->r_rows.ptr, sizeof(float) * vg->r_row_count * vg->r_row_channels, hipMemcpyDeviceToDevice,
		                        static_cast<hipStream_t>(stream)));
	return NNRT_OK;
}

nnrt_status nnrt_voxel_grid_warped_block_boxes(const nnrt_voxel_grid* vg, const int32_t* d_block_keys, int64_t count, const nnrt_warp_field* wf,
                                               const double* h_E, float* d_boxes, void* stream) {
	NNRT_CHECK_ARG(vg && wf && (count == 0 || (d_block_keys && d_boxes)) && count >= 0, "invalid arguments");
	GridGuard guard(vg->device);
	const WarpFieldView wv = warp_field_view(wf);
	NNRT_CHECK_ARG(wv.anchor_count >= 1 && wv.anchor_count <= TSDF_MAX_ANCHORS, "anchor_count must be in [1, 8]");
	if (count == 0) return NNRT_OK;
	const float side = static_cast<float>(vg->res) * vg->voxel_size;
	const Xform ex = make_xform(nullptr, h_E);
	hipStream_t bs = static_cast<hipStream_t>(stream);
	switch (wv.anchor_count) {
#define NNRT_BOX_CASE(KK)                                                                                  \
	case KK: k_warped_block_boxes<KK><<<grid_of(8 * count, BOX_BLOCK), BOX_BLOCK, 0, bs>>>(d_block_keys, count, side, wv, ex, 2.f * wv.coverage, d_boxes); break;
		NNRT_BOX_CASE(1) NNRT_BOX_CASE(2) NNRT_BOX_CASE(3) NNRT_BOX_CASE(4) NNRT_BOX_CASE(5) NNRT_BOX_CASE(6) NNRT_BOX_CASE(7) NNRT_BOX_CASE(8)
#undef NNRT_BOX_CASE
	}
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

nnrt_status nnrt_boxes_intersecting_surface_mask(const float* d_boxes, int64_t count, const void* d_depth, int32_t depth_dtype, int32_t height,
                                                 int32_t width, const double* h_K, float depth_scale, float depth_max, int32_t stride,
                                                 float truncation_distance, uint8_t* d_mask, void* stream) {
	NNRT_CHECK_ARG((count == 0 || (d_boxes && d_mask)) && d_depth && h_K && height > 0 && width > 0 && stride >= 1 && count >= 0,
	               "invalid arguments");
	NNRT_CHECK_ARG(depth_dtype == NNRT_DTYPE_UINT16 || depth_dtype == NNRT_DTYPE_FLOAT32, "depth must be uint16 or float32");
	hipStream_t s = static_cast<hipStream_t>(stream);
	if (count == 0) return NNRT_OK;
	const int64_t nseg = static_cast<int64_t>(height / stride) * (width / stride);
	Seg* segs = nullptr;
	NNRT_HIP(hipMallocAsync(reinterpret_cast<void**>(&segs), sizeof(Seg) * std::max<int64_t>(nseg, 1), s));
	const ImageView im = make_image(d_depth, depth_dtype, height, width, nullptr, 0, 0, depth_scale, depth_max);
	if (nseg > 0) k_make_segments<<<grid_of(nseg), 256, 0, s>>>(im, stride, make_xform(h_K, nullptr), truncation_distance, segs);
	k_boxes_mask<<<grid_of(count), 256, 0, s>>>(d_boxes, count, segs, nseg, d_mask);
	hipError_t le = hipGetLastError();
	hipFreeAsync(segs, s);
	NNRT_HIP(le);
	return NNRT_OK;
}

nnrt_status nnrt_voxel_grid_find_blocks_intersecting_truncation_region(nnrt_voxel_grid* vg, const void* d_depth, int32_t depth_dtype, int32_t height,
                                                                       int32_t width, const nnrt_warp_field* wf, const double* h_K, const double* h_E,
                                                                       float depth_scale, float depth_max, float trunc_voxel_multiplier,
                                                                       int64_t* h_count, void* stream) {
	NNRT_CHECK_ARG(vg && wf && d_depth && h_K && h_count, "invalid arguments");
	GridGuard guard(vg->device);
	hipStream_t s = static_cast<hipStream_t>(stream);
	int64_t n = 0;
	nnrt_status st;
	if ((st = inactive_neighbors(vg, s, &n))) return st;
	if ((st = compact_found_coords(vg, n, s))) return st;   // r_coords = inactive neighbour coordinates
	const int64_t m = vg->r_coord_count;
	*h_count = 0;
	if (m == 0) return NNRT_OK;
	if ((st = vg->s_boxes.ensure(6 * static_cast<size_t>(m))) || (st = vg->s_mask.ensure(m)) || (st = vg->s_coords.ensure(3 * static_cast<size_t>(m))))
		return st;
	NNRT_HIP(hipMemcpyAsync(vg->s_coords.ptr, vg->r_coords.ptr, sizeof(int32_t) * 3 * m, hipMemcpyDeviceToDevice, s));
	if ((st = nnrt_voxel_grid_warped_block_boxes(vg, vg->s_coords.ptr, m, wf, h_E, vg->s_boxes.ptr, stream))) return st;
	// NonRigidSurfaceVoxelBlockGrid.cpp:163-166: stride 4, truncation = voxel_size * trunc_voxel_multiplier (default 8)
	if ((st = nnrt_boxes_intersecting_surface_mask(vg->s_boxes.ptr, m, d_depth, depth_dtype, height, width, h_K, depth_scale, depth_max, 4,
	                                               vg->voxel_size * trunc_voxel_multiplier, vg->s_mask.ptr, stream)))
		return st;
	if ((st = vg->s_found.ensure(m)) || (st = vg->s_rank.ensure(m))) return st;
	k_and_mask<<<grid_of(m), 256, 0, s>>>(vg->s_found.ptr, vg->s_mask.ptr, m);
	NNRT_LAUNCH_CHECK();
	if ((st = compact_found_coords(vg, m, s))) return st;
	*h_count = vg->r_coord_count;
	return NNRT_OK;
}

nnrt_status nnrt_voxel_grid_activate_sleeve_blocks(nnrt_voxel_grid* vg, int64_t* h_count, void* stream) {
	NNRT_CHECK_ARG(vg && h_count, "invalid arguments");
	GridGuard guard(vg->device);
	hipStream_t s = static_cast<hipStream_t>(stream);
	int64_t n = 0;
	nnrt_status st;
	if ((st = inactive_neighbors(vg, s, &n))) return st;
	if ((st = compact_found_coords(vg, n, s))) return st;
	const int64_t m = vg->r_coord_count;
	*h_count = m;   // the reference returns the count with duplicates (:109)
	if (m == 0) return NNRT_OK;
	if ((st = vg->s_coords.ensure(3 * static_cast<size_t>(m)))) return st;
	NNRT_HIP(hipMemcpyAsync(vg->s_coords.ptr, vg->r_coords.ptr, sizeof(int32_t) * 3 * m, hipMemcpyDeviceToDevice, s));
	return activate_coords(vg, vg->s_coords.ptr, m, s);
}

nnrt_status nnrt_voxel_grid_extract_triangle_mesh(nnrt_voxel_grid* vg, float weight_threshold, int64_t* h_vertex_count, int64_t* h_triangle_count,
                                                  void* stream) {
	NNRT_CHECK_ARG(vg && h_vertex_count && h_triangle_count, "invalid arguments");
	GridGuard guard(vg->device);
	hipStream_t s = static_cast<hipStream_t>(stream);
	nnrt_status st;
	if ((st = upload_mc_tables())) return st;
	vg->r_nv = vg->r_nt = 0;
	*h_vertex_count = *h_triangle_count = 0;
	const int64_t nb = vg->active, nvox = nb * vg->res3;
	if (nb == 0) return NNRT_OK;
	if ((st = vg->s_nbr.ensure(27 * static_cast<size_t>(nb))) || (st = vg->s_cube.ensure(nvox)) || (st = vg->s_ntri.ensure(nvox)) ||
	    (st = vg->s_toff.ensure(nvox)) || (st = vg->s_eflag.ensure(3 * static_cast<size_t>(nvox))) || (st = vg->s_vidx.ensure(3 * static_cast<size_t>(nvox))))
		return st;
	MeshGridView m{vg->view(), vg->s_nbr.ptr, weight_threshold};
	k_block_neighbors<<<grid_of(27 * nb), 256, 0, s>>>(m.g, nb, vg->s_nbr.ptr);
	NNRT_HIP(hipMemsetAsync(vg->s_eflag.ptr, 0, sizeof(int) * 3 * nvox, s));
	k_mc_cubes<<<grid_of(nvox), 256, 0, s>>>(m, nb, vg->s_cube.ptr, vg->s_ntri.ptr, vg->s_eflag.ptr);
	NNRT_LAUNCH_CHECK();
	int64_t nv = 0, nt = 0;
	if ((st = scan_total(vg, vg->s_eflag.ptr, vg->s_vidx.ptr, 3 * nvox, s, &nv))) return st;
	if ((st = scan_total(vg, vg->s_ntri.ptr, vg->s_toff.ptr, nvox, s, &nt))) return st;
	if ((st = vg->r_vpos.ensure(3 * static_cast<size_t>(std::max<int64_t>(nv, 1)))) || (st = vg->r_vnrm.ensure(3 * static_cast<size_t>(std::max<int64_t>(nv, 1)))) ||
	    (st = vg->r_vcol.ensure(3 * static_cast<size_t>(std::max<int64_t>(nv, 1)))) || (st = vg->r_tris.ensure(3 * static_cast<size_t>(std::max<int64_t>(nt, 1)))))
		return st;
	k_mc_vertices<<<grid_of(3 * nvox), 256, 0, s>>>(m, nb, vg->s_eflag.ptr, vg->s_vidx.ptr, vg->r_vpos.ptr, vg->r_vnrm.ptr,
	                                                  vg->color_type != ST_NONE ? vg->r_vcol.ptr : nullptr);
	k_mc_triangles<<<grid_of(nvox), 256, 0, s>>>(m, nb, vg->s_cube.ptr, vg->s_toff.ptr, vg->s_vidx.ptr, vg->r_tris.ptr);
	NNRT_LAUNCH_CHECK();
	NNRT_HIP(hipStreamSynchronize(s));
	vg->r_nv = nv;
	vg->r_nt = nt;
	*h_vertex_count = nv;
	*h_triangle_count = nt;
	return NNRT_OK;
}

nnrt_status nnrt_voxel_grid_copy_mesh(const nnrt_voxel_grid* vg, float* d_vertices, float* d_normals, float* d_colors, int64_t* d_triangles, void* stream) {
	NNRT_CHECK_ARG(vg, "null grid");
	GridGuard guard(vg->device);
	hipStream_t s = static_cast<hipStream_t>(stream);
	const size_t nv = static_cast<size_t>(vg->r_nv), nt = static_cast<size_t>(vg->r_nt);
	if (nv && d_vertices) NNRT_HIP(hipMemcpyAsync(d_vertices, vg->r_vpos.ptr, sizeof(float) * 3 * nv, hipMemcpyDeviceToDevice, s));
	if (nv && d_normals) NNRT_HIP(hipMemcpyAsync(d_normals, vg->r_vnrm.ptr, sizeof(float) * 3 * nv, hipMemcpyDeviceToDevice, s));
	if (nv && d_colors && vg->color_type != ST_NONE) NNRT_HIP(hipMemcpyAsync(d_colors, vg->r_vcol.ptr, sizeof(float) * 3 * nv, hipMemcpyDeviceToDevice, s));
	if (nt && d_triangles) NNRT_HIP(hipMemcpyAsync(d_triangles, vg->r_tris.ptr, sizeof(int64_t) * 3 * nt, hipMemcpyDeviceToDevice, s));
	return NNRT_OK;
}

// the marching-cubes triangle table in emission order (host copy, for tests): tri [256][31] int8 (edge triples, -1 terminated)
nnrt_status nnrt_marching_cubes_table(int8_t* h_tri, uint16_t* h_edge_mask) {
	NNRT_CHECK_ARG(h_tri || h_edge_mask, "null output");
	const McTables t = build_mc_tables();
	if (h_tri) std::memcpy(h_tri, t.tri, sizeof(t.tri));
	if (h_edge_mask) std::memcpy(h_edge_mask, t.edge_mask, sizeof(t.edge_mask));
	return NNRT_OK;
}

} // extern "C"
