// =====================================================================================================================
// tsdf_oracle.cpp -- TEST INFRASTRUCTURE ONLY (parity oracle). NOT PART OF THE PRODUCT PATH.
//
// Plain C++ restatement of the TSDF voxel block grid around the fitter:
//   * NNRT's NonRigidSurfaceVoxelBlockGrid (cpp/geometry/NonRigidSurfaceVoxelBlockGrid.cpp:33-224,
//     cpp/geometry/kernel/NonRigidSurfaceVoxelBlockGridImpl.h:52-652, cpp/geometry/kernel/Segment.h) -- pinned by the
//     reference's own known-answer tests (cpp/tests/test_non_rigid_surface_voxel_block_grid.cpp:60-351, transcribed in
//     tests/golden/kat_literals.py);
//   * the Open3D 0.17 kernels NNRT's VoxelBlockGrid calls (HashMap::Activate, voxel_grid::DepthTouch / Integrate /
//     ExtractTriangleMesh) -- third-party, absent from the reference tree: restated from Open3D's published algorithm
//     (the DepthTouch sampling and the Integrate update are also exercised by the IntegrateNonRigid KAT, whose volume is
//     built with them); the marching-cubes triangulation is the published Lorensen-Cline / Bourke table Open3D indexes
//     (mc_table_oracle.hpp; no Open3D output fixture exists here, so mesh parity with Open3D stays unpinned).
// Deterministic policies (shared with the HIP path by specification, not by code): blocks are numbered in first-
// activation order (first occurrence within an activation call); anchors of a voxel are the K nearest nodes among those
// within 2 * (largest) coverage, ascending node order, replace-the-maximum insertion.
// =====================================================================================================================
#include "mc_table_oracle.hpp"
#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <map>
#include <tuple>
#include <vector>

#define ORC_API extern "C" __attribute__((visibility("default")))

namespace {

enum { DT_NONE = -1, DT_F32 = 0, DT_U16 = 1, DT_U8 = 2 };

float cr_exp(float x) { return static_cast<float>(std::exp(static_cast<double>(x))); }

struct Cam {   // Open3D TransformIndexer: float rows of the 3x4 extrinsic, float intrinsics
	float m[12];
	float fx, fy, cx, cy;
	void rigid(float x, float y, float z, float& a, float& b, float& c) const {
		a = ((x * m[0] + y * m[1]) + z * m[2]) + m[3];
		b = ((x * m[4] + y * m[5]) + z * m[6]) + m[7];
		c = ((x * m[8] + y * m[9]) + z * m[10]) + m[11];
	}
	void project(float x, float y, float z, float& u, float& v) const {
		const float iz = 1.0f / z;
		u = (fx * x) * iz + cx;
		v = (fy * y) * iz + cy;
	}
	void unproject(float u, float v, float d, float& x, float& y, float& z) const {
		x = ((u - cx) * d) / fx;
		y = ((v - cy) * d) / fy;
		z = d;
	}
};
Cam make_cam(const double* K, const double* E) {
	Cam c{};
	for (int r = 0; r < 3; r++)
		for (int k = 0; k < 4; k++) c.m[4 * r + k] = E ? static_cast<float>(E[4 * r + k]) : (r == k ? 1.f : 0.f);
	c.fx = K ? static_cast<float>(K[0]) : 1.f;
	c.fy = K ? static_cast<float>(K[4]) : 1.f;
	c.cx = K ? static_cast<float>(K[2]) : 0.f;
	c.cy = K ? static_cast<float>(K[5]) : 0.f;
	return c;
}
bool inverse4(const double* a, double* out) {   // Gauss-Jordan, partial pivoting
	double m[4][8];
	for (int r = 0; r < 4; r++)
		for (int c = 0; c < 8; c++) m[r][c] = c < 4 ? a[4 * r + c] : (c - 4 == r);
	for (int c = 0; c < 4; c++) {
		int p = c;
		for (int r = c + 1; r < 4; r++)
			if (std::fabs(m[r][c]) > std::fabs(m[p][c])) p = r;
		if (m[p][c] == 0.0) return false;
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
		for (int c = 0; c < 4; c++) out[4 * r + c] = m[r][4 + c];
	return true;
}
bool in_bounds(float u, float v, int H, int W) { return u >= 0.f && v >= 0.f && u <= static_cast<float>(W) - 1.0f && v <= static_cast<float>(H) - 1.0f; }

struct Img {
	const void* depth;
	int dtype, H, W;
	const void* color;
	int Hc, Wc;
	float scale, dmax;
	float d(int u, int v) const {
		const int64_t i = static_cast<int64_t>(v) * W + u;
		return dtype == DT_U16 ? static_cast<float>(static_cast<const uint16_t*>(depth)[i]) : static_cast<const float*>(depth)[i];
	}
	float c(int u, int v, int ch) const {
		const int64_t i = (static_cast<int64_t>(v) * Wc + u) * 3 + ch;
		return dtype == DT_U16 ? static_cast<float>(static_cast<const uint8_t*>(color)[i]) : static_cast<const float*>(color)[i];
	}
};

float store_cast(int dt, float v) {   // typed store (C++ float -> integer truncates toward zero) read back as float
	if (dt == DT_U16) return static_cast<float>(static_cast<uint16_t>(static_cast<uint32_t>(v)));
	if (dt == DT_U8) return static_cast<float>(static_cast<uint8_t>(static_cast<uint32_t>(v)));
	return v;
}

using Key = std::tuple<int, int, int>;

struct Grid {
	float voxel;
	int res, res3;
	int wdt, cdt;
	std::map<Key, int> index;
	std::vector<Key> keys;
	std::vector<float> tsdf, weight, color;   // values held as float, stored through store_cast

	int find(int x, int y, int z) const {
		auto it = index.find(Key(x, y, z));
		return it == index.end() ? -1 : it->second;
	}
	void activate(const int32_t* c, int64_t n) {
		for (int64_t i = 0; i < n; i++) {
			const Key k(c[3 * i], c[3 * i + 1], c[3 * i + 2]);
			if (index.count(k)) continue;
			index[k] = static_cast<int>(keys.size());
			keys.push_back(k);
			tsdf.resize(tsdf.size() + res3, 0.f);
			weight.resize(weight.size() + res3, 0.f);
			if (cdt != DT_NONE) color.resize(color.size() + 3 * res3, 0.f);
		}
	}
	void voxel_xyz(int b, int vi, int& x, int& y, int& z) const {
		x = std::get<0>(keys[b]) * res + vi % res;
		y = std::get<1>(keys[b]) * res + (vi / res) % res;
		z = std::get<2>(keys[b]) * res + vi / (res * res);
	}
	// voxel at global (x, y, z), -1 if its block is inactive
	int64_t at(int x, int y, int z) const {
		auto fdiv = [&](int a) { return a >= 0 ? a / res : -((-a + res - 1) / res); };
		const int bx = fdiv(x), by = fdiv(y), bz = fdiv(z);
		const int b = find(bx, by, bz);
		if (b < 0) return -1;
		return static_cast<int64_t>(b) * res3 + (x - bx * res) + res * ((y - by * res) + res * (z - bz * res));
	}
};

// ---- anchors with the node-distance threshold (WarpUtilities.h:131-153, :319-341; KnnUtilities.h:146-220) ----------
struct Field {
	int N, K, min_valid;
	const float* nodes;   // [N,3]
	const float* R;       // [N,9]
	const float* t;       // [N,3]
	const float* c2;      // [N] squared coverage (variable) or null
	float coverage;
};
bool anchors(const Field& f, const float* p, float range, int* idx, float* w) {
	for (int k = 0; k < f.K; k++) {
		idx[k] = -1;
		w[k] = INFINITY;
	}
	float maxd = INFINITY;
	int max_at = 0;
	for (int n = 0; n < f.N; n++) {
		const float dx = f.nodes[3 * n] - p[0], dy = f.nodes[3 * n + 1] - p[1], dz = f.nodes[3 * n + 2] - p[2];
		const float d = std::sqrt((dx * dx + dy * dy) + dz * dz);
		if (!(d <= range)) continue;
		if (maxd > d) {
			w[max_at] = d;
			idx[max_at] = n;
			max_at = 0;
			maxd = w[0];
			for (int k = 1; k < f.K; k++)
				if (w[k] > maxd) {
					max_at = k;
					maxd = w[k];
				}
		}
	}
	float sum = 0.f;
	int valid = 0;
	for (int k = 0; k < f.K; k++) {
		if (idx[k] < 0) continue;
		const float sq = w[k] * w[k];
		const float c2 = f.c2 ? f.c2[idx[k]] : f.coverage * f.coverage;
		if (sq > 4 * c2) {
			idx[k] = -1;
			continue;
		}
		const float wt = cr_exp(-sq / (2 * c2));
		sum += wt;
		w[k] = wt;
		valid++;
	}
	if (valid < f.min_valid) return false;
	if (sum > 0.0f) {
		for (int k = 0; k < f.K; k++) w[k] /= sum;
	} else if (valid > 0) {
		for (int k = 0; k < f.K; k++) w[k] = 1.0f / static_cast<float>(valid);
	}
	return true;
}
void blend(const Field& f, const int* idx, const float* w, const float* p, float* o) {
	o[0] = o[1] = o[2] = 0.f;
	for (int k = 0; k < f.K; k++) {
		const int n = idx[k];
		if (n < 0) continue;
		const float* g = f.nodes + 3 * n;
		const float* R = f.R + 9 * n;
		const float d[3] = {p[0] - g[0], p[1] - g[1], p[2] - g[2]};
		float r[3];
		for (int i = 0; i < 3; i++) r[i] = (R[3 * i] * d[0] + R[3 * i + 1] * d[1]) + R[3 * i + 2] * d[2];
		for (int i = 0; i < 3; i++) o[i] += w[k] * ((g[i] + r[i]) + f.t[3 * n + i]);
	}
}

// ---- marching-cubes table: the published Lorensen-Cline / Bourke table Open3D indexes (oracle copy: mc_table_oracle.hpp);
// each triangle (a, b, c) is emitted as (c, b, a): Open3D stores table vertex v at slot 2 - v (faces away from negative
// tsdf; the slot order is restated from Open3D's published source, third-party and absent: parity unpinned) ----
struct McTable {
	uint16_t mask[256];
	std::vector<int> tri[256];
};
const McTable& mc_table() {
	static McTable T;
	static bool built = false;
	if (built) return T;
	const int ev[12][2] = {{0, 1}, {1, 2}, {2, 3}, {3, 0}, {4, 5}, {5, 6}, {6, 7}, {7, 4}, {0, 4}, {1, 5}, {2, 6}, {3, 7}};
	for (int cfg = 0; cfg < 256; cfg++) {
		uint16_t mask = 0;
		for (int e = 0; e < 12; e++)
			if (((cfg >> ev[e][0]) & 1) != ((cfg >> ev[e][1]) & 1)) mask |= static_cast<uint16_t>(1 << e);
		T.mask[cfg] = mask;
		for (int i = 0; i < 16 && ORC_MC_TRI_TABLE[cfg][i] >= 0; i += 3)
			T.tri[cfg].insert(T.tri[cfg].end(), {ORC_MC_TRI_TABLE[cfg][i + 2], ORC_MC_TRI_TABLE[cfg][i + 1], ORC_MC_TRI_TABLE[cfg][i]});
	}
	built = true;
	return T;
}
const int k_owner[12][4] = {{0, 0, 0, 0}, {1, 0, 0, 1}, {0, 1, 0, 0}, {0, 0, 0, 1}, {0, 0, 1, 0}, {1, 0, 1, 1},
                            {0, 1, 1, 0}, {0, 0, 1, 1}, {0, 0, 0, 2}, {1, 0, 0, 2}, {1, 1, 0, 2}, {0, 1, 0, 2}};
const int k_corner[8][3] = {{0, 0, 0}, {1, 0, 0}, {1, 1, 0}, {0, 1, 0}, {0, 0, 1}, {1, 0, 1}, {1, 1, 1}, {0, 1, 1}};

} // namespace

ORC_API void* orc_grid_create(float voxel, int res, int weight_dtype, int color_dtype) {
	Grid* g = new Grid();
	g->voxel = voxel;
	g->res = res;
	g->res3 = res * res * res;
	g->wdt = weight_dtype;
	g->cdt = color_dtype;
	return g;
}
ORC_API void orc_grid_destroy(void* h) { delete static_cast<Grid*>(h); }
ORC_API int64_t orc_grid_block_count(void* h) { return static_cast<int64_t>(static_cast<Grid*>(h)->keys.size()); }
ORC_API void orc_grid_block_coords(void* h, int32_t* out) {
	const Grid* g = static_cast<Grid*>(h);
	for (size_t b = 0; b < g->keys.size(); b++) {
		out[3 * b] = std::get<0>(g->keys[b]);
		out[3 * b + 1] = std::get<1>(g->keys[b]);
		out[3 * b + 2] = std::get<2>(g->keys[b]);
	}
}
ORC_API void orc_grid_activate(void* h, const int32_t* coords, int64_t n) { static_cast<Grid*>(h)->activate(coords, n); }

// Open3D DepthTouch: stride 4, 4 samples on [max(d - trunc, 0), min(d + trunc, dmax)]; unique in first-occurrence order
ORC_API int64_t orc_grid_touch(void* h, const void* depth, int dtype, int H, int W, const double* K, const double* E, float scale, float dmax,
                               float trunc_mult, int32_t* out, int64_t cap) {
	const Grid* g = static_cast<Grid*>(h);
	static const double I4[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
	double Ei[16];
	inverse4(E ? E : I4, Ei);
	const Cam c = make_cam(K, Ei);
	const Img im{depth, dtype, H, W, nullptr, 0, 0, scale, dmax};
	const float trunc = g->voxel * trunc_mult, bs = g->voxel * static_cast<float>(g->res);
	std::map<Key, bool> seen;
	int64_t n = 0;
	for (int yy = 0; yy < H / 4; yy++)
		for (int xx = 0; xx < W / 4; xx++) {
			const int x = xx * 4, y = yy * 4;
			const float d = im.d(x, y) / scale;
			if (!(d > 0.f && d < dmax)) continue;
			float xc, yc, zc, xg, yg, zg;
			c.unproject(static_cast<float>(x), static_cast<float>(y), 1.0f, xc, yc, zc);
			c.rigid(xc, yc, zc, xg, yg, zg);
			const float xo = c.m[3], yo = c.m[7], zo = c.m[11];
			const float xd = xg - xo, yd = yg - yo, zd = zg - zo;
			const float t0 = std::max(d - trunc, 0.0f), t1 = std::min(d + trunc, dmax);
			const float step = (t1 - t0) / 3.0f;
			float t = t0;
			for (int s = 0; s <= 3; s++, t += step) {
				const Key k(static_cast<int>(std::floor((xo + t * xd) / bs)), static_cast<int>(std::floor((yo + t * yd) / bs)),
				            static_cast<int>(std::floor((zo + t * zd) / bs)));
				if (seen.count(k)) continue;
				seen[k] = true;
				if (n < cap) {
					out[3 * n] = std::get<0>(k);
					out[3 * n + 1] = std::get<1>(k);
					out[3 * n + 2] = std::get<2>(k);
				}
				n++;
			}
		}
	return n;
}

// Open3D voxel_grid::Integrate over the listed blocks (activated first)
ORC_API void orc_grid_integrate(void* h, const int32_t* coords, int64_t n, const void* depth, int dtype, int H, int W, const void* color, int Hc,
                                int Wc, const double* Kd, const double* Kc, const double* E, float scale, float dmax, float trunc_mult) {
	Grid* g = static_cast<Grid*>(h);
	g->activate(coords, n);
	const Cam cd = make_cam(Kd, E), cc = make_cam(Kc ? Kc : Kd, nullptr);
	const Img im{depth, dtype, H, W, color, Hc, Wc, scale, dmax};
	const float trunc = g->voxel * trunc_mult, mult = dtype == DT_F32 ? 255.0f : 1.0f;
	for (int64_t i = 0; i < n; i++) {
		const int b = g->find(coords[3 * i], coords[3 * i + 1], coords[3 * i + 2]);
		for (int vi = 0; vi < g->res3; vi++) {
			int X, Y, Z;
			g->voxel_xyz(b, vi, X, Y, Z);
			const float x = static_cast<float>(X) * g->voxel, y = static_cast<float>(Y) * g->voxel, z = static_cast<float>(Z) * g->voxel;
			float xc, yc, zc, u, v;
			cd.rigid(x, y, z, xc, yc, zc);
			cd.project(xc, yc, zc, u, v);
			if (!in_bounds(u, v, H, W)) continue;
			int ui = static_cast<int>(std::round(u)), vr = static_cast<int>(std::round(v));
			const float dd = im.d(ui, vr) / scale;
			float sdf = dd - zc;
			if (dd <= 0.0f || dd > dmax || zc <= 0.0f || sdf < -trunc) continue;
			sdf = sdf < trunc ? sdf : trunc;
			sdf /= trunc;
			const int64_t lin = static_cast<int64_t>(b) * g->res3 + vi;
			const float w = g->weight[lin], inv = 1.0f / (w + 1);
			g->tsdf[lin] = (w * g->tsdf[lin] + sdf) * inv;
			if (g->cdt != DT_NONE && color) {
				float xu, yu, zu, uc, vc;
				cd.unproject(static_cast<float>(ui), static_cast<float>(vr), 1.0f, xu, yu, zu);
				cc.project(xu, yu, zu, uc, vc);
				if (in_bounds(uc, vc, Hc, Wc)) {
					ui = static_cast<int>(std::round(uc));
					vr = static_cast<int>(std::round(vc));
					for (int ch = 0; ch < 3; ch++)
						g->color[3 * lin + ch] = store_cast(g->cdt, (w * g->color[3 * lin + ch] + im.c(ui, vr, ch) * mult) * inv);
				}
			}
			g->weight[lin] = store_cast(g->wdt, w + 1);
		}
	}
}

// IntegrateNonRigid (NonRigidSurfaceVoxelBlockGridImpl.h:52-229) over all active blocks (after activating `coords`).
// apply_oblique_test = 0 drops the `cosine > 0.5` skip (used only to check the reference KAT, see tests).
ORC_API void orc_grid_integrate_non_rigid(void* h, const int32_t* coords, int64_t n, const float* nodes, const float* R, const float* t,
                                          const float* c2, int N, float coverage, int K, int min_valid, const void* depth, int dtype, int H, int W,
                                          const void* color, int Hc, int Wc, const float* normals, const double* Kd, const double* Kc,
                                          const double* E, float scale, float dmax, float trunc_mult, float* cos_out, int apply_oblique_test) {
	Grid* g = static_cast<Grid*>(h);
	g->activate(coords, n);
	const Field f{N, K, min_valid, nodes, R, t, c2, coverage};
	float range = 2.f * coverage;
	if (c2) {
		float mx = 0.f;
		for (int i = 0; i < N; i++) mx = std::max(mx, c2[i]);
		range = 2.f * std::sqrt(mx);
	}
	const Cam cd = make_cam(Kd, E), cc = make_cam(Kc ? Kc : Kd, nullptr);
	const Img im{depth, dtype, H, W, color, Hc, Wc, scale, dmax};
	const float trunc = g->voxel * trunc_mult, mult = dtype == DT_F32 ? 255.0f : 1.0f;
	std::fill(cos_out, cos_out + static_cast<int64_t>(H) * W, 0.f);
	for (size_t b = 0; b < g->keys.size(); b++)
		for (int vi = 0; vi < g->res3; vi++) {
			int X, Y, Z;
			g->voxel_xyz(static_cast<int>(b), vi, X, Y, Z);
			float p[3];
			cd.rigid(static_cast<float>(X) * g->voxel, static_cast<float>(Y) * g->voxel, static_cast<float>(Z) * g->voxel, p[0], p[1], p[2]);
			int idx[8];
			float w[8];
			if (!anchors(f, p, range, idx, w)) continue;
			float wp[3];
			blend(f, idx, w, p, wp);
			if (wp[2] < 0) continue;
			float u, v;
			cd.project(wp[0], wp[1], wp[2], u, v);
			if (!in_bounds(u, v, H, W)) continue;
			int ui = static_cast<int>(std::round(u)), vr = static_cast<int>(std::round(v));
			const float dd = im.d(ui, vr) / scale;
			if (dd <= 0.0f || dd > dmax) continue;
			const float psdf = dd - wp[2];
			float vd[3] = {-wp[0], -wp[1], -wp[2]};
			const float vn2 = (vd[0] * vd[0] + vd[1] * vd[1]) + vd[2] * vd[2];
			if (vn2 > 0.f) {
				const float vn = std::sqrt(vn2);
				for (float& q : vd) q /= vn;
			}
			const int64_t pix = static_cast<int64_t>(vr) * W + ui;
			const float cosine = (vd[0] * normals[3 * pix] + vd[1] * normals[3 * pix + 1]) + vd[2] * normals[3 * pix + 2];
			cos_out[pix] = cosine;   // racy in the reference; the serial last writer (highest voxel index) here and on the GPU
			if (psdf <= -trunc || (apply_oblique_test && cosine > 0.5f)) continue;
			const int64_t lin = static_cast<int64_t>(b) * g->res3 + vi;
			const float tn = (psdf < trunc ? psdf : trunc) / trunc;
			const float wt = g->weight[lin], inv = 1.0f / (wt + 1);
			g->tsdf[lin] = (wt * g->tsdf[lin] + tn) * inv;
			if (g->cdt != DT_NONE && color) {
				float xu, yu, zu, uc, vc;
				cd.unproject(static_cast<float>(ui), static_cast<float>(vr), 1.0f, xu, yu, zu);
				cc.project(xu, yu, zu, uc, vc);
				if (in_bounds(uc, vc, Hc, Wc)) {
					ui = static_cast<int>(std::round(uc));
					vr = static_cast<int>(std::round(vc));
					for (int ch = 0; ch < 3; ch++)
						g->color[3 * lin + ch] = store_cast(g->cdt, (wt * g->color[3 * lin + ch] + im.c(ui, vr, ch) * mult) * inv);
				}
			}
		}
}

// ExtractVoxelValuesAt (NonRigidSurfaceVoxelBlockGridImpl.h:581-652, global-coordinate indexing quirk reproduced);
// returns the number of rows (queries whose block x / res, y / res, z / res is active)
ORC_API int64_t orc_grid_values_at(void* h, const int32_t* q, int64_t n, float* out) {
	const Grid* g = static_cast<Grid*>(h);
	const int C = g->cdt != DT_NONE ? 8 : 5;
	int64_t rows = 0;
	for (int64_t i = 0; i < n; i++) {
		const int x = q[3 * i], y = q[3 * i + 1], z = q[3 * i + 2];
		const int b = g->find(x / g->res, y / g->res, z / g->res);
		if (b < 0) continue;
		float* o = out + rows * C;
		for (int c = 0; c < C; c++) o[c] = -2.f;
		const int64_t lin = static_cast<int64_t>(b) * g->res3 + (static_cast<int64_t>(x) + static_cast<int64_t>(g->res) * (y + static_cast<int64_t>(g->res) * z));
		rows++;
		if (lin < 0 || lin >= static_cast<int64_t>(g->tsdf.size())) continue;
		o[0] = static_cast<float>(x) * g->voxel;
		o[1] = static_cast<float>(y) * g->voxel;
		o[2] = static_cast<float>(z) * g->voxel;
		o[3] = g->tsdf[lin];
		o[4] = g->weight[lin];
		if (C > 5)
			for (int c = 0; c < 3; c++) o[5 + c] = g->color[3 * lin + c];
	}
	return rows;
}
ORC_API void orc_grid_values_all(void* h, float* out) {
	const Grid* g = static_cast<Grid*>(h);
	const int C = g->cdt != DT_NONE ? 8 : 5;
	for (size_t b = 0; b < g->keys.size(); b++)
		for (int vi = 0; vi < g->res3; vi++) {
			int X, Y, Z;
			g->voxel_xyz(static_cast<int>(b), vi, X, Y, Z);
			const int64_t lin = static_cast<int64_t>(b) * g->res3 + vi;
			float* o = out + lin * C;
			o[0] = static_cast<float>(X) * g->voxel;
			o[1] = static_cast<float>(Y) * g->voxel;
			o[2] = static_cast<float>(Z) * g->voxel;
			o[3] = g->tsdf[lin];
			o[4] = g->weight[lin];
			if (C > 5)
				for (int c = 0; c < 3; c++) o[5 + c] = g->color[3 * lin + c];
		}
}

// GetBoundingBoxesOfWarpedBlocks (NonRigidSurfaceVoxelBlockGridImpl.h:289-356), quirks as written (key used as the
// metric corner, if / else-if min-max, anchors' failure ignored: unnormalized weights then)
ORC_API void orc_warped_block_boxes(const int32_t* keys, int64_t n, float side, const float* nodes, const float* R, const float* t, int N,
                                    float coverage, int K, int min_valid, const double* E, float* boxes) {
	const Cam ex = make_cam(nullptr, E);
	const Field f{N, K, min_valid, nodes, R, t, nullptr, coverage};
	for (int64_t i = 0; i < n; i++) {
		const float x0 = static_cast<float>(keys[3 * i]), y0 = static_cast<float>(keys[3 * i + 1]), z0 = static_cast<float>(keys[3 * i + 2]);
		const float x1 = x0 + side, y1 = y0 + side, z1 = z0 + side;
		const float cs[8][3] = {{x0, y0, z0}, {x0, y0, z1}, {x0, y1, z0}, {x1, y0, z0}, {x0, y1, z1}, {x1, y0, z1}, {x1, y1, z0}, {x1, y1, z1}};
		float mn[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, mx[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
		for (const auto& c : cs) {
			float p[3];
			ex.rigid(c[0], c[1], c[2], p[0], p[1], p[2]);
			int idx[8];
			float w[8];
			// nodes within 2 c (the only possible valid anchors; both implementations search those), fixed coverage; the
			// result is used whatever the valid count (anchors() returns before normalizing when valid < min_valid: the raw
			// Gaussian weights are blended then)
			anchors(f, p, 2.f * coverage, idx, w);
			float wp[3];
			blend(f, idx, w, p, wp);
			for (int k = 0; k < 3; k++) {
				if (mn[k] > wp[k]) mn[k] = wp[k];
				else if (mx[k] < wp[k]) mx[k] = wp[k];
			}
		}
		for (int k = 0; k < 3; k++) {
			boxes[6 * i + k] = mn[k];
			boxes[6 * i + 3 + k] = mx[k];
		}
	}
}

// GetAxisAlignedBoxesInterceptingSurfaceMask (NonRigidSurfaceVoxelBlockGridImpl.h:359-437) + Segment.h
ORC_API void orc_boxes_mask(const float* boxes, int64_t n, const void* depth, int dtype, int H, int W, const double* K, float scale, float dmax,
                            int stride, float trunc, uint8_t* mask) {
	const Cam c = make_cam(K, nullptr);
	const Img im{depth, dtype, H, W, nullptr, 0, 0, scale, dmax};
	struct S {
		float o[3], inv[3];
		int sign[3];
	};
	std::vector<S> segs;
	for (int yy = 0; yy < H / stride; yy++)
		for (int xx = 0; xx < W / stride; xx++) {
			const int u = xx * stride, v = yy * stride;
			const float d = im.d(u, v) / scale;
			if (!(d > 0 && d < dmax)) continue;
			float a[3], e[3];
			c.unproject(static_cast<float>(u), static_cast<float>(v), d - trunc, a[0], a[1], a[2]);
			c.unproject(static_cast<float>(u), static_cast<float>(v), d + trunc, e[0], e[1], e[2]);
			S s;
			for (int k = 0; k < 3; k++) {
				s.o[k] = a[k];
				s.inv[k] = 1.f / (e[k] - a[k]);
				s.sign[k] = s.inv[k] < 0;
			}
			segs.push_back(s);
		}
	for (int64_t i = 0; i < n; i++) {
		const float* bounds[2] = {boxes + 6 * i, boxes + 6 * i + 3};
		mask[i] = 0;
		for (const S& s : segs) {
			float t0 = (bounds[s.sign[0]][0] - s.o[0]) * s.inv[0], t1 = (bounds[1 - s.sign[0]][0] - s.o[0]) * s.inv[0];
			const float y0 = (bounds[s.sign[1]][1] - s.o[1]) * s.inv[1], y1 = (bounds[1 - s.sign[1]][1] - s.o[1]) * s.inv[1];
			if (t0 > y1 || y0 > t1) continue;
			if (y0 > t0) t0 = y0;
			if (y1 < t1) t1 = y1;
			const float z0 = (bounds[s.sign[2]][2] - s.o[2]) * s.inv[2], z1 = (bounds[1 - s.sign[2]][2] - s.o[2]) * s.inv[2];
			if (t0 > z1 || z0 > t1) continue;
			if (z0 > t0) t0 = z0;
			if (z1 < t1) t1 = z1;
			if (!(t1 < 0.0f || t0 > 1.0f)) {
				mask[i] = 1;
				break;
			}
		}
	}
}

// inactive neighbours of the active blocks, neighbour-major (NonRigidSurfaceVoxelBlockGrid.cpp:68-96), duplicates kept
ORC_API int64_t orc_grid_inactive_neighbors(void* h, int32_t* out, int64_t cap) {
	const Grid* g = static_cast<Grid*>(h);
	int64_t n = 0;
	for (int nb = 0; nb < 27; nb++)
		for (size_t b = 0; b < g->keys.size(); b++) {
			const int x = std::get<0>(g->keys[b]) + nb % 3 - 1, y = std::get<1>(g->keys[b]) + (nb % 9) / 3 - 1, z = std::get<2>(g->keys[b]) + nb / 9 - 1;
			if (g->find(x, y, z) >= 0) continue;
			if (n < cap) {
				out[3 * n] = x;
				out[3 * n + 1] = y;
				out[3 * n + 2] = z;
			}
			n++;
		}
	return n;
}

// ExtractTriangleMesh: vertices on owned edges of valid surface cubes (blocks in activation order, voxels in block order,
// edges x, y, z), normals from interpolated central-difference gradients (missing neighbour -> centre value), colors
// interpolated / 255; returns (vertex count, triangle count) through the pointers
ORC_API void orc_grid_mesh(void* h, float weight_threshold, float* vpos, float* vnrm, float* vcol, int64_t* tris, int64_t vcap, int64_t tcap,
                           int64_t* nv_out, int64_t* nt_out) {
	const Grid* g = static_cast<Grid*>(h);
	const McTable& T = mc_table();
	const int64_t nvox = static_cast<int64_t>(g->keys.size()) * g->res3;
	std::vector<uint8_t> cube(nvox, 0);
	std::vector<int64_t> vid(3 * nvox, -1);
	std::vector<uint8_t> need(3 * nvox, 0);
	auto tsdf_or = [&](int x, int y, int z, float fb) {
		const int64_t v = g->at(x, y, z);
		return v < 0 ? fb : g->tsdf[v];
	};
	for (size_t b = 0; b < g->keys.size(); b++)
		for (int vi = 0; vi < g->res3; vi++) {
			int X, Y, Z;
			g->voxel_xyz(static_cast<int>(b), vi, X, Y, Z);
			int idx = 0;
			bool ok = true;
			for (int c = 0; c < 8 && ok; c++) {
				const int64_t v = g->at(X + k_corner[c][0], Y + k_corner[c][1], Z + k_corner[c][2]);
				if (v < 0 || !(g->weight[v] > weight_threshold)) ok = false;
				else if (g->tsdf[v] < 0) idx |= 1 << c;
			}
			if (!ok || idx == 0 || idx == 255) continue;
			const int64_t w = static_cast<int64_t>(b) * g->res3 + vi;
			cube[w] = static_cast<uint8_t>(idx);
			for (int e = 0; e < 12; e++)
				if (T.mask[idx] >> e & 1) need[3 * g->at(X + k_owner[e][0], Y + k_owner[e][1], Z + k_owner[e][2]) + k_owner[e][3]] = 1;
		}
	int64_t nv = 0;
	for (int64_t i = 0; i < 3 * nvox; i++) {
		if (!need[i]) continue;
		const int64_t w = i / 3;
		const int d = static_cast<int>(i % 3);
		int X, Y, Z;
		g->voxel_xyz(static_cast<int>(w / g->res3), static_cast<int>(w % g->res3), X, Y, Z);
		const int ex = d == 0, ey = d == 1, ez = d == 2;
		const int64_t ve = g->at(X + ex, Y + ey, Z + ez);
		const float to = g->tsdf[w], te = g->tsdf[ve];
		const float r = (0.0f - to) / (te - to);
		if (nv < vcap) {
			vpos[3 * nv] = (static_cast<float>(X) + r * ex) * g->voxel;
			vpos[3 * nv + 1] = (static_cast<float>(Y) + r * ey) * g->voxel;
			vpos[3 * nv + 2] = (static_cast<float>(Z) + r * ez) * g->voxel;
			const float no[3] = {tsdf_or(X + 1, Y, Z, to) - tsdf_or(X - 1, Y, Z, to), tsdf_or(X, Y + 1, Z, to) - tsdf_or(X, Y - 1, Z, to),
			                     tsdf_or(X, Y, Z + 1, to) - tsdf_or(X, Y, Z - 1, to)};
			const int Xe = X + ex, Ye = Y + ey, Ze = Z + ez;
			const float ne[3] = {tsdf_or(Xe + 1, Ye, Ze, te) - tsdf_or(Xe - 1, Ye, Ze, te), tsdf_or(Xe, Ye + 1, Ze, te) - tsdf_or(Xe, Ye - 1, Ze, te),
			                     tsdf_or(Xe, Ye, Ze + 1, te) - tsdf_or(Xe, Ye, Ze - 1, te)};
			float n[3];
			for (int k = 0; k < 3; k++) n[k] = (1 - r) * no[k] + r * ne[k];
			const float nn = std::sqrt((n[0] * n[0] + n[1] * n[1]) + n[2] * n[2]);
			for (int k = 0; k < 3; k++) vnrm[3 * nv + k] = nn > 0.f ? n[k] / nn : 0.f;
			if (vcol && g->cdt != DT_NONE)
				for (int k = 0; k < 3; k++) vcol[3 * nv + k] = ((1 - r) * g->color[3 * w + k] + r * g->color[3 * ve + k]) / 255.0f;
		}
		vid[i] = nv++;
	}
	int64_t nt = 0;
	for (int64_t w = 0; w < nvox; w++) {
		if (!cube[w]) continue;
		int X, Y, Z;
		g->voxel_xyz(static_cast<int>(w / g->res3), static_cast<int>(w % g->res3), X, Y, Z);
		const auto& tri = T.tri[cube[w]];
		for (size_t k = 0; k < tri.size(); k += 3, nt++)
			for (int j = 0; j < 3; j++) {
				const int e = tri[k + j];
				if (nt < tcap) tris[3 * nt + j] = vid[3 * g->at(X + k_owner[e][0], Y + k_owner[e][1], Z + k_owner[e][2]) + k_owner[e][3]];
			}
	}
	*nv_out = nv;
	*nt_out = nt;
}

// test helper: overwrite every voxel's tsdf / weight (block order, voxel order)
ORC_API void orc_grid_set_values(void* h, const float* tsdf, const float* weight) {
	Grid* g = static_cast<Grid*>(h);
	std::copy(tsdf, tsdf + g->tsdf.size(), g->tsdf.begin());
	std::copy(weight, weight + g->weight.size(), g->weight.begin());
}

// the table in emission order (tests): tri [256][16] int8 edge triples, -1 terminated
ORC_API int orc_marching_cubes_table(int8_t* tri) {
	const McTable& T = mc_table();
	for (int cfg = 0; cfg < 256; cfg++)
		for (int i = 0; i < 16; i++) tri[16 * cfg + i] = i < static_cast<int>(T.tri[cfg].size()) ? static_cast<int8_t>(T.tri[cfg][i]) : -1;
	return 0;
}
