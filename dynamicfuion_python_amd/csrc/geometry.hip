// Geometry stages of the hot path on gfx950: anchors (once per frame), mesh warp (+ warped-surface Jacobians),
// NDC face extraction, depth unprojection, attribute interpolation, Rodrigues.
#include "kernels.hpp"

#include <cstdlib>

namespace nnrt {

// =====================================================================================================================
// Anchors: brute-force K-NN in ascending node order with replace-the-current-maximum insertion
// (cpp/core/kernel/KnnUtilities.h:64-117) + Gaussian weights (WarpUtilities.h:34-247, WarpAnchorComputationImpl.h:42-140).
// One lane per point, one wave per workgroup. Nodes are loaded 64 at a time (one per lane, a batch ahead) and
// broadcast by readlane (SGPR operands, no LDS); squared distances of a group of ANCHOR_UNROLL nodes are formed with packed f32
// (the reference's (dx dx + dy dy) + dz dz, no contraction); only the group's nodes that some lane has below its
// current maximum at the group's start run the insertion (maxd only decreases, so every other node would have been
// skipped by the serial loop too), in node order, exactly as the serial loop.
// =====================================================================================================================
constexpr int ANCHOR_BLOCK = 64;
constexpr int ANCHOR_UNROLL = 8;

__device__ inline float lane_read(float v, int src) {
	return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), src));
}

template <int K>
__global__ __launch_bounds__(ANCHOR_BLOCK) void k_compute_anchors(const float* __restrict__ points, int64_t point_count,
                                                                    const float* __restrict__ nodes, int node_count,
                                                                    float coverage_squared, const float* __restrict__ node_weights,
                                                                    int threshold, int minimum_valid, int32_t* __restrict__ anchors,
                                                                    float* __restrict__ weights) {
	typedef float f2 __attribute__((ext_vector_type(2)));
	const int64_t i = static_cast<int64_t>(blockIdx.x) * ANCHOR_BLOCK + threadIdx.x;
	const bool active = i < point_count;
	float px = 0.f, py = 0.f, pz = 0.f;
	if (active) {
		px = points[3 * i];
		py = points[3 * i + 1];
		pz = points[3 * i + 2];
	}
	int32_t idx[K];
	float d2[K];
#pragma unroll
	for (int k = 0; k < K; k++) {
		idx[k] = -1;
		d2[k] = INFINITY;
	}
	int max_at = 0;
	float maxd = active ? INFINITY : -INFINITY;   // inactive lanes never insert
	auto insert = [&](float sq, int j) {
		if (sq < maxd) {
#pragma unroll
			for (int k = 0; k < K; k++) {
				if (k == max_at) {
					d2[k] = sq;
					idx[k] = j;
				}
			}
			max_at = 0;
			maxd = d2[0];
#pragma unroll
			for (int k = 1; k < K; k++) {
				if (d2[k] > maxd) {
					max_at = k;
					maxd = d2[k];
				}
			}
		}
	};
	const f2 PX = {px, px}, PY = {py, py}, PZ = {pz, pz};
	// batches of 64 nodes: lane l loads node base + l (coalesced, one batch ahead); the batch's coordinates are then
	// broadcast to the wave by readlane (SGPR operands)
	const int full = node_count - node_count % 64;
	float bx = 0.f, by = 0.f, bz = 0.f;
	const int lane = static_cast<int>(threadIdx.x & 63);
	if (full > 0) {
		bx = nodes[3 * lane];
		by = nodes[3 * lane + 1];
		bz = nodes[3 * lane + 2];
	}
	for (int base = 0; base < full; base += 64) {
		const float cx = bx, cy = by, cz = bz;
		if (base + 64 < full) {
			const int64_t j = base + 64 + lane;
			bx = nodes[3 * j];
			by = nodes[3 * j + 1];
			bz = nodes[3 * j + 2];
		}
#pragma unroll
		for (int g = 0; g < 64; g += ANCHOR_UNROLL) {
			float sq[ANCHOR_UNROLL];
#pragma unroll
			for (int q = 0; q < ANCHOR_UNROLL; q += 2) {
				const f2 dx = f2{lane_read(cx, g + q), lane_read(cx, g + q + 1)} - PX;
				const f2 dy = f2{lane_read(cy, g + q), lane_read(cy, g + q + 1)} - PY;
				const f2 dz = f2{lane_read(cz, g + q), lane_read(cz, g + q + 1)} - PZ;
				const f2 s2 = (dx * dx + dy * dy) + dz * dz;
				sq[q] = s2.x;
				sq[q + 1] = s2.y;
			}
			// the group runs the (divergent, node-ordered) insertions only if some lane has one of its distances below its
			// maximum at the group's start (maxd only decreases, so otherwise the serial loop would skip all of them)
			float m = sq[0];
#pragma unroll
			for (int q = 1; q < ANCHOR_UNROLL; q++) m = fminf(m, sq[q]);
			if (__any(m < maxd)) {
#pragma unroll
				for (int q = 0; q < ANCHOR_UNROLL; q++) insert(sq[q], base + g + q);
			}
		}
	}
	for (int j = full; j < node_count; j++) {
		const float dx = nodes[3 * j] - px, dy = nodes[3 * j + 1] - py, dz = nodes[3 * j + 2] - pz;
		insert((dx * dx + dy * dy) + dz * dz, j);
	}
	if (!active) return;
	float w[K];
	float sum = 0.f;
	int valid = 0;
	bool normalize = true;
	if (threshold) {
#pragma unroll
		for (int k = 0; k < K; k++) {
			// a slot left empty (node_count < K: index -1, distance inf) fails the 2c test whatever its c^2 (the reference
			// reads node_weights[-1] there)
			const float c2 = node_weights ? (idx[k] >= 0 ? node_weights[idx[k]] : 1.f) : coverage_squared;
			w[k] = d2[k];   // reference repurposes the weight array for squared distances
			if (d2[k] > 4 * c2) {
				idx[k] = -1;
				continue;
			}
			const float wt = exp_cr(-d2[k] / (2 * c2));
			sum += wt;
			w[k] = wt;
			valid++;
		}
		if (valid < minimum_valid) normalize = false;   // WarpUtilities.h:242-244
	} else {
#pragma unroll
		for (int k = 0; k < K; k++) {
			const float c2 = node_weights ? (idx[k] >= 0 ? node_weights[idx[k]] : 1.f) : coverage_squared;   // empty slot: exp(-inf) = 0
			const float wt = exp_cr(-d2[k] / (2 * c2));
			sum += wt;
			w[k] = wt;
		}
		valid = K;
	}
	if (normalize) {
		if (sum > 0.0f) {
#pragma unroll
			for (int k = 0; k < K; k++) w[k] /= sum;
		} else if (valid > 0) {
#pragma unroll
			for (int k = 0; k < K; k++) w[k] = 1.0f / static_cast<float>(valid);
		}
	}
#pragma unroll
	for (int k = 0; k < K; k++) {
		anchors[i * K + k] = idx[k];
		weights[i * K + k] = w[k];
	}
}

nnrt_status launch_compute_anchors(const float* points, int64_t V, const float* nodes, int N, int K, float coverage,
                                   const float* node_weights, int minimum_valid, int32_t* anchors, float* weights, hipStream_t stream,
                                   int threshold) {
	if (threshold < 0) threshold = minimum_valid > 0;   // WarpAnchorComputation.cpp (kernel dispatch): threshold iff minimum > 0
	NNRT_CHECK_ARG(K >= 1 && K <= MAX_ANCHORS, "anchor_count must be in [1, 8]");
	NNRT_CHECK_ARG(N >= 0, "negative node count");   // N < K leaves slots at -1 with weight 0 (the reference's brute-force K-NN)
	if (V == 0) return NNRT_OK;
	const dim3 grid(static_cast<unsigned>(ceil_div(V, ANCHOR_BLOCK)));
	const float c2 = coverage * coverage;
#define NNRT_ANCHOR_CASE(KK)                                                                                                 \
	case KK:                                                                                                                 \
		k_compute_anchors<KK><<<grid, ANCHOR_BLOCK, 0, stream>>>(points, V, nodes, N, c2, node_weights, threshold, minimum_valid, anchors, weights); \
		break;
	switch (K) {
		NNRT_ANCHOR_CASE(1)
		NNRT_ANCHOR_CASE(2)
		NNRT_ANCHOR_CASE(3)
		NNRT_ANCHOR_CASE(4)
		NNRT_ANCHOR_CASE(5)
		NNRT_ANCHOR_CASE(6)
		NNRT_ANCHOR_CASE(7)
		NNRT_ANCHOR_CASE(8)
	}
#undef NNRT_ANCHOR_CASE
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

// =====================================================================================================================
// Warp + warped-surface Jacobians, fused (S1 + S6). One thread per vertex.
//   warped point  v' = sum_k w_k (g_k + R_k (E v - g_k) + t_k)        Warp3dPointsAndNormalsImpl.h:334-390, WarpUtilities.h:448-467
//   warped normal n' = sum_k w_k R_k (E_R n)    (not normalized: A12)
//   Jv[v,k] = (-w R_k (v - g_k), w) ; Jn[v,k] = -w R_k n   (canonical v, n)   WarpedSurfaceJacobiansImpl.h:117-156
// Outputs: float4 warped positions / normals [V] (w unused), Jacobian rows [V,K] of 24 B (store_jacobian_row).
// =====================================================================================================================
__global__ __launch_bounds__(256) void k_warp_mesh(const float* __restrict__ points, const float* __restrict__ normals, int64_t V,
                                                   const float* __restrict__ node_state, const int32_t* __restrict__ anchors,
                                                   const float* __restrict__ weights, int K, WarpExtrinsics E, float4* __restrict__ out_p,
                                                   float4* __restrict__ out_n, float2* __restrict__ jrows) {
	const int64_t v = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (v >= V) return;
	const f3 p = make3(points[3 * v], points[3 * v + 1], points[3 * v + 2]);
	const f3 n = make3(normals[3 * v], normals[3 * v + 1], normals[3 * v + 2]);
	f3 pc = p, nc = n;
	if (!E.identity) {
		pc = make3(((p.x * E.m[0] + p.y * E.m[1]) + p.z * E.m[2]) + E.m[3], ((p.x * E.m[4] + p.y * E.m[5]) + p.z * E.m[6]) + E.m[7],
		           ((p.x * E.m[8] + p.y * E.m[9]) + p.z * E.m[10]) + E.m[11]);
		nc = make3((n.x * E.m[0] + n.y * E.m[1]) + n.z * E.m[2], (n.x * E.m[4] + n.y * E.m[5]) + n.z * E.m[6],
		           (n.x * E.m[8] + n.y * E.m[9]) + n.z * E.m[10]);
	}
	f3 wp = make3(0.f, 0.f, 0.f), wn = make3(0.f, 0.f, 0.f);
	for (int k = 0; k < K; k++) {
		const int32_t a = anchors[v * K + k];
		float4 ojv = make_float4(0.f, 0.f, 0.f, 0.f), ojn = make_float4(0.f, 0.f, 0.f, 0.f);
		if (a != -1) {
			const float w = weights[v * K + k];
			const float* ns = node_state + static_cast<int64_t>(a) * NODE_STRIDE;
			const f3 g = make3(ns[0], ns[1], ns[2]);
			const f3 t = make3(ns[3], ns[4], ns[5]);
			const float* R = ns + 6;
			const f3 Rd = matvec3(R, sub3(pc, g));
			wp.x += w * ((g.x + Rd.x) + t.x);
			wp.y += w * ((g.y + Rd.y) + t.y);
			wp.z += w * ((g.z + Rd.z) + t.z);
			const f3 Rn = matvec3(R, nc);
			wn.x += w * Rn.x;
			wn.y += w * Rn.y;
			wn.z += w * Rn.z;
			{
				const f3 Rj = E.identity ? Rd : matvec3(R, sub3(p, g));
				const f3 Rnj = E.identity ? Rn : matvec3(R, n);
				ojv = make_float4(-w * Rj.x, -w * Rj.y, -w * Rj.z, w);
				ojn = make_float4(-w * Rnj.x, -w * Rnj.y, -w * Rnj.z, 0.f);
			}
		}
		if (jrows) store_jacobian_row(jrows, v * K + k, ojv, ojn);
	}
	out_p[v] = make_float4(wp.x, wp.y, wp.z, 0.f);
	out_n[v] = make_float4(wn.x, wn.y, wn.z, 0.f);
}

// K <= 4: one lane per (vertex, anchor slot) -- 4x the waves of a lane-per-vertex launch, so the node-state gathers of
// neighbouring lanes are in flight together; Jv/Jn rows are stored coalesced (lane = slot). The quad's slot-0 lane sums
// the slot contributions in slot order (DPP quad broadcasts), the reference's serial accumulation order.
template <int CTRL>
__device__ inline float quad_bcast(float x) {
	return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xf, 0xf, false));
}

// IDENTITY: every node at R = I, t = 0 without reading them (iterate-from-identity, the benchmark protocol); the
// arithmetic is the same as with the identity loaded from memory.
#ifdef NNRT_KERNEL_STAMPS
__device__ unsigned long long g_warp_stamps[16384][4];
extern "C" int nnrt_dev_warp_stamps(unsigned long long* out) {
	return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_warp_stamps), sizeof(g_warp_stamps)) == hipSuccess ? 0 : 1;
}
#endif

// workgroups per launch, the quads strided over them (development; round 5: a cap of 1024 / 2048 -- every wave
// resident, looping -- measured 74.0 / 67.8 µs at C3 against 62.4 µs with one quad step per lane)
#ifndef NNRT_WARP_MAX_WGS
#define NNRT_WARP_MAX_WGS (int64_t{1} << 40)
#endif
constexpr int64_t WARP_MAX_WGS = NNRT_WARP_MAX_WGS;
#ifndef NNRT_WARP_UNROLL
#define NNRT_WARP_UNROLL 1
#endif
constexpr int WARP_UNROLL = NNRT_WARP_UNROLL;
template <bool IDENTITY>
__global__ __launch_bounds__(256) void k_warp_mesh_quad(const float* __restrict__ points, const float* __restrict__ normals, int64_t V,
                                                        const float* __restrict__ node_state, const int32_t* __restrict__ anchors,
                                                        const float* __restrict__ weights, int K, WarpExtrinsics E, float4* __restrict__ out_p,
                                                        float4* __restrict__ out_n, float2* __restrict__ jrows) {
	NNRT_WAVE_STAMP(g_warp_stamps, 0, __builtin_amdgcn_s_memrealtime());
	NNRT_WAVE_STAMP(g_warp_stamps, 3, NNRT_STAMP_HWID());
	// The input loads (canonical vertex, normal, anchor, weight) are issued unconditionally at clamped indices, so they
	// leave together ahead of the node-state gathers (round 5: C3 74.7 -> 62.4 µs against the loads inside the
	// `slot_ok` branch). WARP_UNROLL quads per lane per step (development: 2 / 4 measured no faster -- the extra
	// registers cost waves) over a workgroup-strided loop (one step per lane unless WARP_MAX_WGS caps the launch).
	constexpr int U = WARP_UNROLL;
	const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
	for (int64_t base = static_cast<int64_t>(blockIdx.x) * blockDim.x; base < 4 * V; base += U * stride) {
		int64_t v[U];
		int k[U];
		bool vertex_ok[U], slot_ok[U];
		f3 p[U], n[U];
		int32_t a[U];
		float w[U];
#pragma unroll
		for (int u = 0; u < U; u++) {   // inputs (clamped indices: every load is issued, the unused ones ignored)
			const int64_t tid = base + u * stride + threadIdx.x;
			v[u] = tid >> 2;
			k[u] = static_cast<int>(tid & 3);
			vertex_ok[u] = v[u] < V;
			slot_ok[u] = vertex_ok[u] && k[u] < K;
			const int64_t vv = vertex_ok[u] ? v[u] : 0;
			const int kk = slot_ok[u] ? k[u] : 0;
			p[u] = make3(points[3 * vv], points[3 * vv + 1], points[3 * vv + 2]);
			n[u] = make3(normals[3 * vv], normals[3 * vv + 1], normals[3 * vv + 2]);
			a[u] = anchors[vv * K + kk];
			w[u] = weights[vv * K + kk];
		}
#pragma unroll
		for (int u = 0; u < U; u++) {
			f3 cp = make3(0.f, 0.f, 0.f), cn = make3(0.f, 0.f, 0.f);   // this slot's contribution
			const bool valid = slot_ok[u] && a[u] != -1;
			{
				f3 pc = p[u], nc = n[u];
				if (!E.identity) {
					pc = apply_extrinsics_point(E, p[u]);
					nc = apply_extrinsics_normal(E, n[u]);
				}
				float4 ojv = make_float4(0.f, 0.f, 0.f, 0.f), ojn = make_float4(0.f, 0.f, 0.f, 0.f);
				if (valid) warp_slot<IDENTITY>(node_state, a[u], w[u], p[u], n[u], pc, nc, E.identity, cp, cn, ojv, ojn);
				if (jrows && slot_ok[u]) store_jacobian_row(jrows, v[u] * K + k[u], ojv, ojn);
			}
			// serial slot-order sum on the quad's first lane: ((0 + c0) + c1) + c2) + c3, skipping invalid anchors
			const float vf = valid ? 1.f : 0.f;
			float c[4][7];
			const float mine[7] = {cp.x, cp.y, cp.z, cn.x, cn.y, cn.z, vf};
#pragma unroll
			for (int i = 0; i < 7; i++) {
				c[0][i] = quad_bcast<0x00>(mine[i]);
				c[1][i] = quad_bcast<0x55>(mine[i]);
				c[2][i] = quad_bcast<0xAA>(mine[i]);
				c[3][i] = quad_bcast<0xFF>(mine[i]);
			}
			if (vertex_ok[u] && k[u] == 0) {
				float acc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
				for (int q = 0; q < 4; q++) {
					if (q >= K || c[q][6] == 0.f) continue;
#pragma unroll
					for (int i = 0; i < 6; i++) acc[i] += c[q][i];
				}
				out_p[v[u]] = make_float4(acc[0], acc[1], acc[2], 0.f);
				out_n[v[u]] = make_float4(acc[3], acc[4], acc[5], 0.f);
			}
		}
	}
	NNRT_WAVE_STAMP(g_warp_stamps, 2, __builtin_amdgcn_s_memrealtime());
}

// Meshes of 64 k vertices and more (C1 / C2 / C5: 77 k, C3: 2.25 M): one lane per vertex, its K <= 4 anchor slots' loads (anchors and weights as one
// 16-B load each when K = 4) and node-state gathers issued together, the slots summed in slot order as the quad kernel's
// slot-0 lane sums them (warp_slot's contributions, invalid slots skipped): bit-identical positions and normals, a
// quarter of the waves, four gathers in flight per lane (round 6; the quad kernel's 140 k waves ran 17 residency rounds
// of two dependent memory round trips each: C3 61.7 -> 45 us; C2 4.9 -> 4.7 us). Smaller meshes keep the quad kernel's
// four lanes per vertex (more waves for a launch that is mostly latency). Positions and normals only (the fitter's warp:
// no Jacobian rows).
template <bool IDENTITY, bool VEC4>
__global__ __launch_bounds__(256) void k_warp_mesh_vertex(const float* __restrict__ points, const float* __restrict__ normals, int64_t V,
                                                          const float* __restrict__ node_state, const int32_t* __restrict__ anchors,
                                                          const float* __restrict__ weights, int K, WarpExtrinsics E, float4* __restrict__ out_p,
                                                          float4* __restrict__ out_n, const uint2* __restrict__ anchors16) {
	const int64_t v = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (v >= V) return;
	const f3 p = make3(points[3 * v], points[3 * v + 1], points[3 * v + 2]);
	const f3 n = make3(normals[3 * v], normals[3 * v + 1], normals[3 * v + 2]);
	int32_t a[4];
	float w[4];
	if constexpr (VEC4) {
		if (anchors16) {   // the per-frame 16-bit copy (launch_pack_anchors16): 8 B per vertex instead of 16
			const uint2 q = anchors16[v];
			const uint32_t h[4] = {q.x & 0xFFFFu, q.x >> 16, q.y & 0xFFFFu, q.y >> 16};
#pragma unroll
			for (int k = 0; k < 4; k++) a[k] = h[k] == 0xFFFFu ? -1 : static_cast<int32_t>(h[k]);
		} else {
			const int4 a4 = reinterpret_cast<const int4*>(anchors)[v];
			a[0] = a4.x, a[1] = a4.y, a[2] = a4.z, a[3] = a4.w;
		}
		const float4 w4 = reinterpret_cast<const float4*>(weights)[v];
		w[0] = w4.x, w[1] = w4.y, w[2] = w4.z, w[3] = w4.w;
	} else {
#pragma unroll
		for (int k = 0; k < 4; k++) {
			a[k] = k < K ? anchors[v * K + k] : -1;
			w[k] = k < K ? weights[v * K + k] : 0.f;
		}
	}
	f3 pc = p, nc = n;
	if (!E.identity) {
		pc = apply_extrinsics_point(E, p);
		nc = apply_extrinsics_normal(E, n);
	}
	// every slot's node state first (clamped indices, no branch: the four gathers leave together)
	float4 ns[4][4];
#pragma unroll
	for (int k = 0; k < 4; k++) load_warp_state<IDENTITY>(node_state, (k < K && a[k] != -1) ? a[k] : 0, ns[k]);
	f3 wp = make3(0.f, 0.f, 0.f), wn = make3(0.f, 0.f, 0.f);
#pragma unroll
	for (int k = 0; k < 4; k++) {
		const bool valid = k < K && a[k] != -1;
		f3 cp, cn;
		float4 ojv, ojn;   // (unused: no rows on this path)
		warp_slot_state<IDENTITY>(ns[k], w[k], p, n, pc, nc, E.identity, cp, cn, ojv, ojn);
		if (valid) {
			wp.x += cp.x;
			wp.y += cp.y;
			wp.z += cp.z;
			wn.x += cn.x;
			wn.y += cn.y;
			wn.z += cn.z;
		}
	}
	out_p[v] = make_float4(wp.x, wp.y, wp.z, 0.f);
	out_n[v] = make_float4(wn.x, wn.y, wn.z, 0.f);
}

static bool warp_vertex_path(int64_t V) {
	if (const char* e = std::getenv("NNRT_WARP_VERTEX")) return *e == '1';   // development switch: 0 / 1 force a path
	return V >= (int64_t{1} << 16);
}

// [V, 4] int32 anchors (every index < 65535, -1 for none) -> 4 x 16 bits per vertex (0xFFFF: none), for the
// lane-per-vertex warp's anchor loads (C3: 36 of its ~200 MB per launch as int32)
__global__ void k_pack_anchors16(const int4* __restrict__ anchors, int64_t V, uint2* __restrict__ out) {
	const int64_t v = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (v >= V) return;
	const int4 a = anchors[v];
	auto h = [](int x) { return x < 0 ? 0xFFFFu : static_cast<uint32_t>(x); };
	out[v] = make_uint2(h(a.x) | h(a.y) << 16, h(a.z) | h(a.w) << 16);
}
nnrt_status launch_pack_anchors16(const int32_t* anchors, int64_t V, uint2* out, hipStream_t stream) {
	if (V == 0) return NNRT_OK;
	k_pack_anchors16<<<static_cast<unsigned>(ceil_div(V, 256)), 256, 0, stream>>>(reinterpret_cast<const int4*>(anchors), V, out);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

nnrt_status launch_warp_mesh(const float* points, const float* normals, int64_t V, const float* node_state, const int32_t* anchors,
                             const float* weights, int K, const WarpExtrinsics& E, float4* out_p, float4* out_n, float2* jrows,
                             hipStream_t stream, bool from_identity, const uint2* anchors16) {
	if (V == 0) return NNRT_OK;
	if (K <= 4 && !jrows && warp_vertex_path(V)) {
		const unsigned grid = static_cast<unsigned>(ceil_div(V, 256));
		const bool vec4 = K == 4 && (reinterpret_cast<uintptr_t>(anchors) & 15) == 0 && (reinterpret_cast<uintptr_t>(weights) & 15) == 0;
		if (from_identity) {
			if (vec4) k_warp_mesh_vertex<true, true><<<grid, 256, 0, stream>>>(points, normals, V, node_state, anchors, weights, K, E, out_p, out_n, vec4 ? anchors16 : nullptr);
			else k_warp_mesh_vertex<true, false><<<grid, 256, 0, stream>>>(points, normals, V, node_state, anchors, weights, K, E, out_p, out_n, vec4 ? anchors16 : nullptr);
		} else {
			if (vec4) k_warp_mesh_vertex<false, true><<<grid, 256, 0, stream>>>(points, normals, V, node_state, anchors, weights, K, E, out_p, out_n, vec4 ? anchors16 : nullptr);
			else k_warp_mesh_vertex<false, false><<<grid, 256, 0, stream>>>(points, normals, V, node_state, anchors, weights, K, E, out_p, out_n, vec4 ? anchors16 : nullptr);
		}
		NNRT_LAUNCH_CHECK();
		return NNRT_OK;
	}
	if (K <= 4) {
		const unsigned grid = static_cast<unsigned>(std::min<int64_t>(ceil_div(4 * V, 256), WARP_MAX_WGS));
		if (from_identity)
			k_warp_mesh_quad<true><<<grid, 256, 0, stream>>>(points, normals, V, node_state, anchors, weights, K, E, out_p, out_n, jrows);
		else
			k_warp_mesh_quad<false><<<grid, 256, 0, stream>>>(points, normals, V, node_state, anchors, weights, K, E, out_p, out_n, jrows);
		NNRT_LAUNCH_CHECK();
		return NNRT_OK;
	}
	if (from_identity) {
		set_error("launch_warp_mesh: from_identity needs K <= 4");
		return NNRT_ERROR_ARGUMENT;
	}
	k_warp_mesh<<<static_cast<unsigned>(ceil_div(V, 256)), 256, 0, stream>>>(points, normals, V, node_state, anchors, weights, K, E, out_p,
	                                                                          out_n, jrows);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

// =====================================================================================================================
// Point / point+normal warp of the nnrt.geometry.functional API (warp_triangle_mesh, warp_point_cloud): supplied
// anchors (online anchors are computed first by k_compute_anchors, the reference's Find* then BlendWarp split).
//   minimum_valid < 0: BlendWarp over the non-(-1) slots (Warp3dPointsAndNormalsImpl.h:173-193, :393-414);
//   minimum_valid >= 0: BlendWarp_ValidAnchorCountThreshold (WarpUtilities.h:505-580): the point (and normal) stays
//   zero unless at least minimum_valid slots are valid. For online threshold anchors this is FindAnchors...Threshold
//   returning false (WarpUtilities.h:242-244): the slots failing the 2c test are exactly the -1 slots.
// Extrinsics act on the point (rigid) and the normal (rotation) before blending (:369-378). One lane per point, outputs
// [V,3] as the reference's tensors.
// =====================================================================================================================
template <bool NORMALS>
__global__ __launch_bounds__(256) void k_warp_points(const float* __restrict__ points, const float* __restrict__ normals, int64_t V,
                                                     const float* __restrict__ node_state, const int32_t* __restrict__ anchors,
                                                     const float* __restrict__ weights, int K, int minimum_valid, WarpExtrinsics E,
                                                     float* __restrict__ out_p, float* __restrict__ out_n) {
	const int64_t v = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (v >= V) return;
	int valid = 0;
	for (int k = 0; k < K; k++) valid += anchors[v * K + k] != -1;
	f3 wp = make3(0.f, 0.f, 0.f), wn = make3(0.f, 0.f, 0.f);
	if (minimum_valid < 0 || valid >= minimum_valid) {
		const f3 p = make3(points[3 * v], points[3 * v + 1], points[3 * v + 2]);
		const f3 pc = E.identity ? p : apply_extrinsics_point(E, p);
		f3 nc = make3(0.f, 0.f, 0.f);
		if constexpr (NORMALS) {
			const f3 n = make3(normals[3 * v], normals[3 * v + 1], normals[3 * v + 2]);
			nc = E.identity ? n : apply_extrinsics_normal(E, n);
		}
		for (int k = 0; k < K; k++) {
			const int32_t a = anchors[v * K + k];
			if (a == -1) continue;
			const float w = weights[v * K + k];
			const float* ns = node_state + static_cast<int64_t>(a) * NODE_STRIDE;
			const f3 g = make3(ns[0], ns[1], ns[2]);
			const f3 t = make3(ns[3], ns[4], ns[5]);
			const f3 Rd = matvec3(ns + 6, sub3(pc, g));
			wp.x += w * ((g.x + Rd.x) + t.x);
			wp.y += w * ((g.y + Rd.y) + t.y);
			wp.z += w * ((g.z + Rd.z) + t.z);
			if constexpr (NORMALS) {
				const f3 Rn = matvec3(ns + 6, nc);
				wn.x += w * Rn.x;
				wn.y += w * Rn.y;
				wn.z += w * Rn.z;
			}
		}
	}
	out_p[3 * v] = wp.x;
	out_p[3 * v + 1] = wp.y;
	out_p[3 * v + 2] = wp.z;
	if constexpr (NORMALS) {
		out_n[3 * v] = wn.x;
		out_n[3 * v + 1] = wn.y;
		out_n[3 * v + 2] = wn.z;
	}
}

nnrt_status launch_warp_points(const float* points, const float* normals, int64_t V, const float* node_state, const int32_t* anchors,
                               const float* weights, int K, int minimum_valid, const WarpExtrinsics& E, float* out_p, float* out_n,
                               hipStream_t stream) {
	if (V == 0) return NNRT_OK;
	const unsigned grid = static_cast<unsigned>(ceil_div(V, 256));
	if (normals)
		k_warp_points<true><<<grid, 256, 0, stream>>>(points, normals, V, node_state, anchors, weights, K, minimum_valid, E, out_p, out_n);
	else
		k_warp_points<false><<<grid, 256, 0, stream>>>(points, nullptr, V, node_state, anchors, weights, K, minimum_valid, E, out_p, nullptr);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

// ComputePointToPlaneDistances (PointToPlaneDistancesImpl.h:26-50): d = n1 . (v1 - v2), one lane per point. The
// three-term dot is summed left to right, as every dot product of this library and of the oracle.
__global__ __launch_bounds__(256) void k_point_to_plane(const float* __restrict__ n1, const float* __restrict__ v1, const float* __restrict__ v2,
                                                        int64_t count, float* __restrict__ out) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= count) return;
	const f3 n = make3(n1[3 * i], n1[3 * i + 1], n1[3 * i + 2]);
	const f3 d = sub3(make3(v1[3 * i], v1[3 * i + 1], v1[3 * i + 2]), make3(v2[3 * i], v2[3 * i + 1], v2[3 * i + 2]));
	out[i] = dot3(n, d);
}

nnrt_status launch_point_to_plane(const float* n1, const float* v1, const float* v2, int64_t count, float* out, hipStream_t stream) {
	if (count == 0) return NNRT_OK;
	k_point_to_plane<<<static_cast<unsigned>(ceil_div(count, 256)), 256, 0, stream>>>(n1, v1, v2, count, out);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

__global__ void k_pack_nodes(const float* __restrict__ nodes, const float* __restrict__ R, const float* __restrict__ t, int N,
                             float* __restrict__ state) {
	const int n = blockIdx.x * blockDim.x + threadIdx.x;
	if (n >= N) return;
	float* s = state + static_cast<int64_t>(n) * NODE_STRIDE;
	for (int c = 0; c < 3; c++) {
		s[c] = nodes[3 * n + c];
		s[3 + c] = t ? t[3 * n + c] : 0.f;
	}
	for (int c = 0; c < 9; c++) s[6 + c] = R ? R[9 * n + c] : ((c % 4 == 0) ? 1.f : 0.f);
	s[15] = 0.f;
}

__global__ void k_unpack_float4x3(const float4* __restrict__ in, int64_t count, float* __restrict__ out) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= count) return;
	const float4 v = in[i];
	out[3 * i] = v.x;
	out[3 * i + 1] = v.y;
	out[3 * i + 2] = v.z;
}

nnrt_status launch_pack_nodes(const float* nodes, const float* R, const float* t, int N, float* state, hipStream_t stream) {
	if (N == 0) return NNRT_OK;
	k_pack_nodes<<<static_cast<unsigned>(ceil_div(N, 256)), 256, 0, stream>>>(nodes, R, t, N, state);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

nnrt_status launch_unpack_float4x3(const float4* in, int64_t count, float* out, hipStream_t stream) {
	if (count == 0) return NNRT_OK;
	k_unpack_float4x3<<<static_cast<unsigned>(ceil_div(count, 256)), 256, 0, stream>>>(in, count, out);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

// =====================================================================================================================
// NDC face extraction + clip mask: ExtractClippedFaceVerticesImpl.h:108-179 (near/far OR test: A6). Clipped faces are
// zero-filled (the reference leaves them uninitialized). Vertices given as [V,3] floats or float4.
// =====================================================================================================================
template <typename TVertexLoader>
__device__ inline void extract_face(int64_t f, const int64_t* faces, TVertexLoader load, const NdcSetup& s, float near_clip, float far_clip,
                                    float* out, uint8_t* mask) {
	f3 v[3];
	for (int i = 0; i < 3; i++) v[i] = load(faces[3 * f + i]);
	bool in_range = false;
	for (int i = 0; i < 3; i++) {
		in_range |= v[i].z >= near_clip;
		in_range |= v[i].z <= far_clip;
	}
	bool inlier = false;
	float xy[3][2];
	if (in_range) {
		for (int i = 0; i < 3; i++) {
			s.ndc.project_rn(v[i].x, v[i].y, v[i].z, &xy[i][0], &xy[i][1]);
			inlier |= (xy[i][1] >= s.min_y && xy[i][0] >= s.min_x && xy[i][1] <= s.max_y && xy[i][0] <= s.max_x);
		}
	}
	if (!in_range || !inlier) {
		mask[f] = 0;
		for (int i = 0; i < 9; i++) out[9 * f + i] = 0.f;
		return;
	}
	mask[f] = 1;
	for (int i = 0; i < 3; i++) {
		out[9 * f + 3 * i] = xy[i][0];
		out[9 * f + 3 * i + 1] = xy[i][1];
		out[9 * f + 3 * i + 2] = v[i].z;
	}
}

__global__ void k_extract_face_ndc(const float* __restrict__ verts, const int64_t* __restrict__ faces, int64_t F, NdcSetup s, float near_clip,
                                   float far_clip, float* __restrict__ out, uint8_t* __restrict__ mask) {
	const int64_t f = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (f >= F) return;
	extract_face(f, faces, [&](int64_t i) { return make3(verts[3 * i], verts[3 * i + 1], verts[3 * i + 2]); }, s, near_clip, far_clip, out, mask);
}

nnrt_status launch_extract_face_ndc(const float* verts, const int64_t* faces, int64_t F, const NdcSetup& s, float near_clip, float far_clip,
                                    float* out, uint8_t* mask, hipStream_t stream) {
	if (F == 0) return NNRT_OK;
	k_extract_face_ndc<<<static_cast<unsigned>(ceil_div(F, 256)), 256, 0, stream>>>(verts, faces, F, s, near_clip, far_clip, out, mask);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

// =====================================================================================================================
// Unprojection (UnprojectRasterWithoutDepthFiltering, PerspectiveProjectionImpl.h:60-146) and attribute interpolation
// (InterpolateFaceAttributesImpl.h:30-75). Depth uint16 or float32, divided by depth_scale in float (the reference's
// `*depth / depth_scale`); kept iff 0 < d < depth_max: Open3D TransformIndexer::Unproject ((u - cx) d / fx, ...) then
// RigidTransform by pose = extrinsics^-1 (skipped for the identity, where it is exact). Rejected pixels: zero point,
// mask 0 (the reference's Zeros-initialised outputs).
// =====================================================================================================================
template <typename T>
__global__ void k_unproject(const T* __restrict__ depth, int H, int W, Camera K, WarpExtrinsics pose, float scale, float depth_max,
                            float* __restrict__ pts, uint8_t* __restrict__ mask) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= static_cast<int64_t>(H) * W) return;
	const int y = static_cast<int>(i / W), x = static_cast<int>(i % W);
	const float d = static_cast<float>(depth[i]) / scale;
	if (d > 0 && d < depth_max) {
		f3 c = make3((static_cast<float>(x) - K.cx) * d / K.fx, (static_cast<float>(y) - K.cy) * d / K.fy, d);
		if (!pose.identity) c = apply_extrinsics_point(pose, c);
		pts[3 * i] = c.x;
		pts[3 * i + 1] = c.y;
		pts[3 * i + 2] = c.z;
		mask[i] = 1;
	} else {
		pts[3 * i] = pts[3 * i + 1] = pts[3 * i + 2] = 0.f;
		mask[i] = 0;
	}
}

nnrt_status launch_unproject(const void* depth, int depth_dtype, int H, int W, const Camera& K, const WarpExtrinsics& pose, float scale,
                             float depth_max, float* pts, uint8_t* mask, hipStream_t stream) {
	const int64_t P = static_cast<int64_t>(H) * W;
	if (P == 0) return NNRT_OK;
	const unsigned grid = static_cast<unsigned>(ceil_div(P, 256));
	if (depth_dtype == NNRT_DTYPE_UINT16)
		k_unproject<uint16_t><<<grid, 256, 0, stream>>>(static_cast<const uint16_t*>(depth), H, W, K, pose, scale, depth_max, pts, mask);
	else
		k_unproject<float><<<grid, 256, 0, stream>>>(static_cast<const float*>(depth), H, W, K, pose, scale, depth_max, pts, mask);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

// =====================================================================================================================
// Depth back-projection to an ordered [H, W, 3] point image (cpp/cpu/image_proc.cpp:275-339): depth = d / normalizer,
// p = (depth * (x - cx) / fx, depth * (y - cy) / fy, depth), zeros where depth <= 0. Four pixels per lane: 8 B (u16) or
// 16 B (f32) in, three 16-B stores out, so a wave writes 3 KB of contiguous point image.
// =====================================================================================================================
template <typename T>
__device__ __forceinline__ void backproject_one(T raw, int x, int y, const BackprojectCamera& c, float& px, float& py, float& pz) {
	const float depth = static_cast<float>(raw) / c.normalizer;
	if (depth > 0.f) {
		px = depth * (static_cast<float>(x) - c.cx) / c.fx;
		py = depth * (static_cast<float>(y) - c.cy) / c.fy;
		pz = depth;
	} else {
		px = py = pz = 0.f;
	}
}

template <typename T>
__global__ void k_backproject_depth_x4(const T* __restrict__ depth, int H, int W, BackprojectCamera c, float4* __restrict__ out) {
	const int64_t q = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;   // quad of pixels 4q .. 4q+3
	if (q * 4 >= static_cast<int64_t>(H) * W) return;
	T d[4];
	if constexpr (sizeof(T) == 2) {
		const uint2 v = reinterpret_cast<const uint2*>(depth)[q];
		d[0] = static_cast<T>(v.x & 0xffffu); d[1] = static_cast<T>(v.x >> 16);
		d[2] = static_cast<T>(v.y & 0xffffu); d[3] = static_cast<T>(v.y >> 16);
	} else {
		const float4 v = reinterpret_cast<const float4*>(depth)[q];
		d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
	}
	float p[12];
	const int y = static_cast<int>((q * 4) / W), x0 = static_cast<int>((q * 4) % W);   // W % 4 == 0: one row per quad
#pragma unroll
	for (int k = 0; k < 4; ++k) backproject_one(d[k], x0 + k, y, c, p[3 * k], p[3 * k + 1], p[3 * k + 2]);
	out[3 * q] = make_float4(p[0], p[1], p[2], p[3]);
	out[3 * q + 1] = make_float4(p[4], p[5], p[6], p[7]);
	out[3 * q + 2] = make_float4(p[8], p[9], p[10], p[11]);
}

template <typename T>
__global__ void k_backproject_depth(const T* __restrict__ depth, int H, int W, BackprojectCamera c, float* __restrict__ out) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= static_cast<int64_t>(H) * W) return;
	backproject_one(depth[i], static_cast<int>(i % W), static_cast<int>(i / W), c, out[3 * i], out[3 * i + 1], out[3 * i + 2]);
}

template <typename T>
static nnrt_status backproject_depth(const T* depth, int H, int W, const BackprojectCamera& c, float* out, hipStream_t stream) {
	const int64_t P = static_cast<int64_t>(H) * W;
	if (P == 0) return NNRT_OK;
	const bool vec = (W % 4 == 0) && (reinterpret_cast<uintptr_t>(depth) % (4 * sizeof(T)) == 0) &&
	                 (reinterpret_cast<uintptr_t>(out) % 16 == 0);
	if (vec) {
		k_backproject_depth_x4<T><<<static_cast<unsigned>(ceil_div(P / 4, 256)), 256, 0, stream>>>(depth, H, W, c,
		                                                                                         reinterpret_cast<float4*>(out));
	} else {
		k_backproject_depth<T><<<static_cast<unsigned>(ceil_div(P, 256)), 256, 0, stream>>>(depth, H, W, c, out);
	}
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

nnrt_status launch_backproject_depth_u16(const uint16_t* depth, int H, int W, const BackprojectCamera& c, float* out, hipStream_t stream) {
	return backproject_depth<uint16_t>(depth, H, W, c, out, stream);
}

nnrt_status launch_backproject_depth_f32(const float* depth, int H, int W, const BackprojectCamera& c, float* out, hipStream_t stream) {
	return backproject_depth<float>(depth, H, W, c, out, stream);
}

__global__ void k_interpolate(const int64_t* __restrict__ pixel_faces, const float* __restrict__ bary, int64_t P, int Kf,
                              const float* __restrict__ attrs, int C, float* __restrict__ out) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= P * C) return;
	const int64_t p = i / C;
	const int c = static_cast<int>(i % C);
	bool done = false;
	for (int k = 0; k < Kf; k++) {
		const int64_t f = done ? -1 : pixel_faces[p * Kf + k];
		if (f < 0) done = true;
		float acc = 0.0f;
		if (!done) {
			for (int v = 0; v < 3; v++) acc += bary[(p * Kf + k) * 3 + v] * attrs[f * 3 * C + v * C + c];
		}
		out[(p * Kf + k) * C + c] = acc;
	}
}

nnrt_status launch_interpolate(const int64_t* pixel_faces, const float* bary, int64_t P, int Kf, const float* attrs, int C, float* out,
                               hipStream_t stream) {
	if (P * C == 0) return NNRT_OK;
	k_interpolate<<<static_cast<unsigned>(ceil_div(P * C, 256)), 256, 0, stream>>>(pixel_faces, bary, P, Kf, attrs, C, out);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

// Matmul3D (cpp/core/linalg/Matmul3D.cpp:25-83, the batched GEMM behind R <- R dR): C[b] = A[b] B[b], row-major
// [batch, m, k] x [batch, k, n] (n = 1 for an array of vectors). One lane per output element, products summed in k order.
__global__ void k_matmul3d(const float* __restrict__ A, const float* __restrict__ B, int64_t batch, int m, int k, int n, float* __restrict__ C) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	const int64_t per = static_cast<int64_t>(m) * n;
	if (i >= batch * per) return;
	const int64_t b = i / per;
	const int r = static_cast<int>((i % per) / n), c = static_cast<int>(i % n);
	const float* a = A + b * m * k + static_cast<int64_t>(r) * k;
	const float* bb = B + b * k * n + c;
	float acc = 0.f;
	for (int j = 0; j < k; j++) acc += a[j] * bb[static_cast<int64_t>(j) * n];
	C[i] = acc;
}

nnrt_status launch_matmul3d(const float* A, const float* B, int64_t batch, int m, int k, int n, float* C, hipStream_t stream) {
	const int64_t total = batch * m * n;
	if (total == 0) return NNRT_OK;
	k_matmul3d<<<static_cast<unsigned>(ceil_div(total, 256)), 256, 0, stream>>>(A, B, batch, m, k, n, C);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

__global__ void k_rodrigues(const float* __restrict__ w, int N, float* __restrict__ R) {
	const int n = blockIdx.x * blockDim.x + threadIdx.x;
	if (n >= N) return;
	float m[9];
	rodrigues_device(w[3 * n], w[3 * n + 1], w[3 * n + 2], m);
	for (int i = 0; i < 9; i++) R[9 * n + i] = m[i];
}

nnrt_status launch_rodrigues(const float* w, int N, float* R, hipStream_t stream) {
	if (N == 0) return NNRT_OK;
	k_rodrigues<<<static_cast<unsigned>(ceil_div(N, 256)), 256, 0, stream>>>(w, N, R);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

} // namespace nnrt
