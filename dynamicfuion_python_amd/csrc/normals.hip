// Triangle, vertex and ordered-point-cloud normals (cpp/geometry/functional/kernel/NormalsOperationsImpl.h).
//
// The reference accumulates vertex normals with float atomics (order-nondeterministic, A18); here every vertex
// gathers its incident faces in ascending face order from a vertex -> face CSR built on the device, which is the
// reference's serial (CPU, single-thread) summation order exactly.
#include "kernels.hpp"

namespace nnrt {

__device__ inline f3 load3(const float* p, int64_t i) { return make3(p[3 * i], p[3 * i + 1], p[3 * i + 2]); }

// Eigen::Vector3f::normalize(): divide by the root of the squared norm when it is positive (zero stays zero), then
// NormalizeVectors3d maps NaN to (0, 0, 1) (NormalsOperationsImpl.h:75-93)
__device__ inline f3 normalize_like_eigen(f3 v) {
	const float n2 = (v.x * v.x + v.y * v.y) + v.z * v.z;
	if (n2 > 0.f) {
		const float n = sqrtf(n2);
		v = make3(v.x / n, v.y / n, v.z / n);
	}
	if (v.x != v.x) v = make3(0.f, 0.f, 1.f);
	return v;
}

// ComputeTriangleNormals (:39-68): (v1 - v0) x (v2 - v0)
__device__ inline f3 triangle_normal(const float* verts, const int64_t* faces, int64_t f) {
	const f3 v0 = load3(verts, faces[3 * f]), v1 = load3(verts, faces[3 * f + 1]), v2 = load3(verts, faces[3 * f + 2]);
	const f3 a = sub3(v1, v0), b = sub3(v2, v0);
	return make3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}

__global__ void k_triangle_normals(const float* __restrict__ verts, int64_t V, const int64_t* __restrict__ faces, int64_t F, int normalized,
                                   float* __restrict__ out, int* error_flag) {
	const int64_t f = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (f >= F) return;
	const int64_t i0 = faces[3 * f], i1 = faces[3 * f + 1], i2 = faces[3 * f + 2];
	if (i0 < 0 || i0 >= V || i1 < 0 || i1 >= V || i2 < 0 || i2 >= V) {   // no gather outside the vertex array
		atomicOr(error_flag, 1);
		out[3 * f] = out[3 * f + 1] = out[3 * f + 2] = __builtin_nanf("");
		return;
	}
	f3 n = triangle_normal(verts, faces, f);
	if (normalized) n = normalize_like_eigen(n);
	out[3 * f] = n.x;
	out[3 * f + 1] = n.y;
	out[3 * f + 2] = n.z;
}

__global__ void k_vertex_face_count(const int64_t* __restrict__ faces, int64_t F, int64_t V, int* __restrict__ count, int* error_flag) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= 3 * F) return;
	const int64_t v = faces[i];
	if (v < 0 || v >= V) {
		atomicOr(error_flag, 1);
		return;
	}
	atomicAdd(count + v, 1);
}

// single-workgroup exclusive scan of the per-vertex counts (V + 1 offsets), 1024 threads, chunked
__global__ __launch_bounds__(1024) void k_exclusive_scan(const int* __restrict__ in, int64_t n, int* __restrict__ out) {
	__shared__ int s_part[1024];
	const int t = threadIdx.x;
	const int64_t per = (n + 1023) / 1024;
	const int64_t lo = t * per, hi = lo + per < n ? lo + per : n;
	int sum = 0;
	for (int64_t i = lo; i < hi; i++) sum += in[i];
	s_part[t] = sum;
	__syncthreads();
	for (int d = 1; d < 1024; d <<= 1) {   // Hillis-Steele inclusive scan of the chunk sums
		const int v = t >= d ? s_part[t - d] : 0;
		__syncthreads();
		s_part[t] += v;
		__syncthreads();
	}
	int run = t > 0 ? s_part[t - 1] : 0;
	for (int64_t i = lo; i < hi; i++) {
		out[i] = run;
		run += in[i];
	}
	if (t == 1023) out[n] = s_part[1023];
}

__global__ void k_vertex_face_fill(const int64_t* __restrict__ faces, int64_t F, const int* __restrict__ offsets, int* __restrict__ cursor,
                                   int* __restrict__ list) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= 3 * F) return;
	const int64_t v = faces[i];   // indices were validated by k_vertex_face_count before this launch
	const int slot = atomicAdd(cursor + v, 1);
	list[offsets[v] + slot] = static_cast<int>(i / 3);
}

// per vertex: incident faces sorted ascending (insertion sort in place; lists are short), then the serial sum
__global__ void k_vertex_normals(const float* __restrict__ verts, const int64_t* __restrict__ faces, int64_t V, const int* __restrict__ offsets,
                                 int* __restrict__ list, int normalized, float* __restrict__ out) {
	const int64_t v = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (v >= V) return;
	const int b = offsets[v], e = offsets[v + 1];
	for (int i = b + 1; i < e; i++) {
		const int key = list[i];
		int j = i - 1;
		while (j >= b && list[j] > key) {
			list[j + 1] = list[j];
			j--;
		}
		list[j + 1] = key;
	}
	float x = 0.f, y = 0.f, z = 0.f;
	for (int i = b; i < e; i++) {
		const f3 n = triangle_normal(verts, faces, list[i]);   // the unnormalized triangle normal (:52-57)
		x += n.x;
		y += n.y;
		z += n.z;
	}
	f3 r = make3(x, y, z);
	if (normalized) r = normalize_like_eigen(r);
	out[3 * v] = r.x;
	out[3 * v + 1] = r.y;
	out[3 * v + 2] = r.z;
}

// ComputeOrderedPointCloudNormals (:170-214): border pixels get 0; else normalize((right - left) x (top - bottom)),
// flipped to face the camera (n.z <= 0)
__global__ void k_ordered_point_cloud_normals(const float* __restrict__ pts, int H, int W, float* __restrict__ out) {
	const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
	if (i >= static_cast<int64_t>(H) * W) return;
	const int y = static_cast<int>(i / W), x = static_cast<int>(i % W);
	f3 n = make3(0.f, 0.f, 0.f);
	if (!(x == 0 || x == W - 1 || y == 0 || y == H - 1)) {
		const f3 l = load3(pts, i - 1), r = load3(pts, i + 1), t = load3(pts, i - W), b = load3(pts, i + W);
		const f3 dh = sub3(r, l), dv = sub3(t, b);
		n = make3(dh.y * dv.z - dh.z * dv.y, dh.z * dv.x - dh.x * dv.z, dh.x * dv.y - dh.y * dv.x);
		const float n2 = (n.x * n.x + n.y * n.y) + n.z * n.z;   // Eigen normalized(): zero vectors stay zero
		if (n2 > 0.f) {
			const float s = sqrtf(n2);
			n = make3(n.x / s, n.y / s, n.z / s);
		}
		if (n.z > 0.f) n = make3(-n.x, -n.y, -n.z);
	}
	out[3 * i] = n.x;
	out[3 * i + 1] = n.y;
	out[3 * i + 2] = n.z;
}

} // namespace nnrt

using namespace nnrt;

extern "C" {

nnrt_status nnrt_compute_triangle_normals(const float* d_vertices, int64_t vertex_count, const int64_t* d_faces, int64_t face_count,
                                          int32_t normalized, float* d_out, void* stream) {
	if (face_count == 0) return NNRT_OK;
	NNRT_CHECK_ARG(d_vertices && d_faces && d_out && face_count > 0 && vertex_count >= 0, "invalid arguments");
	hipStream_t s = static_cast<hipStream_t>(stream);
	int* flag = nullptr;
	NNRT_HIP(hipMallocAsync(reinterpret_cast<void**>(&flag), sizeof(int), s));
	NNRT_HIP(hipMemsetAsync(flag, 0, sizeof(int), s));
	k_triangle_normals<<<static_cast<unsigned>(ceil_div(face_count, 256)), 256, 0, s>>>(d_vertices, vertex_count, d_faces, face_count, normalized,
	                                                                                    d_out, flag);
	hipError_t le = hipGetLastError();
	int host_flag = 0;
	hipError_t ce = hipMemcpyAsync(&host_flag, flag, sizeof(int), hipMemcpyDeviceToHost, s);
	hipError_t se = hipStreamSynchronize(s);
	hipFreeAsync(flag, s);
	NNRT_HIP(le);
	NNRT_HIP(ce);
	NNRT_HIP(se);
	if (host_flag) {
		set_error("triangle index out of range");
		return NNRT_ERROR_ARGUMENT;
	}
	return NNRT_OK;
}

nnrt_status nnrt_compute_vertex_normals(const float* d_vertices, int64_t vertex_count, const int64_t* d_faces, int64_t face_count,
                                        int32_t normalized, float* d_out, void* stream) {
	NNRT_CHECK_ARG(d_vertices && d_out && vertex_count >= 0 && face_count >= 0 && (face_count == 0 || d_faces), "invalid arguments");
	if (vertex_count == 0) return NNRT_OK;
	hipStream_t s = static_cast<hipStream_t>(stream);
	int *count = nullptr, *offsets = nullptr, *list = nullptr, *flag = nullptr;
	const int64_t V = vertex_count, n3 = 3 * face_count;
	NNRT_HIP(hipMallocAsync(reinterpret_cast<void**>(&count), sizeof(int) * V, s));
	NNRT_HIP(hipMallocAsync(reinterpret_cast<void**>(&offsets), sizeof(int) * (V + 1), s));
	NNRT_HIP(hipMallocAsync(reinterpret_cast<void**>(&list), sizeof(int) * (n3 > 0 ? n3 : 1), s));
	NNRT_HIP(hipMallocAsync(reinterpret_cast<void**>(&flag), sizeof(int), s));
	NNRT_HIP(hipMemsetAsync(count, 0, sizeof(int) * V, s));
	NNRT_HIP(hipMemsetAsync(flag, 0, sizeof(int), s));
	if (n3 > 0) k_vertex_face_count<<<static_cast<unsigned>(ceil_div(n3, 256)), 256, 0, s>>>(d_faces, face_count, V, count, flag);
	{   // validate every index before anything gathers through the faces (the fill and the sums index by them)
		hipError_t le = hipGetLastError();
		int host_flag = 0;
		hipError_t ce = hipMemcpyAsync(&host_flag, flag, sizeof(int), hipMemcpyDeviceToHost, s);
		hipError_t se = hipStreamSynchronize(s);
		if (le != hipSuccess || ce != hipSuccess || se != hipSuccess || host_flag) {
			for (void* p : {static_cast<void*>(count), static_cast<void*>(offsets), static_cast<void*>(list), static_cast<void*>(flag)}) hipFreeAsync(p, s);
			NNRT_HIP(le);
			NNRT_HIP(ce);
			NNRT_HIP(se);
			set_error("triangle index out of range");
			return NNRT_ERROR_ARGUMENT;
		}
	}
	k_exclusive_scan<<<1, 1024, 0, s>>>(count, V, offsets);
	NNRT_HIP(hipMemsetAsync(count, 0, sizeof(int) * V, s));
	if (n3 > 0) k_vertex_face_fill<<<static_cast<unsigned>(ceil_div(n3, 256)), 256, 0, s>>>(d_faces, face_count, offsets, count, list);
	k_vertex_normals<<<static_cast<unsigned>(ceil_div(V, 256)), 256, 0, s>>>(d_vertices, d_faces, V, offsets, list, normalized, d_out);
	hipError_t le = hipGetLastError();
	hipError_t se = hipStreamSynchronize(s);
	for (void* p : {static_cast<void*>(count), static_cast<void*>(offsets), static_cast<void*>(list), static_cast<void*>(flag)}) hipFreeAsync(p, s);
	NNRT_HIP(le);
	NNRT_HIP(se);
	return NNRT_OK;
}

nnrt_status nnrt_compute_ordered_point_cloud_normals(const float* d_points, int64_t point_count, int32_t height, int32_t width, float* d_out,
                                                     void* stream) {
	NNRT_CHECK_ARG(d_points && d_out, "null pointer");
	if (point_count != static_cast<int64_t>(height) * width) {
		set_error("Point cloud point count (got " + std::to_string(point_count) + ") must equal the multiple of dimensions (got " +
		          std::to_string(height) + " * " + std::to_string(width) + ")");
		return NNRT_ERROR_ARGUMENT;
	}
	if (point_count == 0) return NNRT_OK;
	k_ordered_point_cloud_normals<<<static_cast<unsigned>(ceil_div(point_count, 256)), 256, 0, static_cast<hipStream_t>(stream)>>>(d_points, height,
	                                                                                                                               width, d_out);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

} // extern "C"
