// Build (not committed as a binary): hipcc --offload-arch=gfx950 -O3 tools/dev/rcp_check.hip -o tools/dev/rcp_check
// Exhaustive check (development): rcp_rn_fast(b) == RN(1/b) = (float)(1.0 / (double)b) for every float bit pattern.
// rcp_rn_fast: hardware double reciprocal estimate + one Newton step in double, rounded to float.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstring>

__device__ inline float rcp_ref(float b) { return static_cast<float>(1.0 / static_cast<double>(b)); }
__device__ inline float rcp_fast64(float b) {
	const double bd = b;
	double r = __builtin_amdgcn_rcp(bd);
	const double e = __builtin_fma(-bd, r, 1.0);
	r = __builtin_fma(r, e, r);
	return static_cast<float>(r);
}
// hardware float estimate + one Newton step with FMA
__device__ inline float rcp_fast32(float b) {
	const float y = __builtin_amdgcn_rcpf(b);
	const float e = __builtin_fmaf(-b, y, 1.0f);
	return __builtin_fmaf(e, y, y);
}

template <int V>
__global__ void k_check(uint64_t lo, uint64_t n, unsigned long long* bad, uint32_t* first) {
	const uint64_t stride = static_cast<uint64_t>(gridDim.x) * blockDim.x;
	unsigned long long mine = 0;
	for (uint64_t i = static_cast<uint64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
		const uint32_t u = static_cast<uint32_t>(lo + i);
		const float b = __uint_as_float(u);
		const float x = rcp_ref(b), y = V == 64 ? rcp_fast64(b) : rcp_fast32(b);
		const float ab = fabsf(b);
		if (ab < 0x1p-125f || ab > 0x1p125f) continue;   // normal domain: b and 1/b normal
		const bool same = __float_as_uint(x) == __float_as_uint(y) || (x != x && y != y);
		if (!same) {
			mine++;
			const unsigned long long k = atomicAdd(bad + 1, 1ull);
			if (k < 16) first[k] = u;
		}
	}
	if (mine) atomicAdd(bad, mine);
}

int main() {
	unsigned long long* bad;
	uint32_t* first;
	hipMalloc(&bad, 16);
	hipMalloc(&first, 64);
	for (int v : {32, 64}) {
		hipMemset(bad, 0, 16);
		hipMemset(first, 0, 64);
		if (v == 32) hipLaunchKernelGGL(k_check<32>, dim3(8192), dim3(256), 0, 0, 0ull, 1ull << 32, bad, first);
		else hipLaunchKernelGGL(k_check<64>, dim3(8192), dim3(256), 0, 0, 0ull, 1ull << 32, bad, first);
		if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 2; }
		unsigned long long h[2];
		uint32_t f[16];
		hipMemcpy(h, bad, 16, hipMemcpyDeviceToHost);
		hipMemcpy(f, first, 64, hipMemcpyDeviceToHost);
		printf("rcp_fast%d: mismatches vs RN(1/b) over all float patterns with |b| in [2^-125, 2^125]: %llu\n", v, h[0]);
		for (int i = 0; i < (h[0] < 16 ? static_cast<int>(h[0]) : 16); i++) {
			float bb;
			memcpy(&bb, &f[i], 4);
			printf("  0x%08x  %g\n", f[i], bb);
		}
	}
	return 0;
}
