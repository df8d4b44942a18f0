// Probe of the gfx950 cross-lane primitives used by the wave reductions (run once on the GPU box).
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void probe(int* out) {
	const int l = threadIdx.x;
	const unsigned a = 1000 + l, b = 2000 + l;
	auto r32 = __builtin_amdgcn_permlane32_swap(a, b, false, false);
	auto r16 = __builtin_amdgcn_permlane16_swap(a, b, false, false);
	out[l * 4 + 0] = r32[0];
	out[l * 4 + 1] = r32[1];
	out[l * 4 + 2] = r16[0];
	out[l * 4 + 3] = r16[1];
}

int main() {
	int* d;
	hipMalloc(&d, 64 * 4 * sizeof(int));
	probe<<<1, 64>>>(d);
	int h[256];
	hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
	for (int l = 0; l < 64; l++) printf("lane %2d: p32 (%d, %d)  p16 (%d, %d)\n", l, h[4 * l], h[4 * l + 1], h[4 * l + 2], h[4 * l + 3]);
	hipFree(d);
	return 0;
}
