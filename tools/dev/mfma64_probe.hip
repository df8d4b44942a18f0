// Probe: v_mfma_f64_16x16x4f64 operand/result layout with exact data, and issue rate (1 and 4 chains per wave).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void layout(double* out) {
	const int l = threadIdx.x;
	// A[i][k] = 100*i + k ; B[k][j] = (k == j) ? 1 : 0  -> C = A * B = A[i][j] for j < 4
	const double a = 100.0 * (l & 15) + (l >> 4);
	const double b = ((l >> 4) == (l & 15)) ? 1.0 : 0.0;
	d4 c = {0, 0, 0, 0};
	c = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
	for (int r = 0; r < 4; r++) out[l * 4 + r] = c[r];
}

template <int CHAINS>
__global__ void rate(double* out, int iters) {
	const int l = threadIdx.x & 63;
	double a = 1.0 + l * 1e-3, b = 1.0 - l * 1e-3;
	d4 c[CHAINS];
	for (int i = 0; i < CHAINS; i++) c[i] = d4{0, 0, 0, 0};
	for (int it = 0; it < iters; it++)
#pragma unroll
		for (int i = 0; i < CHAINS; i++) c[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[i], 0, 0, 0);
	double s = 0;
	for (int i = 0; i < CHAINS; i++) s += c[i][0] + c[i][1] + c[i][2] + c[i][3];
	if (s == 12345.0) out[0] = s;
}

int main() {
	double* d;
	hipMalloc(&d, 64 * 4 * sizeof(double));
	layout<<<1, 64>>>(d);
	std::vector<double> h(256);
	hipMemcpy(h.data(), d, 256 * sizeof(double), hipMemcpyDeviceToHost);
	int bad = 0;
	for (int l = 0; l < 64; l++)
		for (int r = 0; r < 4; r++) {
			const int row = (l >> 4) + 4 * r, col = l & 15;   // guide: col = lane & 15, row = (lane >> 4) + 4 * reg
			const double expect = col < 4 ? 100.0 * row + col : 0.0;
			if (h[l * 4 + r] != expect) bad++;
		}
	printf("layout mismatches vs guide map: %d\n", bad);
	for (int l = 0; l < 64; l += 17) printf("lane %d: %g %g %g %g\n", l, h[4 * l], h[4 * l + 1], h[4 * l + 2], h[4 * l + 3]);
	hipEvent_t e0, e1;
	hipEventCreate(&e0);
	hipEventCreate(&e1);
	const int iters = 4096;
	// one wave per SIMD: 256 CUs x 4 SIMDs = 1024 waves of 64
	for (int pass = 0; pass < 2; pass++) {
		hipEventRecord(e0);
		rate<1><<<1024, 64>>>(d, iters);
		hipEventRecord(e1);
		hipEventSynchronize(e1);
		float ms1;
		hipEventElapsedTime(&ms1, e0, e1);
		hipEventRecord(e0);
		rate<4><<<1024, 64>>>(d, iters);
		hipEventRecord(e1);
		hipEventSynchronize(e1);
		float ms4;
		hipEventElapsedTime(&ms4, e0, e1);
		// ns per MFMA per wave (each SIMD runs one wave): time / (iters * chains)
		printf("1 chain: %.3f ms -> %.2f ns/mfma ; 4 chains: %.3f ms -> %.2f ns/mfma\n", ms1, ms1 * 1e6 / iters, ms4, ms4 * 1e6 / (4.0 * iters));
	}
	hipFree(d);
	return 0;
}
