// Host timing of the warp-field hierarchy construction (csrc/warp_field.cpp) on grid-like node sets:
//   g++ -O3 -std=c++17 -Iinclude -Idynamicfuion_python_amd/csrc tools/hierarchy_host_timing.cpp \
//       dynamicfuion_python_amd/csrc/warp_field.cpp -o /tmp/hierarchy_host_timing
#include "warp_field.hpp"

#include <chrono>
#include <cmath>
#include <cstdio>
#include <random>

namespace nnrt {
void set_error(const std::string&) {}
}

int main() {
	for (int N : {1500, 5000, 20000}) {
		std::mt19937 rng(1);
		std::uniform_real_distribution<float> U(-1.f, 1.f);
		std::vector<float> nodes(3 * static_cast<size_t>(N));
		const int side = static_cast<int>(std::sqrt(static_cast<double>(N)));
		for (int i = 0; i < N; i++) {
			nodes[3 * i] = static_cast<float>(i % side) * 0.025f + U(rng) * 1e-3f;
			nodes[3 * i + 1] = static_cast<float>(i / side) * 0.025f;
			nodes[3 * i + 2] = 1.5f + 0.01f * U(rng);
		}
		const auto t0 = std::chrono::steady_clock::now();
		nnrt::Hierarchy h;
		nnrt::build_hierarchy(nodes.data(), N, 0.03f, 2, 4, nullptr, h);
		const auto t1 = std::chrono::steady_clock::now();
		std::vector<float> w;
		nnrt::node_coverage_weights(nodes.data(), N, 0.03f, w);
		const auto t2 = std::chrono::steady_clock::now();
		std::printf("N=%d hierarchy (2 layers) %.2f ms, coverage weights %.2f ms\n", N,
		            std::chrono::duration<double, std::milli>(t1 - t0).count(), std::chrono::duration<double, std::milli>(t2 - t1).count());
	}
	return 0;
}
