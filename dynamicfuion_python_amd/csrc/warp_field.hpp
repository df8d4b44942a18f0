#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "nnrt_mi355x.h"

namespace nnrt {

void set_error(const std::string& message);

#ifndef NNRT_CHECK_ARG
#define NNRT_CHECK_ARG(cond, msg)                                                                                        \
	do {                                                                                                                 \
		if (!(cond)) {                                                                                                   \
			::nnrt::set_error(std::string("invalid argument: ") + (msg));                                              \
			return NNRT_ERROR_ARGUMENT;                                                                                  \
		}                                                                                                                \
	} while (0)
#endif

struct Hierarchy {
	std::vector<int64_t> virtual_indices;   // virtual -> original
	std::vector<int> layer_counts;          // fine -> coarse
	std::vector<float> radii;               // per layer decimation radius (layer 0: coverage)
	std::vector<int32_t> edges;             // [E,2] virtual
	std::vector<int8_t> edge_layers;        // [E]
};

nnrt_status build_hierarchy(const float* nodes, int N, float coverage, int layer_count, int max_degree, const float* radii, Hierarchy& h);
void node_coverage_weights(const float* nodes, int N, float coverage, std::vector<float>& out);

} // namespace nnrt
