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

// The O(n^2) steps of the construction (hierarchy.hip implements them on the GPU).
class HierarchyOps {
public:
	virtual ~HierarchyOps() = default;
	// median-grid subsample: flags[i] = 1 iff point i is the medoid of its cell of size `cell`
	virtual nnrt_status medoid_flags(const std::vector<float>& pts, float cell, std::vector<uint8_t>& flags) = 0;
	// rows [n_fine, k]: k nearest coarse points by (squared distance, index), sorted by descending index, -1 padded
	virtual nnrt_status knn_rows(const std::vector<float>& fine, const std::vector<float>& coarse, int k, std::vector<int32_t>& rows) = 0;
	// WarpField.cpp:249-263 coverage weights (squared nearest-other-node distance)
	virtual nnrt_status coverage_weights(const float* nodes, int N, float coverage, std::vector<float>& out) = 0;
};
HierarchyOps& device_hierarchy_ops();

nnrt_status build_hierarchy(const float* nodes, int N, float coverage, int layer_count, int max_degree, const float* radii, HierarchyOps& ops,
                            Hierarchy& h);

} // namespace nnrt
