// Host-side hierarchy construction for the warp field -- HierarchicalGraphWarpField::RebuildRegularizationLayers
// (cpp/geometry/HierarchicalGraphWarpField.cpp:74-199): median-grid subsampling per layer
// (GeometrySamplingMedian.h:260-290, GeometrySamplingGridBinning.h:27-46), K-NN edges from each finer layer into the next
// coarser one, sorted descending and laid out in flipped source order (HierarchicalGraphWarpFieldImpl.h:218-297).
// Runs once per warp field (not per GN iteration). Order-nondeterministic parts of the reference (hash-map bin order,
// atomic bin fill) are made deterministic: bins visited in ascending point order, coarse samples in ascending index.
#include "warp_field.hpp"

#include <algorithm>
#include <cmath>
#include <map>
#include <tuple>

namespace nnrt {

namespace {
std::vector<int> median_grid_subsample(const std::vector<float>& pts, float cell) {
	const int n = static_cast<int>(pts.size() / 3);
	std::map<std::tuple<int, int, int>, std::vector<int>> bins;
	std::vector<std::tuple<int, int, int>> order;
	for (int i = 0; i < n; i++) {
		auto key = std::make_tuple(static_cast<int>(std::floor(pts[3 * i] / cell)), static_cast<int>(std::floor(pts[3 * i + 1] / cell)),
		                           static_cast<int>(std::floor(pts[3 * i + 2] / cell)));
		auto it = bins.find(key);
		if (it == bins.end()) {
			bins[key] = {i};
			order.push_back(key);
		} else {
			it->second.push_back(i);
		}
	}
	std::vector<int> sample;
	sample.reserve(order.size());
	for (const auto& key : order) {
		const auto& members = bins[key];
		float best = 3.402823466e+38f;
		int best_i = members[0];
		for (int a : members) {
			float sum = 0.f;
			for (int b : members) {
				const float dx = pts[3 * b] - pts[3 * a], dy = pts[3 * b + 1] - pts[3 * a + 1], dz = pts[3 * b + 2] - pts[3 * a + 2];
				sum += std::sqrt((dx * dx + dy * dy) + dz * dz);
			}
			if (sum < best) {
				best = sum;
				best_i = a;
			}
		}
		sample.push_back(best_i);
	}
	std::sort(sample.begin(), sample.end());
	return sample;
}

void knn_sorted(const float* q, const std::vector<float>& ref, int k, int32_t* out) {
	const int n = static_cast<int>(ref.size() / 3);
	std::vector<std::pair<float, int>> d(n);
	for (int i = 0; i < n; i++) {
		const float dx = ref[3 * i] - q[0], dy = ref[3 * i + 1] - q[1], dz = ref[3 * i + 2] - q[2];
		d[i] = {(dx * dx + dy * dy) + dz * dz, i};
	}
	const int kk = std::min(k, n);
	std::partial_sort(d.begin(), d.begin() + kk, d.end());
	for (int j = 0; j < k; j++) out[j] = j < n ? d[j].second : -1;
}
} // namespace

nnrt_status build_hierarchy(const float* nodes, int N, float coverage, int layer_count, int max_degree, const float* radii, Hierarchy& h) {
	NNRT_CHECK_ARG(layer_count >= 1, "layer_count must be a positive integer");
	struct Layer {
		std::vector<int64_t> idx;
		std::vector<float> pos;
		std::vector<int32_t> edges;
		float radius = 0.f;
	};
	std::vector<Layer> layers(layer_count);
	layers[0].radius = coverage;
	for (int i = 0; i < N; i++) {
		layers[0].idx.push_back(i);
		for (int c = 0; c < 3; c++) layers[0].pos.push_back(nodes[3 * i + c]);
	}
	for (int l = 1; l < layer_count; l++) {
		Layer& finer = layers[l - 1];
		Layer& cur = layers[l];
		cur.radius = radii ? radii[l] : static_cast<float>(l + 1) * coverage;
		const std::vector<int> sample = median_grid_subsample(finer.pos, cur.radius * 2);
		if (sample.size() == finer.idx.size()) {
			set_error("Attempting to generate a coarser layer of the same size as the finer layer; reduce the layer count or increase "
			          "the decimation radius (HierarchicalGraphWarpField.cpp:96-101)");
			return NNRT_ERROR_ARGUMENT;
		}
		std::vector<char> keep(finer.idx.size(), 1);
		for (int s : sample) {
			keep[s] = 0;
			cur.idx.push_back(finer.idx[s]);
			for (int c = 0; c < 3; c++) cur.pos.push_back(finer.pos[3 * s + c]);
		}
		std::vector<int64_t> fidx;
		std::vector<float> fpos;
		for (size_t i = 0; i < finer.idx.size(); i++) {
			if (!keep[i]) continue;
			fidx.push_back(finer.idx[i]);
			for (int c = 0; c < 3; c++) fpos.push_back(finer.pos[3 * i + c]);
		}
		finer.idx.swap(fidx);
		finer.pos.swap(fpos);
	}
	std::vector<int> first_virtual(layer_count);
	h.layer_counts.assign(layer_count, 0);
	h.radii.assign(layer_count, 0.f);
	int vc = 0;
	for (int l = 0; l < layer_count; l++) {
		first_virtual[l] = vc;
		h.layer_counts[l] = static_cast<int>(layers[l].idx.size());
		h.radii[l] = layers[l].radius;
		vc += h.layer_counts[l];
	}
	for (int l = layer_count - 1; l >= 1; l--) {
		Layer& cur = layers[l];
		Layer& finer = layers[l - 1];
		const int ns = static_cast<int>(finer.idx.size());
		std::vector<int32_t> adj(static_cast<size_t>(ns) * max_degree);
		for (int s = 0; s < ns; s++) {
			int32_t* row = &adj[static_cast<size_t>(s) * max_degree];
			knn_sorted(&finer.pos[3 * s], cur.pos, max_degree, row);
			std::sort(row, row + max_degree, std::greater<int32_t>());
		}
		std::vector<int32_t> raw(static_cast<size_t>(ns) * max_degree * 2, -1);
		for (int s = 0; s < ns; s++)
			for (int k = 0; k < max_degree; k++) {
				const int32_t t = adj[static_cast<size_t>(s) * max_degree + k];
				int32_t* out = &raw[(static_cast<size_t>(ns - 1 - s) * max_degree + k) * 2];
				if (t != -1) {
					out[0] = first_virtual[l - 1] + s;
					out[1] = first_virtual[l] + t;
				}
			}
		for (size_t e = 0; e < raw.size() / 2; e++) {
			if (raw[2 * e] == -1) continue;
			finer.edges.push_back(raw[2 * e]);
			finer.edges.push_back(raw[2 * e + 1]);
		}
	}
	h.edges.clear();
	h.edge_layers.clear();
	for (int l = layer_count - 1; l >= 0; l--) {
		if (l >= layer_count - 1) continue;
		for (size_t e = 0; e < layers[l].edges.size() / 2; e++) {
			h.edges.push_back(layers[l].edges[2 * e]);
			h.edges.push_back(layers[l].edges[2 * e + 1]);
			h.edge_layers.push_back(static_cast<int8_t>(l + 1));
		}
	}
	h.virtual_indices.clear();
	for (int l = 0; l < layer_count; l++)
		for (int64_t i : layers[l].idx) h.virtual_indices.push_back(i);
	return NNRT_OK;
}

// WarpField.cpp:249-263: squared distance to the nearest other node (N == 1: coverage, un-squared as written)
void node_coverage_weights(const float* nodes, int N, float coverage, std::vector<float>& out) {
	out.assign(N, 0.f);
	if (N == 1) {
		out[0] = coverage;
		return;
	}
	for (int i = 0; i < N; i++) {
		float d2[2] = {INFINITY, INFINITY};
		int max_at = 0;
		float maxd = INFINITY;
		for (int j = 0; j < N; j++) {
			const float dx = nodes[3 * j] - nodes[3 * i], dy = nodes[3 * j + 1] - nodes[3 * i + 1], dz = nodes[3 * j + 2] - nodes[3 * i + 2];
			const float sq = (dx * dx + dy * dy) + dz * dz;
			if (sq < maxd) {
				d2[max_at] = sq;
				max_at = d2[1] > d2[0] ? 1 : 0;
				maxd = d2[max_at];
			}
		}
		const float d = std::sqrt(std::max(d2[0], d2[1]));
		out[i] = d * d;
	}
}

} // namespace nnrt
