// Hierarchy construction bookkeeping for the warp field -- HierarchicalGraphWarpField::RebuildRegularizationLayers
// (cpp/geometry/HierarchicalGraphWarpField.cpp:74-199): median-grid subsampling per layer
// (GeometrySamplingMedian.h:260-290, GeometrySamplingGridBinning.h:27-46), K-NN edges from each finer layer into the next
// coarser one, sorted descending and laid out in flipped source order (HierarchicalGraphWarpFieldImpl.h:218-297).
// Runs once per warp field (not per GN iteration). Order-nondeterministic parts of the reference (hash-map bin order,
// atomic bin fill) are made deterministic: medoid sums in ascending point order, coarse samples in ascending index.
// The O(n^2) steps (medoids, K-NN rows, coverage weights) run through HierarchyOps: hierarchy.hip on the GPU.
#include "warp_field.hpp"

#include <algorithm>

namespace nnrt {

nnrt_status build_hierarchy(const float* nodes, int N, float coverage, int layer_count, int max_degree, const float* radii, HierarchyOps& ops,
                            Hierarchy& h) {
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
		std::vector<uint8_t> medoid;
		if (nnrt_status st = ops.medoid_flags(finer.pos, cur.radius * 2, medoid)) return st;
		std::vector<int> sample;   // ascending
		for (size_t i = 0; i < medoid.size(); i++)
			if (medoid[i]) sample.push_back(static_cast<int>(i));
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
		std::vector<int32_t> adj;
		if (nnrt_status st = ops.knn_rows(finer.pos, cur.pos, max_degree, adj)) return st;
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

} // namespace nnrt
