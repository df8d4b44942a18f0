// Schur corner of the arrowhead solve: tile-sparse supernodal Cholesky (SolveBlockSparseArrowheadCholesky.cpp:30-95
// factors S = C - B^T D^-1 B with a dense potrf; SolveCholesky{CPU,CUDA}.cpp). The corner of a deformation-graph hierarchy
// is the Schur complement of a 2-D node grid: every corner node couples only to the corner nodes it shares a stem node
// with (and to its own corner edges, >= 3 layers), so S and its factor are sparse. Here:
//
//   host (once per hierarchy, CornerSolver::prepare): nested-dissection order of the corner nodes (coordinate bisection
//   when node positions are given, else BFS level-set separators; separators thinned; leaves of ND_LEAF nodes), every ND group starting on a 64-unknown tile boundary (identity padding), the
//   tile structure of L (symbolic factorisation over the tile elimination tree) and its levels (tile columns whose
//   subtrees are independent share a level);
//   device: one launch per level (k_corner_factor). Its panel workgroups factor the level's tile columns -- each stages
//   its diagonal tile and its panel tile with the updates of the previous level's columns applied (f32 MFMA), then one
//   wave eliminates the 64 columns in registers (L_JJ and L_IJ = A_IJ L_JJ^-T in one pass, the right-hand side riding
//   along as the diagonal workgroup's augmented row); its trailing workgroups apply the previous level's updates to
//   every later structurally non-zero tile. Back substitution runs one launch per level from the root down
//   (k_corner_back). Only structurally non-zero tiles are stored (slot-major 64 x 64 tiles).
//
// Race freedom: a launch reads only tiles finished by earlier launches and writes tiles no other workgroup of the same
// launch reads: the diagonal factor L_JJ goes to its own array (ldiag), never over A_JJ, which the column's other panel
// workgroups stage concurrently. Nothing depends on workgroup co-residency or dispatch order; the corner size is bounded
// by memory only.
//
// Numerics: the same float operations per tile as a right-looking blocked Cholesky (MFMA tile products, column
// eliminations in ascending order); the elimination order (nested dissection) differs from the reference's natural
// order, which changes float rounding only (the tests hold the solve against the oracle and an fp64 solution).
#include <algorithm>
#include <cfloat>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <tuple>

#include "arrow_device.hpp"

namespace nnrt {

constexpr int CT = 256;                       // threads per workgroup of the corner kernels
constexpr int CTF = 512;                      // threads per workgroup of the factor launches (k_corner_factor)
constexpr int TILE = CORNER_NB;               // 64
constexpr int TILE_ELEMS = TILE * TILE;
constexpr int CS4 = TILE + 4;                 // LDS row stride of staged tiles (16-B aligned rows for ds_read_b128)
#ifndef NNRT_ND_LEAF
#define NNRT_ND_LEAF 42
#endif
constexpr int ND_LEAF = NNRT_ND_LEAF;         // nodes per nested-dissection leaf: 252 unknowns = four tiles

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

// ===================================================================================================================
// host: ordering, symbolic factorisation, launch plan
// ===================================================================================================================
namespace {

struct Dissection {
	const std::vector<std::vector<int>>* adj = nullptr;
	const float* pos = nullptr;         // [nc, 3] corner node positions (nullable: graph-only separators)
	std::vector<int> sub, vis, level, mark;   // epoch marks: subset membership, BFS visit / side; BFS levels; separator
	int epoch = 0;
	std::vector<std::vector<int>> groups;   // elimination order: leaves and separators, post-order

	// BFS inside the subset marked `sep` from src; returns the visit order, level[] of every visited node
	void bfs(int sep, int src, std::vector<int>& order) {
		const int vep = ++epoch;
		order.clear();
		order.push_back(src);
		vis[src] = vep;
		level[src] = 0;
		for (size_t h = 0; h < order.size(); h++) {
			const int u = order[h];
			for (int v : (*adj)[u])
				if (sub[v] == sep && vis[v] != vep) {
					vis[v] = vep;
					level[v] = level[u] + 1;
					order.push_back(v);
				}
		}
	}

	void leaf(std::vector<int> nodes) {
		std::sort(nodes.begin(), nodes.end());
		if (!nodes.empty()) groups.push_back(std::move(nodes));
	}

	void dissect(std::vector<int> nodes) {
		if (static_cast<int>(nodes.size()) <= ND_LEAF) return leaf(std::move(nodes));
		std::sort(nodes.begin(), nodes.end());
		const int sep = ++epoch;
		for (int u : nodes) sub[u] = sep;
		// connected components (in ascending order of their smallest node)
		std::vector<std::vector<int>> comps;
		{
			const int cep = ++epoch;
			std::vector<int> order;
			for (int u : nodes) {
				if (vis[u] == cep) continue;
				bfs(sep, u, order);
				for (int v : order) vis[v] = cep;
				comps.push_back(order);
			}
		}
		if (comps.size() > 1) {   // independent subtrees; small components share leaves (no false coupling: same chain)
			std::vector<int> small;
			for (auto& c : comps) {
				if (static_cast<int>(c.size()) > ND_LEAF) {
					dissect(std::move(c));
					continue;
				}
				if (small.size() + c.size() > static_cast<size_t>(ND_LEAF)) {
					leaf(std::move(small));
					small.clear();
				}
				small.insert(small.end(), c.begin(), c.end());
			}
			leaf(std::move(small));
			return;
		}
		std::vector<int> left, right, mid;
		if (pos ? split_geometric(nodes, left, mid, right) : split_bfs(sep, nodes, left, mid, right)) {
			refine(left, mid, right);
			dissect(std::move(left));
			dissect(std::move(right));
			leaf(std::move(mid));
		} else {
			leaf(std::move(nodes));
		}
	}

	// separator from coordinate bisection: the half-sets at the median of the longest axis (ties by node index), the
	// separator the smaller of the two boundary sets (nodes with a neighbour across)
	bool split_geometric(const std::vector<int>& nodes, std::vector<int>& left, std::vector<int>& mid, std::vector<int>& right) {
		float lo[3] = {FLT_MAX, FLT_MAX, FLT_MAX}, hi[3] = {-FLT_MAX, -FLT_MAX, -FLT_MAX};
		for (int u : nodes)
			for (int c = 0; c < 3; c++) {
				lo[c] = std::min(lo[c], pos[3 * u + c]);
				hi[c] = std::max(hi[c], pos[3 * u + c]);
			}
		int ax = 0;
		for (int c = 1; c < 3; c++)
			if (hi[c] - lo[c] > hi[ax] - lo[ax]) ax = c;
		std::vector<int> order(nodes);
		std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return pos[3 * x + ax] < pos[3 * y + ax]; });
		const size_t half = order.size() / 2;
		const int side_l = ++epoch, side_r = ++epoch;
		for (size_t i = 0; i < order.size(); i++) vis[order[i]] = i < half ? side_l : side_r;
		std::vector<int> bl, br;
		for (int u : nodes) {
			const int other = vis[u] == side_l ? side_r : side_l;
			bool across = false;
			for (int v : (*adj)[u]) across |= vis[v] == other;
			if (across) (vis[u] == side_l ? bl : br).push_back(u);
		}
		const bool use_l = bl.size() <= br.size();
		const int sep_ep = ++epoch;
		for (int u : use_l ? bl : br) mark[u] = sep_ep;
		for (int u : nodes) {
			if (mark[u] == sep_ep) mid.push_back(u);
			else (vis[u] == side_l ? left : right).push_back(u);
		}
		return !left.empty() && !right.empty();
	}

	// separator from BFS level sets: the level at which the cumulative count first reaches half the nodes, BFS from a
	// pseudo-peripheral node (repeated BFS from the farthest node while the eccentricity grows)
	bool split_bfs(int sep, const std::vector<int>& nodes, std::vector<int>& left, std::vector<int>& mid, std::vector<int>& right) {
		std::vector<int> order;
		int start = nodes.front();
		bfs(sep, start, order);
		int ecc = level[order.back()];
		for (int it = 0; it < 4; it++) {
			const int far = order.back();
			std::vector<int> o2;
			bfs(sep, far, o2);
			if (level[o2.back()] <= ecc) break;
			ecc = level[o2.back()];
			start = far;
			order.swap(o2);
		}
		bfs(sep, start, order);
		const int L = level[order.back()];
		if (L < 2) return false;
		std::vector<int> cnt(static_cast<size_t>(L) + 1, 0);
		for (int u : nodes) cnt[static_cast<size_t>(level[u])]++;
		int s = 0, cum = 0;
		for (; s <= L; s++) {
			cum += cnt[static_cast<size_t>(s)];
			if (2 * cum >= static_cast<int>(nodes.size())) break;
		}
		s = std::min(std::max(s, 1), L - 1);
		for (int u : nodes) (level[u] < s ? left : level[u] > s ? right : mid).push_back(u);
		return true;
	}

	// a separator node with no neighbour on one side joins the other side (repeat until none moves): thinner separators,
	// shorter chains at the top of the elimination tree
	void refine(std::vector<int>& left, std::vector<int>& mid, std::vector<int>& right) {
		const int el = ++epoch, er = ++epoch, em = ++epoch;
		for (int u : left) vis[u] = el;
		for (int u : right) vis[u] = er;
		for (int u : mid) vis[u] = em;
		for (bool moved = true; moved;) {
			moved = false;
			std::vector<int> keep;
			for (int u : mid) {
				bool nl = false, nr = false;
				for (int v : (*adj)[u]) {
					nl |= vis[v] == el;
					nr |= vis[v] == er;
				}
				if (!nr) {
					vis[u] = el;
					left.push_back(u);
					moved = true;
				} else if (!nl) {
					vis[u] = er;
					right.push_back(u);
					moved = true;
				} else {
					keep.push_back(u);
				}
			}
			mid.swap(keep);
		}
	}
};

} // namespace

struct CornerPlan {
	int nc = 0, ld = 0, T = 0, H = 0;
	std::vector<int> node_row;        // [nc] first (permuted) unknown of each corner node
	std::vector<int> row_node;        // [ld] 8 * node + component, -1 on identity padding
	std::vector<int> tile_slot;       // [T * T] slot of tile (I, J), I >= J; -1: structurally zero
	std::vector<int2> slot_ij;        // [slots] (I, J)
	std::vector<int> level_off, level_panel;   // [H + 1] task offsets per factor launch, [H] panel tasks first
	std::vector<CornerTask> tasks;
	std::vector<int4> srcs;           // (slot X, slot Y, column k, 0): X Y^T update terms; rhs term L_k y_k uses X and k
	std::vector<int> back_off;        // [launches + 1] back-substitution chains per launch
	std::vector<int2> back_chains;    // (first column entry, column count): a chain of the elimination tree, root end first
	std::vector<int4> back_cols;      // (J, entry offset, entry count, outside entries)
	std::vector<int2> back_ent;       // (slot of L_IJ, I): per column the entries whose I lies outside the column's chain
	                                  // (x from earlier launches) first, then those inside it
	std::vector<int> back_pre_off;    // [launches + 1] per launch, its columns with outside entries (pre-sum launches)
	std::vector<int2> back_pre;       // (column index into back_cols, 1)
	// forward substitution L y = b (iterative refinement): the back chains in reverse (deepest launch first, each chain
	// from its bottom column up); per column its row entries (slot of L_Jk, k), k < J
	std::vector<int> fwd_off;
	std::vector<int2> fwd_chains;     // (first column entry, column count)
	std::vector<int4> fwd_cols;       // (J, entry offset, entry count, outside entries)
	std::vector<int2> fwd_ent;        // (slot of L_Jk, k): outside the column's chain first, then inside
	std::vector<int> fwd_pre_off;
	std::vector<int2> fwd_pre;
	// single-workgroup walks (k_corner_walk): per stream element (array: 0 tiles slot / 1 L_JJ^-1 / 2 L_JJ, index, x_off,
	// info); back: columns T-1 .. 0, each its entries L_IJ (ascending I) then its head; forward: columns 0 .. T-1, each its
	// row entries L_Jk (ascending k) then its head
	std::vector<int4> walk_back, walk_fwd;
	std::vector<int> corner_edges;    // edges between two corner nodes (>= 3 layers)
	// dataflow launches (k_corner_flow): per back chain b (back column first, column count, forward column first, parent
	// back chain or -1); columns + child chains; the back chain of every tile column
	std::vector<int4> flow_chains;
	std::vector<int> flow_need, col_chain;
};

static CornerPlan plan_corner(const int32_t* edges, int E, int n0, int N, const float* corner_pos, bool trim = true) {
	CornerPlan p;
	const int nc = N - n0;
	p.nc = nc;
	if (nc <= 0) return p;
	// corner adjacency: corner edges + pairs of corner nodes sharing a stem node (the Schur fill B^T D^-1 B)
	std::vector<std::vector<int>> adj(static_cast<size_t>(nc)), stem_targets(static_cast<size_t>(std::max(n0, 0)));
	for (int e = 0; e < E; e++) {
		const int i = edges[2 * e], j = edges[2 * e + 1];
		if (i >= n0) {
			adj[static_cast<size_t>(i - n0)].push_back(j - n0);
			adj[static_cast<size_t>(j - n0)].push_back(i - n0);
			p.corner_edges.push_back(e);
		} else {
			stem_targets[static_cast<size_t>(i)].push_back(j - n0);
		}
	}
	for (auto& ts : stem_targets)
		for (int a : ts)
			for (int b : ts)
				if (a != b) adj[static_cast<size_t>(a)].push_back(b);
	for (auto& a : adj) {
		std::sort(a.begin(), a.end());
		a.erase(std::unique(a.begin(), a.end()), a.end());
	}
	// nested dissection
	Dissection nd;
	nd.adj = &adj;
	nd.pos = corner_pos;
	nd.mark.assign(static_cast<size_t>(nc), 0);
	nd.sub.assign(static_cast<size_t>(nc), 0);
	nd.vis.assign(static_cast<size_t>(nc), 0);
	nd.level.assign(static_cast<size_t>(nc), 0);
	{
		std::vector<int> all(static_cast<size_t>(nc));
		for (int a = 0; a < nc; a++) all[static_cast<size_t>(a)] = a;
		nd.dissect(std::move(all));
	}
	// layout: every group starts on a tile boundary
	p.node_row.assign(static_cast<size_t>(nc), -1);
	int off = 0;
	for (const auto& g : nd.groups) {
		off = (off + TILE - 1) / TILE * TILE;
		for (int a : g) {
			p.node_row[static_cast<size_t>(a)] = off;
			off += 6;
		}
	}
	p.ld = (off + TILE - 1) / TILE * TILE;
	const int T = p.T = p.ld / TILE;
	p.row_node.assign(static_cast<size_t>(p.ld), -1);
	for (int a = 0; a < nc; a++)
		for (int c = 0; c < 6; c++) p.row_node[static_cast<size_t>(p.node_row[static_cast<size_t>(a)] + c)] = 8 * a + c;
	// initial tile structure (strictly lower tiles per column), then the symbolic factorisation over the elimination tree
	std::vector<std::vector<int>> cs(static_cast<size_t>(T));   // cs[J]: rows I > J of column J's non-zero tiles
	for (int a = 0; a < nc; a++) {
		const int ra = p.node_row[static_cast<size_t>(a)];
		for (int b : adj[static_cast<size_t>(a)]) {
			const int rb = p.node_row[static_cast<size_t>(b)];
			for (int ti = ra / TILE; ti <= (ra + 5) / TILE; ti++)
				for (int tj = rb / TILE; tj <= (rb + 5) / TILE; tj++)
					if (ti > tj) cs[static_cast<size_t>(tj)].push_back(ti);
		}
		if (ra / TILE != (ra + 5) / TILE) cs[static_cast<size_t>(ra / TILE)].push_back((ra + 5) / TILE);   // a node straddling two tiles
	}
	std::vector<int> parent(static_cast<size_t>(T), -1), lvl(static_cast<size_t>(T), 0);
	for (int J = 0; J < T; J++) {
		auto& c = cs[static_cast<size_t>(J)];
		std::sort(c.begin(), c.end());
		c.erase(std::unique(c.begin(), c.end()), c.end());
		if (c.empty()) continue;
		const int par = c.front();
		parent[static_cast<size_t>(J)] = par;
		auto& pc = cs[static_cast<size_t>(par)];
		pc.insert(pc.end(), c.begin() + 1, c.end());
	}
	for (int J = 0; J < T; J++)
		if (parent[static_cast<size_t>(J)] >= 0)
			lvl[static_cast<size_t>(parent[static_cast<size_t>(J)])] =
			    std::max(lvl[static_cast<size_t>(parent[static_cast<size_t>(J)])], lvl[static_cast<size_t>(J)] + 1);
	p.H = 0;
	for (int J = 0; J < T; J++) p.H = std::max(p.H, lvl[static_cast<size_t>(J)] + 1);
	// slots: per column its diagonal tile, then its panel tiles
	p.tile_slot.assign(static_cast<size_t>(T) * T, -1);
	for (int J = 0; J < T; J++) {
		p.tile_slot[static_cast<size_t>(J) * T + J] = static_cast<int>(p.slot_ij.size());
		p.slot_ij.push_back(make_int2(J, J));
		for (int I : cs[static_cast<size_t>(J)]) {
			p.tile_slot[static_cast<size_t>(I) * T + J] = static_cast<int>(p.slot_ij.size());
			p.slot_ij.push_back(make_int2(I, J));
		}
	}
	auto slot = [&](int I, int J) { return p.tile_slot[static_cast<size_t>(I) * T + J]; };
	// update terms: column k contributes L_Ik L_Jk^T to every tile (I, J), I >= J in its structure, applied at launch
	// lvl[k] + 1 -- by the panel of column J if J sits at that level, else by a trailing workgroup
	std::map<std::tuple<int, int, int>, std::vector<int>> contrib;   // (launch, J, I) -> columns k, ascending
	for (int k = 0; k < T; k++) {
		const auto& c = cs[static_cast<size_t>(k)];
		for (size_t x = 0; x < c.size(); x++)
			for (size_t y = 0; y <= x; y++) contrib[std::make_tuple(lvl[static_cast<size_t>(k)] + 1, c[y], c[x])].push_back(k);
	}
	auto terms = [&](int launch, int J, int I) -> const std::vector<int>* {
		auto it = contrib.find(std::make_tuple(launch, J, I));
		return it == contrib.end() ? nullptr : &it->second;
	};
	// per column: its real rows, a prefix (every ND group starts on a tile boundary); else all 64
	std::vector<int> col_real(static_cast<size_t>(T), TILE);
	for (int J = 0; J < T && trim; J++) {
		int nreal = 0;
		for (int r = 0; r < TILE; r++) nreal += p.row_node[static_cast<size_t>(J) * TILE + r] >= 0;
		for (int r = 0; r < TILE; r++)
			if ((p.row_node[static_cast<size_t>(J) * TILE + r] >= 0) != (r < nreal)) nreal = TILE;
		col_real[static_cast<size_t>(J)] = nreal;
	}
	// a term over source column k runs the MFMA steps s < its real columns (the 32 x 32 x 2 step s consumes k-columns s
	// and 32 + s; the padding columns of L_Ik are exact zeros), in groups of four: srcs.w
	auto src = [&](int a, int b, int k) {
		const int nr = col_real[static_cast<size_t>(k)];
		return make_int4(a, b, k, nr > TILE / 2 ? 8 : (nr + 3) / 4);
	};
	p.level_off.push_back(0);
	for (int l = 0; l < p.H; l++) {
		int panels = 0;
		for (int J = 0; J < T; J++) {
			if (lvl[static_cast<size_t>(J)] != l) continue;
			const std::vector<int>* dterms = terms(l, J, J);
			std::vector<int> rows(1, J);
			rows.insert(rows.end(), cs[static_cast<size_t>(J)].begin(), cs[static_cast<size_t>(J)].end());
			const int nreal = col_real[static_cast<size_t>(J)];
			for (int I : rows) {
				CornerTask t{};
				t.I = I;
				t.J = J;
				t.nreal = nreal;
				t.slot_t = slot(I, J);
				t.slot_d = slot(J, J);
				t.src = static_cast<int>(p.srcs.size());
				if (dterms)
					for (int k : *dterms) p.srcs.push_back(src(slot(J, k), slot(J, k), k));
				t.nd = dterms ? static_cast<int>(dterms->size()) : 0;
				if (I != J) {
					const std::vector<int>* pterms = terms(l, J, I);
					if (pterms)
						for (int k : *pterms) p.srcs.push_back(src(slot(I, k), slot(J, k), k));
					t.np = pterms ? static_cast<int>(pterms->size()) : 0;
				}
				p.tasks.push_back(t);
				panels++;
			}
		}
		p.level_panel.push_back(panels);
		for (auto it = contrib.lower_bound(std::make_tuple(l, -1, -1)); it != contrib.end() && std::get<0>(it->first) == l; ++it) {
			const int J = std::get<1>(it->first), I = std::get<2>(it->first);
			if (lvl[static_cast<size_t>(J)] == l) continue;   // the panel's own staging
			CornerTask t{};
			t.I = I;
			t.J = J;
			t.nreal = TILE;
			t.slot_t = slot(I, J);
			t.slot_d = -1;
			t.src = static_cast<int>(p.srcs.size());
			for (int k : it->second) p.srcs.push_back(src(slot(I, k), slot(J, k), k));
			t.nd = static_cast<int>(it->second.size());
			p.tasks.push_back(t);
		}
		p.level_off.push_back(static_cast<int>(p.tasks.size()));
	}

	// back substitution over chains of the elimination tree: a chain starts at a root or at a child of a node with two or
	// more children and follows single children down; one workgroup walks a chain from its root end, so a launch holds
	// every chain at the same number of branchings below the root (x of every column above a chain's top is known
	// before its launch: struct(J) holds ancestors only)
	std::vector<std::vector<int>> kids(static_cast<size_t>(T));
	for (int J = 0; J < T; J++)
		if (parent[static_cast<size_t>(J)] >= 0) kids[static_cast<size_t>(parent[static_cast<size_t>(J)])].push_back(J);
	std::vector<std::vector<int>> chains_at;   // chain tops per depth
	std::vector<std::pair<int, int>> stack;    // (chain top, depth)
	for (int J = T - 1; J >= 0; J--)
		if (parent[static_cast<size_t>(J)] < 0) stack.push_back({J, 0});
	std::vector<std::vector<int>> chain_cols;
	std::vector<int> chain_depth;
	while (!stack.empty()) {
		const auto [top, d] = stack.back();
		stack.pop_back();
		std::vector<int> cols(1, top);
		while (kids[static_cast<size_t>(cols.back())].size() == 1) cols.push_back(kids[static_cast<size_t>(cols.back())][0]);
		for (int c : kids[static_cast<size_t>(cols.back())]) stack.push_back({c, d + 1});
		chain_cols.push_back(std::move(cols));
		chain_depth.push_back(d);
	}
	int depth_max = 0;
	for (int d : chain_depth) depth_max = std::max(depth_max, d);
	std::vector<int> chain_of(static_cast<size_t>(T), -1);
	for (size_t c = 0; c < chain_cols.size(); c++)
		for (int J : chain_cols[c]) chain_of[static_cast<size_t>(J)] = static_cast<int>(c);
	p.back_off.push_back(0);
	p.back_pre_off.push_back(0);
	std::vector<int> bidx(chain_cols.size(), -1);   // chain -> back chain index
	for (int d = 0; d <= depth_max; d++) {
		for (size_t c = 0; c < chain_cols.size(); c++) {
			if (chain_depth[c] != d) continue;
			bidx[c] = static_cast<int>(p.back_chains.size());
			p.back_chains.push_back(make_int2(static_cast<int>(p.back_cols.size()), static_cast<int>(chain_cols[c].size())));
			for (int J : chain_cols[c]) {
				const auto& cc = cs[static_cast<size_t>(J)];
				int outside = 0;
				for (int I : cc) outside += chain_of[static_cast<size_t>(I)] != static_cast<int>(c);
				if (outside > 0) p.back_pre.push_back(make_int2(static_cast<int>(p.back_cols.size()), 1));
				p.back_cols.push_back(make_int4(J, static_cast<int>(p.back_ent.size()), static_cast<int>(cc.size()), outside));
				for (int pass = 0; pass < 2; pass++)
					for (int I : cc)
						if ((chain_of[static_cast<size_t>(I)] == static_cast<int>(c)) == (pass == 1)) p.back_ent.push_back(make_int2(slot(I, J), I));
			}
		}
		p.back_off.push_back(static_cast<int>(p.back_chains.size()));
		p.back_pre_off.push_back(static_cast<int>(p.back_pre.size()));
	}
	// single-workgroup walk streams
	{
		std::vector<std::vector<int>> rowk(static_cast<size_t>(T));   // rowk[J]: k < J with a stored tile (J, k), ascending
		for (int k = 0; k < T; k++)
			for (int I : cs[static_cast<size_t>(k)]) rowk[static_cast<size_t>(I)].push_back(k);
		auto head = [&](int J) { return make_int4(1, J, J * TILE, 1); };   // L_JJ^-1 of every column (k_corner_invert)
		for (int J = T - 1; J >= 0; J--) {
			for (int I : cs[static_cast<size_t>(J)]) p.walk_back.push_back(make_int4(0, slot(I, J), I * TILE, -1));
			p.walk_back.push_back(head(J));
		}
		for (int J = 0; J < T; J++) {
			for (int k : rowk[static_cast<size_t>(J)]) p.walk_fwd.push_back(make_int4(0, slot(J, k), k * TILE, -1));
			p.walk_fwd.push_back(head(J));
		}
	}
	// dataflow plan: chain parents (the chain of the top column's parent), columns + child chains, column -> chain
	p.flow_chains.assign(p.back_chains.size(), make_int4(0, 0, 0, -1));
	p.flow_need.assign(p.back_chains.size(), 0);
	p.col_chain.assign(static_cast<size_t>(T), -1);
	for (size_t c = 0; c < chain_cols.size(); c++) {
		const int b = bidx[c];
		const int top = chain_cols[c].front(), bottom = chain_cols[c].back();
		const int par = parent[static_cast<size_t>(top)];
		p.flow_chains[static_cast<size_t>(b)] = make_int4(p.back_chains[static_cast<size_t>(b)].x, p.back_chains[static_cast<size_t>(b)].y, 0,
		                                                  par < 0 ? -1 : bidx[static_cast<size_t>(chain_of[static_cast<size_t>(par)])]);
		p.flow_need[static_cast<size_t>(b)] = static_cast<int>(chain_cols[c].size() + kids[static_cast<size_t>(bottom)].size());
		for (int J : chain_cols[c]) p.col_chain[static_cast<size_t>(J)] = b;
	}
	// forward chains: row entries of every column, then the back launches in reverse with each chain reversed
	std::vector<std::vector<int2>> rows(static_cast<size_t>(T));
	for (size_t sl = 0; sl < p.slot_ij.size(); sl++)
		if (p.slot_ij[sl].x != p.slot_ij[sl].y) rows[static_cast<size_t>(p.slot_ij[sl].x)].push_back(make_int2(static_cast<int>(sl), p.slot_ij[sl].y));
	p.fwd_off.push_back(0);
	p.fwd_pre_off.push_back(0);
	for (int l = static_cast<int>(p.back_off.size()) - 2; l >= 0; l--) {
		for (int c = p.back_off[static_cast<size_t>(l)]; c < p.back_off[static_cast<size_t>(l) + 1]; c++) {
			const int2 ch = p.back_chains[static_cast<size_t>(c)];
			p.flow_chains[static_cast<size_t>(c)].z = static_cast<int>(p.fwd_cols.size());
			p.fwd_chains.push_back(make_int2(static_cast<int>(p.fwd_cols.size()), ch.y));
			for (int q = ch.y - 1; q >= 0; q--) {
				const int4 bc = p.back_cols[static_cast<size_t>(ch.x + q)];
				const int own = chain_of[static_cast<size_t>(bc.x)];
				const auto& rw = rows[static_cast<size_t>(bc.x)];
				int outside = 0;
				for (const int2& e : rw) outside += chain_of[static_cast<size_t>(e.y)] != own;
				if (outside > 0) p.fwd_pre.push_back(make_int2(static_cast<int>(p.fwd_cols.size()), 1));
				p.fwd_cols.push_back(make_int4(bc.x, static_cast<int>(p.fwd_ent.size()), static_cast<int>(rw.size()), outside));
				for (int pass = 0; pass < 2; pass++)
					for (const int2& e : rw)
						if ((chain_of[static_cast<size_t>(e.y)] == own) == (pass == 1)) p.fwd_ent.push_back(e);
			}
		}
		p.fwd_off.push_back(static_cast<int>(p.fwd_chains.size()));
		p.fwd_pre_off.push_back(static_cast<int>(p.fwd_pre.size()));
	}
	return p;
}

// ===================================================================================================================
// device
// ===================================================================================================================
__device__ inline float lane_bcast(float v, int src) {
	return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), src));
}

__global__ void k_corner_init(CornerInitArgs a, const float* __restrict__ diag, const float* __restrict__ rhs) {
	corner_init_thread(static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x, a, diag, rhs);
}

// corner off-diagonal blocks (edges between two corner nodes, >= 3 layers; the reference drops them, A3): each entry of
// the wing block is added once, at its lower-triangle position (S is symmetric)
__global__ void k_corner_offdiag(const int* __restrict__ corner_edges, int n0, const int32_t* __restrict__ edges, const float* __restrict__ wing,
                                 CornerMap m) {
	const int e = corner_edges[blockIdx.x];
	const int t = threadIdx.x;
	if (t >= 36) return;
	const int a = edges[2 * e] - n0, b = edges[2 * e + 1] - n0;
	int R = m.node_row[a] + t / 6, C = m.node_row[b] + t % 6;
	if (R < C) {
		const int x = R;
		R = C;
		C = x;
	}
	atomicAdd(corner_entry(m, R, C), wing[static_cast<int64_t>(e) * 36 + t]);
}

__device__ inline int quad_row(int v, int lane) { return (v & 3) + 8 * (v >> 2) + 4 * (lane >> 5); }

// 32 MFMA steps of quadrant (qr, qc) of X Y^T for 64 x 64 tiles: lane l feeds A[i = l & 31][k'] = X[32 qr + i][32 (l >> 5) + s]
// and B[k'][j] = Y[32 qc + j][32 (l >> 5) + s] to step s (vx / vy: the lane's 32 contiguous floats of its X / Y row), so
// the 32 steps x 2 lane halves cover the 64-wide k range. C/D map: column l & 31, row (v & 3) + 8 (v >> 2) + 4 (l >> 5).
__device__ __forceinline__ f32x16 term_mfma(const float4 (&vx)[8], const float4 (&vy)[8], f32x16 acc) {
#pragma unroll
	for (int q = 0; q < 8; q++) {
		acc = __builtin_amdgcn_mfma_f32_32x32x2f32(vx[q].x, vy[q].x, acc, 0, 0, 0);
		acc = __builtin_amdgcn_mfma_f32_32x32x2f32(vx[q].y, vy[q].y, acc, 0, 0, 0);
		acc = __builtin_amdgcn_mfma_f32_32x32x2f32(vx[q].z, vy[q].z, acc, 0, 0, 0);
		acc = __builtin_amdgcn_mfma_f32_32x32x2f32(vx[q].w, vy[q].w, acc, 0, 0, 0);
	}
	return acc;
}

// s_waitcnt vmcnt(n) for a run-time n (even values up to 62: two DMA instructions per wave per tile)
__device__ __forceinline__ void wait_vmcnt(int n) {
	switch (n) {
#define W_(k) \
	case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
		W_(0) W_(2) W_(4) W_(6) W_(8) W_(10) W_(12) W_(14) W_(16) W_(18) W_(20) W_(22) W_(24) W_(26) W_(28) W_(30)
		W_(32) W_(34) W_(36) W_(38) W_(40) W_(42) W_(44) W_(46) W_(48) W_(50) W_(52) W_(54) W_(56) W_(58) W_(60) W_(62)
#undef W_
		default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
	}
}
// workgroup barrier for LDS traffic only: retires this wave's LDS operations, leaves LDS-DMA loads in flight
__device__ __forceinline__ void lds_barrier() {
	asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
	__builtin_amdgcn_s_barrier();
}

// ---- panel staging through LDS (k_corner_factor's panel tasks) ----
// A term's operand tiles X, Y (64 x 64, row-major) arrive in LDS by LDS-DMA (global_load_lds, 16 B per lane, 1 KB per
// instruction: every request reads whole lines), laid out with the 16-B chunks of row r XOR-swizzled by r mod 16 so that
// the MFMA operand reads -- lane l: 32 contiguous floats of row 32 q + (l mod 32) -- fall in distinct banks; a group of
// four waves double-buffers its terms (the next term's DMA in flight while the current term's MFMAs run). Direct loads
// of the operands streamed them into the MFMAs one pair at a time, a memory round trip per quarter term (round 5 stamps:
// 4.7 k cycles per term, 2 k of them MFMA; issuing all 16 loads of a term first was slower still, the 64 lines of a
// lane group's rows then missed L1 8 times over). LDS-DMA staging: C5 staging 22 k -> 17 k cycles per level.
typedef __attribute__((address_space(3))) void factor_lds_t;
typedef const __attribute__((address_space(1))) void factor_global_t;
constexpr int TERM_FLOATS = 2 * TILE_ELEMS;   // one term's X and Y
constexpr int STAGE_WORDS = 2 * 2 * TERM_FLOATS;   // two groups x two buffers
static_assert(2 * TILE * CS4 <= 2 * TERM_FLOATS, "the staged tiles alias the first buffers");
// wave w (0..3) of a group: its 8 of the term's 32 pieces (4 of X, 4 of Y), swizzled
__device__ __forceinline__ void term_dma(const float* tiles, int4 s, float* buf, int w, int lane) {
#pragma unroll
	for (int h = 0; h < 2; h++) {
		const float* src = tiles + static_cast<int64_t>(h == 0 ? s.x : s.y) * TILE_ELEMS;
		float* dst = buf + h * TILE_ELEMS;
#pragma unroll
		for (int i = 0; i < 4; i++) {
			const int piece = 4 * w + i;                // rows 4 piece .. 4 piece + 3
			const int r = 4 * piece + (lane >> 4);      // this lane's row and physical chunk
			const int c = (lane & 15) ^ (r & 15);       // the logical chunk that lands there
			__builtin_amdgcn_global_load_lds((factor_global_t*)(src + r * TILE + 4 * c), (factor_lds_t*)(dst + piece * 256), 16, 0, 0);
		}
	}
}
// the term's MFMA steps for quadrant (qr, qc) from a staged (swizzled) buffer: the first 4 nq of the 32 (nq = srcs.w:
// the steps past the source column's real columns multiply exact zeros, and adding them changes nothing)
__device__ __forceinline__ f32x16 term_mfma_lds(const float* buf, int qr, int qc, int lane, f32x16 acc, int nq) {
	const int half = lane >> 5, l32 = lane & 31;
	const int rx = 32 * qr + l32, ry = 32 * qc + l32;
	if (nq >= 8) {
		float4 vx[8], vy[8];
#pragma unroll
		for (int q = 0; q < 8; q++) {
			vx[q] = *reinterpret_cast<const float4*>(buf + rx * TILE + 4 * ((8 * half + q) ^ (rx & 15)));
			vy[q] = *reinterpret_cast<const float4*>(buf + TILE_ELEMS + ry * TILE + 4 * ((8 * half + q) ^ (ry & 15)));
		}
		return term_mfma(vx, vy, acc);
	}
#pragma unroll
	for (int q = 0; q < 8; q++) {
		if (q < nq) {   // wave-uniform
			const float4 vx = *reinterpret_cast<const float4*>(buf + rx * TILE + 4 * ((8 * half + q) ^ (rx & 15)));
			const float4 vy = *reinterpret_cast<const float4*>(buf + TILE_ELEMS + ry * TILE + 4 * ((8 * half + q) ^ (ry & 15)));
			acc = __builtin_amdgcn_mfma_f32_32x32x2f32(vx.x, vy.x, acc, 0, 0, 0);
			acc = __builtin_amdgcn_mfma_f32_32x32x2f32(vx.y, vy.y, acc, 0, 0, 0);
			acc = __builtin_amdgcn_mfma_f32_32x32x2f32(vx.z, vy.z, acc, 0, 0, 0);
			acc = __builtin_amdgcn_mfma_f32_32x32x2f32(vx.w, vy.w, acc, 0, 0, 0);
		}
	}
	return acc;
}

// (L y) row t >> 2 for a 64 x 64 tile L and the 64-vector y: 4 threads per row, 16 columns each (all 4 get the sum)
__device__ inline float rhs_row_update(const float* L, const float* y, int t) {
	const int r = t >> 2, q4 = t & 3;
	const float* Lr = L + r * TILE + 16 * q4;
	const float* yq = y + 16 * q4;
	float s0 = 0.f, s1 = 0.f;
#pragma unroll
	for (int c = 0; c < 16; c += 2) {
		s0 += Lr[c] * yq[c];
		s1 += Lr[c + 1] * yq[c + 1];
	}
	float s = s0 + s1;
	s += __shfl_xor(s, 1);
	s += __shfl_xor(s, 2);
	return s;
}

__device__ inline float rhs_updates(const float* tiles, const int4* src, int n, const float* cb, int t) {
	float s = 0.f;
	for (int e = 0; e < n; e++) {
		const int4 q = src[e];
		s += rhs_row_update(tiles + static_cast<int64_t>(q.x) * TILE_ELEMS, cb + static_cast<int64_t>(q.z) * TILE, t);
	}
	return s;
}

// Column eliminations J0 <= j < J1 of the row pairs ap (lane = row), applied to the columns c < J1 only, in blocks of
// four: the four columns are factored among themselves, then applied to every later column c with four packed FMAs
// whose multipliers L_c,jb..jb+3 are read from lane c by readlane (scalar operands: nothing on the elimination path
// waits on LDS). Every element sees its updates in ascending column order.
template <int J0, int J1>
__device__ inline void eliminate_columns(f32x2 (&ap)[TILE], int lane, int& bad) {
	__shared__ float4 s_l4[2][TILE];   // s_l4[.][c] = (L_c,jb .. L_c,jb+3)
#pragma clang loop unroll(full)
	for (int jb = J0; jb < J1; jb += 4) {
		// The 4 x 4 diagonal sub-block is read once (10 independent readlanes) and factored wave-uniformly; every lane
		// then runs the same operations on its own row with the uniform multipliers (the values lanes jb..jb+3 compute).
		float M[4][4], Lu[4][4], rsv[4];
#pragma unroll
		for (int q = 0; q < 4; q++)
#pragma unroll
			for (int i = q; i < 4; i++) M[i][q] = lane_bcast(ap[jb + q].x, jb + i);
#pragma unroll
		for (int q = 0; q < 4; q++) {
			float piv = M[q][q];   // A_jj after the first j eliminations
			bad |= !(piv > 0.f);
			piv = piv > 0.f ? piv : 1.f;
			rsv[q] = __builtin_amdgcn_rsqf(piv);
#pragma unroll
			for (int i = q; i < 4; i++) Lu[i][q] = M[i][q] * rsv[q];
#pragma unroll
			for (int q2 = q + 1; q2 < 4; q2++)
#pragma unroll
				for (int i = q2; i < 4; i++) M[i][q2] = __builtin_fmaf(-Lu[i][q], Lu[q2][q], M[i][q2]);
		}
		float lx[4];
		f32x2 nl[4];
#pragma unroll
		for (int q = 0; q < 4; q++) {
			const f32x2 l = ap[jb + q] * rsv[q];   // (L_rj for rows r >= j of the diagonal block, panel / rhs entry)
			ap[jb + q] = l;
			lx[q] = l.x;
			nl[q] = -l;
#pragma unroll
			for (int q2 = q + 1; q2 < 4; q2++) {
				const float lc = Lu[q2][q];
				ap[jb + q2] = __builtin_elementwise_fma(nl[q], f32x2{lc, lc}, ap[jb + q2]);
			}
		}
		// next block's columns first (readlane: on the pivot chain), the rest from a wave-uniform 16-B LDS broadcast
		// whose latency hides behind them
		float4* row = &s_l4[(jb >> 2) & 1][0];
		if (jb + 8 < J1) row[lane] = make_float4(lx[0], lx[1], lx[2], lx[3]);
#pragma unroll
		for (int q = 0; q < 4; q++)   // q outer: consecutive FMAs are independent
#pragma unroll
			for (int c = jb + 4; c < J1 && c < jb + 8; c++) {
				const float lc = lane_bcast(lx[q], c);   // L_c,jb+q, c > jb + 3
				ap[c] = __builtin_elementwise_fma(nl[q], f32x2{lc, lc}, ap[c]);
			}
#pragma unroll
		for (int c0 = jb + 8; c0 < J1; c0 += 8) {   // chunks of 8 columns: 8 broadcasts in flight
			float4 L4[8];
#pragma unroll
			for (int u = 0; u < 8; u++)
				if (c0 + u < J1) L4[u] = row[c0 + u];
#pragma unroll
			for (int u = 0; u < 8; u++)
				if (c0 + u < J1) ap[c0 + u] = __builtin_elementwise_fma(nl[0], f32x2{L4[u].x, L4[u].x}, ap[c0 + u]);
#pragma unroll
			for (int u = 0; u < 8; u++)
				if (c0 + u < J1) ap[c0 + u] = __builtin_elementwise_fma(nl[1], f32x2{L4[u].y, L4[u].y}, ap[c0 + u]);
#pragma unroll
			for (int u = 0; u < 8; u++)
				if (c0 + u < J1) ap[c0 + u] = __builtin_elementwise_fma(nl[2], f32x2{L4[u].z, L4[u].z}, ap[c0 + u]);
#pragma unroll
			for (int u = 0; u < 8; u++)
				if (c0 + u < J1) ap[c0 + u] = __builtin_elementwise_fma(nl[3], f32x2{L4[u].w, L4[u].w}, ap[c0 + u]);
		}
	}
}

// Multi-wave elimination of a panel (k_corner_factor, NNRT_CORNER_ELIM_WAVES = EW > 0): the tile's 16 four-column
// blocks are dealt cyclically over EW waves (block b on wave b mod EW, lane = row, the A_JJ row and the panel row as
// one f32x2 per column as in eliminate_columns). Per block: its owner factors it (the 4 x 4 diagonal sub-block by
// readlane, wave-uniform, then every row), writes the block's L columns of every row to LDS, one workgroup barrier, and
// each wave applies them to its own later blocks (four packed FMAs per column, multipliers L_c,jb..jb+3 from a
// wave-uniform 16-B LDS read), nearest block first: the next owner's block is ready one update after the barrier, the
// other updates run on the other waves while it factors. Every element sees its updates in ascending column order.
#ifndef NNRT_CORNER_ELIM_WAVES
#define NNRT_CORNER_ELIM_WAVES 8
#endif
#ifndef NNRT_CORNER_ELIM_BW
#define NNRT_CORNER_ELIM_BW 4
#endif
#ifndef NNRT_CORNER_ELIM_PRIO
#define NNRT_CORNER_ELIM_PRIO 1
#endif
constexpr bool ELIM_PRIO = NNRT_CORNER_ELIM_PRIO != 0;   // the next block's owner at raised wave priority
constexpr int ELIM_WAVES = NNRT_CORNER_ELIM_WAVES;
constexpr int ELIM_BW = NNRT_CORNER_ELIM_BW;   // columns per block (8: two four-column sub-blocks factored by the owner)
static_assert(ELIM_WAVES == 0 || ELIM_WAVES == 4 || ELIM_WAVES == 8, "elimination waves");
static_assert((ELIM_BW == 4 || ELIM_BW == 8) && TILE / ELIM_BW >= ELIM_WAVES, "elimination blocks");
__device__ __forceinline__ void factor_block(f32x2* c4, int jb, int& bad) {
#ifdef NNRT_DEV_ELIM_NOFACTOR   // timing build only: no factorization (values meaningless)
	(void)jb;
	(void)bad;
#pragma unroll
	for (int q = 0; q < 4; q++) c4[q] = c4[q] * 0.5f;
	return;
#endif
	float M[4][4], Lu[4][4], rsv[4];
#pragma unroll
	for (int q = 0; q < 4; q++)
#pragma unroll
		for (int i = q; i < 4; i++) M[i][q] = lane_bcast(c4[q].x, jb + i);
#pragma unroll
	for (int q = 0; q < 4; q++) {
		const float piv = M[q][q];   // (not clamped: a non-positive pivot flags the factorization, whose values are dropped)
		bad |= !(piv > 0.f);
		rsv[q] = __builtin_amdgcn_rsqf(piv);
#pragma unroll
		for (int i = q; i < 4; i++) Lu[i][q] = M[i][q] * rsv[q];
#pragma unroll
		for (int q2 = q + 1; q2 < 4; q2++)
#pragma unroll
			for (int i = q2; i < 4; i++) M[i][q2] = __builtin_fmaf(-Lu[i][q], Lu[q2][q], M[i][q2]);
	}
#pragma unroll
	for (int q = 0; q < 4; q++) {
		const f32x2 l = c4[q] * rsv[q];
		c4[q] = l;
		const f32x2 nl = -l;
#pragma unroll
		for (int q2 = q + 1; q2 < 4; q2++) {
			const float lc = Lu[q2][q];
			c4[q2] = __builtin_elementwise_fma(nl, f32x2{lc, lc}, c4[q2]);
		}
	}
}

// development timing build only (-DNNRT_CORNER_STAMPS, tools/dev/stamps_build.sh): shader-clock stamps of the first
// workgroup of each factor launch at its phase boundaries, read back by nnrt_dev_corner_stamps
#ifdef NNRT_CORNER_STAMPS
// [level][workgroup][8]: shader clock at the phase boundaries 0-5 of every workgroup, the constant-rate clock at its start
// (6) and end (7, bit 62 set for trailing tasks)
__device__ unsigned long long g_corner_stamps[64][512][8];
// [level][workgroup][block][4]: multi-wave elimination, shader clock of block b + 1's owner at the start of iteration b,
// after its update by block b, after publishing block b + 1, and after the iteration's barrier
__device__ unsigned long long g_elim_stamps[16][128][16][4];
#ifdef NNRT_ELIM_STAMPS
#define ELIM_STAMP(blk, i)                                                                                              \
	do {                                                                                                                \
		if (lane == 0 && a.level < 16 && blockIdx.x < 128 && (blk) < 16) g_elim_stamps[a.level][blockIdx.x][blk][i] = __builtin_amdgcn_s_memtime(); \
	} while (0)
#else
#define ELIM_STAMP(blk, i) \
	do {                   \
	} while (0)
#endif
#define CORNER_STAMP(i)                                                                                                  \
	do {                                                                                                                 \
		if (threadIdx.x == 0 && a.level < 64 && blockIdx.x < 512) g_corner_stamps[a.level][blockIdx.x][i] = __builtin_amdgcn_s_memtime(); \
	} while (0)
#define CORNER_RT(i, flag)                                                                                               \
	do {                                                                                                                 \
		if (threadIdx.x == 0 && a.level < 64 && blockIdx.x < 512)                                                        \
			g_corner_stamps[a.level][blockIdx.x][i] = __builtin_amdgcn_s_memrealtime() | (flag);                         \
	} while (0)
#else
#define CORNER_RT(i, flag) \
	do {                   \
	} while (0)
#define CORNER_STAMP(i) \
	do {                \
	} while (0)
#define ELIM_STAMP(blk, i) \
	do {                   \
	} while (0)
#endif

// minimum over the 64 lanes (DPP row shifts, then row broadcasts into lane 63), wave-uniform result
__device__ inline int corner_wave_min_i32(int v) {
	constexpr int ID = 0x7fffffff;
	v = min(v, __builtin_amdgcn_update_dpp(ID, v, 0x111, 0xf, 0xf, false));   // row_shr:1
	v = min(v, __builtin_amdgcn_update_dpp(ID, v, 0x112, 0xf, 0xf, false));   // row_shr:2
	v = min(v, __builtin_amdgcn_update_dpp(ID, v, 0x114, 0xf, 0xf, false));   // row_shr:4
	v = min(v, __builtin_amdgcn_update_dpp(ID, v, 0x118, 0xf, 0xf, false));   // row_shr:8
	v = min(v, __builtin_amdgcn_update_dpp(ID, v, 0x142, 0xa, 0xf, false));   // row_bcast:15
	v = min(v, __builtin_amdgcn_update_dpp(ID, v, 0x143, 0xc, 0xf, false));   // row_bcast:31
	return __builtin_amdgcn_readlane(v, 63);
}

struct CornerFactorArgs {
	float* tiles;            // [slots, 64, 64]
	float* ldiag;            // [T, 64, 64] L_JJ (lower part; the part above the diagonal is not meaningful)
	float* cb;               // [ld] b_C -> y (forward substitution)
	const CornerTask* tasks; // this launch's tasks, panels first
	const int4* srcs;
	int n_panel;
	int* error_flag;
	int level;
	const float* sdiag;      // [ld] diag(S) before the factorization (nullable)
	unsigned* pivot_word;    // atomic minimum of pivot / diag(S) over the diagonal tasks (nullable)
	// the last level's launch (fold_invert: no k_corner_invert launch): its diagonal tasks invert their own tile after
	// the elimination, and n_inv extra workgroups (blockIdx >= n_tasks) invert the earlier levels' tiles inv_cols[.]
	int n_tasks, n_inv, invert_self;
	const int* inv_cols;
	float* minv;             // [T, 64, 64] M = L_JJ^-1
	unsigned* flow_ctl;      // zeroed by block 0 (the dataflow substitution's control words; nullable)
	int n_ctl;
};

// M = L^-1 for the 64 x 64 lower-triangular factor L (row-major lower part; the staging zeroes the part above the diagonal) in LDS. Forward
// substitution against the identity, all four waves: column c of M belongs to the lane quad (16 columns per wave), lane q
// of the quad holds M[4 i + q][c] and sums the terms k = q mod 4 of each row (the zero upper part of L lets every lane
// run the same unrolled stream); the quad's partials are summed by DPP and row r's entry is the sum times 1 / L_rr (the
// 64 reciprocals formed up front), so a row waits on one FMA, two DPP adds and a multiply instead of a division.
__device__ __forceinline__ float quad_xor(float v, int ctrl_sel) {   // 0: lanes 1,0,3,2; 1: lanes 2,3,0,1
	const int x = __builtin_bit_cast(int, v);
	return __builtin_bit_cast(float, ctrl_sel == 0 ? __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xf, 0xf, false)
	                                               : __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xf, 0xf, false));
}
// the lower part of the row-major tile L (global) into s_l (row stride CS4), zeros above the diagonal; nt threads
__device__ __forceinline__ void lower_to_lds(const float* L, float* s_l, int t, int nt) {
	const float4* L4 = reinterpret_cast<const float4*>(L);
	for (int i = t; i < TILE_ELEMS / 4; i += nt) {
		const int r = i >> 4, c0 = 4 * (i & 15);
		const float4 v = L4[i];
		*reinterpret_cast<float4*>(s_l + r * CS4 + c0) =
		    make_float4(c0 <= r ? v.x : 0.f, c0 + 1 <= r ? v.y : 0.f, c0 + 2 <= r ? v.z : 0.f, c0 + 3 <= r ? v.w : 0.f);
	}
}
// M = L^-1 from s_l (written and made visible by the caller); s_y: 64 floats of scratch LDS. Every thread of the
// workgroup calls it (one barrier inside); threads t < CT (four waves) compute and store M.
__device__ __forceinline__ void invert_lower_lds(const float* s_l, float* s_y, float* __restrict__ M, int t) {
	if (t < TILE) s_y[t] = 1.f / s_l[t * CS4 + t];
	__syncthreads();
	if (t >= CT) return;
	const int lane = t & 63, c = 16 * (t >> 6) + (lane >> 2), q = lane & 3;
	float m[TILE / 4];   // m[i] = M[4 i + q][c]
#pragma unroll
	for (int i = 0; i < TILE / 4; i++) m[i] = 0.f;
	// row r's L values (k = 4 i + q <= r + 3: L_rk = 0 above the diagonal, m = 0 where unset) are read one row ahead, so
	// a row's sum waits on its last product only, not on LDS
	float lr[TILE / 4], ln[TILE / 4];
	lr[0] = s_l[q];
#pragma unroll
	for (int r = 0; r < TILE; r++) {
		if (r + 1 < TILE) {
#pragma unroll
			for (int i = 0; i <= ((r + 1) >> 2); i++) ln[i] = s_l[(r + 1) * CS4 + 4 * i + q];
		}
		float a0 = 0.f, a1 = 0.f;
#pragma unroll
		for (int i = 0; i <= (r >> 2); i++) {
			if (i & 1) a1 = __builtin_fmaf(lr[i], m[i], a1);
			else a0 = __builtin_fmaf(lr[i], m[i], a0);
		}
#pragma unroll
		for (int i = 0; i < TILE / 4; i++) lr[i] = ln[i];
		float part = a0 + a1;
		part += quad_xor(part, 0);
		part += quad_xor(part, 1);
		const float v = ((c == r ? 1.f : 0.f) - part) * s_y[r];
		m[r >> 2] = q == (r & 3) ? v : m[r >> 2];
	}
#pragma unroll
	for (int i = 0; i < TILE / 4; i++) M[(4 * i + q) * TILE + c] = m[i];
}

// (workgroup 0 also zeroes the control words of the dataflow substitution launches that follow: k_corner_flow)
__global__ __launch_bounds__(CT) void k_corner_invert(const float* __restrict__ ldiag, float* __restrict__ minv, unsigned* __restrict__ flow_ctl,
                                                     int n_ctl) {
	__shared__ __attribute__((aligned(16))) float s_l[TILE * CS4];
	__shared__ float s_y[TILE];
	const int t = threadIdx.x;
	const int64_t J = blockIdx.x;
	if (J == 0)
		for (int i = t; i < n_ctl; i += CT) flow_ctl[i] = 0u;
	lower_to_lds(ldiag + J * TILE_ELEMS, s_l, t, CT);
	__syncthreads();
	invert_lower_lds(s_l, s_y, minv + J * TILE_ELEMS, t);
}

// One launch per level of the tile elimination tree; workgroups of 8 waves (CTF threads).
//   panel (I, J) (blockIdx < n_panel): s_d = A_JJ - sum_k L_Jk L_Jk^T and s_p = A_IJ - sum_k L_Ik L_Jk^T over the columns k of
//   the previous level (MFMA, one 32 x 32 quadrant per wave): waves 0-3 stage s_d while waves 4-7 stage s_p (below the
//   diagonal) or the augmented row b_J - sum_k L_Jk y_k (the diagonal workgroup), so a panel's two tiles' update terms run
//   side by side. Wave 0 then holds both (lane = row) in registers and eliminates the column's real columns (a tile
//   whose last rows are identity padding stops there: the padding's columns are the identity, their elimination changes
//   nothing), applying each to the panel row as it goes (one packed FMA per column pair): up to 32 columns in one run,
//   else two 32-column halves joined by a rank-32 MFMA update on waves 1-3.
//   trailing (blockIdx >= n_panel): A_IJ -= sum_k L_Ik L_Jk^T (and b_J -= sum_k L_Jk y_k on diagonal tiles), waves 0-3.
__global__ __launch_bounds__(CTF) void k_corner_factor(CornerFactorArgs a) {
	// the term buffers of the panel staging; then A_JJ (s_d) and A_IJ (s_p) after the previous level's updates, in the
	// first buffers of groups 0 and 1
	__shared__ __attribute__((aligned(16))) float s_stage[STAGE_WORDS];
	float* const s_d = s_stage;
	float* const s_p = s_stage + 2 * TERM_FLOATS;
	__shared__ float s_b[TILE];         // b_J after the previous level's updates (diagonal workgroup)
	const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
	CORNER_STAMP(0);
	CORNER_RT(6, 0ull);
	if (a.flow_ctl && blockIdx.x == 0)
		for (int i = t; i < a.n_ctl; i += CTF) a.flow_ctl[i] = 0u;
	if (static_cast<int>(blockIdx.x) >= a.n_tasks) {   // an earlier level's diagonal inverse (the last launch's extra workgroups)
		const int64_t J = a.inv_cols[blockIdx.x - a.n_tasks];
		lower_to_lds(a.ldiag + J * TILE_ELEMS, s_stage, t, CTF);
		__syncthreads();
		invert_lower_lds(s_stage, s_b, a.minv + J * TILE_ELEMS, t);
		return;
	}
	const CornerTask tk = a.tasks[blockIdx.x];
	const int4* src = a.srcs + tk.src;
	if (static_cast<int>(blockIdx.x) >= a.n_panel) {
		// waves 0-3: the tile's quadrants, the terms double-buffered in LDS as in the panel staging; waves 4-7: b_J's
		// terms on diagonal tiles
		const int w4 = wave & 3, qr = w4 >> 1, qc = w4 & 1;
		const int n_g = wave < 4 ? tk.nd : 0;
		f32x16 acc = {};
		float* C = a.tiles + static_cast<int64_t>(tk.slot_t) * TILE_ELEMS + 32 * qc + (lane & 31);
		float cv[16];   // the tile's own entries first (they land while the terms stream)
		if (wave < 4) {
#pragma unroll
			for (int v = 0; v < 16; v++) cv[v] = C[(32 * qr + quad_row(v, lane)) * TILE];
		}
		if (n_g > 0) term_dma(a.tiles, src[0], s_stage, w4, lane);
		float bs = 0.f, bv = 0.f;
		float* bj = a.cb + static_cast<int64_t>(tk.J) * TILE;
		const int t4 = t - 4 * 64;
		if (wave >= 4 && tk.I == tk.J) {
			bv = (t4 & 3) == 0 ? bj[t4 >> 2] : 0.f;
			bs = rhs_updates(a.tiles, src, tk.nd, a.cb, t4);
		}
		for (int e = 0; e < tk.nd; e++) {
			const bool more = e + 1 < n_g;
			if (more) term_dma(a.tiles, src[e + 1], s_stage + ((e + 1) & 1) * TERM_FLOATS, w4, lane);
			if (e < n_g) wait_vmcnt(more ? 8 : 0);
			lds_barrier();
			if (e < n_g) acc = term_mfma_lds(s_stage + (e & 1) * TERM_FLOATS, qr, qc, lane, acc, src[e].w);
			lds_barrier();
		}
		if (wave < 4) {
#pragma unroll
			for (int v = 0; v < 16; v++) C[(32 * qr + quad_row(v, lane)) * TILE] = cv[v] - acc[v];
		} else if (tk.I == tk.J && (t4 & 3) == 0) {
			bj[t4 >> 2] = bv - bs;
		}
		CORNER_RT(7, 1ull << 62);
		return;
	}
	const bool diag = tk.I == tk.J;
	// the gate's diag(S) entry of this lane's row, loaded now: after the elimination its latency would sit on the
	// level's critical path
	const float sd = diag && a.pivot_word && wave == 0 ? a.sdiag[static_cast<int64_t>(tk.J) * TILE + lane] : 0.f;
	{
		// group 0 (waves 0-3) stages A_JJ with the nd terms, group 1 A_IJ with the np terms (the diagonal task: b_J with
		// direct loads); one quadrant per wave, the terms double-buffered in LDS. Both groups run max(nd, np) rounds of
		// two workgroup barriers each.
		const int g = wave >> 2, w4 = wave & 3, qr = w4 >> 1, qc = w4 & 1;
		const int n_g = g == 0 ? tk.nd : diag ? 0 : tk.np;
		const int4* src_g = g == 0 ? src : src + tk.nd;
		const int rounds = tk.nd > tk.np ? tk.nd : tk.np;
		float* bufs = s_stage + g * 2 * TERM_FLOATS;
		f32x16 acc = {};
		// the staged tile's own entries (this wave's quadrant) and b_J first: their loads land while the terms stream,
		// instead of a memory round trip after the last term
		const float* A = a.tiles + static_cast<int64_t>(g == 0 ? tk.slot_d : tk.slot_t) * TILE_ELEMS;
		float tv[16];
		if (g == 0 || !diag) {
#pragma unroll
			for (int v = 0; v < 16; v++) tv[v] = A[(32 * qr + quad_row(v, lane)) * TILE + 32 * qc + (lane & 31)];
		}
		const int t4 = t - 4 * 64;
		const float cbj = g == 1 && diag && (t4 & 3) == 0 ? a.cb[static_cast<int64_t>(tk.J) * TILE + (t4 >> 2)] : 0.f;
		if (n_g > 0) term_dma(a.tiles, src_g[0], bufs, w4, lane);
		float bs = 0.f;
		if (g == 1 && diag) bs = rhs_updates(a.tiles, src, tk.nd, a.cb, t4);   // b_J's update terms (direct loads, L y)
		for (int e = 0; e < rounds; e++) {
			const bool more = e + 1 < n_g;
			if (more) term_dma(a.tiles, src_g[e + 1], bufs + ((e + 1) & 1) * TERM_FLOATS, w4, lane);
			if (e < n_g) wait_vmcnt(more ? 8 : 0);   // this wave's pieces of term e have landed
			lds_barrier();                           // every wave's have
			if (e < n_g) acc = term_mfma_lds(bufs + (e & 1) * TERM_FLOATS, qr, qc, lane, acc, src_g[e].w);
			lds_barrier();                           // term e's buffer is read: round e + 1 refills it
		}
		if (g == 0 || !diag) {   // s_t = A - sum of the terms (the quadrant of term_mfma's C / D layout)
			float* s_t = g == 0 ? s_d : s_p;
#pragma unroll
			for (int v = 0; v < 16; v++) s_t[(32 * qr + quad_row(v, lane)) * CS4 + 32 * qc + (lane & 31)] = tv[v] - acc[v];
		} else {
			if ((t4 & 3) == 0) s_b[t4 >> 2] = cbj - bs;
		}
	}
	__syncthreads();
	CORNER_STAMP(1);
#if NNRT_CORNER_ELIM_WAVES
	const bool self_inv = diag && a.invert_self;   // the last level's diagonal tasks invert their own tile (all waves)
	{
		constexpr int BW = ELIM_BW, NBO = TILE / BW / ELIM_WAVES;   // block width, blocks per wave
		constexpr int LW = 2 * BW;                                   // LDS words per row of a block's L columns
		const int nb = (tk.nreal + BW - 1) / BW;    // blocks holding real columns (the rest is identity padding: kept)
		float* const s_lb = s_stage + TERM_FLOATS;  // [3][64 rows][LW]: a block's L columns (A_JJ rows, then panel rows)
		int bad = 0;
		f32x2 ap[NBO][BW];
		if (wave < ELIM_WAVES) {
#pragma unroll
			for (int k = 0; k < NBO; k++)
#pragma unroll
				for (int h = 0; h < BW; h += 4) {
					const int c0 = BW * (k * ELIM_WAVES + wave) + h;
					const float4 va = *reinterpret_cast<const float4*>(s_d + lane * CS4 + c0);
					float4 vp;
					if (diag)   // the augmented row: b_J on lane 0, zero elsewhere
						vp = lane == 0 ? *reinterpret_cast<const float4*>(s_b + c0) : make_float4(0.f, 0.f, 0.f, 0.f);
					else
						vp = *reinterpret_cast<const float4*>(s_p + lane * CS4 + c0);
					ap[k][h] = f32x2{va.x, vp.x};
					ap[k][h + 1] = f32x2{va.y, vp.y};
					ap[k][h + 2] = f32x2{va.z, vp.z};
					ap[k][h + 3] = f32x2{va.w, vp.w};
				}
		}
		// block bb's owner: factor it (ap[bb / ELIM_WAVES], all of block bb - 1's updates applied) and publish its L columns
		auto factor_publish = [&](int bb) {
			f32x2* cb = ap[bb / ELIM_WAVES];
			factor_block(cb, BW * bb, bad);
			if (BW == 8) {   // the second sub-block: its columns updated by the first (multipliers by readlane), factored
#pragma unroll
				for (int q = 0; q < 4; q++) {
					const f32x2 nq = -cb[q];
#pragma unroll
					for (int c = 4; c < 8; c++) {
						const float lc = lane_bcast(cb[q].x, BW * bb + c);   // L_c,q
						cb[c] = __builtin_elementwise_fma(nq, f32x2{lc, lc}, cb[c]);
					}
				}
				factor_block(cb + 4, BW * bb + 4, bad);
			}
			float* const out = s_lb + (bb % 3) * (TILE * LW);
#pragma unroll
			for (int h = 0; h < BW; h += 2)   // row-major (A_JJ row, panel row) pairs: the f32x2 registers as they are
				*reinterpret_cast<float4*>(out + lane * LW + 2 * h) = make_float4(cb[h].x, cb[h].y, cb[h + 1].x, cb[h + 1].y);
		};
		// block bb's columns of this wave's block k updated with block b's L columns (published in buf; l: this row's)
		auto apply = [&](int k, int bb, const float* buf, const f32x2 (&l)[BW]) {
			float Lm[BW][BW];   // Lm[c][q] = L_c,q of column c of block bb, q of block b: wave-uniform reads (A_JJ rows)
#pragma unroll
			for (int c = 0; c < BW; c++)
#pragma unroll
				for (int h = 0; h < BW; h += 2) {
					const float4 v = *reinterpret_cast<const float4*>(buf + (BW * bb + c) * LW + 2 * h);
					Lm[c][h] = v.x;
					Lm[c][h + 1] = v.z;
				}
#pragma unroll
			for (int q = 0; q < BW; q++)
#pragma unroll
				for (int c = 0; c < BW; c++) ap[k][c] = __builtin_elementwise_fma(-l[q], f32x2{Lm[c][q], Lm[c][q]}, ap[k][c]);
		};
		// this row's L columns of a published block
		auto row_l = [&](const float* buf, f32x2 (&l)[BW]) {
#pragma unroll
			for (int h = 0; h < BW; h += 2) {
				const float4 v = *reinterpret_cast<const float4*>(buf + lane * LW + 2 * h);
				l[h] = f32x2{v.x, v.y};
				l[h + 1] = f32x2{v.z, v.w};
			}
		};
		if (nb > 0 && wave == 0) factor_publish(0);
		__syncthreads();
		// per block b: block b + 1's owner applies block b to it first, factors and publishes it, and defers block b's
		// updates of its other blocks to iteration b + 1 (before block b + 1's); every other wave applies block b to its
		// later blocks. Three L buffers (block b's stays readable through iteration b + 1); one barrier per block.
#pragma unroll
		for (int b = 0; b < TILE / BW; b++) {
			if (b < nb) {   // workgroup-uniform
				const float* const buf = s_lb + (b % 3) * (TILE * LW);
				if (wave < ELIM_WAVES) {
					const bool owner = b >= 1 && wave == b % ELIM_WAVES;   // published block b in iteration b - 1
					if (b >= 1 && owner) {   // its deferred updates by block b - 1
						const float* const prev = s_lb + ((b - 1) % 3) * (TILE * LW);
						f32x2 np[BW];
						row_l(prev, np);
#pragma unroll
						for (int k = 0; k < NBO; k++) {
							const int b2 = k * ELIM_WAVES + wave;
							if (b2 > b && b2 < nb) apply(k, b2, prev, np);
						}
					}
					f32x2 nl[BW];
					row_l(buf, nl);
					const bool next_owner = b + 1 < nb && wave == (b + 1) % ELIM_WAVES;
					if (b + 1 < TILE / BW && next_owner) {
						ELIM_STAMP(b + 1, 0);
						if (ELIM_PRIO) __builtin_amdgcn_s_setprio(2);   // the critical path: ahead of the SIMD's other wave
						apply((b + 1) / ELIM_WAVES, b + 1, buf, nl);
						ELIM_STAMP(b + 1, 1);
						factor_publish(b + 1);
						if (ELIM_PRIO) __builtin_amdgcn_s_setprio(0);
						ELIM_STAMP(b + 1, 2);
					} else {
#pragma unroll
						for (int k = 0; k < NBO; k++) {
							const int b2 = k * ELIM_WAVES + wave;
							if (b2 > b && b2 < nb) apply(k, b2, buf, nl);   // wave-uniform
						}
					}
				}
#ifdef NNRT_DEV_ELIM_NOBARRIER   // timing build only: no barrier per block (values meaningless)
				__builtin_amdgcn_wave_barrier();
#else
				__syncthreads();
#endif
				if (b + 1 < nb && wave == (b + 1) % ELIM_WAVES) ELIM_STAMP(b + 1, 3);
			}
		}
		CORNER_STAMP(2);
		CORNER_STAMP(3);
		__syncthreads();   // every wave's s_d / s_p reads are done (also when no block was eliminated)
		CORNER_STAMP(4);
		if (wave < ELIM_WAVES) {
#pragma unroll
			for (int k = 0; k < NBO; k++)
#pragma unroll
			for (int h = 0; h < BW; h += 4) {
				const int c0 = BW * (k * ELIM_WAVES + wave) + h;
				const float4 vx = make_float4(ap[k][h].x, ap[k][h + 1].x, ap[k][h + 2].x, ap[k][h + 3].x);
				const float4 vy = make_float4(ap[k][h].y, ap[k][h + 1].y, ap[k][h + 2].y, ap[k][h + 3].y);
				if (diag) {
					// the rows as eliminated (the part above the diagonal is not meaningful: the inverse reads the lower part
					// only), and a copy in LDS with zeros above the diagonal: the pivot gate's and the inverse's input
					*reinterpret_cast<float4*>(a.ldiag + static_cast<int64_t>(tk.J) * TILE_ELEMS + lane * TILE + c0) = vx;
					*reinterpret_cast<float4*>(s_d + lane * CS4 + c0) =
					    make_float4(c0 <= lane ? vx.x : 0.f, c0 + 1 <= lane ? vx.y : 0.f, c0 + 2 <= lane ? vx.z : 0.f, c0 + 3 <= lane ? vx.w : 0.f);
					if (lane == 0) *reinterpret_cast<float4*>(a.cb + static_cast<int64_t>(tk.J) * TILE + c0) = vy;
				} else {
					*reinterpret_cast<float4*>(a.tiles + static_cast<int64_t>(tk.slot_t) * TILE_ELEMS + lane * TILE + c0) = vy;
				}
			}
			if (diag && lane == 0 && bad) atomicOr(a.error_flag, 1);
		}
		if (diag && (a.pivot_word || self_inv)) {
			__syncthreads();   // s_d complete
			if (a.pivot_word && wave == 0) {   // the refinement gate: min over the tile of pivot (L_jj^2) / diag(S)_jj
				const float ljj = s_d[lane * CS4 + lane];
				const float ratio = sd > 0.f ? (ljj * ljj) / sd : 1.f;
				// non-negative floats order like their bit patterns: a DPP integer minimum
				const int rb = corner_wave_min_i32(__float_as_int(fmaxf(ratio, 0.f)));
				if (lane == 0) atomicMin(a.pivot_word, static_cast<unsigned>(rb));
			}
		}
		CORNER_STAMP(5);
		CORNER_RT(7, 0ull);
	}
	if (self_inv) invert_lower_lds(s_d, s_b, a.minv + static_cast<int64_t>(tk.J) * TILE_ELEMS, t);
	return;
#else
	// ap[c] = (A_JJ[lane][c], A_IJ[lane][c]): both rows see the same column operations, so one packed FMA
	// (v_pk_fma_f32) updates the pair. Wave 0 holds them; the other waves join for the rank-32 update between the halves.
	f32x2 ap[TILE];
	int bad = 0;
	const bool full = tk.nreal > TILE / 2;   // workgroup-uniform
	if (wave == 0) {
#pragma unroll
		for (int q = 0; q < TILE / 4; q++) {
			const float4 va = *reinterpret_cast<const float4*>(s_d + lane * CS4 + 4 * q);
			float4 vp;
			if (diag)   // the augmented row: b_J on lane 0, zero elsewhere
				vp = lane == 0 ? *reinterpret_cast<const float4*>(s_b + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
			else
				vp = *reinterpret_cast<const float4*>(s_p + lane * CS4 + 4 * q);
			ap[4 * q] = f32x2{va.x, vp.x};
			ap[4 * q + 1] = f32x2{va.y, vp.y};
			ap[4 * q + 2] = f32x2{va.z, vp.z};
			ap[4 * q + 3] = f32x2{va.w, vp.w};
		}
		// columns past the real ones are identity padding: with at most 32 real ones the first half covers the tile
		eliminate_columns<0, TILE / 2>(ap, lane, bad);
		CORNER_STAMP(2);
		// L[:, 0:32] of the A_JJ rows and of the panel rows -> LDS (s_d / s_p are free once loaded)
		if (full) {
#pragma unroll
			for (int q = 0; q < TILE / 8; q++) {
				*reinterpret_cast<float4*>(s_d + lane * CS4 + 4 * q) = make_float4(ap[4 * q].x, ap[4 * q + 1].x, ap[4 * q + 2].x, ap[4 * q + 3].x);
				*reinterpret_cast<float4*>(s_p + lane * CS4 + 4 * q) = make_float4(ap[4 * q].y, ap[4 * q + 1].y, ap[4 * q + 2].y, ap[4 * q + 3].y);
			}
		}
	}
	if (full) {
	__syncthreads();
	// rank-32 update of columns 32..63: C = L[rows, 0:32] L_JJ[32:64, 0:32]^T on the MFMA, one 32-row block per wave
	// (wave 1: A_JJ rows 32..63; waves 2, 3: panel rows 0..31, 32..63; A_JJ rows 0..31 lie above the diagonal there)
	f32x16 cacc = {};
	if (wave > 0 && wave < 4) {
		const float* X = wave == 1 ? s_d + 32 * CS4 : s_p + 32 * (wave - 2) * CS4;
		const int half = lane >> 5, l32 = lane & 31;
		const float4* x4 = reinterpret_cast<const float4*>(X + l32 * CS4 + 16 * half);
		const float4* y4 = reinterpret_cast<const float4*>(s_d + (32 + l32) * CS4 + 16 * half);
#pragma unroll
		for (int q = 0; q < 4; q++) {
			const float4 vx = x4[q], vy = y4[q];
			cacc = __builtin_amdgcn_mfma_f32_32x32x2f32(vx.x, vy.x, cacc, 0, 0, 0);
			cacc = __builtin_amdgcn_mfma_f32_32x32x2f32(vx.y, vy.y, cacc, 0, 0, 0);
			cacc = __builtin_amdgcn_mfma_f32_32x32x2f32(vx.z, vy.z, cacc, 0, 0, 0);
			cacc = __builtin_amdgcn_mfma_f32_32x32x2f32(vx.w, vy.w, cacc, 0, 0, 0);
		}
	}
	__syncthreads();   // every wave is done reading L before the products overwrite it
	if (wave > 0 && wave < 4) {
		float* Cb = wave == 1 ? s_d + 32 * CS4 : s_p + 32 * (wave - 2) * CS4;
#pragma unroll
		for (int v = 0; v < 16; v++) Cb[quad_row(v, lane) * CS4 + 32 + (lane & 31)] = cacc[v];
	}
	__syncthreads();
	}
	const bool self_inv = diag && a.invert_self;   // the last level's diagonal tasks invert their own tile (all waves)
	if (wave != 0 && !self_inv) return;
	if (wave == 0) {
	if (full) {
#pragma unroll
		for (int q = TILE / 8; q < TILE / 4; q++) {
			const float4 ca = lane >= 32 ? *reinterpret_cast<const float4*>(s_d + lane * CS4 + 4 * q) : make_float4(0.f, 0.f, 0.f, 0.f);
			const float4 cp = *reinterpret_cast<const float4*>(s_p + lane * CS4 + 4 * q);
			ap[4 * q] -= f32x2{ca.x, cp.x};
			ap[4 * q + 1] -= f32x2{ca.y, cp.y};
			ap[4 * q + 2] -= f32x2{ca.z, cp.z};
			ap[4 * q + 3] -= f32x2{ca.w, cp.w};
		}
		CORNER_STAMP(3);
		eliminate_columns<TILE / 2, TILE>(ap, lane, bad);
	}
	CORNER_STAMP(4);
	if (diag) {
		// the rows as eliminated (the part above the diagonal is not meaningful: the inverse reads the lower part only);
		// a copy in LDS with zeros above the diagonal (s_d is this wave's alone now) gives each lane its diagonal entry
		// without a 64-way select, and is the inverse's input (lower_to_lds's layout)
		float4* wa = reinterpret_cast<float4*>(a.ldiag + static_cast<int64_t>(tk.J) * TILE_ELEMS + lane * TILE);
#pragma unroll
		for (int q = 0; q < TILE / 4; q++) {
			const float4 v = make_float4(ap[4 * q].x, ap[4 * q + 1].x, ap[4 * q + 2].x, ap[4 * q + 3].x);
			wa[q] = v;
			const int c0 = 4 * q;
			*reinterpret_cast<float4*>(s_d + lane * CS4 + 4 * q) =
			    make_float4(c0 <= lane ? v.x : 0.f, c0 + 1 <= lane ? v.y : 0.f, c0 + 2 <= lane ? v.z : 0.f, c0 + 3 <= lane ? v.w : 0.f);
		}
		if (a.pivot_word) {   // the refinement gate: min over the tile of pivot (L_jj^2) / diag(S)_jj
			const float ljj = s_d[lane * CS4 + lane];
			const float ratio = sd > 0.f ? (ljj * ljj) / sd : 1.f;
			// non-negative floats order like their bit patterns: a DPP integer minimum
			const int rb = corner_wave_min_i32(__float_as_int(fmaxf(ratio, 0.f)));
			if (lane == 0) atomicMin(a.pivot_word, static_cast<unsigned>(rb));
		}
		if (lane == 0) {
			float4* wb = reinterpret_cast<float4*>(a.cb + static_cast<int64_t>(tk.J) * TILE);
#pragma unroll
			for (int q = 0; q < TILE / 4; q++) wb[q] = make_float4(ap[4 * q].y, ap[4 * q + 1].y, ap[4 * q + 2].y, ap[4 * q + 3].y);
			if (bad) atomicOr(a.error_flag, 1);
		}
	} else {
		float4* wp = reinterpret_cast<float4*>(a.tiles + static_cast<int64_t>(tk.slot_t) * TILE_ELEMS + lane * TILE);
#pragma unroll
		for (int q = 0; q < TILE / 4; q++) wp[q] = make_float4(ap[4 * q].y, ap[4 * q + 1].y, ap[4 * q + 2].y, ap[4 * q + 3].y);
	}
	CORNER_STAMP(5);
	CORNER_RT(7, 0ull);
	}   // wave 0
	if (self_inv) {
		__syncthreads();   // s_d: L_JJ, zeros above the diagonal
		invert_lower_lds(s_d, s_b, a.minv + static_cast<int64_t>(tk.J) * TILE_ELEMS, t);
	}
#endif
}

// development timing build only (-DNNRT_CORNER_STAMPS): per role of the dataflow launch (its ticket), the constant-rate
// clock at its start, the end of its wait and its end ([64]), and per back-chain column q < 64: its start, the end of
// its entry sums, the end of x = M^T z and its end, read back by nnrt_dev_flow_stamps (tools/dev/flow_stamps.py)
#ifdef NNRT_CORNER_STAMPS
__device__ unsigned long long g_flow_stamps[128][66][4];
__shared__ int s_flow_row;
#define FLOW_RT(row, col, i)                                                                                            \
	do {                                                                                                                \
		if (threadIdx.x == 0 && (row) >= 0 && (row) < 128 && (col) < 66) g_flow_stamps[row][col][i] = __builtin_amdgcn_s_memrealtime(); \
	} while (0)
#else
#define FLOW_RT(row, col, i) \
	do {                     \
	} while (0)
#endif

struct CornerBackArgs {
	const unsigned* gate;    // nullable: run only if the pivot ratio word is below ratio (the refinement pass)
	float ratio;
	const float* tiles;
	const float* ldiag;
	const float* minv;       // L_JJ^-1 of the columns whose descriptor says so (w = 1)
	const float* cb;         // y
	float* xp;               // [ld] x in the permuted order
	const int* row_node;
	float* xout;             // [6 nc] x in node order
	const int2* chains;      // this launch's chains (first column, column count)
	const int4* cols;        // (J, entry offset, entry count, outside entries), each chain root end first
	const int2* ent;         // (slot of L_IJ, I)
	float* zx;               // [ld] pre-sums y_J - sum over the outside entries (modes 1, 2)
	int mode;                // 0: every entry; 1: pre-sum launch (outside entries -> zx); 2: inside entries from zx
};
// the entries a column's pass reads (offset, count) and where its y comes from, per substitution mode
__device__ __forceinline__ int2 subst_span(const int4& c, int mode) {
	return mode == 2 ? make_int2(c.y + c.w, c.z - c.w) : mode == 1 ? make_int2(c.y, c.w) : make_int2(c.y, c.z);
}

// Back substitution L^T x = y along chains of the elimination tree (one workgroup per chain, its columns in order; the
// launches run from the root's chain down). Per column J: z = y_J - sum_I L_IJ^T x_I (each wave a quarter of every tile's
// rows, read as 16-B row pieces, BACK_BATCH tiles' loads in flight), then x_J = L_JJ^-T z as the product M^T z with
// M = L_JJ^-1 (k_corner_invert; its tile streams into LDS by LDS-DMA behind the entry loads), a quarter of the rows of M
// per wave. x_J goes to
// global memory before the workgroup barrier, so the chain's next column reads it like the x of earlier launches.
// Per column only the entry tiles and their x are a memory round trip on the chain's path: the chain's column
// descriptors are staged in LDS up front, each column's first 64 entry descriptors are fetched during the previous
// column (wave 1, into LDS before its last barrier), and y_J is loaded ahead of the sums.
constexpr int BACK_BATCH = 8;   // entry tiles per batch of loads (8 x (4 + 1) = 40 outstanding loads per lane)
constexpr int BACK_COLS = 64;   // chain columns whose descriptors are staged in LDS at a time
typedef __attribute__((address_space(3))) void corner_lds_t;
typedef const __attribute__((address_space(1))) void corner_global_t;
// the 64 x 64 tile at src -> LDS dst (row-major, no padding) by LDS-DMA: 16 pieces of 1 KB, four per wave of a
// 256-thread workgroup; complete once the issuing waves wait for their loads (a __syncthreads() does)
__device__ __forceinline__ void tile_to_lds(const float* src, float* dst, int wave, int lane) {
#pragma unroll
	for (int i = 0; i < 4; i++) {
		const int chunk = 4 * wave + i;
		__builtin_amdgcn_global_load_lds((corner_global_t*)(src + chunk * 256 + lane * 4), (corner_lds_t*)(dst + chunk * 256), 16, 0, 0);
	}
}
// the vector accesses of a substitution pass: plain loads / stores between launches; sc1 (L1-bypassing loads,
// write-through stores) for the vectors other workgroups of a dataflow launch (k_corner_flow) write and read
template <bool SC1>
struct SubstVec {
	const float* base;
	__amdgpu_buffer_rsrc_t r;
	__device__ __forceinline__ SubstVec(const float* p, int64_t n) : base(p) {
		if constexpr (SC1) r = flow_rsrc(p, 4 * n);
	}
	// other: the bytes were written by another workgroup of this launch (sc1 load); else by this workgroup or an earlier
	// launch (plain load: L1 holds no older copy of a line this workgroup wrote)
	__device__ __forceinline__ float4 ld4(int64_t i, bool other = true) const {
		if constexpr (SC1) {
			if (other) return ld_sc1_f4(r, static_cast<int>(4 * i));
		}
		return *reinterpret_cast<const float4*>(base + i);
	}
	__device__ __forceinline__ float ld(int64_t i) const {
		if constexpr (SC1) return ld_sc1_f(r, static_cast<int>(4 * i));
		else return base[i];
	}
	__device__ __forceinline__ void st(int64_t i, float v) const {
		if constexpr (SC1) st_sc1(const_cast<float*>(base) + i, v);
		else const_cast<float*>(base)[i] = v;
	}
};

// one chain of the back substitution (the body of k_corner_back; k_corner_flow runs it with SC1 vectors)
template <bool SC1X, bool SC1Y>
__device__ __forceinline__ void corner_back_chain(const CornerBackArgs& a, int2 ch, int ld, int64_t nxout) {
	__shared__ __attribute__((aligned(16))) float s_m[TILE_ELEMS];   // L_JJ^-1 of the current column
	__shared__ __attribute__((aligned(16))) float s_part[4][TILE];
	__shared__ float s_xq[4][TILE];   // quarters of x_J = M^T z
	__shared__ int4 s_cols[BACK_COLS];
	__shared__ int2 s_ent[2][64];   // first 64 entry descriptors of the current (q & 1) and the next column
	const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
	const SubstVec<SC1X> xv_(a.xp, ld), xo_(a.xout, nxout);
	const SubstVec<SC1Y> yv_(a.cb, ld);
	for (int q0 = 0; q0 < ch.y; q0 += BACK_COLS) {
		const int nq = ch.y - q0 < BACK_COLS ? ch.y - q0 : BACK_COLS;
		if (t < nq) s_cols[t] = a.cols[ch.x + q0 + t];
		__syncthreads();
		if (wave == 1) {
			const int2 sp0 = subst_span(s_cols[0], a.mode);
			s_ent[0][lane] = lane < sp0.y ? a.ent[sp0.x + lane] : make_int2(0, 0);
		}
		__syncthreads();
		for (int q = 0; q < nq; q++) {
#ifdef NNRT_CORNER_STAMPS
			const int srow = SC1X ? s_flow_row : -1;
#endif
			FLOW_RT(srow, q0 + q, 0);
			const int4 col = s_cols[q];
			const int J = col.x;
			const int2 sp = subst_span(col, a.mode);
			// M = L_JJ^-1 streams into LDS behind the entry loads; y_J is loaded ahead of the sums (wave 0)
			if (a.mode != 1) tile_to_lds(a.minv + static_cast<int64_t>(J) * TILE_ELEMS, s_m, wave, lane);
			const float yv = a.mode == 2 && col.w > 0 ? a.zx[static_cast<int64_t>(J) * TILE + lane]
			                                          : yv_.ld(static_cast<int64_t>(J) * TILE + lane);   // every wave forms z
			const bool has_next = q + 1 < nq;
			int2 nxt = make_int2(0, 0);
			if (wave == 1 && has_next) {
				const int2 spn = subst_span(s_cols[q + 1], a.mode);
				if (lane < spn.y) nxt = a.ent[spn.x + lane];
			}
			// z partials: lane (row group rq, column group cg) covers rows 16 wave + 4 rq .. + 3 and columns 4 cg .. 4 cg + 3
			// of every entry tile (four 16-B row loads and one 16-B x load per tile), BACK_BATCH tiles' loads in flight; the
			// row groups are then summed across lanes
			const int cg = lane & 15, rq = lane >> 4;
			float acc[4] = {0.f, 0.f, 0.f, 0.f};
			for (int e0 = 0; e0 < sp.y; e0 += 64) {
				const int ne = sp.y - e0 < 64 ? sp.y - e0 : 64;
				const int2 mine = e0 == 0 ? s_ent[q & 1][lane] : lane < ne ? a.ent[sp.x + e0 + lane] : make_int2(0, 0);
				for (int e = 0; e < ne; e += BACK_BATCH) {
					float4 l[BACK_BATCH][4], xv[BACK_BATCH];
#pragma unroll
					for (int j = 0; j < BACK_BATCH; j++) {
						const bool ok = e + j < ne;   // a missing entry repeats entry e's tile against x = 0 (exact zeros)
						const int sj = __shfl(mine.x, ok ? e + j : e);
						const int ij = __shfl(mine.y, ok ? e + j : e);
						const float* Lj = a.tiles + static_cast<int64_t>(sj) * TILE_ELEMS + (16 * wave + 4 * rq) * TILE + 4 * cg;
#pragma unroll
						for (int k = 0; k < 4; k++) l[j][k] = *reinterpret_cast<const float4*>(Lj + k * TILE);
						// entries outside the chain first (col.w of them: x from other workgroups), then the chain's own
						const float4 x4 = xv_.ld4(static_cast<int64_t>(ij) * TILE + 16 * wave + 4 * rq, e0 + e + j < col.w);
						xv[j] = ok ? x4 : make_float4(0.f, 0.f, 0.f, 0.f);
					}
#pragma unroll
					for (int j = 0; j < BACK_BATCH; j++) {
						const float xk[4] = {xv[j].x, xv[j].y, xv[j].z, xv[j].w};
#pragma unroll
						for (int k = 0; k < 4; k++) {
							acc[0] += l[j][k].x * xk[k];
							acc[1] += l[j][k].y * xk[k];
							acc[2] += l[j][k].z * xk[k];
							acc[3] += l[j][k].w * xk[k];
						}
					}
				}
			}
#pragma unroll
			for (int i = 0; i < 4; i++) {
				acc[i] += __shfl_xor(acc[i], 16);
				acc[i] += __shfl_xor(acc[i], 32);
			}
			if (lane < 16) *reinterpret_cast<float4*>(&s_part[wave][4 * lane]) = make_float4(acc[0], acc[1], acc[2], acc[3]);
			FLOW_RT(srow, q0 + q, 1);
			__syncthreads();   // also retires the M tile's LDS-DMA pieces of every wave
			if (wave == 0 && a.mode == 1) {
				a.zx[static_cast<int64_t>(J) * TILE + lane] = yv - ((s_part[0][lane] + s_part[1][lane]) + (s_part[2][lane] + s_part[3][lane]));
			} else if (a.mode != 1) {
				// x_c = sum_r M_rc z_r: every wave forms z (lane = row) and sums its 16 rows r, z_r broadcast from lane r,
				// column c of M from LDS (conflict-free); the four quarters meet in LDS
				const float z = yv - ((s_part[0][lane] + s_part[1][lane]) + (s_part[2][lane] + s_part[3][lane]));
				float xs[2] = {0.f, 0.f};
#pragma unroll
				for (int k = 0; k < 16; k++) {
					const int r = 16 * wave + k;
					xs[k & 1] = __builtin_fmaf(s_m[r * TILE + lane], lane_bcast(z, r), xs[k & 1]);
				}
				s_xq[wave][lane] = xs[0] + xs[1];
			}
			if (a.mode != 1) {
				FLOW_RT(srow, q0 + q, 2);
				__syncthreads();   // the quarters of x_J
				if (wave == 0) {
					const float x = (s_xq[0][lane] + s_xq[1][lane]) + (s_xq[2][lane] + s_xq[3][lane]);
					const int64_t row = static_cast<int64_t>(J) * TILE + lane;
					xv_.st(row, x);
					const int rn = a.row_node[row];
					if (rn >= 0) xo_.st(6 * static_cast<int64_t>(rn >> 3) + (rn & 7), x);
				}
			}
			if (wave == 1 && has_next) s_ent[(q + 1) & 1][lane] = nxt;
			__syncthreads();   // x_J visible to the chain's next column; s_part, s_xq, s_m free; the next column's entries staged
			FLOW_RT(srow, q0 + q, 3);
		}
	}
}

__global__ __launch_bounds__(CT) void k_corner_back(CornerBackArgs a, int ld, int64_t nxout) {
	if (a.gate && !refine_gate_on(a.gate, a.ratio)) return;
	corner_back_chain<false, false>(a, a.chains[blockIdx.x], ld, nxout);
}

// Forward substitution L y = b along the forward chains (iterative refinement's corner solve; the first solve's forward
// substitution rides in the factorization as the augmented row): per column J, z = b_J - sum_k L_Jk y_k over its row
// entries (lane (row group, column group) covers rows 16 wave + 4 rq .. + 3 and columns 4 cg .. 4 cg + 3 of every entry tile;
// the 16 column groups are summed across lanes, so each row's sum is complete in its wave), then y_J = L_JJ^-1 z, the
// product with M (k_corner_invert; streamed into LDS by LDS-DMA behind the entry loads) split the same way. y_J
// overwrites b_J in yb (a column reads y of its descendants only: earlier launches or earlier in its chain).
struct CornerFwdArgs {
	const unsigned* gate;
	float ratio;
	const float* tiles;
	const float* ldiag;
	const float* minv;
	float* yb;               // [ld] b in, y out (permuted order)
	const int2* chains;
	const int4* cols;        // (J, entry offset, entry count, outside entries)
	const int2* ent;         // (slot of L_Jk, k)
	float* zx;               // [ld] pre-sums (modes 1, 2; as CornerBackArgs)
	int mode;
};
// one chain of the forward substitution (the body of k_corner_fwd; k_corner_flow runs it with SC1 vectors)
template <bool SC1>
__device__ __forceinline__ void corner_fwd_chain(const CornerFwdArgs& a, int2 ch, int ld) {
	__shared__ __attribute__((aligned(16))) float s_m[TILE_ELEMS];   // L_JJ^-1 of the current column
	__shared__ __attribute__((aligned(16))) float s_z[TILE];
	const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
	const SubstVec<SC1> yv_(a.yb, ld);
	const int cg = lane & 15, rq = lane >> 4;   // rows 16 wave + 4 rq .. + 3, columns 4 cg .. 4 cg + 3
	for (int q = 0; q < ch.y; q++) {
		const int4 col = a.cols[ch.x + q];
		const int J = col.x;
		const int2 sp = subst_span(col, a.mode);
		if (a.mode != 1) tile_to_lds(a.minv + static_cast<int64_t>(J) * TILE_ELEMS, s_m, wave, lane);   // behind the entry loads
		float acc[4] = {0.f, 0.f, 0.f, 0.f};   // rows 16 wave + 4 rq + k, partial over this lane's 4 columns
		for (int e0 = 0; e0 < sp.y; e0 += 64) {
			const int ne = sp.y - e0 < 64 ? sp.y - e0 : 64;
			const int2 mine = lane < ne ? a.ent[sp.x + e0 + lane] : make_int2(0, 0);
			for (int e = 0; e < ne; e += BACK_BATCH) {
				float4 l[BACK_BATCH][4], yv[BACK_BATCH];
#pragma unroll
				for (int j = 0; j < BACK_BATCH; j++) {
					const bool ok = e + j < ne;   // a missing entry repeats entry e's tile against y = 0
					const int sj = __shfl(mine.x, ok ? e + j : e);
					const int kj = __shfl(mine.y, ok ? e + j : e);
					const float* Lj = a.tiles + static_cast<int64_t>(sj) * TILE_ELEMS + (16 * wave + 4 * rq) * TILE + 4 * cg;
#pragma unroll
					for (int k = 0; k < 4; k++) l[j][k] = *reinterpret_cast<const float4*>(Lj + k * TILE);
					const float4 y4 = yv_.ld4(static_cast<int64_t>(kj) * TILE + 4 * cg, e0 + e + j < col.w);   // outside entries first
					yv[j] = ok ? y4 : make_float4(0.f, 0.f, 0.f, 0.f);
				}
#pragma unroll
				for (int j = 0; j < BACK_BATCH; j++)
#pragma unroll
					for (int k = 0; k < 4; k++)
						acc[k] += ((l[j][k].x * yv[j].x + l[j][k].y * yv[j].y) + l[j][k].z * yv[j].z) + l[j][k].w * yv[j].w;
			}
		}
#pragma unroll
		for (int k = 0; k < 4; k++)
#pragma unroll
			for (int m = 1; m < 16; m <<= 1) acc[k] += __shfl_xor(acc[k], m);
		if (cg == 0) {
#pragma unroll
			for (int k = 0; k < 4; k++) {
				const int r = 16 * wave + 4 * rq + k;
				const float b = a.mode == 2 && col.w > 0 ? a.zx[static_cast<int64_t>(J) * TILE + r] : yv_.ld(static_cast<int64_t>(J) * TILE + r);
				const float z = b - acc[k];
				if (a.mode == 1) a.zx[static_cast<int64_t>(J) * TILE + r] = z;
				else s_z[r] = z;
			}
		}
		if (a.mode == 1) continue;   // pre-sum launch: one column per workgroup, no barrier needed
		__syncthreads();   // z complete; the M tile's LDS-DMA pieces of every wave retired
		{   // y_r = sum_c M_rc z_c: the same row / column-group split, summed across the 16 column groups
			const float4 z4 = *reinterpret_cast<const float4*>(&s_z[4 * cg]);
			float yk[4];
#pragma unroll
			for (int k = 0; k < 4; k++) {
				const float4 m4 = *reinterpret_cast<const float4*>(&s_m[(16 * wave + 4 * rq + k) * TILE + 4 * cg]);
				yk[k] = ((m4.x * z4.x + m4.y * z4.y) + m4.z * z4.z) + m4.w * z4.w;
#pragma unroll
				for (int m = 1; m < 16; m <<= 1) yk[k] += __shfl_xor(yk[k], m);
			}
			if (cg == 0)
#pragma unroll
				for (int k = 0; k < 4; k++) yv_.st(static_cast<int64_t>(J) * TILE + 16 * wave + 4 * rq + k, yk[k]);
		}
		__syncthreads();   // y_J visible to the chain's next column; s_z, s_m free
	}
}

__global__ __launch_bounds__(CT) void k_corner_fwd(CornerFwdArgs a, int ld) {
	if (a.gate && !refine_gate_on(a.gate, a.ratio)) return;
	corner_fwd_chain<false>(a, a.chains[blockIdx.x], ld);
}

// ===================================================================================================================
// Dataflow substitution launch (k_corner_flow): the corner's back substitution chains and the stem pass that follows
// them, then -- when the refinement gate opens -- the whole refinement step: the correction's corner right-hand side,
// the forward chains, the back chains and the stem pass applying x + d; ONE launch instead of one launch per chain
// depth per substitution plus the stem passes and the refinement's right-hand side (round 4: 2 + 12 launches at C5).
//
// Workgroups take tickets (one relaxed agent-scope atomic add each) and a ticket fixes the role; roles are numbered so
// that every wait is on work of a LOWER ticket: [back chains, root first] [stem workers] [rhs workers, one per tile
// column] [forward chains, deepest first] [back chains, root first] [correction workers] [apply workers] (the last two:
// the safeguarded step, round 6). A back chain waits for its parent
// chain (the refinement's roots: for their own forward chain), the stem workers for every back chain of their pass, the
// rhs workers for the solve's stem workers (the stem residual), a forward chain for its columns' right-hand sides and
// its child chains. A workgroup that holds a ticket is resident and waits only on lower tickets, so by induction every
// wait ends: no assumption on dispatch order, co-residency or timing (the plan emulator checks the chain order:
// tests/test_corner_plan.py). Every spin is bounded (error flag bit 8 on a timeout). With the gate shut the refinement's
// workgroups return right after their ticket.
//
// Hand-offs (MI355X_MICROARCH.md, inter-workgroup visibility, table row 1): the handed-off vectors (x, y, the stem
// residual, the refinement rhs) are stored write-through (sc1) and read by other workgroups with sc1 loads only; every
// storing wave drains its stores (s_waitcnt vmcnt(0)) before the workgroup barrier behind which one lane signals (an
// agent-scope atomic); the waiting workgroup's lane 0 polls relaxed and the other waves load after the barrier it then
// joins. A chain's own earlier columns are read back with plain loads (its own writes); the refinement's back chains use
// their own x buffer (xp2), so no CU holds an L1 copy of a line another workgroup of the launch rewrote. Tiles and
// inverses come from earlier launches (plain loads). The control words are zeroed by k_corner_invert.
// ===================================================================================================================
struct FlowArgs {
	int refine;              // the refinement step's roles follow the solve's (mode 1)
	int nB, T, ld, stem_wg;  // chains, tile columns, permuted length, stem workgroups per pass
	int64_t nxout;           // 6 nc
	unsigned* ctl;           // 2 x flow_ctl_words(nB) control words (zeroed by k_corner_invert)
	const int4* chains;      // [nB] (back column first, column count, forward column first, parent chain or -1), root first
	const int* fwd_need;     // [nB] columns + child chains of chain c
	const int* col_chain;    // [T] chain of tile column J
	const int* node_row;     // [nc] first permuted row of each corner node
	CornerBackArgs back;     // the solve's back chains (chains unused): y = the factorization's, x -> xp, xout = st.x's corner rows
	CornerFwdArgs fwd;       // the refinement's forward chains (chains unused): yb = its corner rhs -> y
	CornerBackArgs back2;    // the refinement's back chains: y = fwd.yb, x -> xp2 (its own buffer), xout = st.dx's corner rows
	FlowStem st;
};
constexpr unsigned FLOW_MAX_SPINS = 1u << 20;   // per wait: ~1 s of polling before the launch gives up (error bit 8)

// lane 0 polls *w until it reaches target (relaxed agent loads, s_sleep between polls); every thread returns whether it
// did (workgroup-uniform)
__device__ __forceinline__ bool flow_wait(const unsigned* w, unsigned target, int* error_flag) {
	__shared__ int s_ok;
	if (threadIdx.x == 0) {
		unsigned spins = 0;
		int ok = 1;
		while (__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
			if (++spins > FLOW_MAX_SPINS) {
				ok = 0;
				atomicOr(error_flag, 8);
				break;
			}
			__builtin_amdgcn_s_sleep(2);
		}
		s_ok = ok;
	}
	__syncthreads();
	return s_ok != 0;
}
// every wave drains its (sc1) stores, then one lane adds 1 to each of the (up to two) counters
__device__ __forceinline__ void flow_signal(unsigned* w0, unsigned* w1 = nullptr) {
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	__syncthreads();
	if (threadIdx.x == 0) {
		__hip_atomic_fetch_add(w0, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
		if (w1) __hip_atomic_fetch_add(w1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
	}
}

// While a dataflow back chain waits for its parent chain (k_corner_flow), it pulls the entry tiles of its columns into
// this XCD's L2: one 16-B LDS-DMA piece per 64-B segment of every tile (256 threads x 64 B = one 16-KB tile per
// instruction), the data itself dropped in a 4-KB LDS scratch. The tiles were written by the factor launches on any XCD;
// the chain's entry sums then hit L2 instead of going to memory on their critical path. Bounded by FLOW_PREFETCH_TILES
// (NNRT_FLOW_PREFETCH=0: off). The DMA completes in the background; the chain's first tile_to_lds wait retires it.
#ifndef NNRT_FLOW_PREFETCH
#define NNRT_FLOW_PREFETCH 64
#endif
constexpr int FLOW_PREFETCH_TILES = NNRT_FLOW_PREFETCH;
__device__ __forceinline__ void flow_prefetch_chain(const CornerBackArgs& a, int2 ch) {
	__shared__ __attribute__((aligned(16))) float s_pf[CT * 4];
	const int t = threadIdx.x, wave = t >> 6;
	int left = FLOW_PREFETCH_TILES;
	for (int q = 0; q < ch.y && left > 0; q++) {
		const int4 col = a.cols[ch.x + q];   // wave-uniform (scalar loads)
		for (int e = 0; e < col.z && left > 0; e++, left--) {
			const int slot = a.ent[col.y + e].x;
			const float* src = a.tiles + static_cast<int64_t>(slot) * TILE_ELEMS + 16 * t;
			__builtin_amdgcn_global_load_lds((corner_global_t*)src, (corner_lds_t*)(s_pf + wave * 256), 16, 0, 0);
		}
	}
}

__global__ __launch_bounds__(CT) void k_corner_flow(FlowArgs a) {
	__shared__ int s_ticket;
	const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
	const bool refining = a.st.gate && refine_gate_on(a.st.gate, a.st.ratio);
	const int nB = a.nB, S = a.stem_wg;
	unsigned* ctl0 = a.ctl;                        // the solve: [0] ticket, [1] back chains done, [2] stem workers done
	unsigned* back_done0 = ctl0 + 4;               // [nB] back chain c finished
	unsigned* ctl1 = a.ctl + flow_ctl_words(nB);   // the refinement step: [1] back chains done
	unsigned* back_done1 = ctl1 + 4;
	unsigned* fwd_cnt = back_done1 + nB;           // [nB] forward chain c's columns' rhs + finished child chains
	unsigned* fwd_done = fwd_cnt + nB;             // [nB] forward chain c (a root) finished
	if (t == 0) s_ticket = static_cast<int>(__hip_atomic_fetch_add(ctl0, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
	__syncthreads();
	int k = s_ticket;
#ifdef NNRT_CORNER_STAMPS
	if (t == 0) s_flow_row = k;
	__syncthreads();
#endif
	FLOW_RT(k, 64, 0);
	const XSc1 x_sc1{flow_rsrc(a.st.x, 24 * static_cast<int64_t>(a.st.N))};
	// ---- the solve: back chains (root first), then the stem pass ----
	if (k < nB) {
		const int4 ch = a.chains[k];
		if (FLOW_PREFETCH_TILES > 0 && ch.w >= 0) flow_prefetch_chain(a.back, make_int2(ch.x, ch.y));
		if (ch.w >= 0 && !flow_wait(back_done0 + ch.w, 1u, a.st.error_flag)) return;
		FLOW_RT(k, 64, 1);
		corner_back_chain<true, false>(a.back, make_int2(ch.x, ch.y), a.ld, a.nxout);
		flow_signal(back_done0 + k, ctl0 + 1);
		FLOW_RT(k, 64, 2);
		return;
	}
	k -= nB;
	if (k < S) {   // x of the stem, every node's update -- or, when the refinement runs, the stem residual for it
		const int i = k * CT + t;
		const bool live = i < a.st.n_update || i < a.st.n0;
		// while the corner chains run: the stem row's indices, and every line it reads after the wait pulled into L2
		// (the refinement's residual pass keeps the general path)
		StemPre pre{};
		pre.n = -1;
		if (live && !refining) {
			if (i < a.st.n0) pre = stem_prefetch(i, a.st.dinv, a.st.edge_offsets, a.st.edge_list, a.st.edges, a.st.wing, a.st.rhs, a.st.node_state ? a.st.state_in : nullptr);
			else if (a.st.node_state) touch_lines(a.st.state_in + static_cast<int64_t>(i) * NODE_STRIDE, NODE_STRIDE);
		}
		if (!flow_wait(ctl0 + 1, static_cast<unsigned>(nB), a.st.error_flag)) return;
		FLOW_RT(k + nB, 64, 1);
		if (live && i < a.st.n0 && pre.n >= 0) {   // arrow_back_node's stem path (mode 0, or mode 1 with the gate shut)
			float o[6];
			stem_solve_pre(i, pre, a.st.dinv, a.st.wing, XPlain{a.st.rhs}, x_sc1, o);
			store6<true>(a.st.x + 6 * static_cast<int64_t>(i), o);
			if (a.st.node_state) arrow_update_node(i, o, a.st.state_in, a.st.node_state, a.st.updates_out);
		} else if (live)
			arrow_back_node<true>(i, a.st.n0, a.st.n_update, a.st.dinv, a.st.edge_offsets, a.st.edge_list, a.st.edges, a.st.wing,
			                      XPlain{a.st.rhs}, a.st.x, x_sc1, a.st.state_in, a.st.node_state, a.st.updates_out, nullptr, XPlain{nullptr},
			                      a.st.mode, refining, a.st.diag, a.st.res);
		if (a.refine) flow_signal(ctl0 + 2);
		FLOW_RT(k + nB, 64, 2);
		return;
	}
	k -= S;
	if (!refining) return;   // the refinement's roles when its gate is shut
	// ---- the refinement step: the correction's corner rhs per tile column, forward chains (deepest first), back chains
	// (root first), the stem pass applying x + d ----
	const XSc1 res_sc1{flow_rsrc(a.st.res, 24 * static_cast<int64_t>(a.st.N))};
	if (k < a.T) {
		if (!flow_wait(ctl0 + 2, static_cast<unsigned>(S), a.st.error_flag)) return;
		const int J = k;
		int seen = 0;
		for (int r = 0; r < TILE; r++) {
			const int rn = a.back.row_node[static_cast<int64_t>(J) * TILE + r];
			if (rn < 0 || ((rn & 7) != 0 && r != 0)) continue;   // a node's first row, or a node entering from column J - 1
			if ((seen++ & 3) != wave) continue;
			const int node = rn >> 3;
			const float v = refine_rhs_node(node, lane, a.st.n0, a.st.dinv_b, a.st.diag, a.st.inc_off, a.st.inc_list, a.st.edges, a.st.wing,
			                                a.st.rhs, x_sc1, res_sc1);
			const int row = a.node_row[node] + lane;
			if (lane < 6 && row >= J * TILE && row < (J + 1) * TILE) st_sc1(a.fwd.yb + row, v);
		}
		flow_signal(fwd_cnt + a.col_chain[J]);
		return;
	}
	k -= a.T;
	if (k < nB) {
		const int c = nB - 1 - k;
		const int4 ch = a.chains[c];
		if (!flow_wait(fwd_cnt + c, static_cast<unsigned>(a.fwd_need[c]), a.st.error_flag)) return;
		corner_fwd_chain<true>(a.fwd, make_int2(ch.z, ch.y), a.ld);
		flow_signal(ch.w >= 0 ? fwd_cnt + ch.w : fwd_done + c);
		return;
	}
	k -= nB;
	if (k < nB) {
		const int4 ch = a.chains[k];
		if (!flow_wait(ch.w >= 0 ? back_done1 + ch.w : fwd_done + k, 1u, a.st.error_flag)) return;
		corner_back_chain<true, true>(a.back2, make_int2(ch.x, ch.y), a.ld, a.nxout);
		flow_signal(back_done1 + k, ctl1 + 1);
		return;
	}
	k -= nB;
	// the safeguarded step (arrow_device.hpp): a correction pass (the stem rows of d, max |d| and max |x| into the guard
	// words), then an apply pass that waits for every correction workgroup and applies x + d -- or x, when the guard
	// rejects the step -- with each node's update
	const XSc1 dx_sc1{flow_rsrc(a.st.dx, 24 * static_cast<int64_t>(a.st.N))};
	unsigned* guard = a.st.guard;
	if (k < S) {
		if (!flow_wait(ctl1 + 1, static_cast<unsigned>(nB), a.st.error_flag)) return;
		refine_correction_node<true>(k * CT + t, a.st.n0, a.st.N, a.st.dinv, a.st.edge_offsets, a.st.edge_list, a.st.edges, a.st.wing, res_sc1,
		                             a.st.dx, dx_sc1, x_sc1, guard);
		flow_signal(guard + REFINE_GUARD_COUNT);
		return;
	}
	k -= S;
	if (!flow_wait(guard + REFINE_GUARD_COUNT, static_cast<unsigned>(S), a.st.error_flag)) return;
	refine_apply_node(k * CT + t, a.st.N, refine_guard_accepts(guard), dx_sc1, x_sc1, a.st.x, a.st.state_in, a.st.node_state, a.st.updates_out);
}

// ===================================================================================================================
// Single-workgroup substitution walks (the corner solves when the permuted vector fits in LDS): one launch walks every
// tile column in order -- back substitution in descending column order (ancestors before descendants), forward in
// ascending order -- keeping the whole solution vector in LDS, while the tiles each column needs stream through an
// LDS ring by LDS-DMA (global_load_lds_dwordx4) issued ahead of their use. A column's stream elements are its entry
// tiles, then its head: L_JJ^-1 (or L_JJ for top-level columns, which take the substitution). Nothing crosses
// workgroups: no inter-workgroup ordering at all.
// ===================================================================================================================
constexpr int WT = 512;        // threads of the walk workgroup (8 waves)
constexpr int WALK_MAX_LD = 8192;
constexpr int WALK_MAX_ELEMS = 1024;
constexpr int WALK_LDS_BUDGET = 160 * 1024;   // the CU's LDS: the walk's dynamic-LDS cap on every device
// one workgroup streams every tile through one CU's load path (≈ 30-60 GB/s): the walk wins only on small corners; above
// this many stream tiles per direction the chain launches (many CUs) take over. Measured at C5 (254 tiles per direction):
// the walk 4 MB / ≈ 140 µs against ≈ 65 µs for the back chains (round 4)
#ifndef NNRT_WALK_MAX_TILES
#define NNRT_WALK_MAX_TILES 48
#endif
struct WalkElem {
	const float* tile;   // 64 x 64 row-major tile
	int x_off;           // entry: first unknown of the tile whose x (back) / y (forward) it multiplies; head: J * 64
	int info;            // entry: -1; head: 1 if the tile is L_JJ^-1, 0 if it is L_JJ
};
struct CornerWalkArgs {
	const unsigned* gate;  // nullable: run only if the pivot ratio word is below ratio (the refinement pass)
	float ratio;
	const WalkElem* fwd;   // forward stream (n_fwd = 0: none)
	const WalkElem* back;  // back stream (n_back = 0: none)
	int n_fwd, n_back;
	const float* rhs;      // [ld] permuted right-hand side (back only: y; forward + back: b)
	const int* row_node;
	float* xout;           // [6 nc] corner-node order
	int ld, ring;
};

typedef __attribute__((address_space(3))) void walk_lds_t;
typedef const __attribute__((address_space(1))) void walk_global_t;

// one pass over a stream; x (LDS, ld floats) holds the right-hand side on entry and the solution on exit
template <bool BACK>
__device__ void walk_pass(const WalkElem* __restrict__ gdesc, int n, int R, WalkElem* desc, float* x, float* red, float* zt, float* ring) {
	const int t = threadIdx.x, wave = t >> 6, lane = t & 63;
	const int rg = t >> 4, cg = t & 15;   // rows 2 rg, 2 rg + 1 and columns 4 cg .. 4 cg + 3 of a tile
	for (int i = t; i < n; i += WT) desc[i] = gdesc[i];
	asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
	lds_barrier();
	int issued = 0;
	auto issue = [&](int e) {   // tile e -> ring slot e % R: 16 KB = 16 DMA pieces of 1 KB, two per wave
		const float* src = desc[e].tile;
		float* dst = ring + (e % R) * TILE_ELEMS;
#pragma unroll
		for (int i = 0; i < 2; i++) {
			const int chunk = 2 * wave + i;
			__builtin_amdgcn_global_load_lds((walk_global_t*)(src + chunk * 256 + lane * 4), (walk_lds_t*)(dst + chunk * 256), 16, 0, 0);
		}
	};
	while (issued < n && issued < R) issue(issued++);
	int p = 0;
	while (p < n) {
		int h = p;   // the column's head (its last element)
		while (desc[h].info < 0) h++;
		const int J64 = desc[h].x_off;
		float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);   // back: columns 4 cg.. partials; forward: .x / .y rows 2 rg / 2 rg + 1
		int q = p;
		while (true) {
			const int last = min(h, q + R - 1);
			wait_vmcnt(2 * (issued - 1 - last));
			lds_barrier();   // every wave's pieces of tiles q .. last have landed
			for (int e = q; e <= last && e < h; e++) {
				const float* T = ring + (e % R) * TILE_ELEMS;
				const float4 a = *reinterpret_cast<const float4*>(T + (2 * rg) * TILE + 4 * cg);
				const float4 b = *reinterpret_cast<const float4*>(T + (2 * rg + 1) * TILE + 4 * cg);
				const int xo = desc[e].x_off;
				if constexpr (BACK) {
					const float x0 = x[xo + 2 * rg], x1 = x[xo + 2 * rg + 1];
					acc.x += a.x * x0 + b.x * x1;
					acc.y += a.y * x0 + b.y * x1;
					acc.z += a.z * x0 + b.z * x1;
					acc.w += a.w * x0 + b.w * x1;
				} else {
					const float4 y = *reinterpret_cast<const float4*>(x + xo + 4 * cg);
					acc.x += ((a.x * y.x + a.y * y.y) + a.z * y.z) + a.w * y.w;
					acc.y += ((b.x * y.x + b.y * y.y) + b.z * y.z) + b.w * y.w;
				}
			}
			if (last == h) break;
			lds_barrier();   // tiles q .. last read by every wave: their slots are free
			while (issued < n && issued <= last + R) issue(issued++);
			q = last + 1;
		}
		// column finish: the head tile (slot h % R) is resident
		const float* Hd = ring + (h % R) * TILE_ELEMS;
		const bool inv = desc[h].info != 0;
		if constexpr (BACK) {
			// z_c = y_c - sum over rows: lanes 16 apart share columns; the 8 waves meet in LDS
#pragma unroll
			for (int m = 16; m < 64; m <<= 1) {
				acc.x += __shfl_xor(acc.x, m);
				acc.y += __shfl_xor(acc.y, m);
				acc.z += __shfl_xor(acc.z, m);
				acc.w += __shfl_xor(acc.w, m);
			}
			if (lane < 16) *reinterpret_cast<float4*>(red + wave * TILE + 4 * lane) = acc;
			lds_barrier();
			if (wave == 0) {
				float zs = 0.f;
#pragma unroll
				for (int w = 0; w < WT / 64; w++) zs += red[w * TILE + lane];
				zt[lane] = x[J64 + lane] - zs;
			}
			lds_barrier();
			if (inv) {   // x_c = sum_r M_rc z_r
				const float4 a = *reinterpret_cast<const float4*>(Hd + (2 * rg) * TILE + 4 * cg);
				const float4 b = *reinterpret_cast<const float4*>(Hd + (2 * rg + 1) * TILE + 4 * cg);
				const float z0 = zt[2 * rg], z1 = zt[2 * rg + 1];
				float4 m4 = make_float4(a.x * z0 + b.x * z1, a.y * z0 + b.y * z1, a.z * z0 + b.z * z1, a.w * z0 + b.w * z1);
#pragma unroll
				for (int m = 16; m < 64; m <<= 1) {
					m4.x += __shfl_xor(m4.x, m);
					m4.y += __shfl_xor(m4.y, m);
					m4.z += __shfl_xor(m4.z, m);
					m4.w += __shfl_xor(m4.w, m);
				}
				if (lane < 16) *reinterpret_cast<float4*>(red + wave * TILE + 4 * lane) = m4;
				lds_barrier();
				if (wave == 0) {
					float xs = 0.f;
#pragma unroll
					for (int w = 0; w < WT / 64; w++) xs += red[w * TILE + lane];
					x[J64 + lane] = xs;
				}
			} else if (wave == 0) {   // column-oriented substitution with L_JJ (lane = column, L_rc from the resident tile)
				float colv[TILE];
#pragma unroll
				for (int r = 0; r < TILE; r++) colv[r] = Hd[r * TILE + lane];
				float z = zt[lane], xv = 0.f;
#pragma unroll
				for (int r = TILE - 1; r >= 0; r--) {
					const float xr = lane_bcast(z, r) / lane_bcast(colv[r], r);
					xv = lane == r ? xr : xv;
					z -= colv[r] * xr;
				}
				x[J64 + lane] = xv;
			}
		} else {
			// row sums across the 16 column groups of each row (within the wave)
#pragma unroll
			for (int m = 1; m < 16; m <<= 1) {
				acc.x += __shfl_xor(acc.x, m);
				acc.y += __shfl_xor(acc.y, m);
			}
			if (cg == 0) {
				zt[2 * rg] = x[J64 + 2 * rg] - acc.x;
				zt[2 * rg + 1] = x[J64 + 2 * rg + 1] - acc.y;
			}
			lds_barrier();
			if (inv) {   // y_r = sum_c M_rc z_c
				const float4 a = *reinterpret_cast<const float4*>(Hd + (2 * rg) * TILE + 4 * cg);
				const float4 b = *reinterpret_cast<const float4*>(Hd + (2 * rg + 1) * TILE + 4 * cg);
				const float4 z = *reinterpret_cast<const float4*>(zt + 4 * cg);
				float y0 = ((a.x * z.x + a.y * z.y) + a.z * z.z) + a.w * z.w;
				float y1 = ((b.x * z.x + b.y * z.y) + b.z * z.z) + b.w * z.w;
#pragma unroll
				for (int m = 1; m < 16; m <<= 1) {
					y0 += __shfl_xor(y0, m);
					y1 += __shfl_xor(y1, m);
				}
				if (cg == 0) {
					x[J64 + 2 * rg] = y0;
					x[J64 + 2 * rg + 1] = y1;
				}
			} else if (wave == 0) {   // row-oriented substitution with L_JJ: lane r holds row r; y_c = z_c / L_cc, z_r -= L_rc y_c
				float rowv[TILE];
#pragma unroll
				for (int c4 = 0; c4 < TILE / 4; c4++) {
					const float4 v = *reinterpret_cast<const float4*>(Hd + lane * TILE + 4 * c4);
					rowv[4 * c4] = v.x;
					rowv[4 * c4 + 1] = v.y;
					rowv[4 * c4 + 2] = v.z;
					rowv[4 * c4 + 3] = v.w;
				}
				float z = zt[lane], yv = 0.f;
#pragma unroll
				for (int c = 0; c < TILE; c++) {
					const float yc = lane_bcast(z, c) / lane_bcast(rowv[c], c);
					yv = lane == c ? yc : yv;
					z -= rowv[c] * yc;   // rows r > c only matter (L_rc = 0 above the diagonal)
				}
				x[J64 + lane] = yv;
			}
		}
		lds_barrier();   // x_J visible; the column's slots (and red / zt) free
		while (issued < n && issued <= h + R) issue(issued++);
		p = h + 1;
	}
}

__global__ __launch_bounds__(WT) void k_corner_walk(CornerWalkArgs a) {
	extern __shared__ __attribute__((aligned(16))) float s_walk[];
	if (a.gate && !refine_gate_on(a.gate, a.ratio)) return;
	const int nd = a.n_fwd > a.n_back ? a.n_fwd : a.n_back;
	WalkElem* desc = reinterpret_cast<WalkElem*>(s_walk);
	float* x = s_walk + 4 * nd;
	float* red = x + ((a.ld + 3) & ~3);
	float* zt = red + (WT / 64) * TILE;
	float* ring = zt + TILE;
	for (int i = threadIdx.x; i < a.ld; i += WT) x[i] = a.rhs[i];
	if (a.n_fwd > 0) walk_pass<false>(a.fwd, a.n_fwd, a.ring, desc, x, red, zt, ring);
	else lds_barrier();
	if (a.n_back > 0) walk_pass<true>(a.back, a.n_back, a.ring, desc, x, red, zt, ring);
	for (int i = threadIdx.x; i < a.ld; i += WT) {
		const int rn = a.row_node[i];
		if (rn >= 0) a.xout[6 * static_cast<int64_t>(rn >> 3) + (rn & 7)] = x[i];
	}
}

// ===================================================================================================================
// CornerSolver
// ===================================================================================================================
template <typename T>
static nnrt_status dev_upload(T*& ptr, const std::vector<T>& host) {
	if (ptr) hipFree(ptr);
	ptr = nullptr;
	NNRT_HIP(hipMalloc(reinterpret_cast<void**>(&ptr), sizeof(T) * std::max<size_t>(host.size(), 1)));
	if (!host.empty()) NNRT_HIP(hipMemcpy(ptr, host.data(), sizeof(T) * host.size(), hipMemcpyHostToDevice));
	return NNRT_OK;
}

static void dev_free(void*& p) {
	if (p) hipFree(p);
	p = nullptr;
}

// development switches (A/B builds without rebuilding): NNRT_CORNER_WALK=1 enables the single-workgroup walk for small
// corners (round 4's default; the dataflow launch measured faster at C1_ARAP, 7,636 vs 7,500 GN it/s, and equal at
// C2_ARAP in round 5), NNRT_CORNER_FLOW=0 disables the dataflow substitution launch, NNRT_CORNER_TRIM=0 the
// padding-trimmed eliminations
static bool env_flag(const char* name, bool dflt) {
	const char* v = std::getenv(name);
	return v ? std::strcmp(v, "0") != 0 : dflt;
}

// The dynamic-LDS cap of k_corner_walk is a property of the kernel on each device, not of a plan: several plans with
// different walk_lds are live at once (every fitter, the arrowhead pool), so the cap is raised once per device to the
// whole LDS budget, which bounds every plan's walk_lds, under a mutex.
static bool walk_lds_cap_set() {
	static std::mutex mu;
	static std::set<int> done;
	int dev = 0;
	if (hipGetDevice(&dev) != hipSuccess) return false;
	std::lock_guard<std::mutex> lk(mu);
	if (done.count(dev)) return true;
	if (hipFuncSetAttribute(reinterpret_cast<const void*>(k_corner_walk), hipFuncAttributeMaxDynamicSharedMemorySize, WALK_LDS_BUDGET) != hipSuccess)
		return false;
	done.insert(dev);
	return true;
}

CornerSolver::~CornerSolver() { release(); }

void CornerSolver::release() {
	for (void** p : {reinterpret_cast<void**>(&tiles), reinterpret_cast<void**>(&ldiag), reinterpret_cast<void**>(&minv),
	                 reinterpret_cast<void**>(&cb2), reinterpret_cast<void**>(&d_fwd_chains), reinterpret_cast<void**>(&d_fwd_cols),
	                 reinterpret_cast<void**>(&sdiag), reinterpret_cast<void**>(&pivot_word),
	                 reinterpret_cast<void**>(&d_fwd_ent), reinterpret_cast<void**>(&d_walk_back), reinterpret_cast<void**>(&d_walk_fwd),
	                 reinterpret_cast<void**>(&cb),
	                 reinterpret_cast<void**>(&xp), reinterpret_cast<void**>(&d_tile_slot), reinterpret_cast<void**>(&d_slot_ij),
	                 reinterpret_cast<void**>(&d_row_node), reinterpret_cast<void**>(&d_node_row), reinterpret_cast<void**>(&d_tasks),
	                 reinterpret_cast<void**>(&d_srcs), reinterpret_cast<void**>(&d_back_cols), reinterpret_cast<void**>(&d_back_ent), reinterpret_cast<void**>(&d_back_chains),
	                 reinterpret_cast<void**>(&d_corner_edges), reinterpret_cast<void**>(&zx), reinterpret_cast<void**>(&d_back_pre),
	                 reinterpret_cast<void**>(&d_fwd_pre), reinterpret_cast<void**>(&d_flow_chains), reinterpret_cast<void**>(&d_flow_need),
	                 reinterpret_cast<void**>(&d_col_chain), reinterpret_cast<void**>(&flow_ctl), reinterpret_cast<void**>(&d_inv_cols)})
		dev_free(*p);
	use_flow = false;
	fold_invert = false;
	n_inv_cols = 0;
	n_chains = n_flow_ctl = 0;
	back_pre_off.clear();
	fwd_pre_off.clear();
	nc = ld = T = H = slots = n_corner_edges = 0;
	level_off.clear();
	level_panel.clear();
	fwd_off.clear();
	back_off.clear();
	key.clear();
}

nnrt_status CornerSolver::prepare(const int32_t* edges, int E, int n0, int N, const float* corner_pos) {
	std::vector<int32_t> k(edges, edges + 2 * static_cast<size_t>(E));
	k.push_back(n0);
	k.push_back(N);
	if (corner_pos) {   // the plan depends on the positions too
		const size_t nf = 3 * static_cast<size_t>(std::max(N - n0, 0));
		const size_t at = k.size();
		k.resize(at + nf);
		std::memcpy(k.data() + at, corner_pos, sizeof(float) * nf);
	}
	if (k == key && (nc == 0 || tiles)) return NNRT_OK;   // same hierarchy: keep the plan and its buffers
	// the old buffers go now: bump the generation first, so that whatever captured them (the fitter's graphs) is dropped
	// even if the new plan fails below; a failure leaves the solver empty (released), never half-built
	release();
	generation++;
	const CornerPlan p = plan_corner(edges, E, n0, N, corner_pos, env_flag("NNRT_CORNER_TRIM", true));
	auto fail = [&](nnrt_status st) {
		release();
		return st;
	};
	auto alloc = [&](float*& ptr, size_t n) -> nnrt_status {
		NNRT_HIP(hipMalloc(reinterpret_cast<void**>(&ptr), sizeof(float) * n));
		return NNRT_OK;
	};
	if (p.nc > 0) {
		nnrt_status st;
		if ((st = alloc(tiles, p.slot_ij.size() * TILE_ELEMS)) || (st = alloc(ldiag, static_cast<size_t>(p.T) * TILE_ELEMS)) ||
		    (st = alloc(minv, static_cast<size_t>(p.T) * TILE_ELEMS)) || (st = alloc(cb2, static_cast<size_t>(p.ld))) ||
		    (st = alloc(sdiag, static_cast<size_t>(p.ld))) || (st = alloc(reinterpret_cast<float*&>(pivot_word), REFINE_WORDS)) ||
		    (st = alloc(cb, static_cast<size_t>(p.ld))) || (st = alloc(xp, static_cast<size_t>(p.ld))) || (st = alloc(xp2, static_cast<size_t>(p.ld))) ||
		    (st = alloc(zx, static_cast<size_t>(p.ld))))
			return fail(st);
		if ((st = dev_upload(d_tile_slot, p.tile_slot)) || (st = dev_upload(d_slot_ij, p.slot_ij)) || (st = dev_upload(d_row_node, p.row_node)) ||
		    (st = dev_upload(d_node_row, p.node_row)) || (st = dev_upload(d_tasks, p.tasks)) || (st = dev_upload(d_srcs, p.srcs)) ||
		    (st = dev_upload(d_back_cols, p.back_cols)) || (st = dev_upload(d_back_ent, p.back_ent)) || (st = dev_upload(d_back_chains, p.back_chains)) ||
		    (st = dev_upload(d_corner_edges, p.corner_edges)) ||
		    (st = dev_upload(d_fwd_chains, p.fwd_chains)) || (st = dev_upload(d_fwd_cols, p.fwd_cols)) || (st = dev_upload(d_fwd_ent, p.fwd_ent)) ||
		    (st = dev_upload(d_back_pre, p.back_pre)) || (st = dev_upload(d_fwd_pre, p.fwd_pre)))
			return fail(st);
		if (hipMemset(cb2, 0, sizeof(float) * static_cast<size_t>(p.ld)) != hipSuccess) {   // identity padding rows stay 0
			set_error("hipMemset failed");
			return fail(NNRT_ERROR_HIP);
		}
	}
	walk_ok = false;
	if (p.nc > 0 && env_flag("NNRT_CORNER_WALK", false) && p.ld <= WALK_MAX_LD && static_cast<int>(std::max(p.walk_back.size(), p.walk_fwd.size())) <= std::min(WALK_MAX_ELEMS, NNRT_WALK_MAX_TILES)) {
		// LDS: descriptors, the solution vector, the reduction rows, then a ring of as many tiles as fit (at least the
		// largest column's elements need not fit: a column streams through the ring in parts)
		const size_t nd = std::max(p.walk_back.size(), p.walk_fwd.size());
		const size_t fixed = 16 * nd + 4 * (static_cast<size_t>((p.ld + 3) & ~3) + (WT / 64) * TILE + TILE);
		const size_t budget = 160 * 1024;
		const int ring_tiles = fixed < budget ? static_cast<int>(std::min<size_t>(8, (budget - fixed) / (4 * TILE_ELEMS))) : 0;
		if (ring_tiles >= 2) {
			std::vector<WalkElem> wb, wf;
			auto elem = [&](const int4& e) {
				const float* base = e.x == 0 ? tiles : e.x == 1 ? minv : ldiag;
				return WalkElem{base + static_cast<int64_t>(e.y) * TILE_ELEMS, e.z, e.w};
			};
			for (const auto& e : p.walk_back) wb.push_back(elem(e));
			for (const auto& e : p.walk_fwd) wf.push_back(elem(e));
			nnrt_status st;
			if ((st = dev_upload(d_walk_back, wb)) || (st = dev_upload(d_walk_fwd, wf))) return fail(st);
			walk_ring = ring_tiles;
			walk_lds = static_cast<int>(fixed + static_cast<size_t>(ring_tiles) * 4 * TILE_ELEMS);
			n_walk_back = static_cast<int>(wb.size());
			n_walk_fwd = static_cast<int>(wf.size());
			if (!walk_lds_cap_set()) {
				set_error("hipFuncSetAttribute (corner walk LDS) failed");
				return fail(NNRT_ERROR_HIP);
			}
			walk_ok = true;
		}
	}
	if (p.nc > 0 && !walk_ok && env_flag("NNRT_CORNER_FLOW", true)) {   // dataflow substitution launches (k_corner_flow)
		nnrt_status st;
		if ((st = dev_upload(d_flow_chains, p.flow_chains)) || (st = dev_upload(d_flow_need, p.flow_need)) || (st = dev_upload(d_col_chain, p.col_chain)))
			return fail(st);
		n_chains = static_cast<int>(p.flow_chains.size());
		n_flow_ctl = 2 * flow_ctl_words(n_chains);
		if ((st = alloc(reinterpret_cast<float*&>(flow_ctl), static_cast<size_t>(n_flow_ctl)))) return fail(st);
		use_flow = true;
	}
	nc = p.nc;
	if (nc > 0) {
		ld = p.ld;
		T = p.T;
		H = p.H;
		slots = static_cast<int>(p.slot_ij.size());
		n_corner_edges = static_cast<int>(p.corner_edges.size());
		level_off = p.level_off;
		level_panel = p.level_panel;
		fwd_off = p.fwd_off;
		back_off = p.back_off;
		fwd_pre_off = p.fwd_pre_off;
		back_pre_off = p.back_pre_off;
		fill_tiles = static_cast<int64_t>(slots);
		n_terms = static_cast<int64_t>(p.srcs.size());
		exec_mfma_flops = 0;
		for (const int4& q : p.srcs) exec_mfma_flops += static_cast<int64_t>(q.w) * 4 * 2 * TILE * TILE * 2;   // 4 nq steps of 64 x 64 x 2
		elim_cols = 0;
		for (int l = 0; l < p.H; l++)
			for (int q = p.level_off[static_cast<size_t>(l)]; q < p.level_off[static_cast<size_t>(l)] + p.level_panel[static_cast<size_t>(l)]; q++) {
				const CornerTask& tk = p.tasks[static_cast<size_t>(q)];
				if (ELIM_WAVES == 0 && tk.nreal > TILE / 2) exec_mfma_flops += 3 * 2 * 32 * 32 * 32;   // the rank-32 products of waves 1-3
				if (tk.I == tk.J) elim_cols += tk.nreal;
			}
		dense_tiles = static_cast<int64_t>(corner_ld(6 * nc) / TILE) * (corner_ld(6 * nc) / TILE + 1) / 2;
		// the diagonal inverses ride in the last factor launch: its diagonal tasks invert their own tile, extra workgroups
		// the other levels' (NNRT_CORNER_FOLD_INV=0: one k_corner_invert launch after the factorization)
		fold_invert = env_flag("NNRT_CORNER_FOLD_INV", true);
		if (fold_invert) {
			const size_t l0 = static_cast<size_t>(p.level_off[static_cast<size_t>(p.H) - 1]);
			std::vector<char> last(static_cast<size_t>(p.T), 0);
			for (size_t q = l0; q < l0 + static_cast<size_t>(p.level_panel[static_cast<size_t>(p.H) - 1]); q++)
				if (p.tasks[q].I == p.tasks[q].J) last[static_cast<size_t>(p.tasks[q].J)] = 1;
			std::vector<int> cols;
			for (int J = 0; J < p.T; J++)
				if (!last[static_cast<size_t>(J)]) cols.push_back(J);
			n_inv_cols = static_cast<int>(cols.size());
			nnrt_status st;
			if (!cols.empty() && (st = dev_upload(d_inv_cols, cols))) return fail(st);
		}
	}
	key.swap(k);
	return NNRT_OK;
}

CornerMap CornerSolver::map() const { return CornerMap{T, d_tile_slot, d_node_row, tiles, sdiag}; }

nnrt_status CornerSolver::launch_init(int n0, const float* diag, const float* rhs, const int32_t* edges, const float* wing, hipStream_t s) const {
	if (nc == 0) return NNRT_OK;
	const CornerInitArgs ia = init_args(n0);
	k_corner_init<<<static_cast<unsigned>(ceil_div(ia.threads(), 256)), 256, 0, s>>>(ia, diag, rhs);
	NNRT_LAUNCH_CHECK();
	return launch_offdiag(n0, edges, wing, s);
}

nnrt_status CornerSolver::launch_offdiag(int n0, const int32_t* edges, const float* wing, hipStream_t s) const {
	if (nc == 0) return NNRT_OK;
	if (n_corner_edges > 0) {
		k_corner_offdiag<<<n_corner_edges, 64, 0, s>>>(d_corner_edges, n0, edges, wing, map());
		NNRT_LAUNCH_CHECK();
	}
	return NNRT_OK;
}

nnrt_status CornerSolver::launch_solve(float* xout, int* error_flag, hipStream_t s) const {
	if (nc == 0) return NNRT_OK;
	nnrt_status st = launch_factor(error_flag, s);
	if (st) return st;
	if (walk_ok) {   // the back substitution as one single-workgroup walk
		const CornerWalkArgs wa{nullptr, 0.f, nullptr, d_walk_back, 0, n_walk_back, cb, d_row_node, xout, ld, walk_ring};
		k_corner_walk<<<1, WT, walk_lds, s>>>(wa);
		NNRT_LAUNCH_CHECK();
		return NNRT_OK;
	}
	return launch_back(cb, xout, s, nullptr, 0.f);
}

nnrt_status CornerSolver::launch_factor(int* error_flag, hipStream_t s) const {
	if (nc == 0) return NNRT_OK;
	CornerFactorArgs fa{};
	fa.tiles = tiles;
	fa.ldiag = ldiag;
	fa.cb = cb;
	fa.srcs = d_srcs;
	fa.error_flag = error_flag;
	fa.sdiag = sdiag;
	fa.pivot_word = pivot_word;
	fa.minv = minv;
	fa.inv_cols = d_inv_cols;
	for (int l = 0; l < H; l++) {
		fa.level = l;
		const int n = level_off[static_cast<size_t>(l) + 1] - level_off[static_cast<size_t>(l)];
		fa.tasks = d_tasks + level_off[static_cast<size_t>(l)];
		fa.n_panel = level_panel[static_cast<size_t>(l)];
		fa.n_tasks = n;
		const bool last = fold_invert && l == H - 1;
		fa.n_inv = last ? n_inv_cols : 0;
		fa.invert_self = last ? 1 : 0;
		fa.flow_ctl = last ? flow_ctl : nullptr;
		fa.n_ctl = last ? n_flow_ctl : 0;
		k_corner_factor<<<n + fa.n_inv, CTF, 0, s>>>(fa);
		NNRT_LAUNCH_CHECK();
	}
	if (!fold_invert) {
		// every diagonal factor's inverse, one workgroup per tile column (the substitutions multiply by them)
		k_corner_invert<<<T, CT, 0, s>>>(ldiag, minv, flow_ctl, n_flow_ctl);
		NNRT_LAUNCH_CHECK();
	}
	return NNRT_OK;
}

nnrt_status CornerSolver::launch_flow(const FlowStem& st, hipStream_t s) const {
	if (nc == 0 || !use_flow) {
		set_error("launch_flow without a dataflow plan");
		return NNRT_ERROR_ARGUMENT;
	}
	FlowArgs a{};
	a.refine = st.mode == 1;
	a.nB = n_chains;
	a.T = T;
	a.ld = ld;
	a.stem_wg = static_cast<int>(ceil_div(std::max(std::max(st.n_update, st.n0), st.mode == 1 ? st.N : 0), CT));
	a.nxout = 6 * static_cast<int64_t>(nc);
	a.ctl = flow_ctl;
	a.chains = d_flow_chains;
	a.fwd_need = d_flow_need;
	a.col_chain = d_col_chain;
	a.node_row = d_node_row;
	a.back = CornerBackArgs{nullptr, 0.f, tiles, ldiag, minv, cb, xp, d_row_node, st.x + 6 * static_cast<int64_t>(st.n0), nullptr, d_back_cols,
	                        d_back_ent, zx, 0};
	a.fwd = CornerFwdArgs{nullptr, 0.f, tiles, ldiag, minv, cb2, nullptr, d_fwd_cols, d_fwd_ent, zx, 0};
	a.back2 = CornerBackArgs{nullptr, 0.f, tiles, ldiag, minv, cb2, xp2, d_row_node, a.refine ? st.dx + 6 * static_cast<int64_t>(st.n0) : nullptr,
	                         nullptr, d_back_cols, d_back_ent, zx, 0};
	a.st = st;
	const int grid = n_chains + a.stem_wg + (a.refine ? T + 2 * n_chains + 2 * a.stem_wg : 0);
	k_corner_flow<<<grid, CT, 0, s>>>(a);
	NNRT_LAUNCH_CHECK();
	return NNRT_OK;
}

// back substitution chains over y (with NNRT_SUBST_PRESUM, each launch preceded by its columns' pre-sums)
nnrt_status CornerSolver::launch_back(const float* y, float* xout, hipStream_t s, const unsigned* gate, float refine_ratio) const {
	CornerBackArgs ba{gate, refine_ratio, tiles, ldiag, minv, y, xp, d_row_node, xout, nullptr, d_back_cols, d_back_ent, zx, 0};
	for (size_t l = 0; l + 1 < back_off.size(); l++) {
		const int n = back_off[l + 1] - back_off[l];
		const int npre = NNRT_SUBST_PRESUM ? back_pre_off[l + 1] - back_pre_off[l] : 0;
		if (npre > 0) {
			ba.chains = d_back_pre + back_pre_off[l];
			ba.mode = 1;
			k_corner_back<<<npre, CT, 0, s>>>(ba, ld, 6 * static_cast<int64_t>(nc));
			NNRT_LAUNCH_CHECK();
		}
		ba.chains = d_back_chains + back_off[l];
		ba.mode = NNRT_SUBST_PRESUM ? 2 : 0;
		k_corner_back<<<n, CT, 0, s>>>(ba, ld, 6 * static_cast<int64_t>(nc));
		NNRT_LAUNCH_CHECK();
	}
	return NNRT_OK;
}

nnrt_status CornerSolver::launch_resolve(float* xout, hipStream_t s, const unsigned* gate, float refine_ratio) const {
	if (nc == 0) return NNRT_OK;
	if (walk_ok) {   // forward and back substitution in one single-workgroup launch
		const CornerWalkArgs wa{gate, refine_ratio, d_walk_fwd, d_walk_back, n_walk_fwd, n_walk_back, cb2, d_row_node, xout, ld, walk_ring};
		k_corner_walk<<<1, WT, walk_lds, s>>>(wa);
		NNRT_LAUNCH_CHECK();
		return NNRT_OK;
	}
	CornerFwdArgs fa{gate, refine_ratio, tiles, ldiag, minv, cb2, nullptr, d_fwd_cols, d_fwd_ent, zx, 0};
	for (size_t l = 0; l + 1 < fwd_off.size(); l++) {
		const int n = fwd_off[l + 1] - fwd_off[l];
		const int npre = NNRT_SUBST_PRESUM ? fwd_pre_off[l + 1] - fwd_pre_off[l] : 0;
		if (npre > 0) {
			fa.chains = d_fwd_pre + fwd_pre_off[l];
			fa.mode = 1;
			k_corner_fwd<<<npre, CT, 0, s>>>(fa, ld);
			NNRT_LAUNCH_CHECK();
		}
		fa.chains = d_fwd_chains + fwd_off[l];
		fa.mode = NNRT_SUBST_PRESUM ? 2 : 0;
		k_corner_fwd<<<n, CT, 0, s>>>(fa, ld);
		NNRT_LAUNCH_CHECK();
	}
	return launch_back(cb2, xout, s, gate, refine_ratio);
}

#ifdef NNRT_CORNER_STAMPS
extern "C" int nnrt_dev_flow_stamps(unsigned long long* out) {   // [128][66][4] stamps of the last dataflow launch
	return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_flow_stamps), sizeof(unsigned long long) * 128 * 66 * 4) == hipSuccess ? 0 : 1;
}
extern "C" int nnrt_dev_corner_stamps(unsigned long long* out) {   // [64][512][8] stamps of the last solve
	return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_corner_stamps), sizeof(unsigned long long) * 64 * 512 * 8) == hipSuccess ? 0 : 1;
}
extern "C" int nnrt_dev_elim_stamps(unsigned long long* out) {   // [16][128][16][4] stamps of the last solve
	return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_elim_stamps), sizeof(unsigned long long) * 16 * 128 * 16 * 4) == hipSuccess ? 0 : 1;
}
#endif

} // namespace nnrt
