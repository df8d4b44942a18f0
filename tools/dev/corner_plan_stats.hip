// Host-only statistics of the Schur-corner plan (csrc/corner.hip plan_corner) for a structure file written by
// tools/dev/corner_plan_stats.py: per factor launch the panel / trailing tasks and update terms, per back-substitution
// launch the chains, their columns and entry tiles. Build: hipcc -O2 -std=c++17 --offload-arch=gfx950 -I include
// -I dynamicfuion_python_amd/csrc -x hip tools/dev/corner_plan_stats.hip -o /tmp/corner_plan_stats
#include "corner.hip"
#include <cstdio>
namespace nnrt { void set_error(const std::string& m) { fprintf(stderr, "%s\n", m.c_str()); } }
using namespace nnrt;
int main(int argc, char** argv) {
	FILE* f = fopen(argv[1], "rb");
	int E, n0, N;
	fread(&E, 4, 1, f); fread(&n0, 4, 1, f); fread(&N, 4, 1, f);
	std::vector<int32_t> edges(2 * E);
	fread(edges.data(), 4, 2 * E, f);
	std::vector<float> pos(3 * (N - n0));
	const bool has_pos = fread(pos.data(), 4, pos.size(), f) == pos.size() && !pos.empty();
	fclose(f);
	CornerPlan p = plan_corner(edges.data(), E, n0, N, has_pos ? pos.data() : nullptr);
	printf("nc %d ld %d T %d H %d slots %zu tasks %zu srcs %zu\n", p.nc, p.ld, p.T, p.H, p.slot_ij.size(), p.tasks.size(), p.srcs.size());
	for (int l = 0; l < p.H; l++) {
		int np = p.level_panel[l], nt = p.level_off[l + 1] - p.level_off[l] - np, cols = 0, maxsrc = 0, sumsrc = 0;
		for (int q = p.level_off[l]; q < p.level_off[l + 1]; q++) {
			const CornerTask& t = p.tasks[q];
			if (q - p.level_off[l] < np && t.I == t.J) cols++;
			maxsrc = std::max(maxsrc, t.nd + t.np);
			sumsrc += t.nd + t.np;
		}
		printf("level %2d: columns %3d panel tasks %3d trailing %4d  update terms max %3d total %5d\n", l, cols, np, nt, maxsrc, sumsrc);
	}
	for (size_t l = 0; l + 1 < p.back_off.size(); l++) {
		int maxlen = 0, maxent = 0, sument = 0, totcols = 0;
		for (int c = p.back_off[l]; c < p.back_off[l + 1]; c++) {
			const int2 ch = p.back_chains[c];
			maxlen = std::max(maxlen, ch.y);
			totcols += ch.y;
			int ent = 0;
			for (int q = 0; q < ch.y; q++) { ent += p.back_cols[ch.x + q].z; maxent = std::max(maxent, p.back_cols[ch.x + q].z); }
			sument += ent;
		}
		// entries whose I lies in the same chain (x produced inside the launch) vs earlier launches; per chain, the
		// tiles the chain's workgroup reads in order (entries + one L_JJ^-1 per column)
		int inchain = 0, maxchain_tiles = 0, maxchain_inner = 0;
		for (int c = p.back_off[l]; c < p.back_off[l + 1]; c++) {
			const int2 ch = p.back_chains[c];
			int tiles = 0, inner = 0;
			for (int q = 0; q < ch.y; q++) {
				const int4 bc = p.back_cols[ch.x + q];
				tiles += bc.z + 1;
				for (int e = 0; e < bc.z; e++) {
					const int I = p.back_ent[bc.y + e].y;
					for (int q2 = 0; q2 < q; q2++)
						if (p.back_cols[ch.x + q2].x == I) { inchain++; inner++; }
				}
				inner++;
			}
			maxchain_tiles = std::max(maxchain_tiles, tiles);
			maxchain_inner = std::max(maxchain_inner, inner);
		}
		printf("back %zu: chains %3d columns %3d longest chain %3d entries/col max %3d total %4d in-chain %4d; heaviest chain %d tiles (%d on the chain's path)\n", l,
		       p.back_off[l + 1] - p.back_off[l], totcols, maxlen, maxent, sument, inchain, maxchain_tiles, maxchain_inner);
	}
	// staging MFMA steps per level (the slowest panel task): every term 32 steps of 32x32x2, against skipping the steps
	// whose k lies in the source column's identity padding (possible when the column has <= 32 real columns)
	{
		std::vector<int> nreal(p.T, 64);
		for (int l = 0; l < p.H; l++)
			for (int q = p.level_off[l]; q < p.level_off[l] + p.level_panel[l]; q++)
				if (p.tasks[q].I == p.tasks[q].J) nreal[p.tasks[q].J] = p.tasks[q].nreal;
		int le32 = 0;
		for (int J = 0; J < p.T; J++) le32 += nreal[J] <= 32;
		long tot_now = 0, tot_skip = 0;
		for (int l = 0; l < p.H; l++) {
			int worst_now = 0, worst_skip = 0;
			for (int q = p.level_off[l]; q < p.level_off[l] + p.level_panel[l]; q++) {
				const CornerTask& tk = p.tasks[q];
				const bool diag = tk.I == tk.J;
				const int rounds = std::max(tk.nd, diag ? 0 : tk.np);
				int now = 0, skip = 0;
				for (int e = 0; e < rounds; e++) {
					int sd = e < tk.nd ? 32 : 0, sp = (!diag && e < tk.np) ? 32 : 0;
					int kd = e < tk.nd ? p.srcs[tk.src + e].z : -1, kp = (!diag && e < tk.np) ? p.srcs[tk.src + tk.nd + e].z : -1;
					int td = kd >= 0 ? (nreal[kd] <= 32 ? nreal[kd] : 32) : 0, tp = kp >= 0 ? (nreal[kp] <= 32 ? nreal[kp] : 32) : 0;
					now += sd + sp;   // both groups share the SIMDs
					skip += td + tp;
				}
				worst_now = std::max(worst_now, now);
				worst_skip = std::max(worst_skip, skip);
			}
			tot_now += worst_now;
			tot_skip += worst_skip;
			printf("level %2d: staging MFMA steps per SIMD (slowest panel) %4d, with padding skipped %4d\n", l, worst_now, worst_skip);
		}
		printf("columns with <= 32 real columns: %d of %d; staging steps over the levels %ld -> %ld\n", le32, p.T, tot_now, tot_skip);
	}
	// the dataflow launch's critical path (k_corner_flow): a back chain starts when its parent chain ends; per chain its
	// columns and entry tiles, the deepest path in columns and entries
	{
		const int nB = static_cast<int>(p.flow_chains.size());
		std::vector<int> depth_cols(nB, 0), depth_ent(nB, 0);
		int best = 0, best_ent = 0;
		for (int c = 0; c < nB; c++) {   // root first: a parent precedes its children
			const int4 ch = p.flow_chains[c];
			int ent = 0;
			for (int q = 0; q < ch.y; q++) ent += p.back_cols[ch.x + q].z;
			depth_cols[c] = ch.y + (ch.w >= 0 ? depth_cols[ch.w] : 0);
			depth_ent[c] = ent + (ch.w >= 0 ? depth_ent[ch.w] : 0);
			if (depth_cols[c] > best) { best = depth_cols[c]; best_ent = depth_ent[c]; }
		}
		printf("flow: chains %d, critical path %d columns with %d entry tiles\n", nB, best, best_ent);
	}
	return 0;
}
