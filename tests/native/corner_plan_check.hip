// Host-only check of the Schur-corner plan (csrc/corner.hip plan_corner), test infrastructure: builds the plan for an
// arrowhead structure read from argv[1] (int32 E, n0, N, edges [E,2], optional float32 corner positions [N-n0,3]),
// then emulates every factor launch in double precision task by task, checking that every structurally non-zero entry
// has a stored tile, that no task of a launch writes anything another task of the same launch reads or writes, that
// the back substitution only reads x of earlier launches or of its own chain, and that the solution of a random SPD
// system with that structure has a residual below 1e-9. Exit code 0 = all checks pass.
#include "corner.hip"   // the product plan code, compiled here for the host (no kernel is launched)
#include <cmath>
#include <cstdio>
#include <random>
#include <set>
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
	printf("positions %d\n", (int)has_pos);
	const int nc = p.nc, m = 6 * nc, T = p.T;
	printf("nc %d ld %d T %d H %d slots %zu tasks %zu srcs %zu back_cols %zu\n", nc, p.ld, T, p.H, p.slot_ij.size(), p.tasks.size(), p.srcs.size(), p.back_cols.size());
	// random SPD corner with the plan's adjacency pattern (natural order)
	std::mt19937 rng(5);
	std::normal_distribution<double> nd(0, 0.3);
	std::vector<double> M((size_t)m * m, 0.0);
	std::vector<std::vector<int>> adj(nc);
	for (int e = 0; e < E; e++) { int i = edges[2*e], j = edges[2*e+1]; if (i >= n0) { adj[i-n0].push_back(j-n0); } }
	std::vector<std::vector<int>> st(n0);
	for (int e = 0; e < E; e++) { int i = edges[2*e], j = edges[2*e+1]; if (i < n0) st[i].push_back(j-n0); }
	for (auto& s : st) for (int a : s) for (int b : s) if (a < b) adj[a].push_back(b);
	for (int a = 0; a < nc; a++) { std::sort(adj[a].begin(), adj[a].end()); adj[a].erase(std::unique(adj[a].begin(), adj[a].end()), adj[a].end()); }
	for (int a = 0; a < nc; a++) for (int b : adj[a]) for (int r = 0; r < 6; r++) for (int c = 0; c < 6; c++) { double v = nd(rng); M[(size_t)(6*a+r)*m + 6*b+c] += v; M[(size_t)(6*b+c)*m + 6*a+r] += v; }
	for (int i = 0; i < m; i++) { double s = 0; for (int j = 0; j < m; j++) if (j != i) s += fabs(M[(size_t)i*m+j]); M[(size_t)i*m+i] = s + 1.0; }
	std::vector<double> bnat(m); for (auto& v : bnat) v = nd(rng);
	// storage
	const int TE = TILE_ELEMS;
	std::vector<double> tiles(p.slot_ij.size() * TE, 0.0), ldiag((size_t)T * TE, 0.0), cb(p.ld, 0.0), xp(p.ld, 0.0), xout(m, 0.0);
	auto ent = [&](int R, int C) -> double { int rn = p.row_node[R], cn = p.row_node[C]; if (rn >= 0 && cn >= 0) return M[(size_t)(6*(rn>>3)+(rn&7))*m + 6*(cn>>3)+(cn&7)]; return R == C ? 1.0 : 0.0; };
	// every non-zero entry of M must land in a stored tile
	for (int a = 0; a < nc; a++) for (int b = 0; b < nc; b++) { bool nz = false; for (int r=0;r<6;r++) for(int c=0;c<6;c++) nz |= M[(size_t)(6*a+r)*m+6*b+c] != 0; if (!nz) continue;
		for (int r=0;r<6;r++) for(int c=0;c<6;c++){ int R = p.node_row[a]+r, C = p.node_row[b]+c; if (R < C) continue; if (p.tile_slot[(size_t)(R/TILE)*T + C/TILE] < 0) { printf("MISSING tile for entry %d %d\n", R, C); return 1; } } }
	for (size_t s = 0; s < p.slot_ij.size(); s++) { int I = p.slot_ij[s].x, J = p.slot_ij[s].y; for (int r = 0; r < TILE; r++) for (int c = 0; c < TILE; c++) tiles[s*TE + r*TILE + c] = ent(I*TILE+r, J*TILE+c); }
	for (int R = 0; R < p.ld; R++) { int rn = p.row_node[R]; cb[R] = rn >= 0 ? bnat[6*(rn>>3)+(rn&7)] : 0.0; }
	auto tile = [&](int s) { return &tiles[(size_t)s * TE]; };
	std::vector<double> minv((size_t)T * TE, 0.0);
	std::vector<int> ldiag_launch(T, -1), inv_launch(T, -1);
	for (int l = 0; l < p.H; l++) {
		std::set<std::pair<int,int>> reads, writes;   // (kind, id): 0 tile slot, 1 ldiag J, 2 cb J, 3 minv J
		std::vector<std::set<std::pair<int,int>>> tr, tw;
		for (int q = p.level_off[l]; q < p.level_off[l+1]; q++) {
			const CornerTask& tk = p.tasks[q];
			const bool panel = q - p.level_off[l] < p.level_panel[l];
			std::set<std::pair<int,int>> r, w;
			const int4* src = &p.srcs[tk.src];
			// a term runs the MFMA steps s < 4 srcs.w only (k-columns s and 32 + s): the skipped ones must be padding
			for (int e = 0; e < tk.nd + tk.np; e++) {
				const int4 q = src[e];
				if (q.w < 1 || q.w > 8) { printf("term step groups %d out of range\n", q.w); return 1; }
				if (q.w < 8)
					for (int k = 4 * q.w; k < TILE; k++)
						if (p.row_node[(size_t)q.z * TILE + k] >= 0) { printf("term over column %d skips its real column %d\n", q.z, k); return 1; }
			}
			auto kin = [](int w, int k) { return w >= 8 || (k & 31) < 4 * w; };
			auto upd = [&](double* out, const double* A, const int4* s, int n) { for (int i=0;i<TILE;i++) for(int j=0;j<TILE;j++){ double v = A[i*TILE+j]; for (int e=0;e<n;e++){ const double* X = tile(s[e].x); const double* Y = tile(s[e].y); for(int k=0;k<TILE;k++) if (kin(s[e].w, k)) v -= X[i*TILE+k]*Y[j*TILE+k]; r.insert({0,s[e].x}); r.insert({0,s[e].y}); } out[i*TILE+j]=v; } };
			auto rhsu = [&](int J, const int4* s, int n) { std::vector<double> o(TILE); for (int i=0;i<TILE;i++){ double v = cb[J*TILE+i]; for(int e=0;e<n;e++){ const double* X = tile(s[e].x); for (int k=0;k<TILE;k++) v -= X[i*TILE+k]*cb[s[e].z*TILE+k]; r.insert({2,s[e].z}); r.insert({0,s[e].x}); } o[i]=v; } return o; };
			if (!panel) {
				std::vector<double> o(TE); upd(o.data(), tile(tk.slot_t), src, tk.nd); r.insert({0,tk.slot_t}); w.insert({0,tk.slot_t});
				std::copy(o.begin(), o.end(), tile(tk.slot_t));
				if (tk.I == tk.J) { auto y = rhsu(tk.J, src, tk.nd); for (int i=0;i<TILE;i++) cb[tk.J*TILE+i] = y[i]; r.insert({2,tk.J}); w.insert({2,tk.J}); }
			} else {
				std::vector<double> d(TE), pp(TE); upd(d.data(), tile(tk.slot_d), src, tk.nd); r.insert({0,tk.slot_d});
				// cholesky of d
				for (int j=0;j<TILE;j++){ double s = d[j*TILE+j]; for(int k=0;k<j;k++) s -= d[j*TILE+k]*d[j*TILE+k]; if (!(s>0)) { printf("not PD\n"); return 1;} s = sqrt(s); d[j*TILE+j]=s; for(int i=j+1;i<TILE;i++){ double t = d[i*TILE+j]; for(int k=0;k<j;k++) t -= d[i*TILE+k]*d[j*TILE+k]; d[i*TILE+j] = t/s; } for (int c=j+1;c<TILE;c++) d[j*TILE+c]=0; }
				if (tk.I == tk.J) {
					auto y = rhsu(tk.J, src, tk.nd); r.insert({2,tk.J});
					for (int i=0;i<TILE;i++){ double v=y[i]; for(int k=0;k<i;k++) v -= d[i*TILE+k]*y[k]; y[i] = v/d[i*TILE+i]; }
					for (int i=0;i<TILE;i++) cb[tk.J*TILE+i] = y[i]; w.insert({2,tk.J});
					std::copy(d.begin(), d.end(), &ldiag[(size_t)tk.J*TE]); w.insert({1,tk.J}); ldiag_launch[tk.J] = l;
				} else {
					upd(pp.data(), tile(tk.slot_t), src + tk.nd, tk.np); r.insert({0,tk.slot_t});
					// L_IJ = pp L_JJ^-T : solve X L^T = pp row by row
					for (int i=0;i<TILE;i++) for (int j=0;j<TILE;j++){ double v = pp[i*TILE+j]; for (int k=0;k<j;k++) v -= pp[i*TILE+k]*d[j*TILE+k]; pp[i*TILE+j] = v / d[j*TILE+j]; }
					std::copy(pp.begin(), pp.end(), tile(tk.slot_t)); w.insert({0,tk.slot_t});
				}
			}
			tr.push_back(r); tw.push_back(w);
		}
		for (size_t a = 0; a < tw.size(); a++) for (size_t b = 0; b < tw.size(); b++) if (a != b) for (auto& x : tw[a]) if (tr[b].count(x) || tw[b].count(x)) { printf("RACE level %d task %zu writes (%d,%d) touched by task %zu\n", l, a, x.first, x.second, b); return 1; }
	}
	// every diagonal factor's inverse, formed after the last factor launch (k_corner_invert)
	for (int J = 0; J < T; J++) {
		if (ldiag_launch[J] < 0) { printf("column %d never factored\n", J); return 1; }
		const double* Ld = &ldiag[(size_t)J*TE]; double* Mi = &minv[(size_t)J*TE];
		for (int c = 0; c < TILE; c++) for (int rr = 0; rr < TILE; rr++) { double v = rr == c ? 1.0 : 0.0; for (int k = 0; k < rr; k++) v -= Ld[rr*TILE+k]*Mi[k*TILE+c]; Mi[rr*TILE+c] = v / Ld[rr*TILE+rr]; }
		inv_launch[J] = p.H;
	}
	std::vector<int> done_launch(T, -1);   // launch index in which x_J was produced
	printf("back launches %zu chains %zu\n", p.back_off.size() - 1, p.back_chains.size());
	// the pre-sum lists: per launch exactly its columns with entries outside their chain, each once
	for (int dir = 0; dir < 2; dir++) {
		const auto& off = dir ? p.fwd_off : p.back_off;
		const auto& chains = dir ? p.fwd_chains : p.back_chains;
		const auto& cols = dir ? p.fwd_cols : p.back_cols;
		const auto& pre_off = dir ? p.fwd_pre_off : p.back_pre_off;
		const auto& pre = dir ? p.fwd_pre : p.back_pre;
		if (pre_off.size() != off.size()) { printf("pre-sum launch count mismatch\n"); return 1; }
		for (size_t l = 0; l + 1 < off.size(); l++) {
			std::set<int> want, got;
			for (int q = off[l]; q < off[l + 1]; q++)
				for (int k = 0; k < chains[q].y; k++)
					if (cols[chains[q].x + k].w > 0) want.insert(chains[q].x + k);
			for (int q = pre_off[l]; q < pre_off[l + 1]; q++) {
				if (pre[q].y != 1 || !got.insert(pre[q].x).second) { printf("pre-sum list malformed\n"); return 1; }
			}
			if (want != got) { printf("pre-sum list of launch %zu (%s) differs from its outside-entry columns\n", l, dir ? "fwd" : "back"); return 1; }
		}
	}
	for (size_t l = 0; l + 1 < p.back_off.size(); l++) {
		for (int q = p.back_off[l]; q < p.back_off[l+1]; q++) {
			int2 chn = p.back_chains[q];
			std::set<int> mine;
			for (int k = 0; k < chn.y; k++) {
				int4 c = p.back_cols[chn.x + k]; int J = c.x;
				std::vector<double> z(TILE); for (int i=0;i<TILE;i++) z[i] = cb[J*TILE+i];
				for (int e=0;e<c.z;e++){ int2 en = p.back_ent[c.y+e];
					bool ok = (done_launch[en.y] >= 0 && done_launch[en.y] < (int)l) || mine.count(en.y);
					if (!ok) { printf("BACK ORDER violation: column %d needs x_%d\n", J, en.y); return 1; }
					// pre-sum split: the first c.w entries are read by the launch's pre-sum pass (earlier launches only),
					// the rest by the chain (its own earlier columns only)
					if ((e < c.w) != !mine.count(en.y)) { printf("BACK split violation: column %d entry %d (x_%d)\n", J, e, en.y); return 1; }
					const double* L = tile(en.x); for (int r=0;r<TILE;r++) for (int cc=0;cc<TILE;cc++) z[cc] -= L[r*TILE+cc]*xp[en.y*TILE+r]; }
				const double* Ld = &ldiag[(size_t)J*TE];
				{   // x_J = M^T z with the inverse formed after the factor launches
					if (inv_launch[J] < 0) { printf("BACK uses an inverse never formed: column %d\n", J); return 1; }
					const double* Mi = &minv[(size_t)J*TE];
					for (int i=0;i<TILE;i++){ double v = 0; for (int r2=0;r2<TILE;r2++) v += Mi[r2*TILE+i]*z[r2]; xp[J*TILE+i] = v; }
					(void)Ld;
				}
				for (int i=0;i<TILE;i++){ int rn = p.row_node[J*TILE+i]; if (rn>=0) xout[6*(rn>>3)+(rn&7)] = xp[J*TILE+i]; }
				mine.insert(J);
			}
			for (int J : mine) done_launch[J] = (int)l;
		}
	}
	for (int J = 0; J < T; J++) if (done_launch[J] < 0) { printf("column %d never solved\n", J); return 1; }
	// residual vs natural-order M
	double res = 0, bmax = 0;
	for (int i=0;i<m;i++){ double s = -bnat[i]; for (int j=0;j<m;j++) s += M[(size_t)i*m+j]*xout[j]; res = std::max(res, fabs(s)); bmax = std::max(bmax, fabs(bnat[i])); }
	printf("residual %.3g (|b| %.3g)\n", res, bmax);
	if (!(res < 1e-9 * bmax)) return 1;
	// refinement's corner solve with the same factor: forward chains (y of every row entry's column produced by an earlier
	// launch or earlier in the chain), then the back chains again; residual of a second right-hand side
	std::vector<double> b2(m); for (auto& v : b2) v = nd(rng);
	std::vector<double> yb(p.ld, 0.0);
	for (int R = 0; R < p.ld; R++) { int rn = p.row_node[R]; yb[R] = rn >= 0 ? b2[6*(rn>>3)+(rn&7)] : 0.0; }
	std::vector<int> fdone(T, -1);
	for (size_t l = 0; l + 1 < p.fwd_off.size(); l++) {
		for (int q = p.fwd_off[l]; q < p.fwd_off[l+1]; q++) {
			int2 chn = p.fwd_chains[q]; std::set<int> mine;
			for (int k = 0; k < chn.y; k++) {
				int4 c = p.fwd_cols[chn.x + k]; int J = c.x;
				std::vector<double> z(TILE); for (int i=0;i<TILE;i++) z[i] = yb[J*TILE+i];
				for (int e = 0; e < c.z; e++) { int2 en = p.fwd_ent[c.y+e];
					bool ok = (fdone[en.y] >= 0 && fdone[en.y] < (int)l) || mine.count(en.y);
					if (!ok) { printf("FWD ORDER violation: column %d needs y_%d\n", J, en.y); return 1; }
					if ((e < c.w) != !mine.count(en.y)) { printf("FWD split violation: column %d entry %d (y_%d)\n", J, e, en.y); return 1; }
					if (p.slot_ij[en.x].x != J || p.slot_ij[en.x].y != en.y) { printf("FWD entry mismatch\n"); return 1; }
					const double* L = tile(en.x); for (int r=0;r<TILE;r++) for (int cc=0;cc<TILE;cc++) z[r] -= L[r*TILE+cc]*yb[en.y*TILE+cc]; }
				const double* Ld = &ldiag[(size_t)J*TE];
				{ if (inv_launch[J] < 0) { printf("FWD uses an inverse never formed\n"); return 1; }
					const double* Mi = &minv[(size_t)J*TE]; for (int r=0;r<TILE;r++){ double v=0; for(int cc=0;cc<TILE;cc++) v += Mi[r*TILE+cc]*z[cc]; yb[J*TILE+r]=v; } (void)Ld; }
				mine.insert(J);
			}
			for (int J : mine) fdone[J] = (int)l;
		}
	}
	for (int J = 0; J < T; J++) if (fdone[J] < 0) { printf("forward: column %d never solved\n", J); return 1; }
	std::vector<double> xp2(p.ld, 0.0), x2(m, 0.0);
	for (size_t l = 0; l + 1 < p.back_off.size(); l++)
		for (int q = p.back_off[l]; q < p.back_off[l+1]; q++) {
			int2 chn = p.back_chains[q];
			for (int k = 0; k < chn.y; k++) {
				int4 c = p.back_cols[chn.x + k]; int J = c.x;
				std::vector<double> z(TILE); for (int i=0;i<TILE;i++) z[i] = yb[J*TILE+i];
				for (int e=0;e<c.z;e++){ int2 en = p.back_ent[c.y+e]; const double* L = tile(en.x); for (int r=0;r<TILE;r++) for (int cc=0;cc<TILE;cc++) z[cc] -= L[r*TILE+cc]*xp2[en.y*TILE+r]; }
				const double* Ld = &ldiag[(size_t)J*TE];
				for (int i=TILE-1;i>=0;i--){ double v = z[i]; for (int k2=i+1;k2<TILE;k2++) v -= Ld[k2*TILE+i]*xp2[J*TILE+k2]; xp2[J*TILE+i] = v/Ld[i*TILE+i]; }
				for (int i=0;i<TILE;i++){ int rn = p.row_node[J*TILE+i]; if (rn>=0) x2[6*(rn>>3)+(rn&7)] = xp2[J*TILE+i]; }
			}
		}
	double res2 = 0, b2max = 0;
	for (int i=0;i<m;i++){ double s2 = -b2[i]; for (int j=0;j<m;j++) s2 += M[(size_t)i*m+j]*x2[j]; res2 = std::max(res2, fabs(s2)); b2max = std::max(b2max, fabs(b2[i])); }
	printf("refinement-solve residual %.3g (|b| %.3g)\n", res2, b2max);
	if (!(res2 < 1e-9 * b2max)) return 1;
	// the dataflow launch (k_corner_flow): the refinement's tickets run [rhs of every column] [forward chains c = nB-1 .. 0]
	// [back chains c = 0 .. nB-1] (after the solve's back chains and stem pass); every wait must be on a lower ticket
	// (deadlock freedom), the counters a chain waits for must be complete exactly when everything it reads is, and
	// executing the roles in ticket order must solve the system
	{
		const int nB = (int)p.flow_chains.size();
		if (nB != (int)p.back_chains.size() || (int)p.flow_need.size() != nB || (int)p.col_chain.size() != T) { printf("FLOW plan size mismatch\n"); return 1; }
		std::vector<int> kids(nB, 0), ncols_of(nB, 0);
		for (int c = 0; c < nB; c++) {
			const int4 f = p.flow_chains[c];
			if (f.x != p.back_chains[c].x || f.y != p.back_chains[c].y) { printf("FLOW chain %d back columns mismatch\n", c); return 1; }
			if (f.w >= c) { printf("FLOW chain %d waits on chain %d (not a lower back ticket)\n", c, f.w); return 1; }
			if (f.w >= 0) kids[f.w]++;
			for (int k = 0; k < f.y; k++) {
				if (p.back_cols[f.x + k].x != p.fwd_cols[f.z + f.y - 1 - k].x) { printf("FLOW chain %d forward columns mismatch\n", c); return 1; }
				if (p.col_chain[p.back_cols[f.x + k].x] != c) { printf("FLOW column chain map wrong\n"); return 1; }
			}
		}
		for (int J = 0; J < T; J++) ncols_of[p.col_chain[J]]++;
		for (int c = 0; c < nB; c++)
			if (p.flow_need[c] != ncols_of[c] + kids[c]) { printf("FLOW chain %d need %d != columns %d + children %d\n", c, p.flow_need[c], ncols_of[c], kids[c]); return 1; }
		std::vector<double> yf(p.ld, 0.0), xf(p.ld, 0.0), xnat(m, 0.0);
		std::vector<int> cnt(nB, 0), fdone_c(nB, 0), bdone_c(nB, 0);
		std::vector<char> ycol(T, 0), xcol(T, 0), rhs_col(T, 0);
		for (int J = 0; J < T; J++) {   // rhs workers
			for (int i = 0; i < TILE; i++) { int rn = p.row_node[J*TILE+i]; yf[J*TILE+i] = rn >= 0 ? b2[6*(rn>>3)+(rn&7)] : 0.0; }
			rhs_col[J] = 1;
			cnt[p.col_chain[J]]++;
		}
		for (int c = nB - 1; c >= 0; c--) {   // forward chains, deepest first
			const int4 f = p.flow_chains[c];
			if (cnt[c] != p.flow_need[c]) { printf("FLOW forward chain %d would wait forever (%d of %d)\n", c, cnt[c], p.flow_need[c]); return 1; }
			for (int k = 0; k < f.y; k++) {
				int4 col = p.fwd_cols[f.z + k]; int J = col.x;
				if (!rhs_col[J]) { printf("FLOW forward reads an unwritten rhs\n"); return 1; }
				std::vector<double> z(TILE); for (int i=0;i<TILE;i++) z[i] = yf[J*TILE+i];
				for (int e = 0; e < col.z; e++) { int2 en = p.fwd_ent[col.y+e];
					if (!ycol[en.y]) { printf("FLOW forward column %d reads y_%d before it is final\n", J, en.y); return 1; }
					const double* L = tile(en.x); for (int r=0;r<TILE;r++) for (int cc=0;cc<TILE;cc++) z[r] -= L[r*TILE+cc]*yf[en.y*TILE+cc]; }
				const double* Mi = &minv[(size_t)J*TE]; for (int r=0;r<TILE;r++){ double v=0; for(int cc=0;cc<TILE;cc++) v += Mi[r*TILE+cc]*z[cc]; yf[J*TILE+r]=v; }
				ycol[J] = 1;
			}
			if (f.w >= 0) cnt[f.w]++; else fdone_c[c] = 1;
		}
		int btotal = 0;
		for (int c = 0; c < nB; c++) {   // back chains, root first
			const int4 f = p.flow_chains[c];
			if (f.w >= 0 ? !bdone_c[f.w] : !fdone_c[c]) { printf("FLOW back chain %d would wait forever\n", c); return 1; }
			for (int k = 0; k < f.y; k++) {
				int4 col = p.back_cols[f.x + k]; int J = col.x;
				if (!ycol[J]) { printf("FLOW back column %d before its y\n", J); return 1; }
				std::vector<double> z(TILE); for (int i=0;i<TILE;i++) z[i] = yf[J*TILE+i];
				for (int e=0;e<col.z;e++){ int2 en = p.back_ent[col.y+e];
					if (!xcol[en.y]) { printf("FLOW back column %d reads x_%d before it is final\n", J, en.y); return 1; }
					const double* L = tile(en.x); for (int r=0;r<TILE;r++) for (int cc=0;cc<TILE;cc++) z[cc] -= L[r*TILE+cc]*xf[en.y*TILE+r]; }
				const double* Mi = &minv[(size_t)J*TE];
				for (int i=0;i<TILE;i++){ double v = 0; for (int r2=0;r2<TILE;r2++) v += Mi[r2*TILE+i]*z[r2]; xf[J*TILE+i] = v; }
				for (int i=0;i<TILE;i++){ int rn = p.row_node[J*TILE+i]; if (rn>=0) xnat[6*(rn>>3)+(rn&7)] = xf[J*TILE+i]; }
				xcol[J] = 1;
			}
			bdone_c[c] = 1;
			btotal++;
		}
		if (btotal != nB) { printf("FLOW stem workers would wait forever\n"); return 1; }
		double res4 = 0;
		for (int i=0;i<m;i++){ double s4 = -b2[i]; for (int j=0;j<m;j++) s4 += M[(size_t)i*m+j]*xnat[j]; res4 = std::max(res4, fabs(s4)); }
		printf("flow-solve residual %.3g\n", res4);
		if (!(res4 < 1e-9 * b2max)) return 1;
	}
	// single-workgroup walk streams (k_corner_walk): forward then back over b2 in stream order; every entry's vector
	// segment must be final when read (forward: column k < J solved; back: column I > J solved), every head's tile formed
	{
		std::vector<double> xw(p.ld, 0.0);
		for (int R = 0; R < p.ld; R++) { int rn = p.row_node[R]; xw[R] = rn >= 0 ? b2[6*(rn>>3)+(rn&7)] : 0.0; }
		for (int dir = 0; dir < 2; dir++) {
			const auto& st = dir == 0 ? p.walk_fwd : p.walk_back;
			std::vector<char> solved(T, 0);
			std::vector<double> acc(TILE, 0.0);
			for (const int4& e : st) {
				const double* tl = e.x == 0 ? tile(e.y) : e.x == 1 ? &minv[(size_t)e.y*TE] : &ldiag[(size_t)e.y*TE];
				if (e.w < 0) {
					const int K = e.z / TILE;
					if (!solved[K]) { printf("WALK reads an unsolved segment %d\n", K); return 1; }
					for (int r = 0; r < TILE; r++) for (int c = 0; c < TILE; c++) {
						if (dir == 0) acc[r] += tl[r*TILE+c]*xw[e.z+c]; else acc[c] += tl[r*TILE+c]*xw[e.z+r]; }
					continue;
				}
				const int J = e.y;
				if (e.x == 1 && inv_launch[J] < 0) { printf("WALK head inverse never formed: %d\n", J); return 1; }
				std::vector<double> z(TILE); for (int i=0;i<TILE;i++) z[i] = xw[J*TILE+i] - acc[i];
				if (e.x == 1) { for (int i=0;i<TILE;i++){ double v=0; for (int k=0;k<TILE;k++) v += (dir==0 ? tl[i*TILE+k] : tl[k*TILE+i]) * z[k]; xw[J*TILE+i] = v; } }
				else if (dir == 0) { for (int i=0;i<TILE;i++){ double v=z[i]; for (int k=0;k<i;k++) v -= tl[i*TILE+k]*xw[J*TILE+k]; xw[J*TILE+i] = v/tl[i*TILE+i]; } }
				else { for (int i=TILE-1;i>=0;i--){ double v=z[i]; for (int k=i+1;k<TILE;k++) v -= tl[k*TILE+i]*xw[J*TILE+k]; xw[J*TILE+i] = v/tl[i*TILE+i]; } }
				solved[J] = 1;
				std::fill(acc.begin(), acc.end(), 0.0);
			}
			for (int J = 0; J < T; J++) if (!solved[J]) { printf("WALK never solved column %d\n", J); return 1; }
		}
		std::vector<double> xw_nat(m, 0.0);
		for (int R = 0; R < p.ld; R++) { int rn = p.row_node[R]; if (rn >= 0) xw_nat[6*(rn>>3)+(rn&7)] = xw[R]; }
		double res3 = 0;
		for (int i=0;i<m;i++){ double s3 = -b2[i]; for (int j=0;j<m;j++) s3 += M[(size_t)i*m+j]*xw_nat[j]; res3 = std::max(res3, fabs(s3)); }
		printf("walk-solve residual %.3g\n", res3);
		if (!(res3 < 1e-9 * b2max)) return 1;
	}
	return 0;
}
