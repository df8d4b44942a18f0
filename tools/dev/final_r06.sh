#!/bin/bash
# round-6 final measurement pass on the GPU box: kernel traces + PMC traffic for C2 / C3 / C5 (copied into profiles/ on
# the box so the bench lines read them), SQ counters at C2, then every results-table bench line and smoke().
# Every GPU step has its own limit (tools/measure.sh, tools/bench_lines.sh); the first failure ends the script.
set -u
export TAG=${TAG:-r06f}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in ${PMC_CONFIGS-C2 C3 C5}; do
	K=""; [ $cfg = C5 ] && K="k_fit_pixels_fused k_raster_scatter_mesh k_warp_mesh_quad|k_warp_mesh_vertex k_arrow_prepare k_init_stem k_stem_schur_rhs k_corner_factor k_corner_flow"
	KERNELS="$K" CONFIG=$cfg STAGES="prof pmc" bash tools/measure.sh || exit 1
	lc=$(echo $cfg | tr 'A-Z' 'a-z')
	cp gpurun_out/$TAG/pmc_traffic_$cfg.json profiles/r06_pmc_traffic_$lc.json || exit 1
done
CONFIG=C2 STAGES=sq bash tools/measure.sh || exit 1
LINES="${LINES:-c2 c5 c3 c1 c1_arap c2_arap_frame replicas8}" bash tools/bench_lines.sh || exit 1
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1 || { tail -5 gpurun_out/$TAG/smoke.log; exit 1; }
tail -1 gpurun_out/$TAG/smoke.log
