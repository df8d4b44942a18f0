#!/bin/bash
# round-6 PMC traffic for the results table's remaining lines (C1, C1_ARAP, the C2_ARAP frame, 8 C2 replicas), copied
# into profiles/ on the box so the bench lines that follow read them; then those bench lines (tools/bench_lines.sh).
# Every GPU step has its own limit (tools/measure.sh); the first failure ends the script.
set -u
export TAG=${TAG:-r06p}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARAPK="k_fit_pixels_fused k_raster_scatter_mesh k_warp_mesh_quad|k_warp_mesh_vertex k_arrow_prepare k_init_stem k_stem_schur_rhs k_corner_factor k_corner_flow"
run() {   # name config kernels bench-args
	KERNELS="$3" CONFIG=$2 STAGES=pmc BENCH_ARGS="$4" bash tools/measure.sh || exit 1
	cp gpurun_out/$TAG/pmc_traffic_$2.json profiles/r06_pmc_traffic_$1.json || exit 1
}
run c1 C1 "" ""
run c1_arap C1_ARAP "$ARAPK" ""
run c2_arap_frame C2_ARAP "$ARAPK" "--step frame --graph-steps 6"
run c2_replicas8 C2 "" "--replicas 8"
LINES="c1 c1_arap c2_arap_frame replicas8" bash tools/bench_lines.sh || exit 1
