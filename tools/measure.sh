#!/bin/bash
# Measurement pass (C2 unless CONFIG is set): bench line with CPU baseline, kernel trace (rocprofv3 --kernel-trace
# --stats), PMC traffic (separate FETCH_SIZE / WRITE_SIZE passes), SQ counters; outputs under gpurun_out/$TAG/.
# Every GPU step has its own time limit; any failure ends the script (no retries).
#   TAG=r04 CONFIG=C2 tools/measure.sh
set -u
TAG=${TAG:-r05}
CONFIG=${CONFIG:-C2}
STAGES=${STAGES:-"bench prof pmc sq"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "$OUT/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 2 "$OUT/$name.log" | cut -c1-300; return $rc; }
B="python3 bench.py --config $CONFIG ${BENCH_ARGS:-}"   # (BENCH_ARGS: e.g. --step frame --graph-steps 10)
for s in $STAGES; do
	case $s in
		bench) step bench_$CONFIG 400 python3 -u bench.py --config $CONFIG ${BENCH_ARGS:-} || exit 1
		       grep '^{' $OUT/bench_$CONFIG.log > $OUT/bench_$CONFIG.json ;;
		prof) step prof_$CONFIG 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$CONFIG -o run -- $B --steps 300 --warmup 30 --no-cpu-baseline || exit 1 ;;
		pmc) step pmc_fetch_$CONFIG 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch_$CONFIG -o run -- $B --steps 20 --warmup 5 --kernel-trials 1 --no-cpu-baseline || exit 1
		     step pmc_write_$CONFIG 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write_$CONFIG -o run -- $B --steps 20 --warmup 5 --kernel-trials 1 --no-cpu-baseline || exit 1
		     W=$(grep -h '^{' $OUT/pmc_fetch_$CONFIG.log | tail -n 1 | python3 -c "import json,sys;print(json.loads(sys.stdin.read())['config']['workload'])")
		     python3 tools/pmc_traffic.py --fetch "$OUT/pmc_fetch_$CONFIG/**/*counter_collection.csv" --write "$OUT/pmc_write_$CONFIG/**/*counter_collection.csv" --workload "$W" ${KERNELS:+--kernels $KERNELS} --out $OUT/pmc_traffic_$CONFIG.json > /dev/null || exit 1 ;;
		sq) step pmc_sq_$CONFIG 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/pmc_sq_$CONFIG -o run -- $B --steps 20 --warmup 5 --kernel-trials 1 --no-cpu-baseline || exit 1
		    f=$(find $OUT/pmc_sq_$CONFIG -name "*counter_collection.csv" | head -1)
		    python3 tools/sq_summary.py "$f" ${SQ_KERNELS:-k_fit_pixels_fused k_raster_scatter_mesh k_warp_mesh k_solve_update} > $OUT/sq_summary_$CONFIG.txt 2>&1 || exit 1 ;;
	esac
done
echo done
