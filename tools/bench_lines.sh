#!/bin/bash
# Bench lines of the round's results table, each with its CPU baseline unless noted; one JSON
# line per workload in gpurun_out/$TAG/line_<name>.json. Every GPU step has its own time limit; a failure ends the script.
#   TAG=r04 LINES="c5 c3 c1 c1_arap c2_arap_frame replicas8" tools/bench_lines.sh
set -u
TAG=${TAG:-r04}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
line() {
	local name=$1 t=$2; shift 2
	echo "== $name"
	timeout -k 10 "$t" python3 -u bench.py "$@" > "$OUT/line_$name.log" 2>&1
	local rc=$?
	echo "== $name rc=$rc"
	[ $rc -eq 0 ] || { tail -n 5 "$OUT/line_$name.log"; return $rc; }
	grep '^{' "$OUT/line_$name.log" | tail -n 1 > "$OUT/line_$name.json"
	cut -c1-300 "$OUT/line_$name.json"
}
for l in ${LINES:-c5 c3 c1 c1_arap c2_arap_frame replicas8}; do
	case $l in
		c2) line c2 400 --config C2 || exit 1 ;;
		c5) line c5 400 --config C5 || exit 1 ;;
		c3) line c3 400 --config C3 --cpu-share-only --cpu-no-warm --cpu-seconds 1 || exit 1 ;;
		c1) line c1 400 --config C1 || exit 1 ;;
		c1_arap) line c1_arap 400 --config C1_ARAP || exit 1 ;;
		c2_arap_frame) line c2_arap_frame 400 --config C2_ARAP --step frame --graph-steps 6 || exit 1 ;;
		replicas8) line replicas8 300 --config C2 --replicas 8 --no-cpu-baseline || exit 1 ;;
	esac
done
echo done
