#!/bin/bash
# GPU-box check used during development: smoke -> parity tests -> bench -> kernel-trace profile.
# Every GPU step runs under its own time limit; a crash/abort/timeout ends the script (no retries).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
STAGES=${STAGES:-"smoke tests bench prof"}
step() {   # name seconds cmd...
	local name=$1 t=$2
	shift 2
	echo "== $name (limit ${t}s)"
	timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
	local rc=$?
	echo "== $name rc=$rc"
	tail -n 5 "gpurun_out/$name.log"
	return $rc
}
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }   # 1 = ordinary test/assert failure; anything else stops the script
for s in $STAGES; do
	case $s in
		smoke) step smoke 400 python -u -c "import __graft_entry__ as g; g.smoke()"; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
		tests) step gpu_tests 900 python -u -m pytest tests -m gpu -q --maxfail=20 -p no:cacheprovider; rc=$?; fatal $rc && exit $rc ;;
		bench) step bench 600 python -u bench.py; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
		prof) step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o r01 -- python3 bench.py --steps 300 --warmup 30 --timed-steps 100 --no-cpu-baseline; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
	esac
done
exit 0
