#!/bin/bash
# GPU-box check used during development: smoke -> parity tests -> bench -> kernel-trace profile.
# Every GPU step runs under its own time limit; a crash/abort/timeout ends the script (no retries).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
STAGES=${STAGES:-"smoke tests bench prof pmc"}
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
		prof) step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 300 --warmup 30 --timed-steps 100 --no-cpu-baseline; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
		sq) step pmc_sq 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pmc_sq -o run -- python3 bench.py --steps 20 --warmup 5 --timed-steps 20 --no-cpu-baseline; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
		pmc) step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 20 --warmup 5 --timed-steps 20 --no-cpu-baseline; rc=$?; [ $rc -eq 0 ] || exit $rc
		     step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 20 --warmup 5 --timed-steps 20 --no-cpu-baseline; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
	esac
done
exit 0
