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
		variants) step variants 900 python -u tools/fit_variants.py C2; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
		probe) step probe 120 tools/dev/permlane_probe; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
		vprof) for v in ${VPROF:-40}; do export NNRT_LIB_PATH=$PWD/dynamicfuion_python_amd/csrc/variants/libnnrt_v$v.so; step vprof_$v 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vprof_$v -o run -- python3 tools/fit_variants.py --child C2 100; rc=$?; unset NNRT_LIB_PATH; [ $rc -eq 0 ] || exit $rc; done ;;
		stamps) step stamps 300 python -u tools/stamps_report.py; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
		cholstamps) step cholstamps 300 python -u tools/chol_stamps.py C5; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
		mfma64) step mfma64 120 tools/dev/mfma64_probe; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
		vtests) for v in ${VTESTS:-9}; do export NNRT_LIB_PATH=$PWD/dynamicfuion_python_amd/csrc/variants/libnnrt_v$v.so; step vtest_$v 600 python -u -m pytest tests/test_gpu_parity.py -q -k "fit_one_iteration or single_mode or arap or tukey" -p no:cacheprovider; rc=$?; unset NNRT_LIB_PATH; fatal $rc && exit $rc; done ;;
		vsq) PMC=${PMC:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"}; for v in ${VSQ:-50}; do i=0; for pm in $(echo "$PMC" | tr ';' ' ' | sed 's/,/ /g' | xargs -n 8 | tr ' ' ','); do i=$((i+1)); if [ "$v" = "0" ]; then unset NNRT_LIB_PATH; else export NNRT_LIB_PATH=$PWD/dynamicfuion_python_amd/csrc/variants/libnnrt_v$v.so; fi; step vsq_${v}_$i 600 rocprofv3 --pmc $(echo $pm | tr ',' ' ') --output-format csv -d gpurun_out/vsq_${v}_$i -o run -- python3 tools/fit_variants.py --child C2 20; rc=$?; unset NNRT_LIB_PATH; [ $rc -eq 0 ] || exit $rc; done; done ;;
		sq) step pmc_sq 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pmc_sq -o run -- python3 bench.py --steps 20 --warmup 5 --timed-steps 20 --no-cpu-baseline; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
		pmc) step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 20 --warmup 5 --timed-steps 20 --no-cpu-baseline; rc=$?; [ $rc -eq 0 ] || exit $rc
		     step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 20 --warmup 5 --timed-steps 20 --no-cpu-baseline; rc=$?; [ $rc -eq 0 ] || exit $rc ;;
	esac
done
exit 0
