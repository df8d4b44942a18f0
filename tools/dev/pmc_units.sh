#!/bin/bash
# Memory-unit PMC passes over a short C2 bench (development): TA busy, TCP stalls, SQ memory-instruction cycles; one
# pass per counter group (rocprofv3 does not split passes), summaries per kernel in gpurun_out/units/summary.txt
set -u
mkdir -p gpurun_out/units
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
CFG=${CONFIG:-C2}
pass() {
	local name=$1; shift
	timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d gpurun_out/units/$name -o run -- python3 bench.py --config $CFG --steps 20 --warmup 5 --kernel-trials 1 --timed-steps 5 --no-cpu-baseline > gpurun_out/units/$name.log 2>&1 || { echo "pass $name failed"; tail -3 gpurun_out/units/$name.log; exit 1; }
}
pass ta TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE GRBM_COUNT
pass tcp TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_GATE_EN2_sum
pass sqm SQ_WAVES SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU
python3 tools/pmc_summary.py "gpurun_out/units/**/*counter_collection.csv" > gpurun_out/units/summary.txt
cat gpurun_out/units/summary.txt
