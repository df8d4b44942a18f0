#!/bin/bash
# development: C5 bench (no CPU baseline) for the product and every variant, plus a kernel trace of the product's C5 bench
set -u
mkdir -p gpurun_out/c5
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
CONFIGS=${CONFIGS:-C5} REPS=1 bash tools/dev/ab.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5/prof -o run -- python3 bench.py --config ${CONFIGS%% *} --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/c5/prof.log 2>&1 || { tail -5 gpurun_out/c5/prof.log; exit 1; }
f=$(find gpurun_out/c5/prof -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | head -25
