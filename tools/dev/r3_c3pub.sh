#!/bin/bash
# round-3: C3 bench line (GPU only: the binned-raster CPU baseline at C3 runs for minutes per iteration) + published points
set -u
mkdir -p gpurun_out/r3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 -u bench.py --config C3 --steps 200 --warmup 20 --timed-steps 40 --no-cpu-baseline > gpurun_out/r3/bench_C3.log 2>&1 || exit 1
grep '^{' gpurun_out/r3/bench_C3.log > gpurun_out/r3/bench_C3.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3/prof_published -o run -- python3 tools/bench_published.py > gpurun_out/r3/published.log 2>&1 || exit 1
grep '^{' gpurun_out/r3/published.log > gpurun_out/r3/published.jsonl
cat gpurun_out/r3/published.jsonl | cut -c1-400
