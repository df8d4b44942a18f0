#!/bin/bash
# round-3: C5 and C1_ARAP lines (CPU baselines included) and the C5 kernel trace, after the ARAP launch fusions
set -u
mkdir -p gpurun_out/r3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in C5 C1_ARAP; do
  timeout -k 10 420 python3 -u bench.py --config $cfg --steps 200 --warmup 20 --timed-steps 40 --cpu-seconds 10 > gpurun_out/r3/bench_$cfg.log 2>&1 || exit 1
  grep '^{' gpurun_out/r3/bench_$cfg.log > gpurun_out/r3/bench_$cfg.json
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3/prof_c5 -o run -- python3 bench.py --config C5 --steps 60 --warmup 10 --timed-steps 20 --no-cpu-baseline > gpurun_out/r3/prof_c5.log 2>&1 || exit 1
echo done
