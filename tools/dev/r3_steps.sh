#!/bin/bash
# bench sensitivity to the driver's short timed region (--steps 20): graph steps per launch
set -u
mkdir -p gpurun_out/st
for g in 10 20 5 2 1; do
  for rep in 1 2; do
    timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 10 --graph-steps $g --no-cpu-baseline --timed-steps 5 > gpurun_out/st/g${g}_$rep.log 2>&1 || exit 1
    python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/st/g${g}_$rep.log') if l.startswith('{')][-1]; print('graph_steps $g rep $rep', round(d['value']), d['ms_per_step'])"
  done
done
timeout -k 10 200 python3 -u bench.py --steps 500 --warmup 50 --graph-steps 1 --no-cpu-baseline --timed-steps 5 > gpurun_out/st/g1_500.log 2>&1 || exit 1
python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/st/g1_500.log') if l.startswith('{')][-1]; print('graph_steps 1 steps 500', round(d['value']), d['ms_per_step'])"
