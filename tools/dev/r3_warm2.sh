#!/bin/bash
set -u
mkdir -p gpurun_out/st
for w in 0 10; do
  timeout -k 10 200 python3 -u bench.py --steps 20 --warmup $w --no-cpu-baseline --timed-steps 5 > gpurun_out/st/v${w}.log 2>&1 || exit 1
  python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/st/v${w}.log') if l.startswith('{')][-1]; print('warmup $w', round(d['value']), d['ms_per_step'])"
done
timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --config C5 --no-cpu-baseline --timed-steps 5 > gpurun_out/st/c5.log 2>&1 || exit 1
python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/st/c5.log') if l.startswith('{')][-1]; print('C5 steps 20', round(d['value']), d['ms_per_step'])"
