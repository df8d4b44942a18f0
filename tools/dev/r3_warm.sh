#!/bin/bash
set -u
mkdir -p gpurun_out/st
for w in 0 10 50 200 1000; do
  timeout -k 10 200 python3 -u bench.py --steps 20 --warmup $w --no-cpu-baseline --timed-steps 5 > gpurun_out/st/w${w}.log 2>&1 || exit 1
  python3 -c "import json,sys; d=[json.loads(l) for l in open('gpurun_out/st/w${w}.log') if l.startswith('{')][-1]; print('warmup $w', round(d['value']), d['ms_per_step'])"
done
