#!/bin/bash
# bench's N > 1 leg with real fitters on a one-GPU box: 2 ranks sharing the GPU, collectives on gloo
set -u
mkdir -p gpurun_out/dist
export NNRT_BENCH_BACKEND=gloo
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 100 --warmup 20 --no-cpu-baseline --timed-steps 5 > gpurun_out/dist/n2.log 2>&1; rc=$?
echo "rc=$rc"; grep '^{' gpurun_out/dist/n2.log | cut -c1-2000; tail -3 gpurun_out/dist/n2.log | cut -c1-300
