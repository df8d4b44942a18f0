#!/bin/bash
# round-6: where the one-rank RCCL bench line loses time against the plain line. Four C2 lines at
# the headline step count: plain; under torch.distributed.run without a process group; with a gloo process group; with
# the RCCL process group (NNRT_BENCH_DIST_ONE_RANK=1). Each line's value and its graph-replay iteration time.
set -u
mkdir -p gpurun_out/rccl
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
show() { python3 -c "
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d['value'],1), 'ms/step', round(d['ms_per_step']*1000,2), 'us; graph iteration', round(d['kernel_ms']['iteration']*1000,2), 'us;', d['config'].get('collectives'))
" "$1" "$2"; }
run() { local tag=$1; shift; timeout -k 10 300 "$@" > gpurun_out/rccl/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/rccl/$tag.log; exit 1; }; show gpurun_out/rccl/$tag.log $tag; }
TR="python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533"
for rep in 1 2; do
	run plain_$rep python3 -u bench.py --no-cpu-baseline
	run torchrun_nopg_$rep $TR bench.py --no-cpu-baseline
	run gloo_$rep env NNRT_BENCH_DIST_ONE_RANK=1 NNRT_BENCH_BACKEND=gloo $TR bench.py --no-cpu-baseline
	run rccl_$rep env NNRT_BENCH_DIST_ONE_RANK=1 $TR bench.py --no-cpu-baseline
done
