#!/bin/bash
# round-3: full GPU suite, then the C5 bench line + kernel trace; outputs under gpurun_out/r3/
set -u
mkdir -p gpurun_out/r3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/r3/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 3 "gpurun_out/r3/$name.log"; return $rc; }
step suite 900 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread || exit 1
step bench_C5 420 python3 -u bench.py --config C5 --steps 200 --warmup 20 --timed-steps 40 --cpu-seconds 10 || exit 1
grep '^{' gpurun_out/r3/bench_C5.log > gpurun_out/r3/bench_C5.json
step prof_c5 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3/prof_c5 -o run -- python3 bench.py --config C5 --steps 60 --warmup 10 --timed-steps 20 --no-cpu-baseline || exit 1
echo done
