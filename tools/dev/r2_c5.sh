# round-2: C5 bench line (with CPU baseline) and its kernel trace
set -u
mkdir -p gpurun_out/r2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 420 python3 -u bench.py --config C5 --steps 200 --warmup 20 --timed-steps 40 --cpu-seconds 10 > gpurun_out/r2/bench_C5.log 2>&1 || exit 1
grep '^{' gpurun_out/r2/bench_C5.log > gpurun_out/r2/bench_C5.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2/prof_c5 -o run -- python3 bench.py --config C5 --steps 60 --warmup 10 --timed-steps 20 --no-cpu-baseline > gpurun_out/r2/prof_c5.log 2>&1 || exit 1
echo done
