# round-3 final lines for the other configs: C5, C1_ARAP, C1 (CPU baselines), C3 (GPU only), the C5 kernel trace and
# the reference's published points; outputs under gpurun_out/r3/
set -u
mkdir -p gpurun_out/r3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/r3/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 1 "gpurun_out/r3/$name.log" | cut -c1-200; return $rc; }
for cfg in C5 C1_ARAP C1; do
  step bench_$cfg 420 python3 -u bench.py --config $cfg --steps 200 --warmup 20 --timed-steps 40 --cpu-seconds 10 || exit 1
  grep '^{' gpurun_out/r3/bench_$cfg.log > gpurun_out/r3/bench_$cfg.json
done
step bench_C3 300 python3 -u bench.py --config C3 --steps 200 --warmup 20 --timed-steps 40 --no-cpu-baseline || exit 1
grep '^{' gpurun_out/r3/bench_C3.log > gpurun_out/r3/bench_C3.json
step prof_c5 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3/prof_c5 -o run -- python3 bench.py --config C5 --steps 60 --warmup 10 --timed-steps 20 --no-cpu-baseline || exit 1
step published 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3/prof_published -o run -- python3 tools/bench_published.py || exit 1
grep '^{' gpurun_out/r3/published.log > gpurun_out/r3/published.jsonl
echo done
