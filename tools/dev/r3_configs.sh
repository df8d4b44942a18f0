# round-3: bench lines for the other BASELINE configs (CPU baselines included) and the published-point comparisons
set -u
mkdir -p gpurun_out/r3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for cfg in ${CFGS:-C1 C1_ARAP C3}; do
  echo "== $cfg"
  timeout -k 10 420 python3 -u bench.py --config $cfg --steps 200 --warmup 20 --timed-steps 40 --cpu-seconds 10 > gpurun_out/r3/bench_$cfg.log 2>&1; rc=$?
  echo "== $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
  grep '^{' gpurun_out/r3/bench_$cfg.log > gpurun_out/r3/bench_$cfg.json
done
echo "== published"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3/prof_published -o run -- python3 tools/bench_published.py > gpurun_out/r3/published.log 2>&1; rc=$?
echo "== published rc=$rc"; [ $rc -eq 0 ] || exit $rc
grep '^{' gpurun_out/r3/published.log > gpurun_out/r3/published.jsonl
echo done
