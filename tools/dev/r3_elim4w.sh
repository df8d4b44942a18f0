# 4-wave column-partitioned corner tile elimination: ARAP GPU tests,
# then kernel-trace A/B at C5 and C1_ARAP (v0 HEAD, v1 change)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_arrowhead.py -m gpu -x -q --timeout 200 --timeout-method thread -k "snapshot or ARAP or arap or arrow or C5 or L4 or layer or corner or block_sparse or cholesky" > gpurun_out/r3/elim4w_tests.log 2>&1 || { tail -30 gpurun_out/r3/elim4w_tests.log; exit 1; }
tail -1 gpurun_out/r3/elim4w_tests.log
for cfg in C5 C1_ARAP; do
  rm -rf gpurun_out/ab
  VS="0 1" BENCH_ARGS="--config $cfg --steps 200 --warmup 20" bash tools/dev/r3_ab3.sh || exit 1
  for f in gpurun_out/ab/b*_*.log; do python3 -c "
import json
d=[json.loads(l) for l in open('$f') if l.startswith('{')][0]
print('$f', d['config']['config'], round(d['value'],1))"; done
  mv gpurun_out/ab gpurun_out/ab_$cfg
done
