# development: warp quad rows stored as six 16-B pieces per vertex (K = 4) -- parity suite,
# (the product code does not carry the experiment: tools/dev/r3_rowsf4.patch holds it)
# full suite, then C2 and C3 A/B (variants: csrc/variants/libnnrt_v0.so = float2 row stores, v1 = this one)
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3/suite_rowsf4.log 2>&1 || { tail -30 gpurun_out/r3/suite_rowsf4.log; exit 1; }
tail -2 gpurun_out/r3/suite_rowsf4.log
VS="0 1" bash tools/dev/r3_ab3.sh || exit 1
mv gpurun_out/ab gpurun_out/ab_c2
VS="0 1" BENCH_ARGS="--config C3" bash tools/dev/r3_ab3.sh || exit 1
mv gpurun_out/ab gpurun_out/ab_c3
grep -h '^{' gpurun_out/ab_c2/b*_*.log gpurun_out/ab_c3/b*_*.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print(d['config']['config'], round(d['value'],1))"
