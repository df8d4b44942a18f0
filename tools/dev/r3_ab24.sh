set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3/suite24.log 2>&1 || { tail -30 gpurun_out/r3/suite24.log; exit 1; }
tail -2 gpurun_out/r3/suite24.log
VS="0 1" bash tools/dev/r3_ab3.sh || exit 1
mv gpurun_out/ab gpurun_out/ab_c2
VS="0 1" BENCH_ARGS="--config C3" bash tools/dev/r3_ab3.sh || exit 1
mv gpurun_out/ab gpurun_out/ab_c3
grep -h '^{' gpurun_out/ab_c2/b*_*.log gpurun_out/ab_c3/b*_*.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print(d['config']['config'], round(d['value'],1))"
