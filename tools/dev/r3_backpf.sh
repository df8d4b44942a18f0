# development: corner back substitution with staged descriptors / early y and diagonal loads -- suite + C5 A/B
# (variants: csrc/variants/libnnrt_v0.so = previous k_corner_back, v1 = this one)
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3/suite_backpf.log 2>&1 || { tail -30 gpurun_out/r3/suite_backpf.log; exit 1; }
tail -2 gpurun_out/r3/suite_backpf.log
VS="0 1" BENCH_ARGS="--config C5" bash tools/dev/r3_ab3.sh || exit 1
grep -h '^{' gpurun_out/ab/b*_*.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print(d['config']['config'], round(d['value'],1))"
