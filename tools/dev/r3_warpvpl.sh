# development: warp quads with load / gather / compute phases, two vertices per quad from 1M vertices -- parity suite,
# (the product code does not carry the experiment: tools/dev/r3_warpvpl.patch holds it)
# full suite, then C2 and C3 A/B (variants: csrc/variants/libnnrt_v0.so = previous warp, v1 = this one, v2 = two vertices per quad at every size)
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3/suite_warpvpl.log 2>&1 || { tail -30 gpurun_out/r3/suite_warpvpl.log; exit 1; }
tail -2 gpurun_out/r3/suite_warpvpl.log
VS="0 1 2" bash tools/dev/r3_ab3.sh || exit 1
mv gpurun_out/ab gpurun_out/ab_c2
VS="0 1 2" BENCH_ARGS="--config C3" bash tools/dev/r3_ab3.sh || exit 1
mv gpurun_out/ab gpurun_out/ab_c3
grep -h '^{' gpurun_out/ab_c2/b*_*.log gpurun_out/ab_c3/b*_*.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print(d['config']['config'], round(d['value'],1))"
