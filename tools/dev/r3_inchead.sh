# development: k_arrow_prepare reads each node's first 32 edge incidences from a fixed-stride copy (no offset load first)
# (the product code does not carry the experiment: tools/dev/r3_inchead.patch holds it)
# -- full suite, then C5 and C1_ARAP A/B (variants: csrc/variants/libnnrt_v0.so = CSR only, v1 = this one)
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
timeout -k 10 700 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3/suite_inchead.log 2>&1 || { tail -30 gpurun_out/r3/suite_inchead.log; exit 1; }
tail -2 gpurun_out/r3/suite_inchead.log
VS="0 1" BENCH_ARGS="--config C5" bash tools/dev/r3_ab3.sh || exit 1
mv gpurun_out/ab gpurun_out/ab_c5
VS="0 1" BENCH_ARGS="--config C1_ARAP" bash tools/dev/r3_ab3.sh || exit 1
mv gpurun_out/ab gpurun_out/ab_c1a
grep -h '^{' gpurun_out/ab_c5/b*_*.log gpurun_out/ab_c1a/b*_*.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print(d['config']['config'], round(d['value'],1))"
