# carried node skips the min reduction in grouping: full GPU suite, then kernel-trace A/B at C2 and C3 (v0 HEAD, v1 change)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r3
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3/suite_cy.log 2>&1 || { tail -30 gpurun_out/r3/suite_cy.log; exit 1; }
tail -2 gpurun_out/r3/suite_cy.log
rm -rf gpurun_out/ab gpurun_out/ab_c2 gpurun_out/ab_c3
VS="0 1" bash tools/dev/r3_ab3.sh || exit 1
mv gpurun_out/ab gpurun_out/ab_c2
VS="0 1" BENCH_ARGS="--config C3" bash tools/dev/r3_ab3.sh || exit 1
mv gpurun_out/ab gpurun_out/ab_c3
for f in gpurun_out/ab_c2/b*_*.log gpurun_out/ab_c3/b*_*.log; do python3 -c "
import json,sys
d=[json.loads(l) for l in open('$f') if l.startswith('{')][0]
print('$f', d['config']['config'], round(d['value'],1))"; done
