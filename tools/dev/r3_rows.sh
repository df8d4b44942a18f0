# development: product suite with the rows-in-raster launch, then the rows-placement A/B (tools/dev/r3_rows_variants.sh)
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r3/suite_rows.log 2>&1 || { tail -30 gpurun_out/r3/suite_rows.log; exit 1; }
tail -2 gpurun_out/r3/suite_rows.log
VS="0 1 2 3" bash tools/dev/r3_ab3.sh || exit 1
grep -h '^{' gpurun_out/ab/b*_*.log | python3 -c "
import sys,json
for l in sys.stdin: d=json.loads(l); print(d['config']['config'], round(d['value'],1))"
