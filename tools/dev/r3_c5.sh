#!/bin/bash
# C5 / arrowhead: parity subset, then C5 bench + kernel trace (gpurun_out/c5/)
set -u
mkdir -p gpurun_out/c5
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_arrowhead.py tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread -k "arrowhead or ARAP or arap or C5 or multilayer or four_layer or concurrent" > gpurun_out/c5/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/c5/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c5/prof -o run -- python3 bench.py --config C5 --steps 200 --warmup 20 --timed-steps 20 --no-cpu-baseline > gpurun_out/c5/bench.log 2>&1 || exit 1
python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/c5/bench.log') if l.startswith('{')][-1]; print('C5', round(d['value']), d['ms_per_step'], d['ms_per_solve'])"
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/c5/prof/run_kernel_stats.csv')))
for r in sorted(rows,key=lambda r:-float(r["TotalDurationNs"]))[:14]:
    print(f'{float(r["AverageNs"])/1000:8.2f} us  x{r["Calls"]:>6}  {r["Name"][:70]}')
PY
