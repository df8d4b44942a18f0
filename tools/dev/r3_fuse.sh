#!/bin/bash
set -u
mkdir -p gpurun_out/fz
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_arrowhead.py tests/test_gpu_parity.py tests/test_gpu_fusion.py tests/test_gpu_block_sparse.py -q -x --timeout 200 --timeout-method thread -k "arrowhead or ARAP or arap or C5 or multilayer or four_layer or concurrent or trajectory or fusion or real or block or linalg" > gpurun_out/fz/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/fz/tests.log; [ $rc -eq 0 ] || exit $rc
for c in C5 C1_ARAP; do
timeout -k 10 300 python3 -u bench.py --config $c --steps 200 --warmup 20 --timed-steps 20 --no-cpu-baseline > gpurun_out/fz/b_$c.log 2>&1 || exit 1
python3 -c "import json; d=[json.loads(l) for l in open('gpurun_out/fz/b_$c.log') if l.startswith('{')][-1]; print('$c', round(d['value']), d['ms_per_step'], d['ms_per_solve'])"
done
