#!/bin/bash
set -u
mkdir -p gpurun_out/r3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_arrowhead.py tests/test_gpu_block_sparse.py tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread -k "arrowhead or Arrowhead or block or linalg" > gpurun_out/r3/arrow_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/r3/arrow_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3/prof_published -o run -- python3 tools/bench_published.py > gpurun_out/r3/published.log 2>&1 || exit 1
grep '^{' gpurun_out/r3/published.log > gpurun_out/r3/published.jsonl
cut -c1-300 gpurun_out/r3/published.jsonl
