#!/bin/bash
# round-end GPU pass (development): whole GPU suite, smoke(), then the C2 and C5 bench lines under gpurun_out/final
set -u
mkdir -p gpurun_out/final
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/final/gpu_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/final/gpu_tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final/smoke.log 2>&1 || { tail -5 gpurun_out/final/smoke.log; exit 1; }
tail -1 gpurun_out/final/smoke.log
TAG=final LINES="c2 c5" bash tools/bench_lines.sh
