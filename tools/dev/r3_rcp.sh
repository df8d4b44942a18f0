#!/bin/bash
set -u
mkdir -p gpurun_out/rcp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mirror.py tests/test_gpu_fusion.py -q -x --timeout 200 --timeout-method thread > gpurun_out/rcp/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/rcp/tests.log; [ $rc -eq 0 ] || exit $rc
TAG=rcp K=none bash tools/dev/prof.sh
