#!/bin/bash
set -u
mkdir -p gpurun_out
NNRT_LIB_PATH=$PWD/dynamicfuion_python_amd/csrc/variants/libnnrt_v1.so timeout -k 10 500 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fusion.py -q -x --timeout 200 --timeout-method thread > gpurun_out/order_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/order_tests.log; [ $rc -eq 0 ] || exit $rc
VS="0 1" bash tools/dev/r3_ab3.sh
VS="0 1" BENCH_ARGS="--config C3" bash tools/dev/r3_ab3.sh
