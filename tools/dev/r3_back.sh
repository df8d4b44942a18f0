#!/bin/bash
set -u
mkdir -p gpurun_out
NNRT_LIB_PATH=$PWD/dynamicfuion_python_amd/csrc/variants/libnnrt_v1.so timeout -k 10 500 python3 -u -m pytest tests/test_gpu_arrowhead.py tests/test_gpu_parity.py tests/test_gpu_block_sparse.py -q -x --timeout 200 --timeout-method thread -k "arrowhead or ARAP or arap or C5 or multilayer or four_layer or concurrent or block or linalg or plan" > gpurun_out/back_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -2 gpurun_out/back_tests.log; [ $rc -eq 0 ] || exit $rc
VS="0 1" BENCH_ARGS="--config C5" bash tools/dev/r3_ab3.sh
