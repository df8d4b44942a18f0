#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu -s"
for v in 0 1; do
NNRT_WARP_VARIANT=$v timeout -k 10 300 $T tests/test_gpu_parity.py -k "C2_ARAP-10" > gpurun_out/c2arap_v$v.log 2>&1
echo "variant $v rc $?"
done
