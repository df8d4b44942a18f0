#!/bin/bash
# warp non-temporal stores A/B (bench + kernel trace) and the C2_ARAP trajectory diagnosis
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 0 1; do
  NNRT_WARP_VARIANT=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/nt_b$v.log 2>&1 || exit 12
  NNRT_WARP_VARIANT=$v timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/nt_prof$v -o run -- python -u bench.py --no-cpu-baseline --steps 200 > gpurun_out/nt_p$v.log 2>&1 || exit 13
done
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu -s"
timeout -k 10 300 $T tests/test_gpu_parity.py -k "C2_ARAP-10" > gpurun_out/c2arap.log 2>&1
echo "c2arap rc $?"
