#!/bin/bash
# round-3 GPU pass: kernel timelines, warp-variant A/B, parity with variant 1, ARAP/TSDF suites, C5 bench
set -o pipefail
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
timeout -k 10 150 python -u tools/dev/kernel_stamps.py C2 > gpurun_out/kst.log 2>&1 || exit 11
for v in 0 1; do
  NNRT_WARP_VARIANT=$v timeout -k 10 200 python -u bench.py --no-cpu-baseline > gpurun_out/bw_$v.log 2>&1 || exit 12
done
NNRT_WARP_VARIANT=1 timeout -k 10 300 $T tests/test_gpu_parity.py -k "one_iteration or synchronised or stored_states or extrinsics" > gpurun_out/par_v1.log 2>&1 || exit 13
timeout -k 10 600 $T tests/test_gpu_tsdf.py tests/test_gpu_fusion.py tests/test_gpu_arrowhead.py tests/test_gpu_parity.py \
  -k "tsdf or fusion or arrowhead or arap or ARAP or C5 or multilayer or concurrent or trajectory or four_layer" > gpurun_out/suite.log 2>&1 || exit 14
timeout -k 10 300 python -u bench.py --config C5 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/c5.log 2>&1 || exit 15
