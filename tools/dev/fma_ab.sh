#!/bin/bash
# development GPU pass for the FMA-formed pixel-node Jacobians (NNRT_JAC_FMA): the whole GPU suite on the product build,
# the trajectory / real-frame / reference-arithmetic tests on the unfused variant (csrc/variants/jacexact.so), then the
# A/B bench lines of tools/dev/ab.sh (CONFIGS, REPS)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider -s > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/gpu_tests.log | tail -8
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
NNRT_LIB_PATH=$PWD/dynamicfuion_python_amd/csrc/variants/jacexact.so timeout -k 10 400 python -u -m pytest tests/test_gpu_fusion.py tests/test_gpu_parity.py -m gpu -q -s -k "real_frame or trajectory or fused_jacobians" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/exact_tests.log 2>&1
rc2=$?; echo "exact-variant tests rc=$rc2"; grep -E "^FAILED|passed|failed" gpurun_out/exact_tests.log | tail -5
[ $rc2 -eq 0 ] || [ $rc2 -eq 1 ] || exit $rc2
bash tools/dev/ab.sh
