#!/bin/bash
# fused pixel kernel: 4 / 2 / 1 waves per workgroup (variants/libnnrt_v<n>.so) -- parity subset + kernel trace
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in 1 2; do
  NNRT_LIB_PATH=$PWD/dynamicfuion_python_amd/csrc/variants/libnnrt_v$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 200 --timeout-method thread -k "fit_one or stored_states or single_mode" > gpurun_out/pw_tests_$v.log 2>&1; rc=$?
  echo "variant $v tests rc=$rc"; tail -2 gpurun_out/pw_tests_$v.log; [ $rc -eq 0 ] || exit $rc
done
TAG=pw K=none VLIBS="1 2" bash tools/dev/prof.sh
