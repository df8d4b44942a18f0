#!/bin/bash
# development GPU pass: the whole GPU suite on the product build, then (only if green) the A/B lines of tools/dev/ab.sh
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider -s > gpurun_out/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/gpu_tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
bash tools/dev/ab.sh
