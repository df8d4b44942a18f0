#!/bin/bash
# development GPU pass: GPU tests (ordinary failures continue, anything else stops), then the A/B of tools/dev/ab.sh
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=${MAXFAIL:-20} --timeout 200 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS:-} ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "tests rc=$rc"; grep -E "^FAILED|passed|failed" gpurun_out/gpu_tests.log | tail -25
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ "${AB:-1}" = 1 ] || exit $rc
bash tools/dev/ab.sh
