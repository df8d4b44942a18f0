#!/bin/bash
# round-6 development GPU pass: the whole GPU suite, then bench A/B lines (CONFIGS / ENVS as tools/dev/ab.sh)
set -u
mkdir -p gpurun_out/r6d
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
if [ "${SKIP_TESTS:-0}" != 1 ]; then
	timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 400 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/r6d/gpu_tests.log 2>&1
	rc=$?; tail -3 gpurun_out/r6d/gpu_tests.log; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
fi
REPS=${REPS:-1} CONFIGS="${CONFIGS:-C2 C3 C5}" ENVS="${ENVS:--}" bash tools/dev/ab.sh
