#!/bin/bash
# GPU-box pass: GPU parity tests, then the measurement stages of tools/measure.sh. Stops at the first failure.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
if [ "${TESTS:-1}" = 1 ]; then
	timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/gpu_tests.log 2>&1; rc=$?
	echo "tests rc=$rc"; tail -n 4 gpurun_out/gpu_tests.log
	[ $rc -eq 0 ] || exit $rc
fi
exec_measure() { bash tools/measure.sh; }
exec_measure
