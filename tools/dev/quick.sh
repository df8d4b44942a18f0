#!/bin/bash
# development GPU pass: optional targeted GPU tests (PYTEST_K / PYTEST_FILES), then bench A/B lines (CONFIGS) and an
# optional kernel trace of one config (PROF_CONFIG). Every GPU step has its own limit; the first failure ends the script.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
if [ -n "${PYTEST_FILES:-}" ]; then
	timeout -k 10 ${TEST_LIMIT:-600} python -u -m pytest ${PYTEST_FILES} -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider ${PYTEST_K:+-k "$PYTEST_K"} -s > gpurun_out/quick_tests.log 2>&1
	rc=$?; echo "tests rc=$rc"; grep -E "passed|failed|error" gpurun_out/quick_tests.log | tail -3
	[ $rc -eq 0 ] || exit $rc
fi
if [ -n "${CONFIGS:-}" ]; then
	bash tools/dev/ab.sh || exit 1
fi
if [ -n "${PROF_CONFIG:-}" ]; then
	timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$PROF_CONFIG -o run -- python3 bench.py --config $PROF_CONFIG --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/prof_$PROF_CONFIG.log 2>&1 || { echo "prof failed"; tail -5 gpurun_out/prof_$PROF_CONFIG.log; exit 1; }
	echo "prof ok"
fi
echo done
