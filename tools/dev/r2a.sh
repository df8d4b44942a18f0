set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py --maxfail=10 -v --timeout 400 --timeout-method thread -s -k "trajectory" > gpurun_out/r2a_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; grep -E "PASS|FAIL|Error|S1:|C2|C5" gpurun_out/r2a_tests.log | tail -30
[ $rc -le 1 ] || exit $rc
