set -u
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/t_mirror.log 2>&1; rc=$?
echo "rc=$rc"; grep -E "FAIL|Error|passed|failed" gpurun_out/t_mirror.log | tail -15
exit $rc
