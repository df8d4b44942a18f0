set -u
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fusion.py tests/test_gpu_mirror.py --maxfail=5 -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/nr_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/nr_tests.log; grep -E "FAIL|Error" gpurun_out/nr_tests.log | head -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 tools/fit_variants.py C2 > gpurun_out/fv.log 2>&1; rc=$?; cat gpurun_out/fv.log; exit $rc
