# raster change check on the GPU box: parity / mirror / fusion tests, stage timings, kernel trace of a short C2 bench
set -u
mkdir -p gpurun_out/rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fusion.py tests/test_gpu_mirror.py --maxfail=5 -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/rc/tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/rc/tests.log; grep -E "FAIL|Error" gpurun_out/rc/tests.log | head -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/fit_variants.py C2 > gpurun_out/rc/fv.log 2>&1 || exit 1
cat gpurun_out/rc/fv.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/rc/prof -o run -- python3 bench.py --steps 300 --warmup 30 --timed-steps 100 --no-cpu-baseline > gpurun_out/rc/prof.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/rc/prof/**/run_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in ("raster", "pixel_jac", "node_reduce", "warp_mesh", "solve_update")):
        print(f'{r["Name"][:60]:60s} calls {r["Calls"]:>6s} avg_us {float(r["AverageNs"])/1000:8.2f}')
PY
timeout -k 10 300 python3 tools/bench_published.py > gpurun_out/rc/published.log 2>&1; cat gpurun_out/rc/published.log
