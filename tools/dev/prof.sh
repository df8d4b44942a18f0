# dev: parity subset + kernel-trace profile of the bench (snapshot step) -> gpurun_out/prof_<tag>/
set -u
TAG=${TAG:-dev}
K=${K:-"rasterize or fit_one or state_synchronised or stored_states or smoke"}
mkdir -p gpurun_out
if [ "$K" != "none" ]; then
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 300 --timeout-method thread -k "$K" > gpurun_out/prof_tests_$TAG.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/prof_tests_$TAG.log
[ $rc -eq 0 ] || exit $rc
fi
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 200 --warmup 20 --timed-steps 50 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof_bench_$TAG.log 2>&1; rc=$?
echo "prof rc=$rc"; tail -c 300 gpurun_out/prof_bench_$TAG.log
[ $rc -eq 0 ] || exit $rc
f=$(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows,key=lambda r:-float(r["TotalDurationNs"]))[:12]:
    print(f'{float(r["AverageNs"])/1000:8.2f} us  x{r["Calls"]:>6}  {r["Name"][:90]}')
PY
for v in ${VLIBS:-}; do
  NNRT_LIB_PATH=$PWD/dynamicfuion_python_amd/csrc/variants/libnnrt_v$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_v$v -o run -- python3 bench.py --steps 200 --warmup 20 --timed-steps 50 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/prof_bench_${TAG}_v$v.log 2>&1; rc=$?
  echo "variant $v prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
  f=$(find gpurun_out/prof_${TAG}_v$v -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows,key=lambda r:-float(r["TotalDurationNs"]))[:7]:
    print(f'{float(r["AverageNs"])/1000:8.2f} us  x{r["Calls"]:>6}  {r["Name"][:90]}')
PY
done
