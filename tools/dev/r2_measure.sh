# round-2 measurement pass on the GPU box: C2 bench line, kernel trace, PMC traffic; outputs under gpurun_out/r2/
set -u
mkdir -p gpurun_out/r2
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/r2/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 2 "gpurun_out/r2/$name.log"; return $rc; }
step bench_c2 400 python3 -u bench.py || exit 1
grep '^{' gpurun_out/r2/bench_c2.log > gpurun_out/r2/bench_c2.json
step prof_c2 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2/prof_c2 -o run -- python3 bench.py --steps 300 --warmup 30 --timed-steps 100 --no-cpu-baseline || exit 1
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r2/pmc_fetch -o run -- python3 bench.py --steps 20 --warmup 5 --timed-steps 20 --no-cpu-baseline || exit 1
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r2/pmc_write -o run -- python3 bench.py --steps 20 --warmup 5 --timed-steps 20 --no-cpu-baseline || exit 1
W=$(python3 -c "import json;print(json.load(open('gpurun_out/r2/bench_c2.json'))['config']['workload'])")
python3 tools/pmc_traffic.py --fetch "gpurun_out/r2/pmc_fetch/**/*counter_collection.csv" --write "gpurun_out/r2/pmc_write/**/*counter_collection.csv" --workload "$W" --out gpurun_out/r2/pmc_traffic.json > /dev/null || exit 1
step bench_c2_traffic 300 python3 -u bench.py --no-cpu-baseline --traffic-file gpurun_out/r2/pmc_traffic.json || exit 1
grep '^{' gpurun_out/r2/bench_c2_traffic.log > gpurun_out/r2/bench_c2_traffic.json
echo done
