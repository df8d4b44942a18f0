# round-3 measurement pass (C2): bench line with CPU baseline, kernel trace, PMC traffic, SQ counters, replicas line,
# per-wave stamps; outputs under gpurun_out/r3/
set -u
mkdir -p gpurun_out/r3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/r3/$name.log" 2>&1; local rc=$?; echo "== $name rc=$rc"; tail -n 2 "gpurun_out/r3/$name.log" | cut -c1-300; return $rc; }
step bench_c2 400 python3 -u bench.py || exit 1
grep '^{' gpurun_out/r3/bench_c2.log > gpurun_out/r3/bench_c2.json
step prof_c2 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3/prof_c2 -o run -- python3 bench.py --steps 300 --warmup 30 --timed-steps 100 --no-cpu-baseline || exit 1
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r3/pmc_fetch -o run -- python3 bench.py --steps 20 --warmup 5 --timed-steps 20 --no-cpu-baseline || exit 1
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r3/pmc_write -o run -- python3 bench.py --steps 20 --warmup 5 --timed-steps 20 --no-cpu-baseline || exit 1
W=$(python3 -c "import json;print(json.load(open('gpurun_out/r3/bench_c2.json'))['config']['workload'])")
python3 tools/pmc_traffic.py --fetch "gpurun_out/r3/pmc_fetch/**/*counter_collection.csv" --write "gpurun_out/r3/pmc_write/**/*counter_collection.csv" --workload "$W" --out gpurun_out/r3/pmc_traffic.json > /dev/null || exit 1
step bench_c2_traffic 300 python3 -u bench.py --no-cpu-baseline --traffic-file gpurun_out/r3/pmc_traffic.json || exit 1
grep '^{' gpurun_out/r3/bench_c2_traffic.log > gpurun_out/r3/bench_c2_traffic.json
step pmc_sq 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/r3/pmc_sq -o run -- python3 bench.py --steps 20 --warmup 5 --timed-steps 20 --no-cpu-baseline || exit 1
f=$(find gpurun_out/r3/pmc_sq -name "*counter_collection.csv" | head -1)
python3 tools/sq_summary.py "$f" k_fit_pixels_fused k_raster_scatter_mesh k_warp_mesh_quad k_solve_update > gpurun_out/r3/sq_summary.txt 2>&1 || exit 1
step bench_rep8 400 python3 -u bench.py --replicas 8 --no-cpu-baseline || exit 1
grep '^{' gpurun_out/r3/bench_rep8.log > gpurun_out/r3/bench_rep8.json
[ "${STAMPS:-1}" = 0 ] && { echo done; exit 0; }   # the stamp steps need the development stamp libraries (tools/dev/stamps_build.sh)
step fit_stamps 150 python3 -u tools/dev/fit_stamps.py C2 gpurun_out/r3/fit_stamps_c2.json || exit 1
step kernel_stamps 150 python3 -u tools/dev/kernel_stamps.py C2 || exit 1
echo done
