# SQ-counter passes over a short C2 bench, one per library (product + csrc/variants/*.so); summaries in gpurun_out/sq/
set -u
mkdir -p gpurun_out/sq
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in dynamicfuion_python_amd/libnnrt_mi355x.so dynamicfuion_python_amd/csrc/variants/*.so; do
	[ -f "$lib" ] || continue
	n=$(basename "$lib" .so)
	NNRT_LIB_PATH=$PWD/$lib timeout -s KILL ${SQ_TIMEOUT:-120} rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/sq/$n -o run -- python3 bench.py --steps 20 --warmup 5 --timed-steps 20 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/sq/$n.log 2>&1 || exit 1
	echo "== $n"
	python3 tools/sq_summary.py $(ls gpurun_out/sq/$n/*/run_counter_collection.csv gpurun_out/sq/$n/run_counter_collection.csv 2>/dev/null | head -1) ${SQ_KEYS:-k_raster_scatter_mesh}
done
