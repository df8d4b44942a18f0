# stage timings of product + variants, then a kernel trace per library (short C2 bench); raster/pixel/node rows only
set -u
mkdir -p gpurun_out/vp
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python3 tools/fit_variants.py ${CONFIG:-C2} > gpurun_out/vp/fv.log 2>&1 || { cat gpurun_out/vp/fv.log; exit 1; }
cat gpurun_out/vp/fv.log
for lib in dynamicfuion_python_amd/libnnrt_mi355x.so dynamicfuion_python_amd/csrc/variants/*.so; do
	[ -f "$lib" ] || continue
	n=$(basename "$lib" .so)
	NNRT_LIB_PATH=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/vp/$n -o run -- python3 bench.py --config ${CONFIG:-C2} --steps 200 --warmup 20 --timed-steps 100 --no-cpu-baseline > gpurun_out/vp/$n.log 2>&1 || exit 1
	python3 - "$n" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/vp/{sys.argv[1]}/**/run_kernel_stats.csv", recursive=True)[0]
out = []
for r in csv.DictReader(open(f)):
    if any(k in r["Name"] for k in ("raster_scatter_mesh", "pixel_jac", "node_reduce", "fit_pixels_fused", "warp_mesh", "solve_update", "chol", "arap")) and int(r["Calls"]) > 50:
        out.append(f'{r["Name"].split("(")[0].replace("void nnrt::","").replace("nnrt::","")[:34]} {float(r["AverageNs"])/1000:.2f}')
print(f"{sys.argv[1]:16s}", " | ".join(out))
PY
done
