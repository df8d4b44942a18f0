#!/bin/bash
# A/B/C of variant libraries (csrc/variants/libnnrt_v<n>.so), kernel trace, two interleaved repetitions
set -u
mkdir -p gpurun_out/ab
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for rep in 1 2; do for v in ${VS:-0 1 2}; do
  NNRT_LIB_PATH=$PWD/dynamicfuion_python_amd/csrc/variants/libnnrt_v$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/p${v}_$rep -o run -- python3 bench.py --steps 300 --warmup 30 --timed-steps 10 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab/b${v}_$rep.log 2>&1 || exit 1
  python3 - gpurun_out/ab/p${v}_$rep/run_kernel_stats.csv $v $rep <<'PY'
import csv,sys
rows=list(csv.DictReader(open(sys.argv[1])))
want=("k_fit_pixels_fused","k_raster_scatter_mesh","k_warp_mesh_quad","k_solve_update","k_corner_factor","k_corner_back","k_init_stem","k_stem_schur_rhs","k_arrow_back","k_arrow_prepare")
out=[]
for r in rows:
    for w in want:
        if w in r["Name"]: out.append(f'{w} {float(r["AverageNs"])/1000:.2f}')
print(f"v{sys.argv[2]} rep{sys.argv[3]}: " + ", ".join(out))
PY
done; done
