#!/bin/bash
# development A/B on the GPU box: bench.py (no CPU baseline) for the product library and every csrc/variants/*.so,
# REPS interleaved repetitions per config; ENVS: space-separated VAR=value settings, each run as a variant of its own
# ("-" = none); one JSON summary line per run in gpurun_out/ab/summary.jsonl
set -u
mkdir -p gpurun_out/ab
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
LIBS="dynamicfuion_python_amd/libnnrt_mi355x.so $(ls dynamicfuion_python_amd/csrc/variants/*.so 2>/dev/null)"
for rep in $(seq 1 ${REPS:-2}); do
	for cfg in ${CONFIGS:-C2}; do
		for lib in $LIBS; do
		for ev in ${ENVS:--}; do
			tag=$(basename $lib .so)_${cfg}_$rep; [ "$ev" = "-" ] || tag=${tag}_$ev
			env ${ev#-} NNRT_LIB_PATH=$PWD/$lib timeout -k 10 300 python3 -u bench.py --config $cfg --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/ab/$tag.log; exit 1; }
			python3 - "$tag" gpurun_out/ab/$tag.log >> gpurun_out/ab/summary.jsonl <<'PY'
import json, sys
line = [l for l in open(sys.argv[2]) if l.startswith("{")][-1]
d = json.loads(line)
print(json.dumps({"tag": sys.argv[1], "value": round(d["value"], 1), "ms_per_step": round(d["ms_per_step"] * 1000, 2),
                  "kernel_us": {k: (round(v * 1000, 2) if v is not None else None) for k, v in d["kernel_ms"].items()}}))
PY
			tail -1 gpurun_out/ab/summary.jsonl
		done
		done
	done
done
