# ARAP snapshot restart folded into the iteration: ARAP / snapshot GPU tests, then C1_ARAP and C5 A/B (v0 copy, v1 folded)
set -u
mkdir -p gpurun_out/r3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_arrowhead.py -m gpu -x -q --timeout 200 --timeout-method thread -k "snapshot or ARAP or arap or arrow or replica or C5 or L4 or layer" > gpurun_out/r3/fold_tests.log 2>&1 || { tail -30 gpurun_out/r3/fold_tests.log; exit 1; }
tail -2 gpurun_out/r3/fold_tests.log
for rep in 1 2; do for v in 0 1; do for c in C1_ARAP C5; do
  NNRT_LIB_PATH=$PWD/dynamicfuion_python_amd/csrc/variants/libnnrt_v$v.so timeout -k 10 300 python3 -u bench.py --config $c --steps 200 --warmup 20 --timed-steps 40 --no-cpu-baseline > gpurun_out/r3/fold_${c}_v${v}_$rep.log 2>&1 || exit 1
  python3 -c "
import json,sys
d=[json.loads(l) for l in open('gpurun_out/r3/fold_${c}_v${v}_$rep.log') if l.startswith('{')][0]
print('$c v$v rep$rep', round(d['value'],1), round(d['ms_per_step']*1000,1))"
done; done; done
