#!/bin/bash
# round-6 development GPU pass: the exact-system / refinement parity tests on the product library (PRODUCT_K), then bench
# lines of the ARAP configs (CONFIGS_AB, each as "config args|..."), printing GN it/s, kernel times and the gate
set -u
mkdir -p gpurun_out/r6b
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
if [ -n "${PRODUCT_K:-}" ]; then
	PRODUCT_K="$PRODUCT_K" bash tools/dev/r6_parity.sh
	rc=$?; [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
fi
IFS='|' read -ra LINES <<< "${CONFIGS_AB:-}"
for cfg in "${LINES[@]}"; do
	tag=$(echo "$cfg" | tr ' -' '__')
	timeout -k 10 300 python3 -u bench.py $cfg --no-cpu-baseline > gpurun_out/r6b/$tag.log 2>&1 || { echo "FAIL $tag"; tail -3 gpurun_out/r6b/$tag.log; exit 1; }
	python3 -c "
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], round(d['value'],1), {k:round(v*1000,1) for k,v in d['kernel_ms'].items() if v}, d['roofline'].get('refinement'))
" gpurun_out/r6b/$tag.log "$tag"
done
exit 0
