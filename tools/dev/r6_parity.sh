#!/bin/bash
# round-6 development GPU pass: the reference-arithmetic / exact-system parity tests on the product library, then on
# variant libraries (VARIANTS: names under csrc/variants, each with its own test selection VARIANT_K_<name>).
# Every GPU step has its own limit; the first failure ends the script.
set -u
mkdir -p gpurun_out/r6
cd /tmp && export TMPDIR=/tmp && cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
run() {   # tag lib k
	local tag=$1 lib=$2 k=$3
	NNRT_LIB_PATH=$PWD/$lib timeout -k 10 ${TEST_LIMIT:-700} python -u -m pytest tests -m gpu -v -s --timeout 400 --timeout-method thread \
		-p no:cacheprovider -k "$k" > gpurun_out/r6/$tag.log 2>&1
	local rc=$?
	echo "$tag rc=$rc"; grep -E "passed|failed|error" gpurun_out/r6/$tag.log | tail -2
	return $rc
}
fatal() { [ "$1" -ne 0 ] && [ "$1" -ne 1 ]; }
if [ -n "${PRODUCT_K:-}" ]; then run product dynamicfuion_python_amd/libnnrt_mi355x.so "$PRODUCT_K"; rc=$?; fatal $rc && exit $rc; fi
for v in ${VARIANTS:-}; do
	kv=VARIANT_K_$v
	run $v dynamicfuion_python_amd/csrc/variants/$v.so "${!kv}"; rc=$?; fatal $rc && exit $rc
done
exit 0
