#!/bin/bash
# development GPU pass: tools/dev/refine_gpu_exact.py on the product build and the refine_none / refine_all variants
set -u
mkdir -p gpurun_out/refine
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for lib in dynamicfuion_python_amd/libnnrt_mi355x.so dynamicfuion_python_amd/csrc/variants/refine_none.so dynamicfuion_python_amd/csrc/variants/refine_all.so; do
	tag=$(basename $lib .so)
	NNRT_LIB_PATH=$PWD/$lib timeout -k 10 400 python3 -u tools/dev/refine_gpu_exact.py ${SCENE:-C5} ${ITERS:-5} > gpurun_out/refine/$tag.log 2>&1 || { echo "FAIL $tag"; tail -5 gpurun_out/refine/$tag.log; exit 1; }
	grep iteration gpurun_out/refine/$tag.log
done
