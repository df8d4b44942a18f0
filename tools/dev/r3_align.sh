#!/bin/bash
set -u
mkdir -p gpurun_out/al
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/al -o run -- python3 tools/dev/align_stamps.py gpurun_out/al/stamps.json > gpurun_out/al/run.log 2>&1 || exit 1
f=$(find gpurun_out/al -name "*kernel_trace.csv" | head -1)
python3 tools/dev/align_report.py gpurun_out/al/stamps.json "$f"
TAG=wv K=none VLIBS="1 2" bash tools/dev/prof.sh
