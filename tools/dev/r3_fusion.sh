#!/bin/bash
set -u
mkdir -p gpurun_out/r3
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fusion.py -m gpu -v -s --timeout 200 --timeout-method thread > gpurun_out/r3/fusion.log 2>&1; echo "fusion rc $?"
grep -n "fp64 rule\|passed\|failed" gpurun_out/r3/fusion.log
