#!/bin/bash
set -u
mkdir -p gpurun_out/r3
timeout -k 10 150 python3 -u tools/dev/fit_stamps.py C2 gpurun_out/r3/fit_stamps_c2.json > gpurun_out/r3/fit_stamps.log 2>&1 || exit 1
timeout -k 10 150 python3 -u tools/dev/kernel_stamps.py C2 > gpurun_out/r3/kernel_stamps.log 2>&1 || exit 1
tail -3 gpurun_out/r3/kernel_stamps.log
