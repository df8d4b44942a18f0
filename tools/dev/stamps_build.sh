#!/bin/bash
# Development timing builds of the library: stamps_build.sh <DEFINE> <output .so>, e.g.
#   NNRT_CORNER_STAMPS tools/dev/libnnrt_stamps.so   (Schur-corner factor phases, tools/dev/corner_stamps.py)
#   NNRT_FIT_STAMPS    tools/dev/libnnrt_fitstamps.so (per-wave timeline of k_fit_pixels_fused, tools/dev/fit_stamps.py)
set -e
DEF=$1
OUT=$(realpath -m "$2")
cd "$(dirname "$0")/../../dynamicfuion_python_amd/csrc"
TMP=/tmp/nnrt_$DEF
mkdir -p $TMP
for f in *.hip; do
	/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -munsafe-fp-atomics \
		-Wno-unused-result -Wno-unused-value -D$DEF ${EXTRA:-} -I../../include -x hip -c "$f" -o "$TMP/${f%.hip}.o" &
done
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -I../../include -c warp_field.cpp -o $TMP/warp_field.o
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$OUT" $TMP/*.o
