#!/bin/bash
# Development timing build of the library with shader-clock stamps in the Schur-corner factor kernel
# (-DNNRT_CORNER_STAMPS) -> tools/dev/libnnrt_stamps.so; tools/dev/corner_stamps.py loads it via NNRT_LIB_PATH.
set -e
cd "$(dirname "$0")/../../dynamicfuion_python_amd/csrc"
mkdir -p /tmp/nnrt_stamps
for f in *.hip; do
	/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -munsafe-fp-atomics \
		-Wno-unused-result -Wno-unused-value -DNNRT_CORNER_STAMPS -I../../include -x hip -c "$f" -o "/tmp/nnrt_stamps/${f%.hip}.o" &
done
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -I../../include -c warp_field.cpp -o /tmp/nnrt_stamps/warp_field.o
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o ../../tools/dev/libnnrt_stamps.so /tmp/nnrt_stamps/*.o
