#!/bin/bash
# development: build a whole-library timing variant with extra flags into csrc/variants/<name>.so
# usage: build_lib_variant.sh name "-DFLAG=1 ..."   (A/B runs: tools/dev/ab.sh)
set -e
cd "$(dirname "$0")/../../dynamicfuion_python_amd/csrc"
name=$1; defs=$2
mkdir -p variants build/var_$name
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -munsafe-fp-atomics -Wno-unused-result -Wno-unused-value -I../../include"
for src in *.hip; do
	/opt/rocm/bin/hipcc $FLAGS $defs -x hip -c $src -o build/var_$name/${src%.hip}.o &
done
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -I../../include -c warp_field.cpp -o build/var_$name/warp_field.o &
wait
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o variants/$name.so build/var_$name/*.o
rm -rf build/var_$name
ls -la variants/$name.so
