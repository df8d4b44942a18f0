# development: build timing variants of one source (VARIANT_SRC, default raster.hip) into csrc/variants/<name>.so
# usage: build_variants.sh name1 "-DFLAG ..." name2 "-DFLAG ..."
set -e
cd "$(dirname "$0")/../../dynamicfuion_python_amd/csrc"
SRC=${VARIANT_SRC:-raster.hip}
mkdir -p variants build/var
rm -f variants/*.so
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -munsafe-fp-atomics -I../../include"
OBJS=$(ls build/*.o | grep -v "build/${REPLACES:-${SRC%.hip}}.o")
while [ $# -gt 0 ]; do
	name=$1; defs=$2; shift 2
	/opt/rocm/bin/hipcc $FLAGS $defs -x hip -c $SRC -o build/var/$name.o &
done
wait
for o in build/var/*.o; do
	/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o variants/$(basename ${o%.o}).so $o $OBJS
done
rm -rf build/var
ls -la variants
