# development: warped-Jacobian rows in the raster launch -- variant libraries (csrc/variants/libnnrt_v<n>.so)
# (the product code does not carry the experiment: apply tools/dev/r3_rows.patch first)
# v0: rows from the warp (previous product); v1: rows in raster, plain stores; v2: non-temporal; v3: agent write-through
set -e
cd "$(dirname "$0")/../../dynamicfuion_python_amd/csrc"
mkdir -p variants build/var
rm -f variants/*.so
FLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -munsafe-fp-atomics -I../../include"
OBJS=$(ls build/*.o | grep -v -e build/raster.o -e build/capi.o)
build() {   # n defs
	/opt/rocm/bin/hipcc $FLAGS $2 -x hip -c raster.hip -o build/var/raster_$1.o
	/opt/rocm/bin/hipcc $FLAGS $2 -x hip -c capi.hip -o build/var/capi_$1.o
	/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o variants/libnnrt_v$1.so build/var/raster_$1.o build/var/capi_$1.o $OBJS
}
build 0 "-DNNRT_ROWS_IN_RASTER=0" &
build 1 "-DNNRT_ROWS_STORE=0" &
build 2 "-DNNRT_ROWS_STORE=1" &
build 3 "-DNNRT_ROWS_STORE=2" &
wait
rm -rf build/var
ls -la variants
