#!/bin/bash
# Print VGPR / scratch / occupancy of every kernel in a csrc/*.hip file (compile-only, no GPU).
cd "$(dirname "$0")/../dynamicfuion_python_amd/csrc"
hipcc -O3 --offload-arch=gfx950 -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -munsafe-fp-atomics -std=c++17 -fPIC \
	-I../../include -x hip -c "${1:-fitter_kernels.hip}" -o /tmp/_kr.o -Rpass-analysis=kernel-resource-usage 2>&1 |
	grep -E "Function Name|VGPRs:|AGPRs:|ScratchSize|Occupancy|LDS Size" | sed -e 's/.*remark: //'
