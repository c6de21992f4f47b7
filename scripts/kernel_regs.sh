#!/bin/bash
# VGPR / scratch / occupancy of every kernel in one HIP source: scripts/kernel_regs.sh <file.hip> [regex]
f=$1; pat=${2:-.}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -c -Wno-unused-function -munsafe-fp-atomics "$f" \
  -o /tmp/_regs.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk '/Function Name:/ {n=$NF} /VGPRs:/ {v=$NF} /ScratchSize/ {s=$NF} /Occupancy/ {print n, "vgpr="v, "scratch="s, "occ="$NF}' |
  sed 's/\[-Rpass-analysis=kernel-resource-usage\]//g' | grep -E "$pat"
