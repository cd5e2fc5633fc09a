#!/bin/bash
# VGPR / scratch use of mip_search_kernel per CU-size class (compile-only, gfx950).
cd "$(dirname "$0")/../vvc-mip-gpu_amd"
for c in $(seq 0 28); do
  (r=$(/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include -Icsrc -DMIP_ONLY_CLASS=$c --cuda-device-only -c \
       -Rpass-analysis=kernel-resource-usage csrc/mip_search.hip -o /tmp/vgpr_c$c.o 2>&1 | grep -E " VGPRs:| ScratchSize" | sed -n 3,4p | awk '{print $(NF-1)}' | tr '\n' ' ')
   echo "class $c: VGPRs/scratch $r") &
done
wait
