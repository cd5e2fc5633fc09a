#!/bin/bash
# VGPR / scratch use of mip_search_kernel per CU-size class (compile-only, gfx950).
cd "$(dirname "$0")/../vvc-mip-gpu_amd"
tmp=$(mktemp -d)
cp csrc/*.h "$tmp"/
for c in $(seq 0 16); do
  (sed "s/  case idx: run_task<W, H>/  case idx: if (idx == $c) run_task<W, H>/" csrc/mip_search.hip > "$tmp/c$c.hip"
   r=$(/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../include -I"$tmp" --cuda-device-only -c \
       -Rpass-analysis=kernel-resource-usage "$tmp/c$c.hip" -o "$tmp/c$c.o" 2>&1 | grep -E " VGPRs:| ScratchSize" | sed -n 3,4p | awk '{print $NF=="" ? "" : $(NF-1)}' | tr '\n' ' ')
   echo "class $c: VGPRs/scratch $r") &
done
wait
rm -rf "$tmp"
