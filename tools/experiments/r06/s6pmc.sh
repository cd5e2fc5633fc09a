#!/bin/bash
# PMC passes (tools/pmc_profile.sh) of the default build and of a variant library, 128 frames.
set -uo pipefail
cd "$(dirname "$0")/../../.."
B="--frames-per-step 128 --steps 3 --warmup 1 --no-cpu-baseline --no-reference-gpu --no-latency --no-end-to-end --no-filter --allow-knobs"
for v in default ${VARIANTS:-s6}; do
  lib=vvc-mip-gpu_amd/lib/libmipgpu.so; [ $v = default ] || lib=tools/bin/lib_$v.so
  # raw CSVs outside gpurun_out (64 MiB return limit), summaries copied back
  MIPGPU_LIB=$PWD/$lib OUT=/tmp/pmc_$v BENCH_ARGS="$B" timeout -k 10 600 bash tools/pmc_profile.sh > /dev/null 2>&1 || { echo "FAILED $v"; exit 1; }
  mkdir -p gpurun_out/${OUTTAG:-r06s6pmc}; cp /tmp/pmc_$v/pmc/summary.txt gpurun_out/${OUTTAG:-r06s6pmc}/$v.txt
  echo "## $v"; grep -A30 "mip_search_kernel" /tmp/pmc_$v/pmc/summary.txt | grep -E "kernel|SQ_" | head -26
done
