#!/bin/bash
# Round 6: compile-time knobs re-checked at six waves per SIMD (tools/bin/lib_k_*.so), same box,
# 384-frame search, default build first in each rep.
set -uo pipefail
cd "$(dirname "$0")/../../.."
A="--frames-per-step 384 --steps 20 --warmup 3 --no-cpu-baseline --no-reference-gpu --no-latency --no-filter --no-end-to-end --allow-knobs"
for r in 1 2; do
  for lib in vvc-mip-gpu_amd/lib/libmipgpu.so tools/bin/lib_k_*.so; do
    MIPGPU_LIB=$PWD/$lib timeout -k 10 200 python bench.py $A 2>/tmp/ab.err | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], d['roofline']['kernel_ms_per_launch'])" || { tail /tmp/ab.err; exit 1; }
  done
done
