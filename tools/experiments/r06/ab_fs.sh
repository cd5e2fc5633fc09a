#!/bin/bash
# Same-box A/B: per-frame status pointer (default) vs one status set per launch (-DMIP_FRAME_STATUS=0)
# vs the round-5 library + bench (abr05/), 384-frame search only, alternating.
set -uo pipefail
cd "$(dirname "$0")/../../.."
A="--frames-per-step 384 --steps 20 --warmup 3 --no-cpu-baseline --no-reference-gpu --no-latency --no-filter --no-end-to-end --allow-knobs"
for r in 1 2 3; do
  for t in abr05 default nofs; do
    b=bench.py; lib=vvc-mip-gpu_amd/lib/libmipgpu.so
    [ $t = abr05 ] && { b=abr05/bench.py; lib=abr05/vvc-mip-gpu_amd/lib/libmipgpu.so; }
    [ $t = nofs ] && lib=tools/bin/lib_nofs.so
    MIPGPU_LIB=$PWD/$lib timeout -k 10 200 python $b $A 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['value'], d['roofline']['kernel_ms_per_launch'])" || exit 1
  done
done
