#!/bin/bash
# Round 6: task cut factor (MIPGPU_CUT_FACTOR: task size cap = a wave's fair share / factor) at
# twelve waves per workgroup, 384-frame search, same box, alternating.
set -uo pipefail
cd "$(dirname "$0")/../../.."
A="--frames-per-step 384 --steps 20 --warmup 3 --no-cpu-baseline --no-reference-gpu --no-latency --no-filter --no-end-to-end --allow-knobs"
for r in 1 2; do
  for cf in 2 1.33 1 3; do
    MIPGPU_CUT_FACTOR=$cf timeout -k 10 200 python bench.py $A 2>/tmp/ab.err | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cut $cf', d['value'], d['roofline']['kernel_ms_per_launch'])" || { tail /tmp/ab.err; exit 1; }
  done
done
