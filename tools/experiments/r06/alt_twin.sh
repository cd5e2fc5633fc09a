#!/bin/bash
# Round 6: small ALT launches on the four-wave twin vs the six-wave kernel (MIPGPU_PIPE_KERNEL=0):
# device-API launches of 1-16 frames and the configs[2] / [4] steps.  Ran with a since-reverted
# mipgpu.cpp rule (alt_small: ALT launches under kSmallLaunchItemsPerGroup items per workgroup
# took the twin); result and why it was dropped: DESIGN.md section 6 (configs sweep).
set -uo pipefail
cd "$(dirname "$0")/../../.."
for envs in "X=1" "MIPGPU_PIPE_KERNEL=0" "X=2" "MIPGPU_PIPE_KERNEL=0"; do
  echo "== $envs"
  env $envs SB_FILTER=filterFrame_2d_float_5x5_quarterCtu:2 SB_CUTS=2 SB_ORDERS=1 SB_SLICES=0 SB_WIDE=auto timeout -k 10 300 python -u tools/small_batch.py 2>/tmp/sb.err | grep -v build_id | python -c "
import json,sys
for l in sys.stdin: print(json.loads(l)['ms_per_launch'])" || { tail /tmp/sb.err; exit 1; }
  env $envs timeout -k 10 200 python bench.py --frames-per-step 2 --refs-filter filterFrame_2d_float_5x5_quarterCtu --kernel-idx 2 --steps 10 --warmup 2 --no-cpu-baseline --no-reference-gpu --no-latency --no-filter --no-end-to-end --allow-knobs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('configs[2]', d['value'], d['ms_per_step'])"
  env $envs timeout -k 10 200 python bench.py --frames-per-step 1 --width 7680 --height 4320 --refs-filter filterFrame_2d_int_quarterCtu --steps 10 --warmup 2 --no-cpu-baseline --no-reference-gpu --no-latency --no-filter --no-end-to-end --allow-knobs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('configs[4]', d['value'], d['ms_per_step'])"
done
