#!/bin/bash
# Round 6: which HIP call blocks the host for ~8 ms when 32 one-frame calls are queued?
set -uo pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06e; mkdir -p $O
for m in 0 1; do
  MIPGPU_SLOW_CALLS=0.3 MIPGPU_MERGE=$m timeout -k 10 200 python -u tools/e2e_probe.py --reps 3 --calls 32 1:dec:pinned:mb=4 > $O/m$m.jsonl 2> $O/m$m.err || { tail $O/m$m.err; exit 1; }
  echo "== merge $m"; cut -c1-300 $O/m$m.jsonl; grep -c "slow call" $O/m$m.err; grep "slow call" $O/m$m.err | sort -t' ' -k4 -rn | head -20
done
