#!/bin/bash
# Same-box A/B: round-5 final library + bench (abr05/, untracked copy of git 0427f2e) vs this tree,
# 384-frame search only, alternating, 3 reps each.
set -uo pipefail
cd "$(dirname "$0")/../../.."
A="--frames-per-step 384 --steps 20 --warmup 3 --no-cpu-baseline --no-reference-gpu --no-latency --no-filter --no-end-to-end"
for r in 1 2 3; do
  for t in abr05 .; do
    timeout -k 10 200 python $t/bench.py $A 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$t', d['value'], d['roofline']['kernel_ms_per_launch'], d.get('build_id'))" || exit 1
  done
done
