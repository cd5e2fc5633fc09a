#!/bin/bash
# Same-box A/B of library builds: tools/ab_bench.sh REPS lib1.so lib2.so ...  (MIPGPU_LIB switch;
# FRAMES = frames per step, EXTRA = further bench.py arguments, e.g. --refs-filter NAME)
set -euo pipefail
cd "$(dirname "$0")/.."
reps=$1; shift
for r in $(seq "$reps"); do
  for lib in "$@"; do
    MIPGPU_LIB=$PWD/$lib timeout -k 10 120 python bench.py --frames-per-step ${FRAMES:-32} --steps 20 \
      --no-cpu-baseline --no-reference-gpu --no-latency --no-filter --no-end-to-end --allow-knobs ${EXTRA:-} 2>/dev/null \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], d['roofline']['kernel_ms_per_launch'])"
  done
done
