#!/bin/bash
# Round 6: merged one-frame calls (8 / 32 queued, decisions only, page-locked, max_batch 4 and 8)
# with the six-wave default and the four-wave build, same box; and configs[2] (2-frame ALT steps).
set -uo pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/${OUTTAG:-r06mab}; mkdir -p $O
for lib in vvc-mip-gpu_amd/lib/libmipgpu.so tools/bin/lib_s0.so; do
  for calls in 8 32; do
    MIPGPU_LIB=$PWD/$lib timeout -k 10 200 python -u tools/e2e_probe.py --reps 15 --calls $calls 1:dec:pinned:mb=4 1:dec:pinned:mb=8 > $O/t.jsonl 2> $O/t.err || { tail $O/t.err; exit 1; }
    python tools/experiments/r06/summ.py 1 1 < $O/t.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('$(basename $lib)', d['case'], d['calls'], 'median', d['median'], 'p25', d['p25'], 'best', d['best'])"
  done
  MIPGPU_LIB=$PWD/$lib timeout -k 10 200 python bench.py --frames-per-step 2 --refs-filter filterFrame_2d_float_5x5_quarterCtu --kernel-idx 2 --steps 10 --warmup 2 --no-cpu-baseline --no-reference-gpu --no-latency --no-filter --no-end-to-end --allow-knobs 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $lib)', 'configs[2]', d['value'], d['ms_per_step'])"
done
