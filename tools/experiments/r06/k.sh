#!/bin/bash
# Round 6: merged vs unmerged queued one-frame calls (1080p, page-locked), 15 rounds each,
# with the HIP runtime's direct dispatch (default) and without (AMD_DIRECT_DISPATCH=0).
set -uo pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/${OUTTAG:-r06k}; mkdir -p $O
: > $O/merge_rates.jsonl
for dd in ${DDS:-1 0}; do
  for m in 1 0; do
    for calls in 8 32; do
      AMD_DIRECT_DISPATCH=$dd MIPGPU_MERGE=$m timeout -k 10 200 python -u tools/e2e_probe.py --reps 15 --calls $calls 1:dec:pinned:mb=4 1:dec:pinned:mb=8 1:full:pinned:mb=4 > $O/t.jsonl 2> $O/t.err || { tail $O/t.err; exit 1; }
      python tools/experiments/r06/summ.py $dd $m < $O/t.jsonl >> $O/merge_rates.jsonl
    done
  done
done
python -c "
import json
for l in open('$O/merge_rates.jsonl'):
    d=json.loads(l); print(d['AMD_DIRECT_DISPATCH'], d['MIPGPU_MERGE'], d['case'], d['calls'], 'median', d['median'], 'p25', d['p25'], 'best', d['best'])
"
