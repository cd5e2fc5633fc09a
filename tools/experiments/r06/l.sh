#!/bin/bash
# Round 6: the flusher thread and the case order (first engine of the process) vs the merged
# 8-call rate.
set -uo pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06l; mkdir -p $O
: > $O/rates.jsonl
for m in 1 nothread 0; do
  for order in "1:dec:pinned:mb=4 1:dec:pinned:mb=8" "1:dec:pinned:mb=8 1:dec:pinned:mb=4"; do
    MIPGPU_MERGE=$m timeout -k 10 200 python -u tools/e2e_probe.py --reps 15 --calls 8 $order > $O/t.jsonl 2> $O/t.err || { tail $O/t.err; exit 1; }
    python tools/experiments/r06/summ.py 1 $([ $m = 0 ] && echo 0 || echo 1) < $O/t.jsonl | sed "s/^{/{\"mode\": \"$m\", \"order\": \"$order\", /" >> $O/rates.jsonl
  done
done
python -c "
import json
for l in open('$O/rates.jsonl'):
    d=json.loads(l); print(d['mode'], '|', d['order'], '|', d['case'], 'median', d['median'], 'best', d['best'])
"
