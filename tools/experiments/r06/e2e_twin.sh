#!/bin/bash
# Round 6: the bench's end-to-end shape (8 queued 128-frame calls, max_batch 384) decisions only
# and full tables, six-wave chunks (default) vs the four-wave twin for every pipeline chunk
# (MIPGPU_PIPE_KERNEL=8), alternating, same box.
set -uo pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/${OUTTAG:-r06e2etw}; mkdir -p $O
for r in 1 2; do
  for envs in "X=1" "MIPGPU_PIPE_KERNEL=8"; do
    env $envs timeout -k 10 300 python -u tools/e2e_probe.py --reps 5 --calls 8 128:dec:pinned:mb=384 128:full:pinned:mb=384 > $O/t.jsonl 2> $O/t.err || { tail $O/t.err; exit 1; }
    python -c "
import json, sys
for l in open('$O/t.jsonl'):
    d = json.loads(l)
    print('%-22s %-24s fps %8.1f all %s' % ('$envs', d.get('case'), d['fps'], d.get('fps_all')))"
  done
done
