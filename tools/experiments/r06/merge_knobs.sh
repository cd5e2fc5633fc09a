#!/bin/bash
# Round 6: merged one-frame decisions-only calls (8 / 32 queued, max_batch 4) of the six-wave
# build under host-pipeline knobs: split unpacking on the search stream, wide launches never /
# always, one search stream, the /opt/rocm runtime (SDMA copies), no direct dispatch.
set -uo pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/${OUTTAG:-r06mk}; mkdir -p $O
for envs in ${ENVS:-"X=1" "MIPGPU_DEC_INLINE=1" "MIPGPU_WIDE=0" "MIPGPU_WIDE=1" "MIPGPU_SEARCH_STREAMS=1" "MIPGPU_NO_TORCH=1" "AMD_DIRECT_DISPATCH=0" "MIPGPU_LIB=$PWD/tools/bin/lib_s0.so"}; do
  for calls in 8 32; do
    env $envs timeout -k 10 200 python -u tools/e2e_probe.py --reps 15 --calls $calls 1:dec:pinned:mb=4 > $O/t.jsonl 2> $O/t.err || { echo "FAILED $envs"; tail -3 $O/t.err; continue; }
    python tools/experiments/r06/summ.py 1 1 < $O/t.jsonl | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print('%-40s' % '${envs##*/}', d['calls'], 'median', d['median'], 'p25', d['p25'], 'best', d['best'])"
  done
done
