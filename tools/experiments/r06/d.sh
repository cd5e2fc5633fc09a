#!/bin/bash
# Round 6: is the host blocked by the HIP runtime's signal pool / AQL queue when many one-frame
# calls are queued?  Same probe under ROC_SIGNAL_POOL_SIZE / ROC_AQL_QUEUE_SIZE.
set -uo pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06d; mkdir -p $O
for envs in "X=1" "ROC_SIGNAL_POOL_SIZE=1024" "ROC_AQL_QUEUE_SIZE=65536" "ROC_SIGNAL_POOL_SIZE=1024 ROC_AQL_QUEUE_SIZE=65536"; do
  for m in 0 1; do
    tag=$(echo "$envs" | tr ' =' '__')_m$m
    env $envs MIPGPU_MERGE=$m timeout -k 10 200 python -u tools/e2e_probe.py --reps 5 --calls 32 1:dec:pinned:mb=4 1:full:pinned:mb=4 > $O/$tag.jsonl 2> $O/$tag.err || { tail $O/$tag.err; exit 1; }
    env $envs MIPGPU_MERGE=$m timeout -k 10 200 python -u tools/e2e_probe.py --reps 5 --calls 8 1:dec:pinned:mb=4 >> $O/$tag.jsonl 2>> $O/$tag.err || { tail $O/$tag.err; exit 1; }
  done
done
python - <<'P'
import json,glob
for f in sorted(glob.glob("gpurun_out/r06d/*.jsonl")):
    for l in open(f):
        d=json.loads(l); print(f.split("/")[-1][:-6], d["case"], d["calls"], d["fps"], "enq", d["enqueue_ms"][-2:], "calls_us", d["last_round_call_us"][:40])
P
