#!/bin/bash
# Round 6: HIP runtime settings vs the host stalls of 32 queued one-frame calls.
set -uo pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/${OUTTAG:-r06f}; mkdir -p $O
i=0
ENVS=${ENVS:-"X=1|MIPGPU_NO_TORCH=1|DEBUG_CLR_BATCH_CPU_SYNC_SIZE=4096|DEBUG_CLR_MAX_BATCH_SIZE=4096|AMD_DIRECT_DISPATCH=0|HIP_FORCE_DEV_KERNARG=1"}
CALLS=${CALLS:-32}
IFS='|' read -ra LIST <<< "$ENVS"
for envs in "${LIST[@]}"; do
  for m in 0 1; do
    i=$((i+1))
    env $envs MIPGPU_SLOW_CALLS=0.5 MIPGPU_MERGE=$m timeout -k 10 120 python -u tools/e2e_probe.py --reps 3 --calls $CALLS 1:dec:pinned:mb=4 > $O/$i.jsonl 2> $O/$i.err || { echo "FAILED $envs"; tail -3 $O/$i.err; continue; }
    python - "$O/$i.jsonl" "$O/$i.err" "$envs m=$m" <<'P'
import json, sys, re
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
slow = [float(m.group(1)) for m in re.finditer(r"slow call: ([0-9.]+) ms (?!hipHost)", open(sys.argv[2]).read())]
print("%-60s fps %7.1f %s  slow calls %d max %.1f ms" % (sys.argv[3], d["fps"], d["fps_all"], len(slow), max(slow or [0])))
P
  done
done
