#!/bin/bash
# Round 6: kernel + copy traces of queued one-frame calls, merged and not (why 8 merged calls
# ran slower than unmerged ones, and why 32 unmerged calls enqueue slowly).
set -uo pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06c; mkdir -p $O
export TMPDIR=/tmp
i=0
for spec in "1 8 1:dec:pinned:mb=8" "0 8 1:dec:pinned:mb=8" "0 32 1:dec:pinned:mb=4" "1 32 1:dec:pinned:mb=4"; do
  set -- $spec
  i=$((i+1))
  rm -rf /tmp/tr$i
  MIPGPU_MERGE=$1 timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/tr$i -o t --output-format csv -- python -u tools/e2e_probe.py --reps 2 --calls $2 $3 > $O/probe_$i.jsonl 2>$O/probe_$i.err || { tail $O/probe_$i.err; exit 1; }
  python tools/trace_timeline.py /tmp/tr$i --last 120 > $O/timeline_$i.txt
  echo "== $spec"; cat $O/probe_$i.jsonl | cut -c1-400; head -3 $O/timeline_$i.txt
done
