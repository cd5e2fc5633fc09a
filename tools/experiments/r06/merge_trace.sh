#!/bin/bash
# Round 6: kernel + copy trace of 8 queued merged one-frame decisions-only calls (max_batch 4),
# six-wave default vs four-wave build: per-segment timelines (tools/trace_timeline.py).
set -uo pipefail
cd "$(dirname "$0")/../../.."
export TMPDIR=/tmp
O=gpurun_out/${OUTTAG:-r06mtr}; mkdir -p $O
for lib in vvc-mip-gpu_amd/lib/libmipgpu.so tools/bin/lib_s0.so; do
  t=$(basename $lib .so)
  rm -rf /tmp/tr_$t
  MIPGPU_LIB=$PWD/$lib timeout -k 10 240 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/tr_$t -o tr --output-format csv -- \
    python -u tools/e2e_probe.py --reps 4 --calls 8 1:dec:pinned:mb=4 > $O/$t.jsonl 2> $O/$t.err || { tail $O/$t.err; exit 1; }
  python tools/trace_timeline.py /tmp/tr_$t --last 40 > $O/$t.timeline.txt 2>&1
  echo "## $t"; tail -48 $O/$t.timeline.txt
done
