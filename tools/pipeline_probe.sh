#!/bin/bash
# Host-pipeline probe on the GPU box: end-to-end rates of per-frame / small calls
# (tools/e2e_probe.py) and one rocprofv3 kernel + memory-copy trace of the same cases,
# summarised by tools/trace_timeline.py.  usage: OUT=gpurun_out/pipe tools/pipeline_probe.sh [CASE...]
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/pipe}
mkdir -p "$OUT"
export TMPDIR=/tmp
F5=filterFrame_2d_float_5x5_quarterCtu
CASES=("$@")
if [ ${#CASES[@]} -eq 0 ]; then
  CASES=(1:dec:pinned 1:full:pinned 1:dec:pageable 1:full:pageable 2:dec:pinned:$F5:2 2:full:pinned:$F5:2
         2:dec:pageable:$F5:2 2:full:pageable:$F5:2)
fi
echo "== rates $(date +%T)"
timeout -k 10 300 python -u tools/e2e_probe.py "${CASES[@]}" | tee "$OUT/rates.jsonl"
echo "== trace $(date +%T)"
rm -rf /tmp/pipe_trace
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/pipe_trace -o pipe --output-format csv -- \
  python -u tools/e2e_probe.py --reps 1 "${CASES[@]}" > "$OUT/trace_rates.jsonl" 2> "$OUT/trace.err" \
  || { tail -20 "$OUT/trace.err"; exit 1; }
python3 tools/trace_timeline.py /tmp/pipe_trace --last 48 > "$OUT/timeline.txt"
head -c 2000 "$OUT/timeline.txt"
echo "== done $(date +%T)"
