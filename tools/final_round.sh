#!/bin/bash
# One GPU-box pass over the final build of a round, in the order that ties the numbers
# together: parity tests, smoke, the kernel-trace + PMC profiles of the bench's workload
# (tools/profile_round.sh), profiles/traffic.json updated with them (same build ID), then the
# bench line (which reads that traffic.json) and the small-launch sweep.  Stops at the first
# failing step.  usage: OUT=gpurun_out/final tools/final_round.sh
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/final}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
if [ -z "${SKIP_TESTS:-}" ]; then
  step pytest
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1 \
    || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
  tail -2 "$OUT/pytest_gpu.log"
  step smoke
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
  cat "$OUT/smoke.log"
fi
step profile
OUT="$OUT/prof" timeout -k 10 1500 tools/profile_round.sh > "$OUT/profile.log" 2>&1 || { tail -30 "$OUT/profile.log"; exit 1; }
python3 - "$OUT" <<'PY'
import json, sys
out = sys.argv[1]
new = json.load(open(out + "/prof/traffic.json"))
d = json.load(open("profiles/traffic.json"))
d.update(new)
json.dump(d, open("profiles/traffic.json", "w"), indent=1)
json.dump(d, open(out + "/traffic.json", "w"), indent=1)
print("traffic.json:", {k: v.get("build_id") for k, v in new.items()})
PY
step bench
timeout -k 10 900 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
step small_batch
SB_CUTS=2 SB_ORDERS=1 SB_SLICES=0 timeout -k 10 300 python -u tools/small_batch.py > "$OUT/small.jsonl" 2> "$OUT/small.err" \
  || { tail -20 "$OUT/small.err"; exit 1; }
cat "$OUT/small.jsonl"
step done
