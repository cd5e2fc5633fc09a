#!/bin/bash
# One GPU-box pass: parity tests, smoke, bench, kernel-trace profile.  Every GPU step has
# its own time limit and the chain stops at the first failure.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out}
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "== $1 $(date +%T)"; }
if [ -z "${SKIP_TESTS:-}" ]; then
step pytest
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread ${PYTEST_ARGS:-} > "$OUT/pytest_gpu.log" 2>&1 || { tail -40 "$OUT/pytest_gpu.log"; exit 1; }
tail -3 "$OUT/pytest_gpu.log"
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { cat "$OUT/smoke.log"; exit 1; }
cat "$OUT/smoke.log"
fi
step ref_runner
timeout -k 10 300 oracle/_ref/ref_runner --bins oracle/_ref --width 1920 --height 1080 --frames 4 --synth 0:1080 --reps 2 > "$OUT/ref_timing.json" 2>&1 || { cat "$OUT/ref_timing.json"; exit 1; }
cat "$OUT/ref_timing.json"
step bench
timeout -k 10 600 python bench.py ${BENCH_ARGS:-} > "$OUT/bench.json" 2> "$OUT/bench.err" || { tail -20 "$OUT/bench.err"; exit 1; }
cat "$OUT/bench.json"
[ -n "${SKIP_PROF:-}" ] && { step done; exit 0; }
step rocprof
rm -rf "$OUT/prof"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- \
  python bench.py --no-cpu-baseline --no-reference-gpu --no-latency --no-end-to-end --steps 10 > "$OUT/prof_bench.json" 2> "$OUT/prof.err" \
  || { tail -20 "$OUT/prof.err"; exit 1; }
find "$OUT/prof" -name "*stats*" | head
step done
