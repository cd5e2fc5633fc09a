#!/bin/bash
# Round 6: the six-wave build (tools/bin/lib_s6.so) through the whole GPU suite, then bench lines
# (all legs but the CPU and reference ones) and the small-launch sweep of both builds, same box.
set -uo pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/${OUTTAG:-r06s6full}; mkdir -p $O
L=${S6LIB:-tools/bin/lib_s6.so}
echo "== tests $(date +%T)"
MIPGPU_LIB=$PWD/$L timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for lib in vvc-mip-gpu_amd/lib/libmipgpu.so $L; do
  t=$(basename $lib .so)
  echo "== bench $t $(date +%T)"
  MIPGPU_LIB=$PWD/$lib timeout -k 10 400 python bench.py --no-cpu-baseline --no-reference-gpu --allow-knobs > $O/bench_$t.json 2> $O/bench_$t.err || { tail $O/bench_$t.err; exit 1; }
  python - $O/bench_$t.json <<'P'
import json, sys
d = json.load(open(sys.argv[1]))
f = d.get("filter", {})
print(d["value"], "ms", d["ms_per_step"], "valu", d["valu"]["frac"], d["valu"].get("dual_issue_share"), "single", d.get("single_frame_ms"),
      "dec", d.get("decisions_device", {}).get("value"), "alt", f.get("alt_refs_search", {}).get("value"),
      "e2e", d.get("end_to_end", {}).get("value"), d.get("end_to_end", {}).get("decisions_value"))
P
  echo "== small $t $(date +%T)"
  MIPGPU_LIB=$PWD/$lib SB_CUTS=2 SB_ORDERS=1 SB_SLICES=0 timeout -k 10 300 python -u tools/small_batch.py > $O/small_$t.jsonl 2> $O/small_$t.err || { tail $O/small_$t.err; exit 1; }
  tail -1 $O/small_$t.jsonl
done
