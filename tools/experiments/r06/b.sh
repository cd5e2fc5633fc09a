#!/bin/bash
# Round 6, first GPU call: merged launches (new tests + the host-pipeline tests), the whole
# GPU suite, then per-frame call rates with and without merging.
set -uo pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06b; mkdir -p $O
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_parity.py -m gpu -k "merged or idle_call or per_frame or async or pipeline or dropped" > $O/t_new.txt 2>&1 || { tail -30 $O/t_new.txt; exit 1; }
tail -3 $O/t_new.txt
timeout -k 10 900 $T tests -m gpu > $O/t_all.txt 2>&1 || { tail -30 $O/t_all.txt; exit 1; }
tail -3 $O/t_all.txt
P="timeout -k 10 300 python -u tools/e2e_probe.py --reps 7"
for calls in 8 32; do
  for m in 1 0; do
    MIPGPU_MERGE=$m $P --calls $calls 1:dec:pinned:mb=4 1:dec:pinned:mb=8 1:dec:pinned:mb=16 1:full:pinned:mb=4 2:dec:pinned:filterFrame_2d_float_5x5_quarterCtu:2:mb=8 > $O/rates_c${calls}_m$m.jsonl 2>$O/rates_c${calls}_m$m.err || exit 1
  done
done
python - <<'P'
import json,glob
for f in sorted(glob.glob("gpurun_out/r06b/rates_*.jsonl")):
    for l in open(f):
        d=json.loads(l); print(f.split("/")[-1], d["case"], d["calls"], d["fps"], d["fps_all"], d.get("host_stats"))
P
echo "== bench --gpus 2 rehearsal (e2e aggregate)"
timeout -k 10 400 python bench.py --gpus 2 --frames-per-step 32 --steps 5 --warmup 1 --no-cpu-baseline --no-reference-gpu --no-latency --no-filter > $O/bench2.json 2> $O/bench2.err || { tail -20 $O/bench2.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench2.json').read().strip().splitlines()[-1]);print(d['value'], d['numa'], json.dumps(d['end_to_end']))"
