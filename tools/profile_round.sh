#!/bin/bash
# Round profiles of the bench's default workload with bounded output (GPU box):
#   1. rocprofv3 --kernel-trace --stats of the bench command (kernel stats CSV kept);
#   2. separate rocprofv3 --pmc passes over the search / filter kernels
#      (--kernel-include-regex), raw CSVs under /tmp, only summaries kept:
#      traffic.json (tools/traffic_json.py) and the PMC summary (tools/pmc_summary.py).
# Raw traces stay out of gpurun_out (a 384-frame PMC pass writes hundreds of MB of CSV).
# usage: OUT=gpurun_out/prof_r03 tools/profile_round.sh [bench args...]
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out/prof}
RAW=/tmp/prof_raw
rm -rf "$RAW"
mkdir -p "$OUT" "$RAW"
export TMPDIR=/tmp
ARGS="--no-cpu-baseline --no-reference-gpu --no-latency --no-end-to-end $*"
FRAMES=$(python3 -c "import sys; a=sys.argv[1:]; print(a[a.index('--frames-per-step')+1] if '--frames-per-step' in a else 384)" $ARGS)
echo "== kernel trace $(date +%T)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$RAW/trace" -o run --output-format csv -- \
  python3 bench.py --steps 10 $ARGS > "$OUT/trace_bench.json" 2> "$RAW/trace.err" || { tail -20 "$RAW/trace.err"; exit 1; }
find "$RAW/trace" -name "*kernel_stats.csv" -exec cp {} "$OUT/kernel_stats.csv" \;
python3 -c "import sys; sys.path.insert(0, 'vvc-mip-gpu_amd'); import mipgpu; print(mipgpu.build_id())" > "$OUT/build_id.txt"
# the dominant kernel over the bench's timed steps only (kernel_stats.csv averages the warmup
# launches in too), next to the bench line of the same profiled command
python3 - "$RAW/trace" "$OUT" <<'PY' || echo "(timed-launch average unavailable)"
import csv, glob, json, sys
raw, out = sys.argv[1], sys.argv[2]
line = json.loads(open(out + "/trace_bench.json").read().strip().splitlines()[-1])
rows = [r for f in glob.glob(raw + "/**/*kernel_trace.csv", recursive=True) for r in csv.DictReader(open(f))
        if "mip_search_kernel<false, false, true, " in r["Kernel_Name"]]  # (12 waves; 8 before round 6)
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
timed = rows[-line["steps"]:]
dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in timed]
rec = {"kernel": rows[0]["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", ""), "build_id": line["build_id"], "launches": len(rows),
       "timed_launches": len(dur), "timed_avg_ms": round(sum(dur) / len(dur), 4), "timed_min_ms": round(min(dur), 4),
       "timed_max_ms": round(max(dur), 4), "bench_ms_per_step_same_run": line["ms_per_step"],
       "bench_kernel_ms_same_run": line["roofline"]["kernel_ms_per_launch"]}
json.dump(rec, open(out + "/kernel_timed.json", "w"), indent=1)
print(json.dumps(rec))
PY
head -5 "$OUT/kernel_stats.csv"
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  echo "== pmc pass $i: $counters $(date +%T)"
  timeout -s KILL 240 rocprofv3 --pmc $counters --kernel-include-regex "mip_search_kernel|filter_kernel" \
    -d "$RAW/pmc/p$i" -o pmc --output-format csv -- \
    python3 bench.py --steps 3 --warmup 1 $ARGS > "$RAW/p$i.log" 2>&1 || { tail -20 "$RAW/p$i.log"; exit 1; }
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
FETCH_SIZE
WRITE_SIZE
SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE
LIST
python3 tools/pmc_summary.py "$RAW/pmc" > "$OUT/pmc_summary.txt"
python3 tools/traffic_json.py "$RAW/pmc" "1920x1080x$FRAMES" "$OUT/traffic.json"
cat "$OUT/pmc_summary.txt"
rm -rf "$RAW"
echo "== done $(date +%T)"
