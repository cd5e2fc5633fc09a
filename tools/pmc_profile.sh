#!/bin/bash
# PMC passes over the search kernel (separate rocprofv3 runs, counters only + kernel trace).
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out}/pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:-"--frames-per-step 128 --steps 3 --warmup 1 --no-cpu-baseline --no-reference-gpu --no-latency --no-end-to-end"}
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  echo "== pass $i: $counters $(date +%T)"
  timeout -k 10 300 rocprofv3 --pmc $counters -d "$OUT/p$i" -o pmc --output-format csv -- \
    python bench.py $ARGS > "$OUT/p$i.log" 2>&1 || { tail -20 "$OUT/p$i.log"; exit 1; }
done <<'LIST'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE
FETCH_SIZE
WRITE_SIZE
SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16 GRBM_GUI_ACTIVE
SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE
LIST
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt" && cat "$OUT/summary.txt"
