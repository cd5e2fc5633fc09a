#!/bin/bash
# End-to-end timing of the CLI (the reference's process surface): N synthetic 1080p frames as
# CSV (the reference's input format) and as raw u16, searched with the reference flags; the
# cost log of frame 0 (13.2 M rows, the reference's default) and optionally per-CU decisions
# of every frame.  Prints wall times and the CLI's own "Elapsed time" line.  GPU box.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out}/cli_bench
N=${N:-16}
mkdir -p "$OUT"
python3 - "$OUT" "$N" <<'PY'
import sys, numpy as np
sys.path.insert(0, "vvc-mip-gpu_amd")
from mipgpu.synth import synth_frames
out, n = sys.argv[1], int(sys.argv[2])
fr = synth_frames(1920, 1080, n, 0x1080, 0)
fr.astype("<u2").tofile(out + "/in.u16")
with open(out + "/in.csv", "w") as f:
    for frame in fr:
        f.write("\n".join(",".join(map(str, row)) for row in frame.tolist()))
        f.write("\n")
PY
CLI=vvc-mip-gpu_amd/bin/mipgpu_cli
run() {
  local name=$1; shift
  local t0=$(date +%s%N)
  timeout -k 10 300 $CLI -s 1920x1080 -f "$N" "$@" > "$OUT/$name.log" 2>&1
  local t1=$(date +%s%N)
  printf "%-16s wall %6d ms  %s\n" "$name" "$(( (t1 - t0) / 1000000 ))" "$(grep -o 'distortion ([0-9]*x), [0-9]*' "$OUT/$name.log")"
}
ls -la "$OUT"/in.csv "$OUT"/in.u16 | awk '{print $5, $9}'
run csv_log0            -o "$OUT/in.csv" -l "$OUT/o1"
run u16_log0            -o "$OUT/in.u16" --InputFormat u16 -l "$OUT/o2"
run csv_nolog           -o "$OUT/in.csv"
run u16_nolog           -o "$OUT/in.u16" --InputFormat u16
run u16_best_all        -o "$OUT/in.u16" --InputFormat u16 --BestModes "$OUT/best.csv"
ls -la "$OUT"/o1.csv "$OUT"/best.csv | awk '{print $5, $9}'
cmp "$OUT/o1.csv" "$OUT/o2.csv" && echo "logs identical (csv vs u16 input)"
rm -f "$OUT"/in.csv "$OUT"/in.u16 "$OUT"/o1.csv "$OUT"/o2.csv "$OUT"/best.csv
