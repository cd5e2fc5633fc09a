#!/bin/bash
# Same-box PMC comparison of library builds: tools/ab_pmc.sh lib1.so lib2.so ...
# One rocprofv3 --pmc pass per library (VALU issue / dual issue / wait counters of the search).
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out}/ab_pmc
mkdir -p "$OUT"
export TMPDIR=/tmp
COUNTERS=${COUNTERS:-"SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_LDS GRBM_GUI_ACTIVE"}
for lib in "$@"; do
  name=$(basename "$lib" .so)
  MIPGPU_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc $COUNTERS -d "$OUT/$name" -o pmc --output-format csv -- \
    python bench.py --frames-per-step 32 --steps 3 --warmup 1 --allow-knobs --no-cpu-baseline --no-reference-gpu --no-latency \
    --no-end-to-end --no-filter > "$OUT/$name.log" 2>&1 || { tail -20 "$OUT/$name.log"; exit 1; }
  python3 - "$OUT/$name" "$name" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for path in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if "mip_search_kernel" in r["Kernel_Name"]:
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (d, c), v in per.items():
        acc[c].append(v)
m = {c: sum(v) / len(v) for c, v in acc.items()}
g = m.get("GRBM_GUI_ACTIVE", 0) / 8
print(sys.argv[2], " ".join("%s=%.4g" % (c, v) for c, v in sorted(m.items())))
if g:
    print("   VALU insts/SIMD-cycle %.3f  quad-cycles VALU %.3f of wave-cycles, dual %.3f of VALU quads" % (
        m["SQ_INSTS_VALU"] / (1024 * g), m["SQ_ACTIVE_INST_VALU"] / max(1, m["SQ_WAVE_CYCLES"]),
        m.get("SQ_ACTIVE_INST_VALU2", 0) / max(1, m["SQ_ACTIVE_INST_VALU"])))
PY
done
