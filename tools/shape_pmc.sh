#!/bin/bash
# Per CU-size-class PMC view of the search kernel (2 dispatches per class, in class order;
# tools/shape_profile.py restricts the search to one class at a time): VALU / LDS / SALU
# instruction counts per frame, VALU issue per SIMD quad-cycle, the dual-issue share
# (SQ_ACTIVE_INST_VALU2) and where waves wait.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out}/shape_pmc
mkdir -p "$OUT"
export TMPDIR=/tmp SHAPE_PROFILE_PMC=1
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE \
  -d "$OUT/raw" -o pmc --output-format csv -- python tools/shape_profile.py "$OUT/times.json" > "$OUT/log.txt" 2>&1 \
  || { tail -20 "$OUT/log.txt"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, json, sys, collections
out = sys.argv[1]
rows = collections.OrderedDict()
for path in glob.glob(out + "/raw/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        if "mip_search" not in r["Kernel_Name"]:
            continue
        rows.setdefault(int(r["Dispatch_Id"]), collections.Counter())[r["Counter_Name"]] += float(r["Counter_Value"])
ids = sorted(rows)
names = [l.split()[0] for l in open(out + "/log.txt") if "us/frame" in l and not l.startswith("all")]
times = json.load(open(out + "/times.json"))
simds = 1024
print("class   us/frame  VALU/frame  LDS/frame  SALU/frame  VALU/quad  dual  active  wait_issue  wait_cnt")
for i, n in enumerate(names + ["all"]):
    d = [rows[k] for k in ids[2 * i:2 * i + 2]]
    if not d: break
    c = d[-1]
    quads = c["GRBM_GUI_ACTIVE"] / 8 / 4 * simds  # GRBM summed over 8 XCDs; SIMD quad-cycles
    wc = max(1.0, c["SQ_WAVE_CYCLES"])
    print("%6s %9s %10.2fM %9.2fM %10.2fM %10.3f %5.3f %7.3f %11.3f %9.3f" % (
        n, times.get(n, {}).get("us_per_frame", "-"), c["SQ_INSTS_VALU"] / 8e6, c["SQ_INSTS_LDS"] / 8e6,
        c["SQ_INSTS_SALU"] / 8e6, c["SQ_INSTS_VALU"] / quads, c["SQ_ACTIVE_INST_VALU2"] / max(1.0, c["SQ_INSTS_VALU"]),
        c["SQ_ACTIVE_INST_ANY"] / wc, c["SQ_WAIT_INST_ANY"] / wc, c["SQ_WAIT_ANY"] / wc))
PY
