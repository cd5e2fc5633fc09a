#!/bin/bash
# Per CU-size-class PMC view of the search kernel (2 dispatches per class, in class order;
# tools/shape_profile.py restricts the search to one class at a time): VALU / LDS / SALU
# instruction counts per frame, VALU issue per SIMD quad-cycle, the dual-issue share
# (SQ_ACTIVE_INST_VALU2), where waves wait, and (second pass) HBM write bytes per cost-table byte.
# MIPGPU_LIB selects a library build (A/B of variants).
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out}/shape_pmc
mkdir -p "$OUT"
export TMPDIR=/tmp SHAPE_PROFILE_PMC=1
rm -rf /tmp/shape_raw
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
  SQ_ACTIVE_INST_ANY SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE \
  -d /tmp/shape_raw/sq -o pmc --output-format csv -- python tools/shape_profile.py "$OUT/times.json" > "$OUT/log.txt" 2>&1 \
  || { tail -20 "$OUT/log.txt"; exit 1; }
# second pass: HBM write bytes per class (WRITE_SIZE, KiB) against the class's cost-table bytes
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE -d /tmp/shape_raw/wr -o pmc --output-format csv -- \
  python tools/shape_profile.py /dev/null > "$OUT/log_wr.txt" 2>&1 || { tail -20 "$OUT/log_wr.txt"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, json, sys, collections
sys.path.insert(0, "vvc-mip-gpu_amd")
from mipgpu import layout
out = sys.argv[1]
def load(d):
    rows = collections.OrderedDict()
    for path in glob.glob("/tmp/shape_raw/%s/**/*counter_collection.csv" % d, recursive=True):
        for r in csv.DictReader(open(path)):
            if "mip_search" not in r["Kernel_Name"]:
                continue
            rows.setdefault(int(r["Dispatch_Id"]), collections.Counter())[r["Counter_Name"]] += float(r["Counter_Value"])
    return rows
rows, wrows = load("sq"), load("wr")
ids, wids = sorted(rows), sorted(wrows)
names = [l.split()[0] for l in open(out + "/log.txt") if "us/frame" in l and not l.startswith("all")]
times = json.load(open(out + "/times.json"))
simds = 1024
nct = layout.num_ctus(1920, 1080)
print("class   us/frame  VALU/frame  LDS/frame  SALU/frame  VALU/quad  dual  active  wait_issue  wait_cnt  write/table")
for i, n in enumerate(names + ["all"]):
    d = [rows[k] for k in ids[2 * i:2 * i + 2]]
    if not d: break
    c = d[-1]
    wr = wrows[wids[2 * i + 1]]["WRITE_SIZE"] * 1024 if len(wids) > 2 * i + 1 else float("nan")
    if n == "all":
        table = layout.COSTS_PER_CTU * 4 * nct * 8
    else:
        w, h = map(int, n.split("x"))
        table = sum(s.ncu * s.total_modes for s in layout.SHAPES if (s.w, s.h) == (w, h)) * 4 * nct * 8
    quads = c["GRBM_GUI_ACTIVE"] / 8 / 4 * simds  # GRBM summed over 8 XCDs; SIMD quad-cycles
    wc = max(1.0, c["SQ_WAVE_CYCLES"])
    print("%6s %9s %10.2fM %9.2fM %10.2fM %10.3f %5.3f %7.3f %11.3f %9.3f %12.3f" % (
        n, times.get(n, {}).get("us_per_frame", "-"), c["SQ_INSTS_VALU"] / 8e6, c["SQ_INSTS_LDS"] / 8e6,
        c["SQ_INSTS_SALU"] / 8e6, c["SQ_INSTS_VALU"] / quads, c["SQ_ACTIVE_INST_VALU2"] / max(1.0, c["SQ_INSTS_VALU"]),
        c["SQ_ACTIVE_INST_ANY"] / wc, c["SQ_WAIT_INST_ANY"] / wc, c["SQ_WAIT_ANY"] / wc, wr / table))
PY
