#!/bin/bash
# LDS bank conflicts per CU-size class (one rocprofv3 --pmc pass over tools/shape_profile.py,
# which restricts the search to one class at a time, 2 dispatches per class): conflict cycles,
# LDS-array cycles, LDS instructions, LDS waits, VALU per 1080p frame.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out}/shape_lds
mkdir -p "$OUT"
export TMPDIR=/tmp SHAPE_PROFILE_PMC=1
rm -rf /tmp/shape_lds_raw
timeout -s KILL 400 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU \
  SQ_WAVE_CYCLES GRBM_GUI_ACTIVE -d /tmp/shape_lds_raw -o pmc --output-format csv -- \
  python tools/shape_profile.py "$OUT/times.json" > "$OUT/log.txt" 2>&1 || { tail -20 "$OUT/log.txt"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
rows = collections.OrderedDict()
for path in glob.glob("/tmp/shape_lds_raw/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        if "mip_search" in r["Kernel_Name"]:
            rows.setdefault(int(r["Dispatch_Id"]), collections.Counter())[r["Counter_Name"]] += float(r["Counter_Value"])
ids = sorted(rows)
names = [l.split()[0] for l in open(out + "/log.txt") if "us/frame" in l and not l.startswith("all")]
print("class   conflict/frame  lds_cycles/frame  conflict_frac  LDS_insts/frame  lds_wait/wave_cycles  VALU/frame")
for i, n in enumerate(names + ["all"]):
    d = [rows[k] for k in ids[2 * i:2 * i + 2]]
    if not d:
        break
    c = d[-1]
    print("%6s %14.2fM %16.2fM %14.3f %15.2fM %21.3f %10.2fM" % (
        n, c["SQ_LDS_BANK_CONFLICT"] / 8e6, c["SQ_LDS_IDX_ACTIVE"] / 8e6,
        c["SQ_LDS_BANK_CONFLICT"] / max(1.0, c["SQ_LDS_IDX_ACTIVE"]), c["SQ_INSTS_LDS"] / 8e6,
        c["SQ_WAIT_INST_LDS"] / max(1.0, c["SQ_WAVE_CYCLES"]), c["SQ_INSTS_VALU"] / 8e6))
PY
