#!/bin/bash
# VALU / LDS instruction counts per CU-size class (2 search dispatches per class, in order).
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out}/shape_pmc
mkdir -p "$OUT"
export TMPDIR=/tmp SHAPE_PROFILE_PMC=1
timeout -k 10 400 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES \
  -d "$OUT/raw" -o pmc --output-format csv -- python tools/shape_profile.py "$OUT/times.json" > "$OUT/log.txt" 2>&1 \
  || { tail -20 "$OUT/log.txt"; exit 1; }
python3 - "$OUT" <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
rows = collections.OrderedDict()
for path in glob.glob(out + "/raw/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(path)):
        if "mip_search" not in r["Kernel_Name"]:
            continue
        rows.setdefault(int(r["Dispatch_Id"]), collections.Counter())[r["Counter_Name"]] += float(r["Counter_Value"])
ids = sorted(rows)
names = [l.split()[0] for l in open(out + "/log.txt") if "us/frame" in l and not l.startswith("all")]
for i, n in enumerate(names + ["all"]):
    d = [rows[k] for k in ids[2 * i:2 * i + 2]]
    if not d: break
    c = d[-1]
    print("%6s VALU/frame %8.2fM  LDS/frame %6.2fM  SALU %6.2fM  waves %6d" % (
        n, c["SQ_INSTS_VALU"] / 8e6, c["SQ_INSTS_LDS"] / 8e6, c["SQ_INSTS_SALU"] / 8e6, c["SQ_WAVES"]))
PY
