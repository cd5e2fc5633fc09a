#!/bin/bash
# tools/dual_census.hip under rocprofv3 PMC at 1 and 4 waves per SIMD: VALU instructions per
# SIMD quad-cycle and the dual-issued share for every instruction form.
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out}/dual_census
mkdir -p "$OUT"
export TMPDIR=/tmp
hipcc --offload-arch=gfx950 -O3 tools/dual_census.hip -o /tmp/dual_census 2>/dev/null
for w in ${WAVES:-1 4}; do
  timeout -s KILL 100 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 GRBM_GUI_ACTIVE -d "$OUT/w$w" -o pmc \
    --output-format csv -- /tmp/dual_census $w > "$OUT/w$w.names" 2>&1
done
WS="${WAVES:-1 4}" python3 - "$OUT" <<'PY'
import csv, glob, os, sys, collections
WS = [int(x) for x in os.environ['WS'].split()]
out = sys.argv[1]
res = {}
for w in WS:
    rows = collections.OrderedDict()
    for p in glob.glob(out + "/w%d/**/*counter_collection.csv" % w, recursive=True):
        for r in csv.DictReader(open(p)):
            rows.setdefault(int(r["Dispatch_Id"]), [r["Kernel_Name"], collections.Counter()])[1][r["Counter_Name"]] += float(r["Counter_Value"])
    for k in sorted(rows):
        n, c = rows[k]
        q = c["GRBM_GUI_ACTIVE"] / 8 / 4 * 1024
        name = n.split("(")[0].replace("probe_", "")
        res.setdefault(name, {})[w] = (c["SQ_INSTS_VALU"] / q, c["SQ_ACTIVE_INST_VALU2"] / max(1, c["SQ_INSTS_VALU"]))
print("%-22s" % "form" + "".join("   %d w/SIMD: VALU/quad dual" % w for w in WS))
for n, v in res.items():
    print("%-22s" % n + "".join("%21.3f %6.3f" % v.get(w, (0, 0)) for w in WS))
PY
