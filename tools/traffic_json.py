#!/usr/bin/env python3
"""Per-launch HBM traffic of the search kernel from rocprofv3 --pmc passes (tools/pmc_profile.sh).

FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  MI355X_MICROARCH.md (HBM / rocprofv3):
on gfx950 FETCH_SIZE counts half the bytes of wide coalesced reads -> doubled here;
WRITE_SIZE is taken as is.  Usage: traffic_json.py PMC_DIR KEY OUT_JSON  (KEY = WxHxFRAMES).
"""
import csv
import glob
import json
import os
import sys

root, key, out = sys.argv[1], sys.argv[2], sys.argv[3]
vals = {"FETCH_SIZE": [], "WRITE_SIZE": [], "SQ_INSTS_VALU": [], "GRBM_GUI_ACTIVE": [], "SQ_LDS_BANK_CONFLICT": [],
        "SQ_LDS_IDX_ACTIVE": []}
for path in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
    per = {}
    for r in csv.DictReader(open(path)):
        if "mip_search_kernel" not in r["Kernel_Name"] or r["Counter_Name"] not in vals:
            continue
        k = (r["Dispatch_Id"], r["Counter_Name"])
        per[k] = per.get(k, 0.0) + float(r["Counter_Value"])
    for (_, c), v in per.items():
        vals[c].append(v)
fetch = 2 * 1024 * sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"])
write = 1024 * sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"])
mean = lambda c: sum(vals[c]) / len(vals[c]) if vals[c] else None
valu, grbm = mean("SQ_INSTS_VALU"), mean("GRBM_GUI_ACTIVE")
# GRBM_GUI_ACTIVE is summed over the 8 XCDs; a wave64 VALU instruction issues in 4 cycles on
# one of the 1024 SIMDs (MI355X_MICROARCH.md).
util = valu * 4 / (1024 * grbm / 8) if valu and grbm else None
d = json.load(open(out)) if os.path.exists(out) else {}
d[key] = {"hbm_bytes_per_launch": round(fetch + write), "fetch_bytes_x2": round(fetch), "write_bytes": round(write),
          "dispatches": [len(vals["FETCH_SIZE"]), len(vals["WRITE_SIZE"])],
          "valu_insts_per_launch": valu, "gui_active_cycles_per_xcd": grbm and grbm / 8,
          "valu_issue_utilization": util and round(util, 4),
          "lds_bank_conflict_frac": mean("SQ_LDS_BANK_CONFLICT") and round(mean("SQ_LDS_BANK_CONFLICT") / mean("SQ_LDS_IDX_ACTIVE"), 4),
          "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes (tools/pmc_profile.sh); "
                    "FETCH_SIZE KiB x1024 x2 (gfx950 correction), WRITE_SIZE KiB x1024"}
json.dump(d, open(out, "w"), indent=1)
print(json.dumps(d[key]))
