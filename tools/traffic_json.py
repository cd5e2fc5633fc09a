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
vals = {"FETCH_SIZE": [], "WRITE_SIZE": []}
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
d = json.load(open(out)) if os.path.exists(out) else {}
d[key] = {"hbm_bytes_per_launch": round(fetch + write), "fetch_bytes_x2": round(fetch), "write_bytes": round(write),
          "dispatches": [len(vals["FETCH_SIZE"]), len(vals["WRITE_SIZE"])],
          "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes (tools/pmc_profile.sh); "
                    "FETCH_SIZE KiB x1024 x2 (gfx950 correction), WRITE_SIZE KiB x1024"}
json.dump(d, open(out, "w"), indent=1)
print(json.dumps(d[key]))
