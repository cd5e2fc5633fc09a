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
COUNTERS = ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU", "GRBM_GUI_ACTIVE", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE",
            "SQ_INSTS_MFMA", "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_VALU_MFMA_MOPS_F16", "SQ_ACTIVE_INST_VALU2")
# original-reference search with the prefetch (the bench `value`): 12 waves since round 6 (8 before)
SEARCH = "mip_search_kernel<false, false, true, "
FILTER = "filter_kernel<2, true, false>"    # BASELINE configs[2] filter (bench `filter`)


def collect(kernel):
    vals = {c: [] for c in COUNTERS}
    vals["_name"] = set()
    for path in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
        per = {}
        for r in csv.DictReader(open(path)):
            if kernel not in r["Kernel_Name"] or r["Counter_Name"] not in vals:
                continue
            vals["_name"].add(r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
                              .replace("void ", "").replace("mipgpu::", ""))
            k = (r["Dispatch_Id"], r["Counter_Name"])
            per[k] = per.get(k, 0.0) + float(r["Counter_Value"])
        for (_, c), v in per.items():
            vals[c].append(v)
    return vals


def mean(vals, c):
    return sum(vals[c]) / len(vals[c]) if vals[c] else None


def traffic(vals):
    fetch, write = mean(vals, "FETCH_SIZE"), mean(vals, "WRITE_SIZE")
    if fetch is None or write is None:
        return None
    fetch, write = 2 * 1024 * fetch, 1024 * write
    return {"hbm_bytes_per_launch": round(fetch + write), "fetch_bytes_x2": round(fetch), "write_bytes": round(write),
            "dispatches": [len(vals["FETCH_SIZE"]), len(vals["WRITE_SIZE"])]}


s_vals = collect(SEARCH)
rec = traffic(s_vals) or {}
valu, grbm = mean(s_vals, "SQ_INSTS_VALU"), mean(s_vals, "GRBM_GUI_ACTIVE")
# GRBM_GUI_ACTIVE is summed over the 8 XCDs.  A SIMD issues one VALU instruction per
# quad-cycle (4 clocks), or two when both are dual-issue eligible (simple VOP1/VOP2 forms
# from two waves, SQ_ACTIVE_INST_VALU2; tools/dual_census.sh): issue rate = VALU
# instructions per SIMD quad-cycle over the 1024 SIMDs.
util = valu * 4 / (1024 * grbm / 8) if valu and grbm else None
dual = mean(s_vals, "SQ_ACTIVE_INST_VALU2")
conf, lds = mean(s_vals, "SQ_LDS_BANK_CONFLICT"), mean(s_vals, "SQ_LDS_IDX_ACTIVE")
rec.update({"kernel": ", ".join(sorted(s_vals["_name"])) or SEARCH, "valu_insts_per_launch": valu, "gui_active_cycles_per_xcd": grbm and grbm / 8,
            "valu_issue_utilization": util and round(util, 4),
            "valu_insts_per_simd_quad_cycle": util and round(util, 4),
            "valu_dual_issue_share": dual and valu and round(dual / valu, 4),
            "lds_bank_conflict_frac": conf and lds and round(conf / lds, 4),
            "method": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes (tools/pmc_profile.sh); "
                      "FETCH_SIZE KiB x1024 x2 (gfx950 correction), WRITE_SIZE KiB x1024"})
# Matrix cores (phase A of the search): MFMA instructions, busy cycles summed over the
# 1024 SIMDs, and f16 MOPs (x512 = flops, as rocprofv3's MfmaFlopsF16 derives them).
mfma, busy, mops = mean(s_vals, "SQ_INSTS_MFMA"), mean(s_vals, "SQ_VALU_MFMA_BUSY_CYCLES"), \
    mean(s_vals, "SQ_INSTS_VALU_MFMA_MOPS_F16")
if mfma is not None:
    rec.update({"mfma_insts_per_launch": mfma, "mfma_f16_flops_per_launch": mops and mops * 512,
                "mfma_busy_utilization": busy and grbm and round(busy / (1024 * grbm / 8), 4)})
f = traffic(collect(FILTER))
if f:
    f["kernel"] = FILTER
    rec["filter"] = f
# the library build the passes profiled (bench.py accepts PMC data only from the same build)
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "vvc-mip-gpu_amd"))
import mipgpu  # noqa: E402
rec["build_id"] = mipgpu.build_id()
d = json.load(open(out)) if os.path.exists(out) else {}
d[key] = rec
json.dump(d, open(out, "w"), indent=1)
print(json.dumps(d[key]))
