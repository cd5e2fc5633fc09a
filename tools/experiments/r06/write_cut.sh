#!/bin/bash
# Round 6: HBM write bytes of the search (WRITE_SIZE, 128 frames) against the task cut factor:
# do the extra writes of the six-wave kernel come from cost lines written by two tasks?
set -uo pipefail
cd "$(dirname "$0")/../../.."
export TMPDIR=/tmp
B="--frames-per-step 128 --steps 3 --warmup 1 --no-cpu-baseline --no-reference-gpu --no-latency --no-end-to-end --no-filter --allow-knobs"
for cf in 2 1.33 1; do
  rm -rf /tmp/wc_$cf
  MIPGPU_CUT_FACTOR=$cf timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d /tmp/wc_$cf -o pmc --output-format csv -- python bench.py $B > /tmp/wc_$cf.log 2>&1 || { tail /tmp/wc_$cf.log; exit 1; }
  python - $cf <<'P'
import csv, glob, sys
cf = sys.argv[1]
per = {}
for p in glob.glob("/tmp/wc_%s/**/*counter_collection.csv" % cf, recursive=True):
    for r in csv.DictReader(open(p)):
        if "mip_search_kernel<false, false, true" in r["Kernel_Name"]:
            per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
v = sorted(per.values())
print("cut", cf, "WRITE GB per 128-frame launch", [round(x * 1024 / 1e9, 3) for x in v], "cost rows", round(128 * 135 * 97840 * 4 / 1e9, 3))
P
done
