#!/bin/bash
# Round 6: cache-policy bits of the cost-row stores (MIP_COST_STORE_AUX: 0 default, 1 sc0,
# 2 nt, 3 sc0 nt): 384-frame search rate (two alternating reps) and HBM writes per 128-frame
# launch (WRITE_SIZE).
set -uo pipefail
cd "$(dirname "$0")/../../.."
export TMPDIR=/tmp
A="--frames-per-step 384 --steps 20 --warmup 3 --no-cpu-baseline --no-reference-gpu --no-latency --no-filter --no-end-to-end --allow-knobs"
B="--frames-per-step 128 --steps 3 --warmup 1 --no-cpu-baseline --no-reference-gpu --no-latency --no-end-to-end --no-filter --allow-knobs"
LIBS="vvc-mip-gpu_amd/lib/libmipgpu.so tools/bin/lib_aux1.so tools/bin/lib_aux2.so tools/bin/lib_aux3.so"
for r in 1 2; do
  for lib in $LIBS; do
    MIPGPU_LIB=$PWD/$lib timeout -k 10 200 python bench.py $A 2>/tmp/ab.err | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$(basename $lib)', d['value'], d['roofline']['kernel_ms_per_launch'])" || { tail /tmp/ab.err; exit 1; }
  done
done
for lib in $LIBS; do
  t=$(basename $lib .so); rm -rf /tmp/wa_$t
  MIPGPU_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d /tmp/wa_$t -o pmc --output-format csv -- python bench.py $B > /tmp/wa_$t.log 2>&1 || { tail /tmp/wa_$t.log; exit 1; }
  python - $t <<'P'
import csv, glob, sys
t = sys.argv[1]
per = {}
for p in glob.glob("/tmp/wa_%s/**/*counter_collection.csv" % t, recursive=True):
    for r in csv.DictReader(open(p)):
        if "mip_search_kernel<false, false, true" in r["Kernel_Name"]:
            per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
print(t, "WRITE GB per 128-frame launch", sorted(round(x * 1024 / 1e9, 3) for x in per.values()))
P
done
