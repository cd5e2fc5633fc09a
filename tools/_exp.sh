set -e
cd /root/repo
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 -L > gpurun_out/avail.txt 2>&1 || true
grep -i "icache\|SQC_" gpurun_out/avail.txt | head -40
timeout -s KILL 120 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE -d gpurun_out/ic -o pmc --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-reference-gpu --no-latency --no-filter --no-end-to-end > gpurun_out/ic.log 2>&1 || { tail -5 gpurun_out/ic.log; exit 1; }
python - <<'PY'
import csv,glob,collections
per=collections.defaultdict(float)
for p in glob.glob("gpurun_out/ic/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(p)):
        if "mip_search" in r["Kernel_Name"]:
            per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
agg=collections.defaultdict(list)
for (d,c),v in per.items(): agg[c].append(v)
print({c: sum(v)/len(v) for c,v in agg.items()})
PY
