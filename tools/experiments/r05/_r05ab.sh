set -e
O=gpurun_out/r05ab; mkdir -p $O
export TMPDIR=/tmp
for env in "HSA_ENABLE_SDMA=1" "HSA_ENABLE_SDMA=0" "HSA_FORCE_SDMA_SIZE=0" "X=1"; do
    rm -rf /tmp/tr
    env $env timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/tr -o t --output-format csv -- python -u tools/e2e_probe.py --reps 1 --calls 3 --torch init 1:full:pinned > $O/tr.jsonl 2>/dev/null
    python3 - $env <<'PY' | tee -a $O/copies.txt
import csv,glob,sys
k=sum(1 for f in glob.glob('/tmp/tr/**/*kernel_trace.csv',recursive=True) for r in csv.DictReader(open(f)) if 'copyBuffer' in r['Kernel_Name'])
m=sum(1 for f in glob.glob('/tmp/tr/**/*memory_copy_trace.csv',recursive=True) for r in csv.DictReader(open(f)) if 'DEVICE_TO_HOST' in r.get('Direction',''))
print(sys.argv[1], 'copyBuffer kernels', k, 'SDMA D2H', m)
PY
    env $env timeout -k 10 200 python -u tools/e2e_probe.py --reps 5 --torch init 8:full:pageable 1:full:pinned 2:full:pageable:filterFrame_2d_float_5x5_quarterCtu:2 1:dec:pageable 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('$env', d['hip_runtime'][0].split('/')[-1], d['case'][:24], d['fps'], d['fps_all'])" | tee -a $O/rates.txt
done
echo done
