set -e
O=gpurun_out/r05aa; mkdir -p $O
export TMPDIR=/tmp
for rt in torch none; do
  for pr in high normal; do
    T=""; [ $rt = torch ] && T="--torch init"
    rm -rf /tmp/tr
    MIPGPU_STREAM_PRIO=$pr timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/tr -o t --output-format csv -- python -u tools/e2e_probe.py --reps 1 --calls 3 $T 1:full:pinned > $O/tr_${rt}_$pr.jsonl 2>/dev/null
    python3 - $rt $pr <<'PY' | tee -a $O/copies.txt
import csv,glob,sys
k=sum(1 for f in glob.glob('/tmp/tr/**/*kernel_trace.csv',recursive=True) for r in csv.DictReader(open(f)) if 'copyBuffer' in r['Kernel_Name'])
m=sum(1 for f in glob.glob('/tmp/tr/**/*memory_copy_trace.csv',recursive=True) for r in csv.DictReader(open(f)) if 'DEVICE_TO_HOST' in r.get('Direction',''))
print(sys.argv[1], sys.argv[2], 'copyBuffer kernels', k, 'SDMA D2H', m)
PY
    MIPGPU_STREAM_PRIO=$pr timeout -k 10 200 python -u tools/e2e_probe.py --reps 5 $T 8:full:pageable 1:full:pinned 2:full:pinned:filterFrame_2d_float_5x5_quarterCtu:2 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('$rt $pr', d['hip_runtime'][0].split('/')[-1], d['case'][:24], d['fps'], d['fps_all'])" | tee -a $O/rates.txt
  done
done
echo done
