set -e
O=gpurun_out/r05ac; mkdir -p $O
export TMPDIR=/tmp
MIPGPU_D2H_KIND=nocu timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "pipeline or pageable or async or per_frame or triple or stress or ticket" > $O/pytest_nocu.log 2>&1 || { tail -30 $O/pytest_nocu.log; exit 1; }
tail -1 $O/pytest_nocu.log
for rt in torch none; do
  for kind in nocu d2h; do
    T=""; [ $rt = torch ] && T="--torch init"
    rm -rf /tmp/tr
    MIPGPU_D2H_KIND=$kind timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/tr -o t --output-format csv -- python -u tools/e2e_probe.py --reps 1 --calls 3 $T 1:full:pinned > /dev/null 2>&1
    python3 - $rt $kind <<'PY' | tee -a $O/copies.txt
import csv,glob,sys
k=sum(1 for f in glob.glob('/tmp/tr/**/*kernel_trace.csv',recursive=True) for r in csv.DictReader(open(f)) if 'copyBuffer' in r['Kernel_Name'])
m=[r.get('Direction','') for f in glob.glob('/tmp/tr/**/*memory_copy_trace.csv',recursive=True) for r in csv.DictReader(open(f))]
print(sys.argv[1], sys.argv[2], 'copyBuffer kernels', k, 'SDMA copies', len(m), sorted(set(m)))
PY
    MIPGPU_D2H_KIND=$kind timeout -k 10 200 python -u tools/e2e_probe.py --reps 5 $T 8:full:pageable 1:full:pinned 2:full:pageable:filterFrame_2d_float_5x5_quarterCtu:2 2:full:pinned:filterFrame_2d_float_5x5_quarterCtu:2 1:dec:pageable 32:full:pinned 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('$rt $kind', d['hip_runtime'][0].split('/')[-1], d['case'][:24], d['fps'], d['fps_all'])" | tee -a $O/rates.txt
  done
done
echo done
