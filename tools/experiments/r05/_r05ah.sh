set -e
O=gpurun_out/r05ah; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "ramped or pipeline or pageable or async or per_frame or chunk" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 0 1 0; do
  MIPGPU_RAMP=$r timeout -k 10 300 python -u tools/e2e_probe.py --reps 5 128:dec:pinned:mb=384 128:full:pinned:mb=384 128:dec:pageable:mb=384 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('ramp=$r 8calls', d['case'][:24], d['fps'], d['fps_all'])" | tee -a $O/rates.txt
  MIPGPU_RAMP=$r timeout -k 10 300 python -u tools/e2e_probe.py --reps 5 --calls 1 128:dec:pinned:mb=384 128:full:pinned:mb=384 64:dec:pinned:mb=64 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('ramp=$r 1call', d['case'][:24], d['fps'], d['fps_all'])" | tee -a $O/rates.txt
done
echo done
