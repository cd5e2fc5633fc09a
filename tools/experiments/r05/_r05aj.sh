set -e
O=gpurun_out/r05aj; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "ramped or pipeline or per_frame or chunk or contract" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 up 0 1 up 0; do
  MIPGPU_RAMP=$r timeout -k 10 300 python -u tools/e2e_probe.py --reps 5 --calls 1 --sync 128:dec:pinned:mb=384 64:dec:pinned:mb=64 32:dec:pinned:mb=32 128:full:pinned:mb=384 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('ramp=$r sync', d['case'][:24], d['fps'], d['fps_all'])" | tee -a $O/rates.txt
done
echo done
