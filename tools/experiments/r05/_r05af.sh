set -e
O=gpurun_out/r05af; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
F5=filterFrame_2d_float_5x5_quarterCtu
for rt in torch none; do
  NT=""; [ $rt = none ] && NT=1
  MIPGPU_NO_TORCH=$NT timeout -k 10 300 python -u tools/e2e_probe.py --reps 7 1:dec:pinned 1:full:pinned 2:dec:pinned:$F5:2 2:full:pinned:$F5:2 1:dec:pageable 1:full:pageable 2:full:pageable:$F5:2 8:full:pageable 32:full:pageable 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('$rt', d['hip_runtime'], d['case'][:24], d['fps'], d['fps_all'])" | tee -a $O/rates.txt
done
echo done
