set -e
O=${O:-gpurun_out/r05al}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
F5=filterFrame_2d_float_5x5_quarterCtu
for ss in 2 1 2 1; do
  MIPGPU_SEARCH_STREAMS=$ss timeout -k 10 300 python -u tools/e2e_probe.py --reps 5 1:dec:pinned 1:full:pinned 2:dec:pinned:$F5:2 2:full:pinned:$F5:2 4:dec:pinned 128:dec:pinned:mb=384 128:full:pinned:mb=384 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('ss=$ss', d['case'][:24], d['fps'], d['fps_all'])" | tee -a $O/rates.txt
  MIPGPU_SEARCH_STREAMS=$ss timeout -k 10 300 python -u tools/e2e_probe.py --reps 5 --calls 1 --sync 128:dec:pinned:mb=384 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('ss=$ss sync', d['case'][:24], d['fps'], d['fps_all'])" | tee -a $O/rates.txt
done
echo done
