set -e
O=gpurun_out/r05m; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
F5=filterFrame_2d_float_5x5_quarterCtu
for t in none stream; do
  a=""; [ $t != none ] && a="--torch $t"
  timeout -k 10 200 python -u tools/e2e_probe.py --reps 5 $a 1:dec:pinned 1:full:pinned 2:dec:pinned:$F5:2 2:full:pinned:$F5:2 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('$t', d['case'][:16], d['fps'], d['fps_all'])" | tee -a $O/rates.txt
done
OUT=$O timeout -k 10 900 tools/config_sweep.sh > $O/sweep.log 2>&1 || { tail -20 $O/sweep.log; exit 1; }
python3 - <<PY
import json
for l in open("$O/configs.jsonl"):
    d=json.loads(l); c=d['config']; e=d.get('end_to_end',{})
    print(c['width'],c['height'],c['frames_per_step'],'alt' if 'alternative' in c['workload'] else 'orig', d['value'], 'e2e', e.get('value'), e.get('pageable_value'), e.get('decisions_value'))
PY
echo done
