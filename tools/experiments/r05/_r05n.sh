set -e
F5=filterFrame_2d_float_5x5_quarterCtu
for v in "--torch init --torch-after stream" "--torch init --device-first 5" "--torch init --torch-after stream --device-first 5"; do
  timeout -k 10 200 python -u tools/e2e_probe.py --reps 4 $v 2:full:pinned:$F5:2 1:full:pinned 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('$v', d['case'][:16], d['fps'], d['fps_all'])"
done
