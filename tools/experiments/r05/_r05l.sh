set -e
for v in "none:" "stream:" "stream:high" "stream:low" "stream:hwq8"; do
  t=${v%%:*}; p=${v#*:}
  a=""; [ $t != none ] && a="--torch $t"
  E=""; case $p in high|low) E="MIPGPU_STREAM_PRIO=$p";; hwq8) E="GPU_MAX_HW_QUEUES=8";; esac
  env $E timeout -k 10 200 python -u tools/e2e_probe.py --reps 3 $a 1:full:pinned 2:full:pinned:filterFrame_2d_float_5x5_quarterCtu:2 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('$v', d['case'][:12], d['fps'], d['fps_all'])"
done
