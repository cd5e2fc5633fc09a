set -e
O=gpurun_out/r05ae; mkdir -p $O
F5=filterFrame_2d_float_5x5_quarterCtu
for rt in none torch; do
for v in 12 16 12 16; do
  T=""; [ $rt = torch ] && T="--torch init"
  MIPGPU_RING_PIECES=$v timeout -k 10 200 python -u tools/e2e_probe.py --reps 7 $T 8:full:pageable 2:full:pageable:$F5:2 1:dec:pageable 1:full:pageable 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('$rt $v', d['case'][:24], d['fps'], d['fps_all'])" | tee -a $O/rates.txt
done
done
echo done
