set -e
O=gpurun_out/r05ad; mkdir -p $O
F5=filterFrame_2d_float_5x5_quarterCtu
for v in 8 10 12 16 8 10 12 16; do
  MIPGPU_STAGE_TRACE=$O/st_$v MIPGPU_RING_PIECES=$v timeout -k 10 200 python -u tools/e2e_probe.py --reps 5 --torch init 8:full:pageable 2:full:pageable:$F5:2 1:dec:pageable 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('$v', d['case'][:24], d['fps'], d['fps_all'])" | tee -a $O/rates.txt
done
echo done
