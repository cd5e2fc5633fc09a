set -e
O=gpurun_out/r05ag; mkdir -p $O
F5=filterFrame_2d_float_5x5_quarterCtu
for rt in torch none; do
 for sy in poll block poll block; do
  NT=""; [ $rt = none ] && NT=1
  MIPGPU_STAGE_SYNC=$sy MIPGPU_NO_TORCH=$NT timeout -k 10 300 python -u tools/e2e_probe.py --reps 7 1:dec:pageable 1:full:pageable 2:full:pageable:$F5:2 8:full:pageable 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('$rt $sy', d['case'][:24], d['fps'], d['fps_all'])" | tee -a $O/rates.txt
 done
done
echo done
