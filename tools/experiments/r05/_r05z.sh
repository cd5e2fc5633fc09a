set -e
O=gpurun_out/r05z; mkdir -p $O
F5=filterFrame_2d_float_5x5_quarterCtu
for v in "A notorch" "P notorch" "A torch" "P torch"; do
  set -- $v
  lib=vvc-mip-gpu_amd/lib/libmipgpu.so; [ $1 = P ] && lib=tools/bin/lib_pieces.so
  T=""; [ $2 = torch ] && T="--torch init"
  MIPGPU_STAGE_TRACE=$O/st_$1_$2 MIPGPU_LIB=$PWD/$lib timeout -k 10 300 python -u tools/e2e_probe.py --reps 5 $T 8:full:pageable 2:full:pageable:$F5:2 1:dec:pageable 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('$v', d['case'][:24], d['fps'], d['fps_all'], d['enqueue_ms'][-1], d['wait_ms'][-1])" | tee -a $O/ab.txt
done
echo done
