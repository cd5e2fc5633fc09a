set -e
O=gpurun_out/r05w; mkdir -p $O
F5=filterFrame_2d_float_5x5_quarterCtu
C="8:full:pageable 1:dec:pageable 2:full:pageable:$F5:2"
for v in "A=4096" "A=65536" "A=1048576" "L=pieces" "A=4096" "A=1048576" "L=pieces"; do
  lib=vvc-mip-gpu_amd/lib/libmipgpu.so; a=4096
  case $v in A=*) a=${v#A=};; L=pieces) lib=tools/bin/lib_pieces.so;; esac
  MIPGPU_RING_ALIGN=$a MIPGPU_LIB=$PWD/$lib timeout -k 10 300 python -u tools/e2e_probe.py --reps 5 --torch init $C 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin: d=json.loads(l); print('$v', d['case'][:24], d['fps'], d['fps_all'], d['enqueue_ms'][-1], d['wait_ms'][-1])" | tee -a $O/ab.txt
done
echo done
