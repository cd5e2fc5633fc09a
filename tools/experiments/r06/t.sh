#!/bin/bash
# Round 6: filter kernel variants (threads per tile) -- parity of each, then all eight filters
# at 384 x 1080p (KernelIdx 2 for the 5x5 ones as bench.py) against the streaming copy.
set -uo pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06t; mkdir -p $O
for v in default f64 f64x2 f256; do
  lib=vvc-mip-gpu_amd/lib/libmipgpu.so; [ $v = default ] || lib=tools/bin/lib_$v.so
  MIPGPU_LIB=$PWD/$lib timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "filters_vs_oracle or small_configs" > $O/parity_$v.txt 2>&1 || { echo "PARITY FAIL $v"; tail -20 $O/parity_$v.txt; exit 1; }
  echo "$v parity: $(tail -1 $O/parity_$v.txt)"
done
for rep in 1 2; do
  for v in default f64 f64x2 f256; do
    lib=vvc-mip-gpu_amd/lib/libmipgpu.so; [ $v = default ] || lib=tools/bin/lib_$v.so
    MIPGPU_LIB=$PWD/$lib FB_FRAMES=384 FB_KIDX=2 timeout -k 10 200 python -u tools/filter_bench.py > $O/fb_${v}_$rep.json 2>$O/fb_${v}_$rep.err || { tail $O/fb_${v}_$rep.err; exit 1; }
    python -c "
import json; d=json.load(open('$O/fb_${v}_$rep.json'))
print('$v rep $rep copy %.0f GB/s' % d['copy_calibration']['GB/s'], ' '.join('%s %.3f' % (k.replace('filterFrame_',''), v['ms_per_launch']) for k, v in d['filters'].items()))"
  done
done
