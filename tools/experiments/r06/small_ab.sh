#!/bin/bash
# Round 6: small launches (1-16 frames) of the six-wave default and the four-wave build: table,
# decisions only, alternative references (2-D float 5x5 k2), engine's wide rule / 16-wave never.
set -uo pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/${OUTTAG:-r06small}; mkdir -p $O
for lib in vvc-mip-gpu_amd/lib/libmipgpu.so ${EXTRA_LIBS:-tools/bin/lib_s0.so}; do
  for mode in table dec alt; do
    env=""; [ $mode = dec ] && env="SB_DEC=1"; [ $mode = alt ] && env="SB_FILTER=filterFrame_2d_float_5x5_quarterCtu:2"
    echo "== $(basename $lib) $mode"
    env $env MIPGPU_LIB=$PWD/$lib SB_CUTS=2 SB_ORDERS=1 SB_SLICES=0 SB_WIDE=${SB_WIDE:-auto,0} timeout -k 10 300 python -u tools/small_batch.py 2>$O/err.txt | grep -v build_id | python -c "
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d['wide'], d['ms_per_launch'])" || { tail $O/err.txt; exit 1; }
  done
done
