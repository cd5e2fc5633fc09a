#!/bin/bash
# Round 6: the six-waves-per-SIMD build with the MIP tables in LDS and chunk-spanning walks
# (-DMIP_SIX_WAVES=3, tools/bin/lib_s6.so): parity (GPU tests through it), then a same-box A/B
# against the default build at 384 frames, alternating, 3 reps.
set -uo pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/${OUTTAG:-r06s6}; mkdir -p $O
L=${S6LIB:-tools/bin/lib_s6.so}
echo "== parity $(date +%T)"
MIPGPU_LIB=$PWD/$L timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_contract.py -m gpu -x -q \
  --timeout 150 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -2 $O/parity.log
echo "== A/B $(date +%T)"
A="--frames-per-step 384 --steps 20 --warmup 3 --no-cpu-baseline --no-reference-gpu --no-latency --no-filter --no-end-to-end --allow-knobs"
for r in 1 2 3; do
  for lib in vvc-mip-gpu_amd/lib/libmipgpu.so $L ${EXTRA_LIBS:-}; do
    MIPGPU_LIB=$PWD/$lib timeout -k 10 200 python bench.py $A 2>$O/ab.err | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib', d['value'], d['roofline']['kernel_ms_per_launch'])" || { tail $O/ab.err; exit 1; }
  done
done
