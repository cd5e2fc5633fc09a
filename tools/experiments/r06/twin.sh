#!/bin/bash
# Round 6: the four-wave twin for the host pipeline's small chunks -- parity (GPU parity +
# contract tests) then merged-call rates against the six-wave half grid and the four-wave build.
set -uo pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/${OUTTAG:-r06twin}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_contract.py -m gpu -x -q --timeout 150 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
ENVS="X=1 MIPGPU_PIPE_KERNEL=6 MIPGPU_LIB=$PWD/tools/bin/lib_s0.so X=2 MIPGPU_PIPE_KERNEL=6" OUTTAG=${OUTTAG:-r06twin}/mk bash tools/experiments/r06/merge_knobs.sh
