#!/bin/bash
# Round 6: merged decisions-only downloads as one gather-copy kernel (MIPGPU_GATHER_DOWN=1):
# parity of the merged-launch tests with it, then merged-call rates against the per-member copies.
set -uo pipefail
cd "$(dirname "$0")/../../.."
MIPGPU_GATHER_DOWN=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "merged or per_frame" --timeout 150 --timeout-method thread > gpurun_out/gather_parity.log 2>&1 || { tail -30 gpurun_out/gather_parity.log; exit 1; }
tail -1 gpurun_out/gather_parity.log
ENVS="X=1 MIPGPU_GATHER_DOWN=1 X=2 MIPGPU_GATHER_DOWN=1" OUTTAG=r06gather bash tools/experiments/r06/merge_knobs.sh
