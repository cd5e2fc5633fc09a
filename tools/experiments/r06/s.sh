#!/bin/bash
# Round 6: merged-launch / churn GPU tests, and the engine sequence with and without the
# device block cache.
set -uo pipefail
cd "$(dirname "$0")/../../.."
O=gpurun_out/r06s; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "churn or merged" > $O/t.txt 2>&1 || { tail -30 $O/t.txt; exit 1; }
tail -2 $O/t.txt
for c in 1 0; do
  echo "== MIPGPU_DEVICE_CACHE=$c"
  MIPGPU_DEVICE_CACHE=$c timeout -k 10 400 python -u tools/engine_sequence.py > $O/seq_cache$c.jsonl 2> $O/seq_cache$c.err || { tail $O/seq_cache$c.err; exit 1; }
  cat $O/seq_cache$c.jsonl
done
