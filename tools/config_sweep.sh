#!/bin/bash
# One bench line per BASELINE.json configuration that fits one GPU (per-GPU share of the
# multi-GPU configs): profiles/<round>_configs.jsonl.  GPU box.
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p "${OUT:-gpurun_out}"
OUT=${OUT:-gpurun_out}/configs.jsonl
: > "$OUT"
COMMON="--no-cpu-baseline --no-reference-gpu --no-latency --no-filter --steps 10 --warmup 2"
run() { echo "== $*" >&2; timeout -k 10 300 python bench.py $COMMON "$@" >> "$OUT"; }
run --frames-per-step 1                                   # configs[1]: 1 x 1080p, original refs
run --frames-per-step 2 --refs-filter filterFrame_2d_float_5x5_quarterCtu --kernel-idx 2   # configs[2]
run --frames-per-step 32                                  # 32 x 1080p
run --frames-per-step 128                                 # 128 x 1080p
run --frames-per-step 384                                 # 384 x 1080p (bench default)
run --frames-per-step 128 --refs-filter filterFrame_2d_float_5x5_quarterCtu --kernel-idx 2
run --frames-per-step 4 --width 3840 --height 2160        # configs[3]: 32 x 4K over 8 GPUs = 4 per GPU
run --frames-per-step 32 --width 3840 --height 2160
run --frames-per-step 1 --width 7680 --height 4320 --refs-filter filterFrame_2d_int_quarterCtu   # configs[4]: 8 x 8K over 8 GPUs
run --frames-per-step 8 --width 7680 --height 4320 --refs-filter filterFrame_2d_int_quarterCtu
cat "$OUT"
