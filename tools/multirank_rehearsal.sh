#!/bin/bash
# Multi-rank GPU path of bench.py on a box with fewer GPUs than ranks (SCALE rehearsal): the
# full search (not --plumbing-check) with world size 2 -- `bench.py --gpus 2` starting its own
# ranks, and torch.distributed.run -- both ranks on device 0 (rank r -> device r % count),
# barriers / timing reductions over gloo; plus the CLI's multi-engine path (--DeviceIndex 0,0).
set -euo pipefail
cd "$(dirname "$0")/.."
OUT=${OUT:-gpurun_out}/multirank
mkdir -p "$OUT"
# (round 6: the end-to-end legs run on every rank at N > 1 -- end_to_end.aggregate)
ARGS="--frames-per-step 128 --steps 10 --warmup 2 --no-cpu-baseline --no-reference-gpu --no-latency --no-filter"
ARGS1="$ARGS --no-end-to-end"
# the driver's 8-GPU launch shape, rehearsed with 8 ranks on this box's one device (round 5:
# launcher, rendezvous, `ranks`, max over 8 ranks; 32 frames per rank keep 8 engines in HBM)
ARGS8="--frames-per-step 32 --steps 10 --warmup 2 --no-cpu-baseline --no-reference-gpu --no-latency --no-filter"
echo "== bench --gpus 8 (own ranks, 8 ranks sharing device 0) $(date +%T)"
timeout -k 10 400 python bench.py --gpus 8 $ARGS8 > "$OUT/bench_gpus8.json" 2> "$OUT/bench_gpus8.err" || { tail -20 "$OUT/bench_gpus8.err"; exit 1; }
cat "$OUT/bench_gpus8.json"
echo "== torch.distributed.run --nproc-per-node 8 $(date +%T)"
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 8 $ARGS8 > "$OUT/bench_torchrun8.json" 2> "$OUT/bench_torchrun8.err" || { tail -20 "$OUT/bench_torchrun8.err"; exit 1; }
cat "$OUT/bench_torchrun8.json"
echo "== bench --gpus 2 (own ranks) $(date +%T)"
timeout -k 10 300 python bench.py --gpus 2 $ARGS > "$OUT/bench_gpus2.json" 2> "$OUT/bench_gpus2.err" || { tail -20 "$OUT/bench_gpus2.err"; exit 1; }
cat "$OUT/bench_gpus2.json"
echo "== torch.distributed.run --nproc-per-node 2 $(date +%T)"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus 2 $ARGS > "$OUT/bench_torchrun2.json" 2> "$OUT/bench_torchrun2.err" || { tail -20 "$OUT/bench_torchrun2.err"; exit 1; }
cat "$OUT/bench_torchrun2.json"
echo "== bench --gpus 1 (same box, reference) $(date +%T)"
timeout -k 10 300 python bench.py $ARGS1 > "$OUT/bench_gpus1.json" 2> "$OUT/bench_gpus1.err" || { tail -20 "$OUT/bench_gpus1.err"; exit 1; }
cat "$OUT/bench_gpus1.json"
echo "== CLI --DeviceIndex 0,0, 2 frames $(date +%T)"
python3 - <<'PY'
import sys
sys.path[:0] = ["vvc-mip-gpu_amd", "tests"]
from mipgpu.synth import synth_frames
f = synth_frames(1920, 1080, 2, 0xC1, 0)
with open("/tmp/mr_in.csv", "w") as fp:
    for fr in f:
        for row in fr:
            fp.write(",".join(map(str, row.tolist())) + "\n")
PY
for dev in 0 0,0; do
  timeout -k 10 300 vvc-mip-gpu_amd/bin/mipgpu_cli -f 2 -s 1920x1080 -o /tmp/mr_in.csv -l /tmp/mr_out_${dev/,/_} \
    --DeviceIndex $dev --AllFrames > "$OUT/cli_dev_${dev/,/_}.txt" 2>&1 || { tail -20 "$OUT/cli_dev_${dev/,/_}.txt"; exit 1; }
done
cmp /tmp/mr_out_0.csv /tmp/mr_out_0_0.csv && echo "CLI logs identical (one engine vs two engines on device 0)" | tee "$OUT/cli_cmp.txt"
sha256sum /tmp/mr_out_0.csv /tmp/mr_out_0_0.csv | tee -a "$OUT/cli_cmp.txt"
tail -3 "$OUT/cli_dev_0_0.txt"
rm -f /tmp/mr_out_0.csv /tmp/mr_out_0_0.csv /tmp/mr_in.csv
echo "== done $(date +%T)"
