#!/bin/bash
# Round 6: small-launch configurations (cut factor x 16-wave rule x slices) for 1 / 2 / 4 frames.
set -uo pipefail
cd "$(dirname "$0")/../../.."
mkdir -p gpurun_out
SB_CUTS=${SB_CUTS:-1,2,3} SB_ORDERS=1 SB_SLICES=${SB_SLICES:-0,1,2,4} SB_WIDE=${SB_WIDE:-auto,0,1} timeout -k 10 500 python -u tools/small_batch.py > gpurun_out/sb_all.jsonl 2> gpurun_out/sb_all.err || { tail gpurun_out/sb_all.err; exit 1; }
python - <<'P'
import json
for l in open("gpurun_out/sb_all.jsonl"):
    d = json.loads(l)
    if "ms_per_launch" in d:
        m = d["ms_per_launch"]
        print(d["cut"], d["wide"], d["slices"], m["1"], m["2"], m["4"])
P
