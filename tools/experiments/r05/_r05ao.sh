set -e
O=gpurun_out/r05ao; mkdir -p $O
export TMPDIR=/tmp
python3 - <<'PY'
import sys, numpy as np
sys.path.insert(0, "vvc-mip-gpu_amd")
from mipgpu.synth import synth_frames
synth_frames(1920, 1080, 64, 0x1080, 0).astype("<u2").tofile("/tmp/in.u16")
PY
rm -rf /tmp/ct
timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d /tmp/ct -o t --output-format csv -- vvc-mip-gpu_amd/bin/mipgpu_cli -s 1920x1080 -f 64 -o /tmp/in.u16 --InputFormat u16 > $O/cli.log 2>&1
grep -o 'distortion ([0-9]*x), [0-9]*' $O/cli.log || true
python3 tools/trace_timeline.py /tmp/ct --last 120 --gap-ms 100 > $O/timeline.txt
echo done
