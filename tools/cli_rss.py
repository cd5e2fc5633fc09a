#!/usr/bin/env python3
"""Peak host memory (max RSS) of the CLI writing the reference's frame-0 cost log of one
large frame (the log writer's buffers must not grow with the thread count).
GPU box:  python tools/cli_rss.py [WIDTHxHEIGHT]   (default 7680x4320; raw u16 input in /tmp)
"""
import os
import resource
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "vvc-mip-gpu_amd"))
from mipgpu.synth import synth_frames  # noqa: E402

w, h = map(int, (sys.argv[1] if len(sys.argv) > 1 else "7680x4320").split("x"))
src, prefix = "/tmp/cli_rss_frame.u16", "/tmp/cli_rss_out"
synth_frames(w, h, 1, 0x8C, 0).astype("<u2").tofile(src)
cli = os.path.join(REPO, "vvc-mip-gpu_amd", "bin", "mipgpu_cli")
t0 = time.time()
r = subprocess.run([cli, "-f", "1", "-s", "%dx%d" % (w, h), "-o", src, "--InputFormat", "u16", "-l", prefix],
                   stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
dt = time.time() - t0
rss_mb = resource.getrusage(resource.RUSAGE_CHILDREN).ru_maxrss / 1024
log = prefix + ".csv"
size = os.path.getsize(log) if os.path.exists(log) else 0
print("%dx%d frame-0 cost log: exit %d, %.1f s, %.2f GB written, peak RSS %.0f MB, %d host threads" %
      (w, h, r.returncode, dt, size / 1e9, rss_mb, os.cpu_count()))
if r.returncode:
    print(r.stderr[-2000:])
for p in (src, log):
    if os.path.exists(p):
        os.remove(p)
sys.exit(r.returncode)
