#!/usr/bin/env python3
"""Opcode histogram of the loops of one size class's search kernel (compile-only,
-DMIP_ONLY_CLASS): tools/class_isa.py CLASS [ALT]."""
import collections
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cls = int(sys.argv[1])
alt = len(sys.argv) > 2 and sys.argv[2] == "1"
out = "/tmp/class_%d.s" % cls
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + REPO + "/include",
                       "-I" + REPO + "/vvc-mip-gpu_amd/csrc", "-DMIP_ONLY_CLASS=%d" % cls, "--cuda-device-only", "-S",
                       "-o", out, REPO + "/vvc-mip-gpu_amd/csrc/mip_search.hip"], stderr=subprocess.DEVNULL)
s = open(out).read()
name = "_ZN6mipgpu12_GLOBAL__N_117mip_search_kernelILb%dELb0ELb%dEEEvNS_10SearchArgsE:" % ((1, 0) if alt else (0, 1))
start = s.index(name)
body = s[start:s.index("s_endpgm", start)].splitlines()
labels = {m.group(1): i for i, l in enumerate(body) for m in [re.match(r"^(\.LBB\S+):", l)] if m}
for i, l in enumerate(body):
    m = re.search(r"s_cbranch_\w+\s+(\.LBB\S+)|s_branch\s+(\.LBB\S+)", l)
    if not m:
        continue
    t = m.group(1) or m.group(2)
    if t in labels and labels[t] < i:
        seg = [x.strip() for x in body[labels[t]:i + 1] if x.strip() and not x.strip().startswith((".", ";"))]
        c = collections.Counter(x.split()[0] for x in seg)
        v = sum(n for k, n in c.items() if k.startswith("v_") and not k.startswith("v_mfma"))
        print("%s lines %d valu %d: %s" % (t, labels[t], v, " ".join("%s:%d" % kv for kv in c.most_common(30))))
