#!/usr/bin/env python3
"""Opcode histogram of the innermost (mode-pair) loop of one size class's search kernel
(compile-only, -DMIP_ONLY_CLASS): tools/loop_isa.py CLASS [ALT] [--dump FILE]; extra -D options
in the KNOBS environment variable (e.g. KNOBS=-DMIP_SIX_WAVES=0)."""
import collections
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
cls = int(sys.argv[1])
alt = len(sys.argv) > 2 and sys.argv[2] == "1"
out = "/tmp/loop_class_%d.s" % cls
subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I" + REPO + "/include",
                       "-I" + REPO + "/vvc-mip-gpu_amd/csrc", "-DMIP_ONLY_CLASS=%d" % cls, "--cuda-device-only", "-S",
                       "-o", out, REPO + "/vvc-mip-gpu_amd/csrc/mip_search.hip"] + os.environ.get("KNOBS", "").split(),
                      stderr=subprocess.DEVNULL)
s = open(out).read()
# the batched kernel (<ALT, table, PF = !ALT, NW = the batched workgroup's waves, not 16)
m = re.search(r"^(_ZN6mipgpu12_GLOBAL__N_117mip_search_kernelILb%dELb0ELb%dELi(?!16)\d+EEEvNS_10SearchArgsE):" %
              ((1, 0) if alt else (0, 1)), s, re.M)
start = m.start()
body = s[start:s.index("s_endpgm", start)].splitlines()
# the mode-pair loop: the smallest backward-branch range holding both the phase-A MFMAs
# and the per-pair cost store
labels = {m.group(1): i for i, l in enumerate(body) for m in [re.match(r"^\.(LBB\S+):", l)] if m}
best = None
for i, l in enumerate(body):
    m = re.search(r"s_(?:cbranch_\w+|branch)\s+\.(LBB\S+)", l)
    if m and m.group(1) in labels and labels[m.group(1)] < i:
        j = labels[m.group(1)]
        txt = "\n".join(body[j:i + 1])
        if "v_mfma" in txt and ("global_store" in txt or "buffer_store" in txt) and (best is None or i - j < best[2] - best[1]):
            best = (m.group(1), j, i + 1)
lab, j, end = best
seg = [x.strip().split(";")[0].strip() for x in body[j:end] if x.strip() and not x.strip().startswith((".", ";"))]
c = collections.Counter(x.split()[0] for x in seg)
valu = sum(n for o, n in c.items() if o.startswith("v_") and not o.startswith("v_mfma"))
print("class %d loop %s: %d instructions, VALU %d" % (cls, lab, len(seg), valu))
print(" ".join("%s:%d" % kv for kv in c.most_common(40)))
if "--dump" in sys.argv:
    open(sys.argv[sys.argv.index("--dump") + 1], "w").write("\n".join(seg) + "\n")
