#!/usr/bin/env python3
"""Disassemble the gfx950 code objects of a built library (no GPU): tools/isa_dump.py LIB OUT.s
[KERNEL_SUBSTRING].  Used to check that an experiment switch leaves the default kernels'
instruction stream unchanged (diff two dumps)."""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
import kernel_resources as K  # noqa: E402

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def main():
    lib, out = sys.argv[1], sys.argv[2]
    want = sys.argv[3] if len(sys.argv) > 3 else ""
    blob = open(lib, "rb").read()
    text = []
    with tempfile.TemporaryDirectory() as d:
        for n, (_, elf) in enumerate(K._code_objects(blob)):
            p = os.path.join(d, "co%d.o" % n)
            open(p, "wb").write(elf)
            text.append(subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", "--no-leading-addr", p],
                                       capture_output=True, text=True, check=True).stdout)
    # keep only the wanted kernels' bodies, without addresses / branch-target offsets
    keep, lines = False, []
    for line in "\n".join(text).splitlines():
        m = re.match(r"^([0-9a-f]+ )?<(.+)>:$", line)
        if m:
            keep = want in m.group(2)
        if keep and "file format" not in line:
            lines.append(re.sub(r"<.*\+0x[0-9a-f]+>", "<L>", line.split("//")[0].rstrip()))
    open(out, "w").write("\n".join(lines) + "\n")
    print(out, len(lines), "lines")


if __name__ == "__main__":
    main()
