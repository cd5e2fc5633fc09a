"""Kernel resource usage read from a built library's gfx950 code objects (no GPU needed).

The HIP fat binary inside libmipgpu.so holds one clang offload bundle per object file; each
gfx950 entry is an ELF code object whose NT_AMDGPU_METADATA note (msgpack) lists every
kernel's VGPR count, scratch bytes per lane, LDS and so on.  Used by tests/test_kernel_resources.py
to catch register spills and occupancy drops of the search kernel at build time (an out-of-line
helper once spilled 192 bytes per lane and cost 12 %).
"""
import struct

import msgpack

_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
_NT_AMDGPU_METADATA = 32


def _code_objects(blob):
    at = blob.find(_MAGIC)
    while at >= 0:
        n = struct.unpack_from("<Q", blob, at + 24)[0]
        p = at + 32
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", blob, p)
            triple = blob[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if "amdgcn" in triple and size:
                yield triple, blob[at + off:at + off + size]
        at = blob.find(_MAGIC, at + len(_MAGIC))


def _metadata(elf):
    if elf[:4] != b"\x7fELF":
        raise ValueError("code object is not an uncompressed ELF")
    shoff = struct.unpack_from("<Q", elf, 0x28)[0]
    shentsize, shnum = struct.unpack_from("<HH", elf, 0x3A)
    for i in range(shnum):
        sh = shoff + i * shentsize
        stype = struct.unpack_from("<I", elf, sh + 4)[0]
        if stype != 7:  # SHT_NOTE
            continue
        off, size = struct.unpack_from("<QQ", elf, sh + 0x18)
        p, end = off, off + size
        while p + 12 <= end:
            namesz, descsz, ntype = struct.unpack_from("<III", elf, p)
            name = elf[p + 12:p + 12 + namesz].rstrip(b"\0")
            d0 = p + 12 + ((namesz + 3) & ~3)
            if name == b"AMDGPU" and ntype == _NT_AMDGPU_METADATA:
                return msgpack.unpackb(elf[d0:d0 + descsz], raw=False)
            p = d0 + ((descsz + 3) & ~3)
    raise ValueError("no AMDGPU metadata note")


def kernels(path):
    """{kernel symbol: metadata dict} over every gfx950 code object of the library."""
    blob = open(path, "rb").read()
    out = {}
    for triple, elf in _code_objects(blob):
        if "gfx950" not in triple:
            continue
        for k in _metadata(elf).get("amdhsa.kernels", []):
            out[k[".name"]] = k
    return out
