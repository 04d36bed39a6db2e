"""Kernel descriptors of the gfx950 code objects inside libqba.so (test helper).

The list kernels' performance rests on two static properties a compiler or
source change can silently break: no scratch (a kernel with a private
segment is dispatched later after the previous kernel) and at
most 64 VGPRs where the kernel is meant to run 8 waves per SIMD.  Both are
fields of the AMDHSA kernel descriptor (`<kernel>.kd`, 64 bytes) of the code
object, which this module reads from the shared library's offload bundles
without a GPU: .hip_fatbin -> clang offload bundles -> the gfx950 ELF ->
symbol table -> descriptor bytes.
"""
from __future__ import annotations

import struct
from pathlib import Path

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"


def _sections(elf: bytes):
    shoff = struct.unpack_from("<Q", elf, 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    secs = []
    for i in range(shnum):
        o = shoff + i * shentsize
        name, typ, _flags, addr, off, size, link, _info, _align, entsize = struct.unpack_from("<IIQQQQIIQQ", elf, o)
        secs.append({"name": name, "type": typ, "addr": addr, "off": off, "size": size, "link": link,
                     "entsize": entsize})
    strtab = secs[shstrndx]
    for s in secs:
        e = elf.index(b"\0", strtab["off"] + s["name"])
        s["name"] = elf[strtab["off"] + s["name"]:e].decode()
    return secs


def _descriptors(elf: bytes) -> dict:
    secs = _sections(elf)
    out = {}
    for s in secs:
        if s["type"] not in (2, 11):  # SYMTAB, DYNSYM
            continue
        strs = secs[s["link"]]
        for i in range(s["size"] // 24):
            name_off, _info, _other, shndx, value, size = struct.unpack_from("<IBBHQQ", elf, s["off"] + 24 * i)
            e = elf.index(b"\0", strs["off"] + name_off)
            name = elf[strs["off"] + name_off:e].decode()
            if not name.endswith(".kd") or shndx == 0 or shndx >= len(secs):
                continue
            sec = secs[shndx]
            kd = elf[sec["off"] + value - sec["addr"]:sec["off"] + value - sec["addr"] + 64]
            group, private, kernarg = struct.unpack_from("<III", kd, 0)
            rsrc1 = struct.unpack_from("<I", kd, 48)[0]
            out[name[:-3]] = {"lds": group, "scratch": private, "kernarg": kernarg,
                              "vgprs": ((rsrc1 & 0x3F) + 1) * 8}  # gfx950, wave64: granules of 8
    return out


def kernel_descriptors(lib: Path) -> dict:
    """{mangled kernel name: {"lds", "scratch", "kernarg", "vgprs"}} over
    every gfx950 code object in `lib`."""
    data = Path(lib).read_bytes()
    secs = _sections(data)
    fat = next(s for s in secs if s["name"] == ".hip_fatbin")
    fb = data[fat["off"]:fat["off"] + fat["size"]]
    out = {}
    pos = 0
    while (i := fb.find(MAGIC, pos)) >= 0:
        n = struct.unpack_from("<Q", fb, i + 24)[0]
        p = i + 32
        for _ in range(n):
            eo, es, tl = struct.unpack_from("<QQQ", fb, p)
            p += 24
            tid = fb[p:p + tl].decode()
            p += tl
            if tid == TARGET and es:
                out.update(_descriptors(fb[i + eo:i + eo + es]))
        pos = i + len(MAGIC)
    return out
