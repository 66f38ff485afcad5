"""Per-kernel resource usage read from the gfx950 code objects inside libtts_hip.so.

The library's .hip_fatbin holds one clang offload bundle per translation unit; each bundle's
gfx950 entry is an ELF whose NT_AMDGPU_METADATA note (msgpack) lists every kernel with its
register counts, spill counts and private (scratch) segment size.  No GPU, no external tool.

usage: python3 tools/kernel_resources.py [lib.so] [--spills]
"""
from __future__ import annotations

import struct
import sys

MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _bundles(blob: bytes):
    """(target id, ELF bytes) of every offload-bundle entry in blob."""
    i = blob.find(MAGIC)
    while i >= 0:
        off = i + len(MAGIC)
        (n,) = struct.unpack_from("<Q", blob, off)
        off += 8
        for _ in range(n):
            o, s, ln = struct.unpack_from("<QQQ", blob, off)
            off += 24
            tid = blob[off:off + ln].decode()
            off += ln
            if s:
                yield tid, blob[i + o:i + o + s]
        i = blob.find(MAGIC, i + len(MAGIC))


def _notes(elf: bytes):
    """(name, type, desc) of every note in the ELF64's SHT_NOTE sections."""
    assert elf[:4] == b"\x7fELF" and elf[4] == 2, "ELF64 expected"
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", elf, 0x3A)
    for k in range(shnum):
        sh = shoff + k * shentsize
        sh_type, = struct.unpack_from("<I", elf, sh + 4)
        if sh_type != 7:  # SHT_NOTE
            continue
        off, size = struct.unpack_from("<QQ", elf, sh + 0x18)
        p, end = off, off + size
        while p + 12 <= end:
            namesz, descsz, ntype = struct.unpack_from("<III", elf, p)
            p += 12
            name = elf[p:p + namesz].rstrip(b"\0").decode()
            p += (namesz + 3) & ~3
            desc = elf[p:p + descsz]
            p += (descsz + 3) & ~3
            yield name, ntype, desc


def kernels(lib_path: str, arch: str = "gfx950"):
    """One dict per kernel: name, vgpr, agpr, sgpr, vgpr_spill, sgpr_spill, scratch, lds."""
    import msgpack
    blob = open(lib_path, "rb").read()
    out = []
    for tid, elf in _bundles(blob):
        if not tid.endswith(arch):
            continue
        for name, ntype, desc in _notes(elf):
            if name != "AMDGPU" or ntype != 32:  # NT_AMDGPU_METADATA
                continue
            md = msgpack.unpackb(desc, raw=False)
            for k in md.get("amdhsa.kernels", []):
                out.append({"name": k[".name"], "vgpr": k.get(".vgpr_count", 0), "agpr": k.get(".agpr_count", 0),
                            "sgpr": k.get(".sgpr_count", 0), "vgpr_spill": k.get(".vgpr_spill_count", 0),
                            "sgpr_spill": k.get(".sgpr_spill_count", 0),
                            "scratch": k.get(".private_segment_fixed_size", 0),
                            "lds": k.get(".group_segment_fixed_size", 0)})
    return out


def main():
    import os
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    lib = args[0] if args else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                            "gonova-tts_amd", "libtts_hip.so")
    ks = kernels(lib)
    if "--spills" in sys.argv:
        ks = [k for k in ks if k["scratch"] or k["vgpr_spill"] or k["sgpr_spill"]]
    for k in sorted(ks, key=lambda k: k["name"]):
        print(f"{k['vgpr']:4d} v {k['agpr']:3d} a {k['sgpr']:3d} s  spill v{k['vgpr_spill']:3d} s{k['sgpr_spill']:3d}"
              f"  scratch {k['scratch']:5d}  lds {k['lds']:6d}  {k['name']}")
    print(f"{len(ks)} kernels", file=sys.stderr)


if __name__ == "__main__":
    main()
