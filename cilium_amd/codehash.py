"""Hashes of the device code in a built library: the gfx950 entries of every
clang offload bundle in the .so (one per HIP translation unit).  A measured
HBM traffic figure depends only on them and the workload, so bench.py accepts
a traffic file whose hash matches even when host code of the library changed
since it was measured.

kernel_md5: md5 of the whole code objects.  Each compile gives its unit a
random `__hip_cuid_<16 hex>` symbol, so this changes with every rebuild of a
device unit, even from the same source.
code_md5: md5 of what the GPU executes and how it is launched -- the ELF
sections .text, .rodata (kernel descriptors) and .note (AMDGPU metadata:
registers, LDS, arguments) of each code object, not its symbol tables -- so
a rebuild of the same source keeps it (tests/test_abi_cpu.py)."""
import hashlib
import struct

_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"
_CODE_SECTIONS = (b".text", b".rodata", b".note")


def _code_objects(data: bytes):
    """(target id, code object bytes) of every amdgcn bundle entry."""
    i = 0
    while True:
        j = data.find(_MAGIC, i)
        if j < 0:
            return
        n = struct.unpack_from("<Q", data, j + len(_MAGIC))[0]
        p = j + len(_MAGIC) + 8
        for _ in range(n):
            off, size, idlen = struct.unpack_from("<QQQ", data, p)
            p += 24
            tid = data[p:p + idlen]
            p += idlen
            if b"amdgcn" in tid:
                yield tid, data[j + off:j + off + size]
        i = j + 1


def kernel_md5(path: str) -> str:
    h = hashlib.md5()
    for tid, obj in _code_objects(open(path, "rb").read()):
        h.update(tid)
        h.update(obj)
    return h.hexdigest()


def _elf_sections(obj: bytes):
    """(name, contents) of the sections of an ELF64 little-endian object."""
    if obj[:4] != b"\x7fELF" or obj[4] != 2:
        raise ValueError("not an ELF64 code object")
    shoff = struct.unpack_from("<Q", obj, 0x28)[0]
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", obj, 0x3A)
    hdrs = [struct.unpack_from("<IIQQQQIIQQ", obj, shoff + k * shentsize) for k in range(shnum)]
    stro = hdrs[shstrndx][4]
    for name_off, stype, _, _, off, size, *_ in hdrs:
        end = obj.index(b"\0", stro + name_off)
        yield obj[stro + name_off:end], (b"" if stype == 8 else obj[off:off + size])  # SHT_NOBITS: no bytes


def code_md5(path: str) -> str:
    """(independent of the order the units were linked in)"""
    digests = []
    for tid, obj in _code_objects(open(path, "rb").read()):
        h = hashlib.md5(tid)
        for name, body in _elf_sections(obj):
            if name in _CODE_SECTIONS:
                h.update(name)
                h.update(struct.pack("<Q", len(body)))
                h.update(body)
        digests.append(h.digest())
    return hashlib.md5(b"".join(sorted(digests))).hexdigest()
