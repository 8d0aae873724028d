"""md5 of the device code objects in a built library: the gfx950 entries of
every clang offload bundle in the .so (one per HIP translation unit).  A
measured HBM traffic figure depends only on them and the workload, so
bench.py accepts a traffic file whose kernel_md5 matches even when host code
of the library changed since it was measured."""
import hashlib
import struct

_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def kernel_md5(path: str) -> str:
    data = open(path, "rb").read()
    h = hashlib.md5()
    i = 0
    while True:
        j = data.find(_MAGIC, i)
        if j < 0:
            break
        n = struct.unpack_from("<Q", data, j + len(_MAGIC))[0]
        p = j + len(_MAGIC) + 8
        for _ in range(n):
            off, size, idlen = struct.unpack_from("<QQQ", data, p)
            p += 24
            tid = data[p:p + idlen]
            p += idlen
            if b"amdgcn" in tid:
                h.update(tid)
                h.update(data[j + off:j + off + size])
        i = j + 1
    return h.hexdigest()
