"""The plain C client (tests/cpp/abi_harness.c) links libl7match.so and,
without a HIP device, every l7m_eval fails loudly with L7M_EDEVICE (there is
no CPU evaluation path)."""
import pytest

from abi_files import run
from cilium_amd import l7match as L
from cilium_amd import workloads as W


def test_c_harness_links_and_fails_without_device(tmp_path):
    if L.device_count() > 0:
        pytest.skip("GPU present")
    rules = W.rules(2, n_rules=20)
    arena, offs = W.requests(2, 0, 64, n_rules=20)
    p, _ = run(str(tmp_path), rules, arena, offs, threads=2, iters=1)
    assert p.returncode == 1
    assert "l7m_eval -6" in p.stderr


def test_kernel_code_hash_covers_both_kernel_objects():
    """bench.py keys measured traffic on the device code objects' hash
    (cilium_amd/codehash.py): the library holds the gfx950 code objects of
    every device translation unit -- the HTTP launcher (search-dialect and
    diagnostic instantiations), the Kafka kernels and the four HTTP feature
    sets (l7m_http_feat.hip) -- and the hash is stable and differs from the
    file hash."""
    import hashlib
    import struct
    from cilium_amd import l7match as L
    from cilium_amd.codehash import kernel_md5, _MAGIC
    data = open(L.LIB_PATH, "rb").read()
    n_gfx = 0
    i = 0
    while (j := data.find(_MAGIC, i)) >= 0:
        n = struct.unpack_from("<Q", data, j + len(_MAGIC))[0]
        p = j + len(_MAGIC) + 8
        for _ in range(n):
            _, size, idlen = struct.unpack_from("<QQQ", data, p)
            p += 24
            n_gfx += b"gfx950" in data[p:p + idlen] and size > 0
            p += idlen
        i = j + 1
    assert n_gfx == 6
    k = kernel_md5(L.LIB_PATH)
    assert k == kernel_md5(L.LIB_PATH) and k != hashlib.md5(data).hexdigest()
    # the code hash reads the ELF sections of every code object (6 of them)
    from cilium_amd.codehash import _code_objects, _elf_sections, code_md5
    objs = list(_code_objects(data))
    assert len(objs) == 6
    for _, obj in objs:
        names = {nm for nm, _ in _elf_sections(obj)}
        assert {b".text", b".rodata", b".note"} <= names
    c = code_md5(L.LIB_PATH)
    assert c == code_md5(L.LIB_PATH) and c != k
