"""Snappy known answers pinned by the snappy format description, not by
golang/snappy's code (both decoders here -- the oracle's go_snappy in
oracle/l7oracle.cc and the GPU second pass's kc_unsnappy in
cilium_amd/csrc/l7m_kcodec.h, host build -- restate golang/snappy
decode_other.go:14-102 and proto/snappy.go, and the reference vendors no
snappy test data).

1. Hand-assembled blocks whose decoded bytes are worked out in the comments,
   one per element form: literal tags with the length inline and in 1, 2, 3
   and 4 extra bytes; copies with 1-byte (11-bit offset), 2-byte and 4-byte
   offsets; overlapping copies; and the conditions decode_other.go reports
   as corrupt.  Both decoders must return exactly these bytes / errors.
2. A format-description encoder with forced element forms
   (kafka_wire.snappy_block_forms) round-trips random data through both.
The compressed-set verdict cases built from it are in kafka_codec_cases
(checked against the oracle here and on the GPU by test_kcodec_gpu)."""
import ctypes
import os
import random
import struct

import pytest

import kafka_wire as K
from oracle import snappy_decode

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

LIT61 = bytes(i % 251 for i in range(291))
# (name, block, decoded bytes or None for "corrupt")
VECTORS = [
    # uvarint 5; literal tag (5-1)<<2 = 0x10; "hello"
    ("literal_inline", b"\x05\x10hello", b"hello"),
    # uvarint 10; literal 'a' (tag 0x00); copy1 length 9 -> (9-4)<<2 | 1 = 0x15,
    # offset 1 (high bits 0 in the tag, low byte 0x01): 'a' + 9 overlapping copies
    ("copy1_rle", b"\x0a\x00a\x15\x01", b"a" * 10),
    # uvarint 12; literal "abcd" (tag 3<<2 = 0x0c); copy2 length 8 -> 7<<2 | 2 = 0x1e, offset 4 LE16
    ("copy2", b"\x0c\x0cabcd\x1e\x04\x00", b"abcd" * 3),
    # uvarint 9; literal "xyz" (tag 2<<2 = 0x08); copy4 length 6 -> 5<<2 | 3 = 0x17, offset 3 LE32
    ("copy4", b"\x09\x08xyz\x17\x03\x00\x00\x00", b"xyz" * 3),
    # uvarint 9; literal "ab" (tag 0x04); copy2 length 7 at offset 2 (overlapping) -> "ababababa"
    ("copy2_overlap", b"\x09\x04ab\x1a\x02\x00", b"ababababa"),
    # uvarint 61 = 0x3d; tag 60 << 2 = 0xf0, length-1 = 60 in one byte
    ("literal_tag60", b"\x3d\xf0\x3c" + bytes(range(61)), bytes(range(61))),
    # uvarint 300 = 0xac 0x02; tag 61 << 2 = 0xf4, length-1 = 299 = 0x012b LE16
    ("literal_tag61", b"\xac\x02\xf4\x2b\x01" + b"q" * 300, b"q" * 300),
    # uvarint 5; tag 62 << 2 = 0xf8, length-1 = 4 in three bytes (a longer form than needed is legal)
    ("literal_tag62", b"\x05\xf8\x04\x00\x00abcde", b"abcde"),
    # uvarint 5; tag 63 << 2 = 0xfc, length-1 = 4 in four bytes
    ("literal_tag63", b"\x05\xfc\x04\x00\x00\x00vwxyz", b"vwxyz"),
    # uvarint 295 = 0xa7 0x02; literal of 291 bytes (tag 61: 0xf4, 290 = 0x0122 LE16);
    # copy1 length 4 at offset 291 = 0x123: tag (0x123 >> 8) << 5 | 0 << 2 | 1 = 0x21, low byte 0x23
    ("copy1_offset_11_bits", b"\xa7\x02\xf4\x22\x01" + LIT61 + b"\x21\x23", LIT61 + LIT61[:4]),
    # uvarint 0: the empty block
    ("empty", b"\x00", b""),
    # copy1 at offset 0 (decode_other.go: offset <= 0 is corrupt)
    ("copy_offset_zero", b"\x05\x00a\x01\x00", None),
    # copy1 at offset 2 with one byte decoded so far (d < offset)
    ("copy_before_start", b"\x05\x00a\x01\x02", None),
    # uvarint 3; 'a'; copy1 length 5 at offset 1 (tag 1<<2 | 1 = 0x05): past the decoded length
    ("copy_past_end", b"\x03\x00a\x05\x01", None),
    # literal of 5 with 3 bytes of input left
    ("literal_past_input", b"\x05\x10hel", None),
    # decoded 5 bytes of a declared 6
    ("short_output", b"\x06\x10hello", None),
    # literal length 2^32 (tag 63, length-1 0xffffffff)
    ("literal_length_2_32", b"\x05\xfc\xff\xff\xff\xffabcde", None),
    # a copy2 tag with one of its two offset bytes
    ("copy2_cut", b"\x05\x00a\x06\x01", None),
    # a tag-60 literal whose length byte is missing
    ("literal_length_cut", b"\x05\xf0", None),
    # uvarint longer than 10 bytes
    ("uvarint_overflow", b"\x80" * 10 + b"\x01", None),
]


def _kcodec_unsnappy():
    lib = ctypes.CDLL(os.path.join(ROOT, "tests", "cpp", "bin", "libkcodec.so"))
    lib.kc_host_unsnappy.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32,
                                     ctypes.POINTER(ctypes.c_uint32)]

    def dec(src, cap=1 << 22):
        out = ctypes.create_string_buffer(cap)
        n = ctypes.c_uint32(0)
        rc = lib.kc_host_unsnappy(src, len(src), out, cap, ctypes.byref(n))
        return rc, (out.raw[:n.value] if rc == 0 else None)
    return dec


@pytest.mark.parametrize("case", VECTORS, ids=lambda c: c[0])
def test_snappy_known_answers_oracle(case):
    name, block, want = case
    rc, got = snappy_decode(block)
    assert (rc, got) == ((0, want) if want is not None else (1, None)), name


@pytest.mark.parametrize("case", VECTORS, ids=lambda c: c[0])
def test_snappy_known_answers_device_decoder(case):
    name, block, want = case
    rc, got = _kcodec_unsnappy()(block)
    assert (rc, got) == ((0, want) if want is not None else (1, None)), name


def test_snappy_known_answers_in_java_framing():
    """proto/snappy.go: the same blocks as snappy-java chunks concatenate."""
    dec = _kcodec_unsnappy()
    ok = [(b, w) for _, b, w in VECTORS if w is not None]
    framed = b"\x82SNAPPY\x00" + struct.pack(">II", 1, 1) + b"".join(struct.pack(">I", len(b)) + b for b, _ in ok)
    want = b"".join(w for _, w in ok)
    assert snappy_decode(framed) == (0, want)
    assert dec(framed) == (0, want)


FORMS = [dict(copy=1), dict(copy=2), dict(copy=4), dict(copy=1, rle=False), dict(copy=0, lit=60),
         dict(copy=0, lit=61), dict(copy=0, lit=62), dict(copy=0, lit=63), dict(copy=4, lit=63)]


@pytest.mark.parametrize("form", FORMS, ids=lambda f: "-".join(f"{k}{v}" for k, v in f.items()))
def test_format_encoder_round_trips_through_both_decoders(form):
    dec = _kcodec_unsnappy()
    rng = random.Random(11)
    seen = set()
    for _ in range(40):
        n = rng.choice((0, 1, 5, 60, 61, 256, 257, 1000, 5000))
        alphabet = rng.choice((b"a", b"ab", b"abc ", bytes(range(256))))
        data = bytes(rng.choice(alphabet) for _ in range(n))
        if rng.random() < 0.5 and n:  # repeated phrases at varied distances
            k = rng.randrange(1, min(n, 3000) + 1)
            data = (data[:k] * (n // k + 1))[:n]
        blk = K.snappy_block_forms(data, **form)
        seen.update(K.snappy_tags(blk))
        assert snappy_decode(blk) == (0, data)
        assert dec(blk) == (0, data)
    # the forced forms were exercised
    if form.get("copy") == 1:
        assert "copy1" in seen
    if form.get("copy") == 4:
        assert "copy4" in seen
    if form.get("lit"):
        assert f"lit{form['lit'] - 59}" in seen
