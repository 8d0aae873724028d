"""Compressed Kafka message sets (messages.go:441-478): requests whose
verdict under the rules [Topic "t"] (and [Topic "x"] for the deny cases)
follows from the reference's decode-and-recurse semantics.

expected: 0 allowed (the set decodes and re-reads without error), -1 denied,
-2 ReadRequest error.  The reasoning for each is in its name / comment; the
oracle (oracle/l7oracle.cc, zlib + restated Go framing) must agree, and the
GPU's second pass must agree with the oracle."""
import struct
import zlib

import kafka_wire as K

INNER = K.message_set(["a", "bb", "ccc" * 40], version=1)


def _deflate_raw(data, **kw):
    co = zlib.compressobj(kw.get("level", 6), zlib.DEFLATED, -15, 8, kw.get("strategy", zlib.Z_DEFAULT_STRATEGY))
    return co.compress(data) + co.flush()


def _gzip_from_raw(raw, data):
    return bytes([0x1F, 0x8B, 8, 0, 0, 0, 0, 0, 0, 255]) + raw + struct.pack("<II", zlib.crc32(data) & 0xFFFFFFFF,
                                                                            len(data))


def _inner_bad_bytes():
    # CRC-valid message whose value length runs past the message: DecodeBytes
    # fails inside the decoded set -> error
    body = struct.pack(">bb", 0, 0) + struct.pack(">q", 1) + K.b(None) + struct.pack(">i", 500) + b"xy"
    m = struct.pack(">I", zlib.crc32(body) & 0xFFFFFFFF) + body
    return struct.pack(">qi", 0, len(m)) + m


def _set_of(*sets):
    return b"".join(sets)


def value_cases():
    """(name, codec, compressed value, version, expected) for ONE compressed
    message carrying the value."""
    g = K.gzip_member
    ok = g(INNER)
    c = []
    c.append(("gzip", K.GZIP, ok, 1, 0))
    c.append(("gzip_v0_no_timestamp", K.GZIP, g(K.message_set(["a"], version=0)), 0, 0))
    c.append(("gzip_stored_blocks", K.GZIP, g(INNER, level=0), 1, 0))
    c.append(("gzip_fixed_codes", K.GZIP, g(INNER, strategy=zlib.Z_FIXED), 1, 0))
    c.append(("gzip_huffman_only", K.GZIP, g(INNER, strategy=zlib.Z_HUFFMAN_ONLY), 1, 0))
    c.append(("gzip_rle", K.GZIP, g(INNER, strategy=zlib.Z_RLE), 1, 0))
    c.append(("gzip_all_header_fields", K.GZIP, g(INNER, fname=b"x.bin", fcomment=b"c", fextra=b"ab", fhcrc=True), 1, 0))
    h = bytearray(g(INNER, fname=b"n", fhcrc=True))
    h[12] ^= 0xFF  # header CRC-16 (after 10 + "n\0")
    c.append(("gzip_bad_header_crc", K.GZIP, bytes(h), 1, -2))
    c.append(("gzip_name_511", K.GZIP, g(INNER, fname=b"n" * 511), 1, 0))
    c.append(("gzip_name_512", K.GZIP, g(INNER, fname=b"n" * 512), 1, -2))  # readString: z.buf is 512 bytes
    k = len(INNER) // 2
    c.append(("gzip_two_members", K.GZIP, g(INNER[:k]) + g(INNER[k:]), 1, 0))
    c.append(("gzip_trailing_5_bytes", K.GZIP, ok + b"\0" * 5, 1, -2))     # ErrUnexpectedEOF
    c.append(("gzip_trailing_10_zero", K.GZIP, ok + b"\0" * 10, 1, -2))    # ErrHeader
    cut = bytes([0x1F, 0x8B, 8, 8, 0, 0, 0, 0, 0, 255]) + b"name-without-nul"
    c.append(("gzip_next_header_cut_in_fname", K.GZIP, ok + cut, 1, 0))  # raw io.EOF ends the stream
    c.append(("gzip_next_header_cut_in_fextra", K.GZIP, ok + bytes([0x1F, 0x8B, 8, 4, 0, 0, 0, 0, 0, 255, 9]), 1, -2))
    bad = bytearray(ok)
    bad[-8] ^= 1
    c.append(("gzip_bad_crc32", K.GZIP, bytes(bad), 1, -2))
    bad = bytearray(ok)
    bad[-4] ^= 1
    c.append(("gzip_bad_isize", K.GZIP, bytes(bad), 1, -2))
    c.append(("gzip_trailer_cut", K.GZIP, ok[:-1], 1, -2))
    c.append(("gzip_data_cut", K.GZIP, ok[:len(ok) // 2], 1, -2))
    c.append(("gzip_bad_magic", K.GZIP, b"\x1f\x8c" + ok[2:], 1, -2))
    c.append(("gzip_cm_not_deflate", K.GZIP, ok[:2] + b"\x07" + ok[3:], 1, -2))
    c.append(("gzip_header_only", K.GZIP, ok[:10], 1, -2))
    c.append(("gzip_block_type_3", K.GZIP, _gzip_from_raw(b"\x07\x00", b""), 1, -2))
    c.append(("gzip_stored_len_mismatch", K.GZIP, _gzip_from_raw(b"\x01\x03\x00\x00\x00abc", b"abc"), 1, -2))
    c.append(("gzip_distance_too_far", K.GZIP, _gzip_from_raw(bytes([0x63, 0x00, 0x02, 0x00]), b""), 1, -2))
    bomb = g(b"\0" * (100 * 65535 + 1), level=9)
    c.append(("gzip_decoded_over_maxParseBufSize", K.GZIP, bomb, 1, -2))
    c.append(("gzip_empty_set", K.GZIP, g(b""), 1, 0))
    c.append(("gzip_inner_bad_crc_ignored", K.GZIP, g(K.message_set(["a", "b"], version=1, bad_crc_at=0)), 1, 0))
    c.append(("gzip_inner_truncated_ignored", K.GZIP, g(INNER[:-3]), 1, 0))
    c.append(("gzip_inner_attr3_nil_nil", K.GZIP, g(K.message_set(["z"], version=1, compression=3)), 1, 0))
    c.append(("gzip_inner_bad_bytes", K.GZIP, g(_inner_bad_bytes()), 1, -2))
    c.append(("gzip_inner_oversized_message", K.GZIP, g(struct.pack(">qi", 0, 100 * 65535 + 1) + b"\0" * 8), 1, -2))
    nested_ok = K.wrapper_set(K.snappy_block(INNER), K.SNAPPY, version=1)
    c.append(("gzip_of_snappy", K.GZIP, g(nested_ok), 1, 0))
    nested_bad = K.wrapper_set(b"\xff\xff\xff", K.SNAPPY, version=1)
    c.append(("gzip_of_corrupt_snappy", K.GZIP, g(nested_bad), 1, -2))
    c.append(("gzip_of_gzip_of_gzip", K.GZIP, g(K.wrapper_set(g(K.wrapper_set(g(INNER), K.GZIP, 1)), K.GZIP, 1)), 1, 0))
    # a set: valid gzip message, then a message with a bad CRC, then garbage
    # gzip: the bad CRC ends the set before the garbage is decoded
    seq = _set_of(K.wrapper_set(ok, K.GZIP, 1), K.message_set(["q"], version=1, bad_crc_at=0),
                  K.wrapper_set(b"garbage", K.GZIP, 1))
    c.append(("gzip_set_stops_at_bad_crc", K.GZIP, g(seq), 1, 0))
    c.append(("snappy_raw", K.SNAPPY, K.snappy_block(INNER), 1, 0))
    c.append(("snappy_java_framing", K.SNAPPY, K.snappy_java(INNER, chunk=50), 1, 0))
    c.append(("snappy_java_version_2", K.SNAPPY, K.snappy_java(INNER, version=2), 1, -2))
    c.append(("snappy_java_10_bytes", K.SNAPPY, b"\x82SNAPPY\x00\x00\x00", 1, -2))  # b[8:12] panics
    c.append(("snappy_java_no_chunks", K.SNAPPY, b"\x82SNAPPY\x00" + struct.pack(">I", 1), 1, 0))
    sj = K.snappy_java(INNER, chunk=64)
    c.append(("snappy_java_chunk_overrun", K.SNAPPY, sj[:-3], 1, -2))          # b[i:i+n] panics
    c.append(("snappy_java_short_length", K.SNAPPY, sj + b"\0\0", 1, -2))      # b[i:i+4] panics
    c.append(("snappy_bad_varint", K.SNAPPY, b"\xff" * 10, 1, -2))
    blk = bytearray(K.snappy_block(INNER))
    c.append(("snappy_length_mismatch", K.SNAPPY, K._uvarint(len(INNER) + 1) + bytes(blk[len(K._uvarint(len(INNER))):]),
              1, -2))
    c.append(("snappy_bad_copy_offset", K.SNAPPY, K._uvarint(8) + bytes([0x0C, 0x61, 0x1E, 0x05, 0x00]), 1, -2))
    c.append(("snappy_decoded_over_maxParseBufSize", K.SNAPPY, K._uvarint(100 * 65535 + 1) + b"\0", 1, -2))
    c.append(("snappy_empty", K.SNAPPY, K._uvarint(0), 1, 0))
    # every snappy element form, written by the format-description encoder
    # (tests/test_snappy_spec_cpu.py pins both decoders on the bytes)
    for nm, kw in (("copy1", dict(copy=1)), ("copy2_no_rle", dict(copy=2, rle=False)), ("copy4", dict(copy=4)),
                   ("lit60", dict(copy=0, lit=60)), ("lit62", dict(copy=0, lit=62)),
                   ("lit63_copy4", dict(copy=4, lit=63))):
        c.append((f"snappy_forms_{nm}", K.SNAPPY, K.snappy_block_forms(INNER, **kw), 1, 0))
    blk4 = K.snappy_block_forms(INNER, copy=4)
    c.append(("snappy_java_forms_copy4", K.SNAPPY,
              b"\x82SNAPPY\x00" + struct.pack(">II", 1, 1) + struct.pack(">I", len(blk4)) + blk4, 1, 0))
    c.append(("snappy_forms_copy4_cut", K.SNAPPY, blk4[:-2], 1, -2))
    return c


def request_cases():
    """(name, record, expected under [Topic t]) including set-level cases."""
    out = []
    for name, codec, val, ver, exp in value_cases():
        out.append((name, K.produce(ver, "c", [("t", [(0, K.wrapper_set(val, codec, ver))])]), exp))
    ok = K.gzip_member(INNER)
    out.append(("gzip_null_value", K.produce(1, "c", [("t", [(0, K.wrapper_set(None, K.GZIP, 1))])]), -2))
    out.append(("gzip_empty_value", K.produce(1, "c", [("t", [(0, K.wrapper_set(b"", K.GZIP, 1))])]), -2))
    out.append(("compressed_wrapper_bad_crc_not_decoded",
                K.produce(1, "c", [("t", [(0, K.wrapper_set(b"junk", K.GZIP, 1, bad_crc=True))])]), 0))
    two = K.wrapper_set(ok, K.GZIP, 1) + K.wrapper_set(b"\xff\xff", K.SNAPPY, 1)
    out.append(("ok_then_corrupt_in_one_set", K.produce(1, "c", [("t", [(0, two)])]), -2))
    parts = [("t", [(0, K.wrapper_set(ok, K.GZIP, 1)), (1, K.wrapper_set(K.snappy_block(INNER), K.SNAPPY, 1))]),
             ("t", [(2, K.wrapper_set(K.gzip_member(INNER, level=1), K.GZIP, 1))])]
    out.append(("three_compressed_partitions", K.produce(1, "c", parts), 0))
    return out


def deny_cases():
    """Under [Topic x]: a decodable set leaves the topic uncovered (-1); a
    corrupt one is a ReadRequest error first (-2)."""
    ok = K.gzip_member(INNER)
    return [("deny_valid_gzip", K.produce(1, "c", [("t", [(0, K.wrapper_set(ok, K.GZIP, 1))])]), -1),
            ("deny_corrupt_gzip", K.produce(1, "c", [("t", [(0, K.wrapper_set(ok[:-2], K.GZIP, 1))])]), -2)]


def deep_nesting(levels):
    """gzip nested `levels` deep around INNER (a set of one gzip message per level)."""
    v = K.gzip_member(INNER)
    for _ in range(levels - 1):
        v = K.gzip_member(K.wrapper_set(v, K.GZIP, 1))
    return K.produce(1, "c", [("t", [(0, K.wrapper_set(v, K.GZIP, 1))])])


def _corrupt(rng, v):
    v = bytearray(v)
    for _ in range(rng.randrange(1, 3)):
        if rng.random() < 0.6 or len(v) < 2:
            v[rng.randrange(len(v))] ^= 1 << rng.randrange(8)
        else:
            del v[rng.randrange(1, len(v)):]
    return bytes(v)


def random_produce_requests(rng, n, framing_stops=False):
    """ProduceReqs of 1-3 topics x 1-3 partitions whose message sets mix plain
    messages and gzip / snappy wrappers (about a third of the compressed
    values corrupted).  framing_stops adds what ends a set early (a bad-CRC
    message, attribute 3, a truncated last message): the reference then
    reads the set's unread bytes as the next partition's fields, which the
    second pass must follow byte for byte."""
    values = [(K.GZIP, K.gzip_member(INNER)), (K.SNAPPY, K.snappy_block(INNER)),
              (K.SNAPPY, K.snappy_java(INNER, chunk=50)), (K.GZIP, K.gzip_member(INNER, level=1))]
    out = []
    for i in range(n):
        ver = rng.choice((0, 1, 2, 3))
        topics = []
        for t in range(rng.randrange(1, 4)):
            parts = []
            for p in range(rng.randrange(1, 4)):
                pieces = []
                for _ in range(rng.randrange(1, 4)):
                    r = rng.random()
                    if r < 0.35:
                        pieces.append(K.message_set(["x" * rng.randrange(0, 40)] * rng.randrange(1, 3), version=ver))
                    else:
                        codec, v = rng.choice(values)
                        if rng.random() < 0.33:
                            v = _corrupt(rng, v)
                        pieces.append(K.wrapper_set(v, codec, ver))
                if framing_stops and rng.random() < 0.3:
                    k = rng.randrange(3)
                    if k == 0:
                        stop = K.message_set(["stop"], version=ver, bad_crc_at=0)
                    elif k == 1:
                        stop = K.message_set(["stop"], version=ver, compression=3)
                    else:
                        stop = K.message_set(["truncated" * 4], version=ver)[:-5]
                    pieces.insert(rng.randrange(len(pieces) + 1), stop)
                parts.append((p, b"".join(pieces)))
            topics.append(("t" if rng.random() < 0.8 else "u", parts))
        out.append(K.produce(ver, "c", topics, txn=None))
    return out
