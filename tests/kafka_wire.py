"""Kafka request encoder for tests (TEST INFRASTRUCTURE).

Writes requests in the wire layout the reference's decoder reads: the
per-kind readers of vendor/github.com/optiopay/kafka/proto/messages.go
(ReadProduceReq :1572-1628, ReadFetchReq :752-809, ReadOffsetReq :1791-1839,
ReadMetadataReq :493-522, ReadOffsetCommitReq :1158-1213, ReadOffsetFetchReq
:1374-1411, ReadConsumerMetadataReq :1018-1039) and readMessageSet
(:357-483; message CRC as writeMessageSet :271-300 computes it).  A record is
the size-prefixed request exactly as proto.ReadReq returns it.
"""
import struct
import zlib

PRODUCE, FETCH, OFFSETS, METADATA, OFFSET_COMMIT, OFFSET_FETCH, CONSUMER_METADATA = 0, 1, 2, 3, 8, 9, 10


def s(x):
    """Kafka STRING (int16 length; None = null, length -1)."""
    if x is None:
        return struct.pack(">h", -1)
    b = x.encode() if isinstance(x, str) else bytes(x)
    return struct.pack(">h", len(b)) + b


def b(x):
    """Kafka BYTES (int32 length; None = null, length -1)."""
    if x is None:
        return struct.pack(">i", -1)
    x = x.encode() if isinstance(x, str) else bytes(x)
    return struct.pack(">i", len(x)) + x


def message_set(values, version=0, compression=0, bad_crc_at=None, key=None, first_offset=0):
    out = b""
    for i, v in enumerate(values):
        body = struct.pack(">bb", 0, compression)
        if version >= 1:
            body += struct.pack(">q", 1_500_000_000_000 + i)
        body += b(key) + b(v)
        crc = zlib.crc32(body) & 0xFFFFFFFF
        if bad_crc_at == i:
            crc ^= 1
        m = struct.pack(">I", crc) + body
        out += struct.pack(">qi", first_offset + i, len(m)) + m
    return out


def request(kind, version, client, body=b"", correlation=1):
    payload = struct.pack(">hhi", kind, version, correlation) + s(client) + body
    return struct.pack(">i", len(payload)) + payload


def produce(version, client, topics, txn=None, acks=-1, timeout=1000):
    """topics: [(name, [(partition, message_set_bytes), ...]), ...]"""
    body = (s(txn) if version >= 3 else b"") + struct.pack(">hi", acks, timeout)
    body += struct.pack(">i", len(topics))
    for name, parts in topics:
        body += s(name) + struct.pack(">i", len(parts))
        for pid, ms in parts:
            body += struct.pack(">ii", pid, len(ms)) + ms
    return request(PRODUCE, version, client, body)


def fetch(version, client, topics):
    """topics: [(name, [partition, ...]), ...]"""
    body = struct.pack(">iii", -1, 500, 1)
    if version >= 3:
        body += struct.pack(">i", 1 << 20)
    if version >= 4:
        body += b"\x00"
    body += struct.pack(">i", len(topics))
    for name, parts in topics:
        body += s(name) + struct.pack(">i", len(parts))
        for pid in parts:
            body += struct.pack(">iq", pid, 42)
            if version >= 5:
                body += struct.pack(">q", 0)
            body += struct.pack(">i", 1 << 20)
    return request(FETCH, version, client, body)


def offsets(version, client, topics):
    body = struct.pack(">i", -1) + (b"\x00" if version >= 2 else b"")
    body += struct.pack(">i", len(topics))
    for name, parts in topics:
        body += s(name) + struct.pack(">i", len(parts))
        for pid in parts:
            body += struct.pack(">iq", pid, -1) + (struct.pack(">i", 1) if version == 0 else b"")
    return request(OFFSETS, version, client, body)


def metadata(version, client, topics):
    """topics: list of names (None = null array, which the decoder rejects)."""
    body = struct.pack(">i", -1 if topics is None else len(topics))
    for name in topics or []:
        body += s(name)
    if version >= 4:
        body += b"\x01"
    return request(METADATA, version, client, body)


def offset_commit(version, client, group, topics):
    body = s(group)
    if version >= 1:
        body += struct.pack(">i", 7) + s("member-1")
    if version >= 2:
        body += struct.pack(">q", 60_000)
    body += struct.pack(">i", len(topics))
    for name, parts in topics:
        body += s(name) + struct.pack(">i", len(parts))
        for pid in parts:
            body += struct.pack(">iq", pid, 100)
            if version == 1:
                body += struct.pack(">q", 1_500_000_000_000)
            body += s("meta")
    return request(OFFSET_COMMIT, version, client, body)


def offset_fetch(version, client, group, topics):
    body = s(group) + struct.pack(">i", len(topics))
    for name, parts in topics:
        body += s(name) + struct.pack(">i", len(parts))
        for pid in parts:
            body += struct.pack(">i", pid)
    return request(OFFSET_FETCH, version, client, body)


def consumer_metadata(version, client, group):
    return request(CONSUMER_METADATA, version, client, s(group) + (b"\x00" if version >= 1 else b""))


def generic(kind, version, client="", body=b"\x00" * 8):
    """A request of a kind ReadRequest does not decode (request == nil)."""
    return request(kind, version, client, body)


def random_requests(rng, n, topics, clients):
    """Well-formed requests of every decoded kind and a few undecoded ones."""
    out = []
    for _ in range(n):
        k = int(rng.integers(0, 9))
        cl = None if rng.random() < 0.05 else str(rng.choice(clients))
        nt = int(rng.integers(0, 4))
        ts = [str(rng.choice(topics)) for _ in range(nt)]
        if k == 0:
            v = int(rng.integers(0, 4))
            parts = [(name, [(0, message_set(["x" * int(rng.integers(0, 20))], version=v)
                              if rng.random() < 0.3 else b"")]) for name in ts]
            out.append(produce(v, cl, parts, txn=None if rng.random() < 0.5 else "tx"))
        elif k == 1:
            out.append(fetch(int(rng.integers(0, 6)), cl, [(t, [0, 1]) for t in ts]))
        elif k == 2:
            out.append(offsets(int(rng.integers(0, 3)), cl, [(t, [0]) for t in ts]))
        elif k == 3:
            out.append(metadata(int(rng.integers(0, 5)), cl, ts))
        elif k == 4:
            out.append(offset_commit(int(rng.integers(0, 3)), cl, "grp", [(t, [1]) for t in ts]))
        elif k == 5:
            out.append(offset_fetch(int(rng.integers(0, 2)), cl, "grp", [(t, [1, 2]) for t in ts]))
        elif k == 6:
            out.append(consumer_metadata(int(rng.integers(0, 2)), cl, "grp"))
        else:
            out.append(generic(int(rng.choice([4, 11, 12, 18, 19, 36, 70, -3])), int(rng.integers(0, 3)), cl or ""))
    return out


def mutate(rng, rec: bytes) -> bytes:
    """One random corruption of a record (truncation, size field, byte flips)."""
    r = bytearray(rec)
    k = int(rng.integers(0, 5))
    if k == 0 and len(r) > 13:  # truncate body, keep the size field honest
        cut = int(rng.integers(12, len(r)))
        r = r[:cut]
        r[0:4] = struct.pack(">i", len(r) - 4)
    elif k == 1:  # lie about the size
        r[0:4] = struct.pack(">i", int(rng.integers(-4, len(r) + 8)))
    elif k == 2 and len(r) > 12:  # flip a byte after the header
        i = int(rng.integers(12, len(r)))
        r[i] ^= int(rng.integers(1, 256))
    elif k == 3 and len(r) > 14:  # huge/negative length in a length field position
        i = int(rng.integers(12, len(r) - 2))
        r[i:i + 2] = struct.pack(">h", int(rng.choice([-1, -2, 0x7FFF, 0])))
    else:  # append garbage (ignored trailing bytes)
        r += bytes(rng.integers(0, 256, size=int(rng.integers(1, 9)), dtype="uint8"))
        r[0:4] = struct.pack(">i", len(r) - 4)
    return bytes(r)


# ---- compressed message sets (messages.go:441-478) ------------------------
GZIP, SNAPPY = 1, 2


def gzip_member(data, level=6, fname=None, fcomment=None, fextra=None, fhcrc=False, strategy=None):
    """One gzip member (RFC 1952) with the optional header fields Go's
    gzip.Reader parses; DEFLATE data from zlib (raw)."""
    flg = (4 if fextra is not None else 0) | (8 if fname is not None else 0) | \
          (16 if fcomment is not None else 0) | (2 if fhcrc else 0)
    hdr = bytes([0x1F, 0x8B, 8, flg]) + struct.pack("<I", 0) + bytes([0, 255])
    if fextra is not None:
        hdr += struct.pack("<H", len(fextra)) + fextra
    if fname is not None:
        hdr += fname + b"\0"
    if fcomment is not None:
        hdr += fcomment + b"\0"
    if fhcrc:
        hdr += struct.pack("<H", zlib.crc32(hdr) & 0xFFFF)
    co = zlib.compressobj(level, zlib.DEFLATED, -15, 8, strategy if strategy is not None else zlib.Z_DEFAULT_STRATEGY)
    body = co.compress(data) + co.flush()
    return hdr + body + struct.pack("<II", zlib.crc32(data) & 0xFFFFFFFF, len(data) & 0xFFFFFFFF)


def _uvarint(n):
    out = b""
    while n >= 0x80:
        out += bytes([(n & 0x7F) | 0x80])
        n >>= 7
    return out + bytes([n])


def snappy_block(data):
    """A valid snappy block (github.com/golang/snappy format): greedy 4-byte
    hash matches as copy-2 elements, literals otherwise."""
    out = bytearray(_uvarint(len(data)))
    table, i, lit = {}, 0, 0

    def emit_literal(a, b):
        n = b - a
        while n > 0:
            k = min(n, 1 << 16)
            if k - 1 < 60:
                out.append((k - 1) << 2)
            elif k - 1 < 256:
                out.extend([60 << 2, k - 1])
            else:
                out.extend([61 << 2, (k - 1) & 0xFF, (k - 1) >> 8])
            out.extend(data[a:a + k])
            a += k
            n -= k

    while i + 4 <= len(data):
        key = bytes(data[i:i + 4])
        j = table.get(key)
        table[key] = i
        if j is not None and i - j < 65536:
            m = 4
            while i + m < len(data) and data[j + m] == data[i + m] and m < 64:
                m += 1
            emit_literal(lit, i)
            out.extend([((m - 1) << 2) | 2, (i - j) & 0xFF, (i - j) >> 8])
            i += m
            lit = i
        else:
            i += 1
    emit_literal(lit, len(data))
    return bytes(out)


def snappy_block_forms(data, lit=None, copy=1, rle=True):
    """A snappy block of `data` written element by element from the snappy
    format description, with chosen element forms (an encoder independent of
    golang/snappy's, for pinning both decoders on every tag form):
      lit   None: shortest literal tag; 60-63: every literal's length-1 in
            1-4 bytes after the tag (longer literals split to fit);
      copy  1: tag 01 (length 4-11, 11-bit offset) where it fits, else tag 10;
            2: tag 10 (16-bit offset); 4: tag 11 (32-bit offset); 0: none;
      rle   runs of one byte are written as an overlapping offset-1 copy."""
    out = bytearray(_uvarint(len(data)))

    def emit_literal(chunk):
        cap = 1 << 16 if lit is None else 1 << (8 * (lit - 59))
        for a in range(0, len(chunk), cap):
            piece = chunk[a:a + cap]
            n = len(piece) - 1
            if lit is None and n < 60:
                out.append(n << 2)
            else:
                k = (lit - 59) if lit is not None else max(1, (n.bit_length() + 7) // 8)
                out.append((59 + k) << 2)
                out.extend(n.to_bytes(k, "little"))
            out.extend(piece)

    def emit_copy(off, m):  # 1 <= m <= 64
        if copy == 1 and 4 <= m <= 11 and off < 2048:
            out.extend([((off >> 8) << 5) | ((m - 4) << 2) | 1, off & 0xFF])
        elif copy in (1, 2):
            out.append(((m - 1) << 2) | 2)
            out.extend(off.to_bytes(2, "little"))
        else:
            out.append(((m - 1) << 2) | 3)
            out.extend(off.to_bytes(4, "little"))

    table, i, start = {}, 0, 0
    while i < len(data):
        best = None
        if copy and rle and i >= 1:
            m = 0
            while i + m < len(data) and m < 64 and data[i + m] == data[i - 1]:
                m += 1
            if m >= 4:
                best = (1, m)
        if copy and best is None and i + 4 <= len(data):
            j = table.get(bytes(data[i:i + 4]))
            if j is not None and i - j < (1 << 16):
                m = 4
                while i + m < len(data) and m < 64 and data[j + m] == data[i + m]:
                    m += 1
                best = (i - j, m)
        if i + 4 <= len(data):
            table[bytes(data[i:i + 4])] = i
        if best:
            emit_literal(data[start:i])
            emit_copy(*best)
            i += best[1]
            start = i
        else:
            i += 1
    emit_literal(data[start:])
    return bytes(out)


def snappy_tags(block):
    """Element tags of a snappy block, in order: 'lit<n>' (n = extra length
    bytes, 0 inline) and 'copy1' / 'copy2' / 'copy4'."""
    p = 0
    while block[p] & 0x80:
        p += 1
    p += 1
    tags = []
    while p < len(block):
        t = block[p] & 3
        if t == 0:
            x = block[p] >> 2
            k = x - 59 if x >= 60 else 0
            n = (int.from_bytes(block[p + 1:p + 1 + k], "little") if k else x) + 1
            tags.append(f"lit{k}")
            p += 1 + k + n
        else:
            tags.append(("copy1", "copy2", "copy4")[t - 1])
            p += (2, 3, 5)[t - 1]
    return tags


def snappy_java(data, chunk=1024, version=1):
    """snappy-java framing (proto/snappy.go): magic, version, compat, chunks."""
    out = b"\x82SNAPPY\x00" + struct.pack(">II", version, 1)
    for k in range(0, len(data), chunk):
        blk = snappy_block(data[k:k + chunk])
        out += struct.pack(">I", len(blk)) + blk
    return out


def wrapper_set(value, codec, version=0, bad_crc=False):
    """A message set holding ONE compressed message whose value is `value`
    (already compressed bytes), attributes = codec."""
    body = struct.pack(">bb", 0, codec)
    if version >= 1:
        body += struct.pack(">q", 1_500_000_000_000)
    body += b(None) + b(value)
    crc = zlib.crc32(body) & 0xFFFFFFFF
    if bad_crc:
        crc ^= 1
    m = struct.pack(">I", crc) + body
    return struct.pack(">qi", 0, len(m)) + m


# ---- deny responses: CreateResponse(ErrTopicAuthorizationFailed) ----------
# Test-side restatement of pkg/kafka/response.go + optiopay Resp.Bytes
# (messages.go:595, 896, 1102, 1327, 1512, 1697, 1956), used to check
# libl7match's l7m_kafka_deny_response.
ERR_TOPIC_AUTHORIZATION_FAILED = 29
ZERO_TIME_MILLIS = -6795364578871  # time.Time{}.UnixNano() (wrapped) / 1e6


def deny_response(kind, version, correlation, topics):
    """topics: [(name, [partition ids])] (names only for metadata)."""
    e = ERR_TOPIC_AUTHORIZATION_FAILED
    out = struct.pack(">i", correlation)
    if kind == PRODUCE:
        out += struct.pack(">i", len(topics))
        for name, parts in topics:
            out += s(name) + struct.pack(">i", len(parts))
            for p in parts:
                out += struct.pack(">ihq", p, e, 0) + (struct.pack(">q", 0) if version >= 2 else b"")
        if version >= 1:
            out += struct.pack(">i", 0)
    elif kind == FETCH:
        out += (struct.pack(">i", 0) if version >= 1 else b"") + struct.pack(">i", len(topics))
        for name, parts in topics:
            out += s(name) + struct.pack(">i", len(parts))
            for p in parts:
                out += struct.pack(">ihq", p, e, 0)
                if version >= 4:
                    out += struct.pack(">q", 0) + (struct.pack(">q", 0) if version >= 5 else b"") + struct.pack(">i", 0)
                out += struct.pack(">i", 0)
    elif kind == OFFSETS:
        out += (struct.pack(">i", 0) if version >= 2 else b"") + struct.pack(">i", len(topics))
        for name, parts in topics:
            out += s(name) + struct.pack(">i", len(parts))
            for p in parts:
                out += struct.pack(">ih", p, e) + (struct.pack(">q", ZERO_TIME_MILLIS) if version >= 1 else b"")
                out += struct.pack(">i", 0)
    elif kind == METADATA:
        out += (struct.pack(">i", 0) if version >= 3 else b"") + struct.pack(">i", 0)
        out += (s("") if version >= 2 else b"") + (struct.pack(">i", 0) if version >= 1 else b"")
        out += struct.pack(">i", len(topics))
        for name in topics:
            out += struct.pack(">h", e) + s(name) + (b"\x00" if version >= 1 else b"") + struct.pack(">i", 0)
    elif kind == OFFSET_COMMIT:
        out += (struct.pack(">i", 0) if version >= 3 else b"") + struct.pack(">i", len(topics))
        for name, parts in topics:
            out += s(name) + struct.pack(">i", len(parts))
            for p in parts:
                out += struct.pack(">ih", p, e)
    elif kind == OFFSET_FETCH:
        out += (struct.pack(">i", 0) if version >= 3 else b"") + struct.pack(">i", len(topics))
        for name, parts in topics:
            out += s(name) + struct.pack(">i", len(parts))
            for p in parts:
                out += struct.pack(">iq", p, 0) + s("") + struct.pack(">h", e)
        if version >= 2:
            out += struct.pack(">h", 0)
    elif kind == CONSUMER_METADATA:
        out += (struct.pack(">i", 0) if version >= 1 else b"") + struct.pack(">h", e)
        out += (s("") if version >= 1 else b"") + struct.pack(">i", 0) + s("") + struct.pack(">i", 0)
    else:
        raise ValueError(kind)
    return struct.pack(">i", len(out)) + out
