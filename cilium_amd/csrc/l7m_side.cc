// l7m_side.cc — verdict side effects on the host (include/l7match.h):
//   * the 403 body Envoy's filter sends on deny (envoy/cilium_l7policy.cc:89-95,
//     169-181);
//   * the Kafka response the proxy sends for a denied request:
//     (*RequestMessage).CreateResponse(proto.ErrTopicAuthorizationFailed)
//     (pkg/kafka/request.go:158-182, pkg/kafka/response.go:81-303) serialised
//     as optiopay's Resp.Bytes(version) (vendor/.../proto/messages.go:595,
//     896, 1102, 1327, 1512, 1697, 1956);
//   * per-endpoint proxy statistics from a batch of verdicts
//     (Endpoint.UpdateProxyStatistics, pkg/endpoint/endpoint.go:2099-2122),
//     flat (l7m_proxy_stats_add) or keyed by (protocol, port, direction,
//     request) as the endpoint keeps them (l7m_proxy_stats_table);
//   * access-log records: the HttpLogEntry protobuf the Envoy filter sends
//     per request (envoy/accesslog.cc:59-170, cilium_l7policy.cc:166-191,
//     envoy/cilium/accesslog.proto) and the Kafka proxy's per-topic log
//     records (pkg/proxy/kafka.go:168-230, pkg/proxy/accesslog/record.go
//     :200-241, pkg/proxy/logger/logger.go:84-357).
// These run only for requests the GPU already decided; no verdict is
// computed here.
#include <algorithm>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/l7match.h"
#include "program.h"

namespace {

// Big-endian request reader with optiopay's sticky-error semantics.
struct Rd {
  const uint8_t* p;
  size_t n, pos = 0;
  bool err = false;
  uint64_t be(size_t k) {
    if (err || n - pos < k) {
      err = true;
      pos = n;
      return 0;
    }
    uint64_t v = 0;
    for (size_t i = 0; i < k; ++i) v = v << 8 | p[pos + i];
    pos += k;
    return v;
  }
  int16_t i16() { return static_cast<int16_t>(be(2)); }
  int32_t i32() { return static_cast<int32_t>(be(4)); }
  std::string str(size_t* at = nullptr) {  // DecodeString: int16 length, < 1 -> ""
    const int16_t k = i16();
    if (at) *at = pos;
    if (err || k < 1) return "";
    if (n - pos < static_cast<size_t>(k)) {
      err = true;
      pos = n;
      return "";
    }
    std::string s(reinterpret_cast<const char*>(p + pos), static_cast<size_t>(k));
    pos += static_cast<size_t>(k);
    return s;
  }
  void skip(size_t k) {
    if (err || n - pos < k) {
      err = true;
      pos = n;
      return;
    }
    pos += k;
  }
  int32_t arraylen() {
    const int32_t v = i32();
    if (v < 0 || v > l7m::kKafkaMaxParseBuf) err = true;
    return err ? 0 : v;
  }
  void bytes() {  // DecodeBytes, value discarded
    const int32_t k = i32();
    if (err || k < 1) return;
    if (k > l7m::kKafkaMaxParseBuf || n - pos < static_cast<size_t>(k)) {
      err = true;
      pos = n;
      return;
    }
    pos += static_cast<size_t>(k);
  }
};

struct Wr {
  std::vector<uint8_t> b;
  void be(uint64_t v, int k) {
    for (int i = k - 1; i >= 0; --i) b.push_back(static_cast<uint8_t>(v >> (8 * i)));
  }
  void i8(int v) { be(static_cast<uint8_t>(v), 1); }
  void i16(int v) { be(static_cast<uint16_t>(v), 2); }
  void i32(int64_t v) { be(static_cast<uint32_t>(v), 4); }
  void i64(int64_t v) { be(static_cast<uint64_t>(v), 8); }
  void str(const std::string& s) {  // Encode(string): uint16 length + bytes
    i16(static_cast<int>(s.size()));
    b.insert(b.end(), s.begin(), s.end());
  }
};

constexpr int kErrTopicAuthorizationFailed = 29;  // vendor/.../proto/errors.go:37
// time.Time{}.UnixNano() / int64(time.Millisecond) on a 64-bit Go: the zero
// Time's nanoseconds overflow int64 and wrap (OffsetResp v>=1 TimeStamp).
constexpr int64_t kZeroTimeMillis = -6795364578871LL;

// Bytes readMessageSet (messages.go:357-483) consumes from its LimitReader:
// it can stop inside the set (a bad CRC, attributes 3), and the request's
// next partition is then read from there.  Only called for requests whose
// verdict is a deny, i.e. whose decode succeeded.
size_t message_set_consumed(const uint8_t* p, size_t avail, int32_t size, int16_t version) {
  const size_t lim = avail < static_cast<size_t>(size) ? avail : static_cast<size_t>(size);
  size_t pos = 0;
  for (;;) {
    if (lim - pos < 12) return lim;  // offset / size: short reads consume the rest
    pos += 8;
    const int32_t msz = static_cast<int32_t>(static_cast<uint32_t>(p[pos]) << 24 | static_cast<uint32_t>(p[pos + 1]) << 16 |
                                             static_cast<uint32_t>(p[pos + 2]) << 8 | p[pos + 3]);
    pos += 4;
    if (msz <= 0) return pos;
    if (lim - pos < static_cast<size_t>(msz)) return lim;
    const uint8_t* m = p + pos;
    pos += static_cast<size_t>(msz);
    if (msz <= 4) return pos;
    uint32_t c = 0xffffffffu;
    for (int32_t i = 4; i < msz; ++i) {
      c ^= m[i];
      for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
    }
    const uint32_t crc = static_cast<uint32_t>(m[0]) << 24 | static_cast<uint32_t>(m[1]) << 16 |
                         static_cast<uint32_t>(m[2]) << 8 | m[3];
    if ((c ^ 0xffffffffu) != crc) return pos;
    const size_t ap = 5;  // crc, magic
    if (msz > static_cast<int32_t>(ap) && (m[ap] & 3) == 3) return pos;
    (void)version;
  }
}

struct TopicParts {
  std::string name;
  size_t at = 0;  // offset of the name's bytes in the request
  std::vector<int32_t> parts;
};

// What GetTopics / CreateResponse need of a request whose decode succeeded
// (pkg/kafka/request.go:88-108,158-182 over optiopay's per-kind readers).
struct KReq {
  int16_t kind = 0, version = 0;
  int32_t corr = 0;
  std::vector<TopicParts> topics;
};

// L7M_OK, L7M_EINVAL (decode error), L7M_EUNSUPPORTED (request == nil: a kind
// ReadRequest leaves untyped, request.go:204-220).
int read_kafka(const uint8_t* req, size_t len, KReq* q) {
  Rd r{req, len};
  r.i32();  // size
  q->kind = r.i16();
  q->version = r.i16();
  q->corr = r.i32();
  if (r.err) return L7M_EINVAL;
  const int16_t version = q->version;
  auto partitions = [&](TopicParts& t, size_t fixed, bool produce, bool commit) {
    const int32_t np = r.arraylen();
    for (int32_t k = 0; k < np && !r.err; ++k) {
      t.parts.push_back(r.i32());
      if (produce) {
        const int32_t sz = r.i32();
        if (r.err) break;
        if (sz < 0 || sz > l7m::kKafkaMaxParseBuf) r.err = true;
        else r.pos += message_set_consumed(r.p + r.pos, r.n - r.pos, sz, version);
      } else if (commit) {
        r.skip(8 + (version == 1 ? 8 : 0));
        r.str();
      } else {
        r.skip(fixed);
      }
    }
  };
  auto read_topics = [&](size_t fixed, bool produce, bool commit, bool names_only) {
    const int32_t nt = r.arraylen();
    for (int32_t k = 0; k < nt && !r.err; ++k) {
      TopicParts t;
      t.name = r.str(&t.at);
      if (!names_only) partitions(t, fixed, produce, commit);
      q->topics.push_back(std::move(t));
    }
  };
  r.str();  // ClientID
  switch (q->kind) {
    case 0:  // ReadProduceReq
      if (version >= 3) r.str();
      r.skip(6);
      read_topics(0, true, false, false);
      break;
    case 1:  // ReadFetchReq
      r.skip(12 + (version >= 3 ? 4 : 0) + (version >= 4 ? 1 : 0));
      read_topics(12 + (version >= 5 ? 8 : 0), false, false, false);
      break;
    case 2:  // ReadOffsetReq
      r.skip(4 + (version >= 2 ? 1 : 0));
      read_topics(8 + (version == 0 ? 4 : 0), false, false, false);
      break;
    case 3:  // ReadMetadataReq
      read_topics(0, false, false, true);
      break;
    case 8:  // ReadOffsetCommitReq
      r.str();
      if (version >= 1) {
        r.skip(4);
        r.str();
      }
      if (version >= 2) r.skip(8);
      read_topics(0, false, true, false);
      break;
    case 9:  // ReadOffsetFetchReq
      r.str();
      read_topics(0, false, false, false);
      break;
    case 10:  // ReadConsumerMetadataReq
      r.str();
      if (version >= 1) r.skip(1);
      break;
    default:
      return L7M_EUNSUPPORTED;
  }
  return r.err ? L7M_EINVAL : L7M_OK;
}

// Protobuf wire writer (proto3: default-valued fields are omitted).
struct Pb {
  std::string b;
  void varint(uint64_t v) {
    while (v >= 0x80) {
      b.push_back(static_cast<char>(v | 0x80));
      v >>= 7;
    }
    b.push_back(static_cast<char>(v));
  }
  void key(uint32_t field, uint32_t wire) { varint(static_cast<uint64_t>(field) << 3 | wire); }
  void u64(uint32_t field, uint64_t v) {
    if (!v) return;
    key(field, 0);
    varint(v);
  }
  void bytes(uint32_t field, const char* p, size_t n) {
    if (!n) return;
    key(field, 2);
    varint(n);
    b.append(p, n);
  }
};

const char* const kApiKeyNames[] = {  // api.KafkaReverseAPIKeyMap (pkg/policy/api/kafka.go:193-227)
    "produce", "fetch", "offsets", "metadata", "leaderandisr", "stopreplica", "updatemetadata",
    "controlledshutdown", "offsetcommit", "offsetfetch", "findcoordinator", "joingroup", "heartbeat",
    "leavegroup", "syncgroup", "describegroups", "listgroups", "saslhandshake", "apiversions",
    "createtopics", "deletetopics", "deleterecords", "initproducerid", "offsetforleaderepoch",
    "addpartitionstotxn", "addoffsetstotxn", "endtxn", "writetxnmarkers", "txnoffsetcommit",
    "describeacls", "createacls", "deleteacls", "describeconfigs", "alterconfigs"};

// Kafka record at offs[i]: the size-prefixed request; false if it does not fit.
bool kafka_rec(const uint8_t* arena, size_t arena_bytes, uint64_t o, size_t* len) {
  if (o > arena_bytes || arena_bytes - o < 4) return false;
  const uint8_t* p = arena + o;
  const uint64_t sz = static_cast<uint64_t>(p[0]) << 24 | static_cast<uint64_t>(p[1]) << 16 |
                      static_cast<uint64_t>(p[2]) << 8 | p[3];
  if (sz > arena_bytes - o - 4) return false;
  *len = static_cast<size_t>(sz + 4);
  return true;
}

// HTTP record fields (include/l7match.h record layout); false if malformed.
struct HttpView {
  uint32_t remote_id = 0, dport = 0, flags = 0, nhdr = 0;
  const uint8_t *method = nullptr, *path = nullptr, *authority = nullptr;
  uint32_t mlen = 0, plen = 0, alen = 0;
  const uint8_t* dir = nullptr;   // n_hdr x {u16 name_len, u16 value_len}
  const uint8_t* names = nullptr; // first header name
};
bool http_rec(const uint8_t* arena, size_t arena_bytes, uint64_t o, HttpView* v) {
  if ((o & 3) || o > arena_bytes || arena_bytes - o < L7M_HTTP_REC_FIXED) return false;
  const uint8_t* r = arena + o;
  uint32_t w[5];
  std::memcpy(w, r, sizeof w);
  if (w[0] > arena_bytes - o) return false;
  v->remote_id = w[1];
  v->dport = w[2] & 0xffffu;
  v->flags = (w[2] >> 16) & 0xffu;
  v->nhdr = w[2] >> 24;
  v->mlen = w[3] & 0xffffu;
  v->plen = w[3] >> 16;
  v->alen = w[4] & 0xffffu;
  uint64_t need = L7M_HTTP_REC_FIXED + 4ull * v->nhdr + v->mlen + v->plen + v->alen;
  if (need > w[0]) return false;
  v->dir = r + L7M_HTTP_REC_FIXED;
  for (uint32_t j = 0; j < v->nhdr; ++j) {
    uint32_t e;
    std::memcpy(&e, v->dir + 4 * j, 4);
    need += (e & 0xffffu) + (e >> 16);
  }
  if (need != w[0]) return false;
  v->method = v->dir + 4u * v->nhdr;
  v->path = v->method + v->mlen;
  v->authority = v->path + v->plen;
  v->names = v->authority + v->alen;
  return true;
}

// FlowVerdict of a decided request: 0 Forwarded, 1 Denied, 2 Error.
uint32_t flow_verdict(int32_t v) { return v >= 0 ? 0u : v == L7M_VERDICT_DENY ? 1u : 2u; }

}  // namespace

extern "C" {

size_t l7m_http_deny_body(const char* configured, char* out, size_t cap) {
  // cilium_l7policy.cc:89-95: empty -> "Access denied"; ensure a trailing CRLF
  std::string b = configured && *configured ? configured : "Access denied";
  const size_t len = b.size();
  if (len < 2 || b[len - 2] != '\r' || b[len - 1] != '\n') b += "\r\n";
  if (out && cap) {
    const size_t k = b.size() < cap - 1 ? b.size() : cap - 1;
    std::memcpy(out, b.data(), k);
    out[k] = 0;
  }
  return b.size();
}

int l7m_kafka_deny_response(const uint8_t* req, size_t len, uint8_t* out, size_t cap, size_t* out_len) {
  if (!req || !out_len) return L7M_EINVAL;
  KReq q;
  const int rc = read_kafka(req, len, &q);
  if (rc != L7M_OK) return rc;
  const int16_t version = q.version;
  const std::vector<TopicParts>& topics = q.topics;
  Wr w;
  w.i32(0);  // size placeholder
  w.i32(q.corr);
  switch (q.kind) {
    case 0:  // ProduceResp.Bytes (messages.go:1697)
      w.i32(static_cast<int64_t>(topics.size()));
      for (const auto& t : topics) {
        w.str(t.name);
        w.i32(static_cast<int64_t>(t.parts.size()));
        for (int32_t id : t.parts) {
          w.i32(id);
          w.i16(kErrTopicAuthorizationFailed);
          w.i64(0);                     // Offset
          if (version >= 2) w.i64(0);   // LogAppendTime
        }
      }
      if (version >= 1) w.i32(0);  // ThrottleTime
      break;
    case 1:  // FetchResp.Bytes (messages.go:896)
      if (version >= 1) w.i32(0);  // ThrottleTime
      w.i32(static_cast<int64_t>(topics.size()));
      for (const auto& t : topics) {
        w.str(t.name);
        w.i32(static_cast<int64_t>(t.parts.size()));
        for (int32_t id : t.parts) {
          w.i32(id);
          w.i16(kErrTopicAuthorizationFailed);
          w.i64(0);  // TipOffset
          if (version >= 4) {
            w.i64(0);                    // LastStableOffset
            if (version >= 5) w.i64(0);  // LogStartOffset
            w.i32(0);                    // AbortedTransactions
          }
          w.i32(0);  // message set size: no messages
        }
      }
      break;
    case 2:  // OffsetResp.Bytes (messages.go:1956)
      if (version >= 2) w.i32(0);  // ThrottleTime
      w.i32(static_cast<int64_t>(topics.size()));
      for (const auto& t : topics) {
        w.str(t.name);
        w.i32(static_cast<int64_t>(t.parts.size()));
        for (int32_t id : t.parts) {
          w.i32(id);
          w.i16(kErrTopicAuthorizationFailed);
          if (version >= 1) w.i64(kZeroTimeMillis);
          w.i32(0);  // Offsets
        }
      }
      break;
    case 3:  // MetadataResp.Bytes (messages.go:595)
      if (version >= 3) w.i32(0);  // ThrottleTime
      w.i32(0);                    // Brokers
      if (version >= 2) w.str("");  // ClusterID
      if (version >= 1) w.i32(0);   // ControllerID
      w.i32(static_cast<int64_t>(topics.size()));
      for (const auto& t : topics) {
        w.i16(kErrTopicAuthorizationFailed);
        w.str(t.name);
        if (version >= 1) w.i8(0);  // IsInternal
        w.i32(0);                   // Partitions
      }
      break;
    case 8:  // OffsetCommitResp.Bytes (messages.go:1327)
      if (version >= 3) w.i32(0);
      w.i32(static_cast<int64_t>(topics.size()));
      for (const auto& t : topics) {
        w.str(t.name);
        w.i32(static_cast<int64_t>(t.parts.size()));
        for (int32_t id : t.parts) {
          w.i32(id);
          w.i16(kErrTopicAuthorizationFailed);
        }
      }
      break;
    case 9:  // OffsetFetchResp.Bytes (messages.go:1512)
      if (version >= 3) w.i32(0);
      w.i32(static_cast<int64_t>(topics.size()));
      for (const auto& t : topics) {
        w.str(t.name);
        w.i32(static_cast<int64_t>(t.parts.size()));
        for (int32_t id : t.parts) {
          w.i32(id);
          w.i64(0);    // Offset
          w.str("");   // Metadata
          w.i16(kErrTopicAuthorizationFailed);
        }
      }
      if (version >= 2) w.i16(0);  // resp.Err: left nil by createOffsetFetchResponse
      break;
    case 10:  // ConsumerMetadataResp.Bytes (messages.go:1102)
      if (version >= 1) w.i32(0);  // ThrottleTime
      w.i16(kErrTopicAuthorizationFailed);
      if (version >= 1) w.str("");  // ErrMsg
      w.i32(0);                     // CoordinatorID
      w.str("");                    // CoordinatorHost
      w.i32(0);                     // CoordinatorPort
      break;
  }
  const uint32_t sz = static_cast<uint32_t>(w.b.size() - 4);
  w.b[0] = static_cast<uint8_t>(sz >> 24);
  w.b[1] = static_cast<uint8_t>(sz >> 16);
  w.b[2] = static_cast<uint8_t>(sz >> 8);
  w.b[3] = static_cast<uint8_t>(sz);
  *out_len = w.b.size();
  if (!out || cap < w.b.size()) return L7M_ENOMEM;
  std::memcpy(out, w.b.data(), w.b.size());
  return L7M_OK;
}

size_t l7m_kafka_api_key_name(int16_t key, char* out, size_t cap) {
  // apiKeyToString (pkg/proxy/kafka.go:161-166): the map's name, else the number
  const std::string s = key >= 0 && key < static_cast<int16_t>(sizeof kApiKeyNames / sizeof *kApiKeyNames)
                            ? kApiKeyNames[key]
                            : std::to_string(key);
  if (out && cap) {
    const size_t k = s.size() < cap - 1 ? s.size() : cap - 1;
    std::memcpy(out, s.data(), k);
    out[k] = 0;
  }
  return s.size();
}

int64_t l7m_http_access_log(const uint8_t* arena, size_t arena_bytes, const uint64_t* offs, size_t n,
                            const int32_t* verdicts, const l7m_access_log_opts* opts, uint8_t* out, size_t cap,
                            uint64_t* entry_offs) {
  if (n && (!arena || !offs || !verdicts || !entry_offs)) return L7M_EINVAL;
  l7m_access_log_opts o{};
  o.http_protocol = 1;  // HTTP11: Envoy's default branch (accesslog.cc:68-79)
  if (opts) {
    const size_t k = opts->struct_size == 0 || opts->struct_size > sizeof o ? sizeof o : opts->struct_size;
    std::memcpy(&o, opts, k);
  }
  const size_t pl = o.policy_name ? std::strlen(o.policy_name) : 0;
  const size_t sl = o.source_address ? std::strlen(o.source_address) : 0;
  const size_t dl = o.destination_address ? std::strlen(o.destination_address) : 0;
  uint64_t total = 0;
  const bool write = out != nullptr;
  Pb pb, kv;
  for (size_t i = 0; i < n; ++i) {
    entry_offs[i] = total;
    HttpView v;
    if (!http_rec(arena, arena_bytes, offs[i], &v) || verdicts[i] <= L7M_VERDICT_PARSE_ERROR) continue;
    const bool denied = verdicts[i] == L7M_VERDICT_DENY;
    const bool ingress = (v.flags & L7M_HTTP_F_INGRESS) != 0;
    pb.b.clear();
    // field order as SerializeToString emits it (accesslog.proto numbers)
    pb.u64(1, o.timestamp_ns);
    pb.u64(2, o.http_protocol);
    pb.u64(3, denied ? 2u : 0u);  // EntryType Denied (encodeHeaders of the 403) / Request
    pb.bytes(4, o.policy_name, pl);
    // 5 cilium_rule_ref: not set by this reference's filter
    pb.u64(6, ingress ? v.remote_id : o.local_identity);  // SocketMarkOption identity_ (the source)
    pb.bytes(7, o.source_address, sl);
    pb.bytes(8, o.destination_address, dl);
    // headers in request order; x-forwarded-proto -> scheme (accesslog.cc:103-131)
    const uint8_t* scheme = nullptr;
    uint32_t scheme_len = 0;
    std::string hdrs;
    const uint8_t* q = v.names;
    for (uint32_t j = 0; j < v.nhdr; ++j) {
      uint32_t e;
      std::memcpy(&e, v.dir + 4 * j, 4);
      const uint32_t nl = e & 0xffffu, vl = e >> 16;
      if (nl == 17 && std::memcmp(q, "x-forwarded-proto", 17) == 0) {
        scheme = q + nl;
        scheme_len = vl;
      } else {
        kv.b.clear();
        kv.bytes(1, reinterpret_cast<const char*>(q), nl);
        kv.bytes(2, reinterpret_cast<const char*>(q + nl), vl);
        Pb f;
        f.key(14, 2);
        f.varint(kv.b.size());
        hdrs += f.b;
        hdrs += kv.b;
      }
      q += nl + vl;
    }
    pb.bytes(9, reinterpret_cast<const char*>(scheme), scheme_len);
    if (v.flags & L7M_HTTP_F_AUTHORITY) pb.bytes(10, reinterpret_cast<const char*>(v.authority), v.alen);
    if (v.flags & L7M_HTTP_F_PATH) pb.bytes(11, reinterpret_cast<const char*>(v.path), v.plen);
    if (v.flags & L7M_HTTP_F_METHOD) pb.bytes(12, reinterpret_cast<const char*>(v.method), v.mlen);
    pb.u64(13, denied ? 403u : 0u);  // responseCode of the local reply
    pb.b += hdrs;
    pb.u64(15, ingress ? 1u : 0u);
    if (write && total + pb.b.size() <= cap) std::memcpy(out + total, pb.b.data(), pb.b.size());
    total += pb.b.size();
  }
  if (n) entry_offs[n] = total;
  return write && total > cap ? static_cast<int64_t>(L7M_ENOMEM) : static_cast<int64_t>(total);
}

int64_t l7m_kafka_access_log(const uint8_t* arena, size_t arena_bytes, const uint64_t* offs, size_t n,
                             const int32_t* verdicts, l7m_kafka_log_record* out, size_t cap) {
  if (n && (!arena || !offs || !verdicts)) return L7M_EINVAL;
  uint64_t k = 0;
  for (size_t i = 0; i < n; ++i) {
    const int32_t vd = verdicts[i];
    // ReadRequest failed: the connection is closed, nothing is logged
    // (pkg/proxy/kafka.go:349-354); -3 (a codec limit of this library) too.
    if (vd == L7M_VERDICT_PARSE_ERROR || vd == L7M_VERDICT_UNSUPPORTED) continue;
    size_t len;
    if (!kafka_rec(arena, arena_bytes, offs[i], &len)) continue;
    KReq q;
    const int rc = read_kafka(arena + offs[i], len, &q);
    if (rc != L7M_OK) continue;  // request == nil: GetTopics() is nil, no records
    // allowed: Forwarded / ErrNone; denied: CreateResponse succeeds for every
    // typed request -> Denied / ErrTopicAuthorizationFailed (kafka.go:240-262,296)
    const uint32_t fv = flow_verdict(vd);
    for (const auto& t : q.topics) {  // one record per topic (kafka.go:207-211)
      if (out && k < cap) {
        l7m_kafka_log_record& r = out[k];
        r.request = i;
        r.verdict = fv;
        r.error_code = fv == 1 ? kErrTopicAuthorizationFailed : 0;
        r.api_key = q.kind;
        r.api_version = q.version;
        r.correlation_id = q.corr;
        r.topic_off = offs[i] + t.at;
        r.topic_len = static_cast<uint32_t>(t.name.size());
        r.pad = 0;
      }
      ++k;
    }
  }
  return out && k > cap ? static_cast<int64_t>(L7M_ENOMEM) : static_cast<int64_t>(k);
}

}  // extern "C"

// Per-endpoint proxy statistics keyed as Endpoint.proxyStatistics
// (pkg/endpoint/endpoint.go:2060-2122): (protocol, port, ingress) -> request /
// response MessageForwardingStatistics.
struct l7m_proxy_stats_table {
  std::mutex mu;
  std::map<std::tuple<uint32_t, uint32_t, uint32_t, uint32_t>, l7m_proxy_stats> m;
};

extern "C" {

l7m_proxy_stats_table* l7m_proxy_stats_table_create(void) { return new (std::nothrow) l7m_proxy_stats_table(); }

void l7m_proxy_stats_table_destroy(l7m_proxy_stats_table* t) { delete t; }

int l7m_proxy_stats_update(l7m_proxy_stats_table* t, uint32_t proto, const uint8_t* arena, size_t arena_bytes,
                           const uint64_t* offs, const int32_t* verdicts, size_t n, uint16_t port, int ingress) {
  if (!t || (n && !verdicts) || (proto != L7M_PROTO_HTTP && proto != L7M_PROTO_KAFKA)) return L7M_EINVAL;
  if (n && (!arena || !offs)) return L7M_EINVAL;
  std::lock_guard<std::mutex> g(t->mu);
  for (size_t i = 0; i < n; ++i) {
    const int32_t vd = verdicts[i];
    uint32_t p = port, ing = ingress ? 1u : 0u;
    if (proto == L7M_PROTO_HTTP) {
      // from the access-log entry: DestinationEndpoint.Port and the entry's
      // direction (pkg/envoy/accesslog_server.go:165-169)
      HttpView v;
      if (!http_rec(arena, arena_bytes, offs[i], &v)) {
        p = port;
      } else {
        p = v.dport;
        ing = (v.flags & L7M_HTTP_F_INGRESS) ? 1u : 0u;
      }
    } else {
      // the redirect's port and direction; port 0 is not counted, nor a
      // request ReadRequest rejected (the connection closes) (kafka.go:213-229,349-354)
      if (vd == L7M_VERDICT_PARSE_ERROR) continue;
    }
    uint32_t fv = flow_verdict(vd);
    if (proto == L7M_PROTO_KAFKA && vd == L7M_VERDICT_DENY) {
      // a denied request is answered with CreateResponse(ErrTopicAuthorizationFailed),
      // which fails for the kinds ReadRequest leaves untyped (request == nil,
      // request.go:174-175): the record is then logged as VerdictError
      // (kafka.go:246-252)
      size_t len = 0;
      KReq q;
      if (kafka_rec(arena, arena_bytes, offs[i], &len) && read_kafka(arena + offs[i], len, &q) == L7M_EUNSUPPORTED)
        fv = 2;
    }
    if (p == 0 && proto == L7M_PROTO_KAFKA) continue;
    l7m_proxy_stats& s = t->m[std::make_tuple(proto, p, ing, 1u)];
    s.received++;
    if (fv == 0) s.forwarded++;
    else if (fv == 1) s.denied++;
    else s.error++;
  }
  return L7M_OK;
}

size_t l7m_proxy_stats_get(l7m_proxy_stats_table* t, l7m_proxy_stats_entry* out, size_t cap) {
  if (!t) return 0;
  std::lock_guard<std::mutex> g(t->mu);
  size_t k = 0;
  for (const auto& e : t->m) {
    if (out && k < cap) {
      l7m_proxy_stats_entry& r = out[k];
      r.proto = std::get<0>(e.first);
      r.port = static_cast<uint16_t>(std::get<1>(e.first));
      r.ingress = static_cast<uint8_t>(std::get<2>(e.first));
      r.request = static_cast<uint8_t>(std::get<3>(e.first));
      r.stats = e.second;
    }
    ++k;
  }
  return k;
}

int l7m_proxy_stats_add(const int32_t* verdicts, size_t n, l7m_proxy_stats* st) {
  if ((n && !verdicts) || !st) return L7M_EINVAL;
  for (size_t i = 0; i < n; ++i) {
    const int32_t v = verdicts[i];
    st->received++;
    if (v >= 0) st->forwarded++;                 // VerdictForwarded
    else if (v == L7M_VERDICT_DENY) st->denied++;  // VerdictDenied
    else st->error++;                            // VerdictError: ReadRequest failed
  }
  return L7M_OK;
}

}  // extern "C"
