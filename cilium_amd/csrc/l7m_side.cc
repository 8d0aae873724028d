// l7m_side.cc — verdict side effects on the host (include/l7match.h):
//   * the 403 body Envoy's filter sends on deny (envoy/cilium_l7policy.cc:89-95,
//     169-181);
//   * the Kafka response the proxy sends for a denied request:
//     (*RequestMessage).CreateResponse(proto.ErrTopicAuthorizationFailed)
//     (pkg/kafka/request.go:158-182, pkg/kafka/response.go:81-303) serialised
//     as optiopay's Resp.Bytes(version) (vendor/.../proto/messages.go:595,
//     896, 1102, 1327, 1512, 1697, 1956);
//   * per-endpoint proxy statistics from a batch of verdicts
//     (Endpoint.UpdateProxyStatistics, pkg/endpoint/endpoint.go:2099-2122).
// These run only for requests the GPU already decided; no verdict is
// computed here.
#include <cstring>
#include <string>
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
  std::string str() {  // DecodeString: int16 length, < 1 -> ""
    const int16_t k = i16();
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
  std::vector<int32_t> parts;
};

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
  Rd r{req, len};
  r.i32();  // size
  const int16_t kind = r.i16(), version = r.i16();
  const int32_t corr = r.i32();
  if (r.err) return L7M_EINVAL;
  std::vector<TopicParts> topics;
  Wr w;
  w.i32(0);  // size placeholder
  w.i32(corr);
  auto partitions = [&](TopicParts& t, size_t fixed, bool produce, bool commit, int16_t v) {
    const int32_t np = r.arraylen();
    for (int32_t k = 0; k < np && !r.err; ++k) {
      t.parts.push_back(r.i32());
      if (produce) {
        const int32_t sz = r.i32();
        if (r.err) break;
        if (sz < 0 || sz > l7m::kKafkaMaxParseBuf) r.err = true;
        else r.pos += message_set_consumed(r.p + r.pos, r.n - r.pos, sz, v);
      } else if (commit) {
        r.skip(8 + (v == 1 ? 8 : 0));
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
      t.name = r.str();
      if (!names_only) partitions(t, fixed, produce, commit, version);
      topics.push_back(std::move(t));
    }
  };
  r.str();  // ClientID
  switch (kind) {
    case 0:  // ReadProduceReq -> ProduceResp.Bytes (messages.go:1697)
      if (version >= 3) r.str();
      r.skip(6);
      read_topics(0, true, false, false);
      if (r.err) return L7M_EINVAL;
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
    case 1:  // ReadFetchReq -> FetchResp.Bytes (messages.go:896)
      r.skip(12 + (version >= 3 ? 4 : 0) + (version >= 4 ? 1 : 0));
      read_topics(12 + (version >= 5 ? 8 : 0), false, false, false);
      if (r.err) return L7M_EINVAL;
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
    case 2:  // ReadOffsetReq -> OffsetResp.Bytes (messages.go:1956)
      r.skip(4 + (version >= 2 ? 1 : 0));
      read_topics(8 + (version == 0 ? 4 : 0), false, false, false);
      if (r.err) return L7M_EINVAL;
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
    case 3:  // ReadMetadataReq -> MetadataResp.Bytes (messages.go:595)
      read_topics(0, false, false, true);
      if (r.err) return L7M_EINVAL;
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
    case 8:  // ReadOffsetCommitReq -> OffsetCommitResp.Bytes (messages.go:1327)
      r.str();
      if (version >= 1) {
        r.skip(4);
        r.str();
      }
      if (version >= 2) r.skip(8);
      read_topics(0, false, true, false);
      if (r.err) return L7M_EINVAL;
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
    case 9:  // ReadOffsetFetchReq -> OffsetFetchResp.Bytes (messages.go:1512)
      r.str();
      read_topics(0, false, false, false);
      if (r.err) return L7M_EINVAL;
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
    case 10:  // ReadConsumerMetadataReq -> ConsumerMetadataResp.Bytes (messages.go:1102)
      r.str();
      if (version >= 1) r.skip(1);
      if (r.err) return L7M_EINVAL;
      if (version >= 1) w.i32(0);  // ThrottleTime
      w.i16(kErrTopicAuthorizationFailed);
      if (version >= 1) w.str("");  // ErrMsg
      w.i32(0);                     // CoordinatorID
      w.str("");                    // CoordinatorHost
      w.i32(0);                     // CoordinatorPort
      break;
    default:  // request == nil: "unsupported request API key" (request.go:176-177)
      return L7M_EUNSUPPORTED;
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
