// l7m_kafka.hip — CDNA4 (gfx950) kernel of the batched Kafka verdict path.
//
// One lane per request record (the raw size-prefixed wire request as
// proto.ReadReq returns it).  Each lane
//   1. decodes the request exactly as kafka.ReadRequest does
//      (pkg/kafka/request.go:186-229 -> vendor/github.com/optiopay/kafka/proto
//      messages.go per-kind readers, decoder error semantics of
//      serialization.go:31-196), including message-set walking with CRC-32
//      checks (messages.go:357-483, CRC table staged in LDS);
//   2. streams every topic name through the Topic -> rules hash table while it
//      is decoded (no per-request topic storage), and
//   3. resolves (*RequestMessage).MatchesRule (pkg/kafka/policy.go:200-225):
//        no topics             -> first rule i with ruleMatches
//        topics T (non-empty)  -> min(first Topic=="" rule with ruleMatches,
//                                     max over t in T of first rule with
//                                     Topic==t and ruleMatches)
//      which is the index at which the reference's ordered loop returns true
//      (the max term is the rule that removes the last uncovered topic).
// Verdicts: -1 deny, -2 ReadRequest error, -3 a compressed message set the
// second pass could not evaluate (queue / slab limits), i >= 0 allowed by rule i.
// Compressed (gzip / snappy) messages: the first pass queues their values and
// decides the request as if they decoded; kafka_codec_kernel then decodes
// each one and re-reads the decoded set (l7m_kcodec.h) and turns the
// request's verdict into -2 where the reference's ReadRequest would fail.
// Records are staged through LDS per wave tile exactly like the HTTP kernel
// (l7m_kernels.hip); the decoder then reads LDS.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../../include/l7match.h"
#include "l7m_device.h"
#include "l7m_kcodec.h"
#include "program.h"

namespace l7m {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// A view of a byte range with the optiopay decoder's sticky-error semantics:
// a short read consumes what is left (io.ReadFull) and sets err.
struct Rd {
  const uint8_t* p;
  uint32_t len;
  uint32_t pos;
  bool err;
};

__device__ __forceinline__ uint64_t rd_be(Rd& d, uint32_t n) {
  if (d.err) return 0;
  if (d.len - d.pos < n) {
    d.pos = d.len;
    d.err = true;
    return 0;
  }
  uint64_t v = 0;
  for (uint32_t i = 0; i < n; ++i) v = (v << 8) | d.p[d.pos + i];
  d.pos += n;
  return v;
}
__device__ __forceinline__ int8_t rd_i8(Rd& d) { return static_cast<int8_t>(rd_be(d, 1)); }
__device__ __forceinline__ int16_t rd_i16(Rd& d) { return static_cast<int16_t>(rd_be(d, 2)); }
__device__ __forceinline__ int32_t rd_i32(Rd& d) { return static_cast<int32_t>(rd_be(d, 4)); }

// n fixed-size bytes whose value is not needed.
__device__ __forceinline__ void rd_skip(Rd& d, uint32_t n) {
  if (d.err) return;
  if (d.len - d.pos < n) {
    d.pos = d.len;
    d.err = true;
    return;
  }
  d.pos += n;
}

// DecodeString (serialization.go:120-153): *off/*len of the bytes, len 0 = "".
__device__ __forceinline__ void rd_str(Rd& d, uint32_t* off, uint32_t* len) {
  *off = 0;
  *len = 0;
  if (d.err) return;
  const int16_t n = rd_i16(d);
  if (d.err || n < 1) return;
  if (d.len - d.pos < static_cast<uint32_t>(n)) {
    d.pos = d.len;
    d.err = true;
    return;
  }
  *off = d.pos;
  *len = static_cast<uint32_t>(n);
  d.pos += static_cast<uint32_t>(n);
}

// DecodeBytes (serialization.go:165-192), value discarded.
__device__ __forceinline__ void rd_skip_bytes(Rd& d) {
  if (d.err) return;
  const int32_t n = rd_i32(d);
  if (d.err || n < 1) return;
  if (n > kKafkaMaxParseBuf) {  // allocParseBuf
    d.err = true;
    return;
  }
  if (d.len - d.pos < static_cast<uint32_t>(n)) {
    d.pos = d.len;
    d.err = true;
    return;
  }
  d.pos += static_cast<uint32_t>(n);
}

// Branch-free forms of the readers for records staged in LDS, where reading
// up to 8 bytes past a range is harmless (the next record or the stage's
// 16-byte slack): the bytes are read unconditionally and the sticky-error
// state is updated with selects, so lanes whose reads fail do not split the
// wave's control flow.  Same results as the readers above.
struct RdL {
  __device__ static __forceinline__ uint64_t be(Rd& d, uint32_t n) {
    const bool ok = !d.err && d.len - d.pos >= n;
    uint64_t v = 0;
    for (uint32_t i = 0; i < n; ++i) v = (v << 8) | d.p[d.pos + i];
    d.err = !ok;
    d.pos = ok ? d.pos + n : d.len;
    return ok ? v : 0;
  }
  __device__ static __forceinline__ void skip(Rd& d, uint32_t n) {
    const bool ok = !d.err && d.len - d.pos >= n;
    d.err = !ok;
    d.pos = ok ? d.pos + n : d.len;
  }
  __device__ static __forceinline__ void str(Rd& d, uint32_t* off, uint32_t* len) {
    const bool was = d.err;
    const int16_t n = static_cast<int16_t>(be(d, 2));
    const bool valid = !d.err && n >= 1;
    const bool fits = valid && d.len - d.pos >= static_cast<uint32_t>(n);
    *off = fits ? d.pos : 0u;
    *len = fits ? static_cast<uint32_t>(n) : 0u;
    d.err = was || d.err || (valid && !fits);
    d.pos = fits ? d.pos + static_cast<uint32_t>(n) : (valid ? d.len : d.pos);
  }
};
// The branchy readers (any source, e.g. records read from HBM).
struct RdG {
  __device__ static __forceinline__ uint64_t be(Rd& d, uint32_t n) { return rd_be(d, n); }
  __device__ static __forceinline__ void skip(Rd& d, uint32_t n) { rd_skip(d, n); }
  __device__ static __forceinline__ void str(Rd& d, uint32_t* off, uint32_t* len) { rd_str(d, off, len); }
};

enum { kMsOk = 0, kMsErr = 1 };

// readMessageSet (messages.go:357-483) over the next `size` bytes of d.
// A gzip / snappy message sets `comp`: its value is decoded, and the request
// re-read, by the second pass (kafka_codec_kernel); a nil value cannot be
// decompressed (gzip.NewReader / snappy.Decode fail).
__device__ int read_message_set(Rd& d, int32_t size, int16_t version, const uint32_t* crc_tab, bool& comp) {
  if (size < 0 || size > kKafkaMaxParseBuf) return kMsErr;
  const uint32_t avail = d.len - d.pos;
  Rd r{d.p + d.pos, avail < static_cast<uint32_t>(size) ? avail : static_cast<uint32_t>(size), 0, false};
  int rc = kMsOk;
  for (;;) {
    rd_be(r, 8);  // offset
    if (r.err) break;
    const int32_t msz = rd_i32(r);
    if (r.err || msz <= 0) break;
    if (msz > kKafkaMaxParseBuf) {
      rc = kMsErr;
      break;
    }
    if (r.len - r.pos < static_cast<uint32_t>(msz)) {  // truncated last message
      r.pos = r.len;
      break;
    }
    const uint8_t* mb = r.p + r.pos;
    r.pos += static_cast<uint32_t>(msz);
    Rd m{mb, static_cast<uint32_t>(msz), 0, false};
    const uint32_t crc = static_cast<uint32_t>(rd_be(m, 4));
    if (msz <= 4) break;
    uint32_t c = 0xffffffffu;
    for (uint32_t i = 4; i < static_cast<uint32_t>(msz); ++i) c = crc_tab[(c ^ mb[i]) & 0xffu] ^ (c >> 8);
    if (crc != (c ^ 0xffffffffu)) break;  // ignore the rest of the set
    rd_i8(m);                              // magic
    const int8_t attr = rd_i8(m);
    if (version >= 1) rd_be(m, 8);         // timestamp
    const int cm = attr & 3;
    if (cm == 3) break;                    // `return nil, err` with err == nil
    rd_skip_bytes(m);                      // key
    const uint32_t vp = m.pos;
    rd_skip_bytes(m);                      // value
    if (m.err || (cm != 0 && m.pos - vp == 4)) {
      rc = kMsErr;
      break;
    }
    comp |= cm != 0;
  }
  d.pos += r.pos;
  return rc;
}

// Diagnostic builds (L7M_PROF, kProf): per-lane cycle accumulators
// (s_memtime): [0] start, [1] decode, [2] topic rounds, [3] ClientID, [4] eval.
#ifdef L7M_PROF
constexpr bool kProf = true;
#else
constexpr bool kProf = false;
#endif

struct KView {
  const uint32_t* prog;
  const KafkaRuleDesc* rules;
  const KafkaTopicSlot* slots;
  const KafkaTopicExt* ext;
  const uint64_t* kind_ok;  // LDS copy of the program's kind_ok table
  const KafkaClientSlot* clients;
  const uint32_t* pool;
  const uint8_t* strings;
  uint32_t n_slots, n_clients;
};

// The first 24 bytes of the name t[0..len) as little-endian words, zero
// past len, from aligned dword reads of the words that hold name bytes
// (records are dword aligned in both the LDS stage and the arena).
constexpr uint32_t kNameWords = kNameHashMinWords;
struct Name {
  uint32_t x[kNameWords];
  uint32_t hash;  // program.h name hash (table key)
};

// kLds: t is in the LDS stage, where reading past the name is harmless, so
// all seven words are read unconditionally; from HBM only the words that
// hold name bytes are.
template <bool kLds, bool kHash = true>
__device__ __forceinline__ Name load_name(const uint8_t* t, uint32_t len) {
  Name nm;
  const uint32_t sh = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(t)) & 3u;
  const uint32_t* a = reinterpret_cast<const uint32_t*>(t - sh);
  uint32_t w[kNameWords + 1];
#pragma unroll
  for (uint32_t k = 0; k <= kNameWords; ++k) w[k] = (kLds || 4 * k < sh + len) ? a[k] : 0u;
  uint32_t h = 0;
#pragma unroll
  for (uint32_t k = 0; k < kNameWords; ++k) {
    nm.x[k] = 0;
    if (__any(4 * k < len)) {  // words past every lane's name are skipped
      const uint32_t v = __builtin_amdgcn_alignbyte(w[k + 1], w[k], sh);
      const int32_t rem = static_cast<int32_t>(len) - static_cast<int32_t>(4 * k);
      nm.x[k] = rem >= 4 ? v : rem <= 0 ? 0u : v & ((1u << (8 * rem)) - 1u);
      if (kHash && rem > 0) h = name_hash_step(h, nm.x[k]);
    }
  }
  nm.hash = 0;
  if (!kHash) return nm;
  for (uint32_t i = 4 * kNameWords; i < len; i += 4) {  // names longer than 24 bytes
    uint32_t x = 0;
    for (uint32_t b = 0; b < 4 && i + b < len; ++b) x |= static_cast<uint32_t>(t[i + b]) << (8 * b);
    h = name_hash_step(h, x);
  }
  nm.hash = name_hash_final(h, len);
  return nm;
}

// t[0..len) (loaded as nm) == the table string whose first kInl bytes are
// inline in pfx (zero padded) and whose whole text is at rest.
template <uint32_t kInl>
__device__ __forceinline__ bool str_eq(const Name& nm, const uint8_t* t, uint32_t len,
                                       const uint32_t (&pfx)[kInl / 4], const uint8_t* rest) {
  static_assert(kInl <= 4 * kNameWords, "inline prefix longer than the loaded name");
  bool eq = true;
#pragma unroll
  for (uint32_t k = 0; k < kInl / 4; ++k) eq &= nm.x[k] == pfx[k];
  if (!eq) return false;
  for (uint32_t i = kInl; i < len; ++i)
    if (t[i] != rest[i]) return false;
  return true;
}

// ruleMatches (policy.go:144-195) minus CheckAPIKeyRole, which list
// membership already guarantees: version, then the ClientID condition when
// `check_client` (typed requests).  client = the request's interned ClientID
// (kNone when no rule names it).
__device__ __forceinline__ bool rest_ok(uint32_t flags, int32_t rversion, uint32_t rclient, int16_t version,
                                        bool check_client, uint32_t client) {
  if ((flags & kKRuleVersion) && rversion != version) return false;
  if (check_client && (flags & kKRuleClient) && rclient != client) return false;
  return true;
}

__device__ __forceinline__ bool key_ok(uint32_t flags, uint32_t keys_lo, uint32_t keys_hi, int32_t kind) {
  if (flags & kKRuleAnyKey) return true;
  if (kind < 0 || kind >= 64) return false;
  return kind < 32 ? ((keys_lo >> kind) & 1u) : ((keys_hi >> (kind - 32)) & 1u);
}

// First rule of an ascending candidate list (ids < limit) that applies to
// the source (gmask: its L7DataMap entries, GetRelevantRules) and passes
// rest_ok.
__device__ uint32_t first_in(const KView& v, Span s, uint32_t skip, uint32_t limit, int32_t kind, bool need_key,
                             int16_t version, bool check_client, uint32_t client, uint64_t gmask) {
  for (uint32_t j = skip; j < s.len; ++j) {
    const uint32_t rid = v.pool[s.off + j];
    if (rid >= limit) break;
    const KafkaRuleDesc r = v.rules[rid];
    if (((gmask >> r.group) & 1ull) && (!need_key || key_ok(r.flags, r.keys_lo, r.keys_hi, kind)) &&
        rest_ok(r.flags, r.version, r.client_idx, version, check_client, client))
      return rid;
  }
  return kNone;
}

// The request ClientID's index among the rules' ClientIDs (kNone if none).
template <bool kLds>
__device__ __forceinline__ uint32_t intern_client(const KView& v, const uint8_t* c, uint32_t len) {
  if (!len || !v.n_clients) return kNone;
  const Name nm = load_name<kLds>(c, len);
  const uint32_t hk = nm.hash;
  for (uint32_t at = hk & (v.n_clients - 1);; at = (at + 1) & (v.n_clients - 1)) {
    const KafkaClientSlot sl = v.clients[at];
    if (sl.hash == 0) return kNone;
    if (sl.hash == hk && sl.str_len == len && str_eq<kClientInline>(nm, c, len, sl.pfx, v.strings + sl.str_off))
      return sl.idx;
  }
}

// The topic's first rule whose CheckAPIKeyRole / version / ClientID
// conditions hold, once slot `at` is known to hold the topic: its first rule
// from the slot's own fields, later ones from the pool (kNone if none).
// kok: the request kind's kind_ok bits.
__device__ __forceinline__ uint32_t slot_first(const KView& v, const KafkaTopicSlot& sl, uint32_t at, uint64_t kok,
                                               int32_t kind, int16_t version, uint32_t client, uint64_t gmask) {
  const uint32_t m = sl.meta;
  if (((gmask >> (sl.r0_client >> 16)) & 1ull) && ((kok >> ((m >> 8) & 63u)) & 1ull) &&
      (!(m & kSlotVersionCond) || static_cast<int16_t>(m >> 16) == version) &&
      (!(m & kSlotClientCond) || (sl.r0_client & 0xffffu) == (client & 0xffffu)))
    return sl.r0 & ~kSlotMore;
  if (!(sl.r0 & kSlotMore)) return kNone;
  return first_in(v, v.ext[at].rules, 1, kNone, kind, true, version, true, client, gmask);
}

// Does slot `at` hold the name nm == t[0..tlen)?
__device__ __forceinline__ bool slot_is(const KView& v, const KafkaTopicSlot& sl, uint32_t at, uint32_t hash,
                                        const Name& nm, const uint8_t* t, uint32_t tlen) {
  if (sl.hash != hash || (sl.meta & 0xffu) != tlen) return false;
  const uint8_t* rest = tlen > kTopicInline ? v.strings + v.ext[at].str_off : nullptr;
  return str_eq<kTopicInline>(nm, t, tlen, sl.pfx, rest);
}

// Probe from slot `at` (already fetched as sl) for the name nm.
__device__ __forceinline__ uint32_t probe_topic(const KView& v, KafkaTopicSlot sl, uint32_t hash, const Name& nm,
                                                const uint8_t* t, uint32_t tlen, uint64_t kok, int32_t kind,
                                                int16_t version, uint32_t client, uint64_t gmask) {
  for (uint32_t at = hash & (v.n_slots - 1);;) {
    if (sl.hash == 0) return kNone;
    if (slot_is(v, sl, at, hash, nm, t, tlen)) return slot_first(v, sl, at, kok, kind, version, client, gmask);
    at = (at + 1) & (v.n_slots - 1);
    sl = v.slots[at];
  }
}

// First rule whose Topic is t[0..tlen) and whose CheckAPIKeyRole / version /
// ClientID conditions hold (kNone if none): the per-topic term of the
// reqTopicsMap coverage walk (policy.go:210-223).
template <bool kLds>
__device__ __forceinline__ uint32_t topic_first(const KView& v, const uint8_t* t, uint32_t tlen, uint64_t kok,
                                                int32_t kind, int16_t version, uint32_t client, uint64_t gmask) {
  if (!tlen || tlen > kMaxTopicLen || !v.n_slots) return kNone;
  const Name nm = load_name<kLds>(t, tlen);
  return probe_topic(v, v.slots[nm.hash & (v.n_slots - 1)], nm.hash, nm, t, tlen, kok, kind, version, client, gmask);
}

// Topics are resolved after the decode, all lanes of the wave together
// (the decode itself diverges by request kind): each lane parks the offsets
// of its first kTopicQ topic names in its LDS column and the lookups run in
// lock-step rounds.  Because MatchesRule's result is
//   min(j, max over topics of f(t))   (f(t) = topic_first, kNone = uncovered)
// with j the first Topic=="" rule, the per-topic terms need neither j nor
// any order, so a lane whose request has more topics resolves the excess
// ones during the decode.
constexpr uint32_t kTopicQ = 4;

// One record whose first `limit` bytes are readable at rec (LDS stage or HBM).
// tq: this lane's topic column in LDS (kTopicQ u16 name offsets, stride 64);
// used by the LDS-staged path only (stage offsets fit 16 bits).
// spans: the header's per-kind candidate lists staged in LDS (kSpanLds);
// kLds: rec is in the LDS stage.
template <bool kLds>
__device__ __forceinline__ int32_t eval_kafka(const KView& v, const Span* spans, const uint8_t* rec,
                                              uint64_t limit, const uint32_t* crc_tab, uint16_t* tq,
                                              uint64_t gmask, bool& comp, uint64_t (&prof)[5]) {
  if constexpr (kProf && kLds) prof[0] = __builtin_amdgcn_s_memtime();
  if (limit < 4) return L7M_VERDICT_PARSE_ERROR;
  const int32_t msize = static_cast<int32_t>((static_cast<uint32_t>(rec[0]) << 24) |
                                             (static_cast<uint32_t>(rec[1]) << 16) |
                                             (static_cast<uint32_t>(rec[2]) << 8) | rec[3]);
  // ReadReq: size <= 0 / short kind read / allocParseBuf; ReadRequest: len < 12.
  if (msize < 8 || static_cast<int64_t>(msize) + 4 > kKafkaMaxParseBuf) return L7M_VERDICT_PARSE_ERROR;
  if (4 + static_cast<uint64_t>(msize) > limit) return L7M_VERDICT_PARSE_ERROR;
  const int32_t kind = static_cast<int16_t>((rec[4] << 8) | rec[5]);
  const int16_t version = static_cast<int16_t>((rec[6] << 8) | rec[7]);  // request.go:72-74
  const uint32_t kidx = (kind >= 0 && kind < 64) ? static_cast<uint32_t>(kind) : 64u;

  using R = typename std::conditional<kLds, RdL, RdG>::type;
  auto arraylen = [](Rd& d, int32_t* n) -> bool {  // DecodeArrayLen (serialization.go:155-163)
    const int32_t v = static_cast<int32_t>(R::be(d, 4));
    if (v < 0 || v > kKafkaMaxParseBuf) return false;
    *n = v;
    return true;
  };
  uint32_t first = kNone;
  const bool typed = kind == 0 || kind == 1 || kind == 2 || kind == 3 || kind == 8 || kind == 9 || kind == 10;
  if (!typed) {
    // request == nil: matchNonTopicRequests (policy.go:54-70), ClientID ignored.
    const bool topic_kind = kind >= 0 && kind < 64 && ((kTopicApiKeyMask >> kind) & 1ull);
    first = first_in(v, topic_kind ? spans[kidx] : spans[kKafkaKinds + kidx], 0, kNone, kind, false,
                     version, false, kNone, gmask);
  } else {
    Rd d{rec, 4u + static_cast<uint32_t>(msize), 12, false};
    uint32_t coff, clen;
    R::str(d, &coff, &clen);
    const uint8_t* client = rec + coff;
    const uint64_t tc0 = kProf ? __builtin_amdgcn_s_memtime() : 0;
    const uint32_t cid = intern_client<kLds>(v, client, clen);
    const uint64_t kok = v.kind_ok[kidx];
    if constexpr (kProf && kLds) prof[3] += __builtin_amdgcn_s_memtime() - tc0;

    int32_t ntop = 0;
    bool ok = true;
    uint32_t maxf = 0, nq = 0;
    auto start_topics = [&](int32_t n) { ntop = n; };
    auto topic = [&]() {
      uint32_t toff, tlen;
      R::str(d, &toff, &tlen);
      if (d.err || maxf == kNone) return;
      if (!tlen) {
        maxf = kNone;
      } else if (kLds && nq < kTopicQ) {
        tq[64 * nq] = static_cast<uint16_t>(toff);
        ++nq;
      } else {
        const uint32_t f = topic_first<kLds>(v, rec + toff, tlen, kok, kind, version, cid, gmask);
        maxf = f > maxf ? f : maxf;
      }
    };
    // The per-kind readers (messages.go) share one shape: kind-specific
    // leading fields, the topic array (name + kind-specific partition
    // array), kind-specific trailing fields.  Only the leading / trailing
    // fields and the variable-size partition entries (Produce message sets,
    // OffsetCommit metadata strings) are decoded per kind; the topic loop is
    // common, so lanes holding different kinds walk it together.  A run of
    // fixed-size reads is one rd_skip: under the sticky-error semantics it
    // fails exactly when one of the reads would.
    uint32_t a, b;
    switch (kind) {
      case 0:  // ReadProduceReq messages.go:1572-1628
        if (version >= 3) R::str(d, &a, &b);  // transactional id
        R::skip(d, 2 + 4);                    // acks, timeout
        break;
      case 1:  // ReadFetchReq messages.go:752-809
        R::skip(d, 12 + (version >= 3 ? 4 : 0) + (version >= 4 ? 1 : 0));
        break;
      case 2:  // ReadOffsetReq messages.go:1791-1839
        R::skip(d, 4 + (version >= 2 ? 1 : 0));
        break;
      case 8:  // ReadOffsetCommitReq messages.go:1158-1213
        R::str(d, &a, &b);
        if (version >= 1) {
          R::skip(d, 4);
          R::str(d, &a, &b);
        }
        if (version >= 2) R::skip(d, 8);
        break;
      case 9:  // ReadOffsetFetchReq messages.go:1374-1411
        R::str(d, &a, &b);
        break;
      case 10:  // ReadConsumerMetadataReq messages.go:1018-1039: no topics
        R::str(d, &a, &b);
        if (version >= 1) R::skip(d, 1);
        break;
      default:  // 3: ReadMetadataReq messages.go:493-522
        break;
    }
    int32_t n = 0;
    if (kind != 10 && !arraylen(d, &n)) ok = false;
    start_topics(n);
    // Fixed partition entry sizes (0: variable or no partition array).
    const uint32_t esz = kind == 1 ? 16u + (version >= 5 ? 8u : 0u)
                       : kind == 2 ? 12u + (version == 0 ? 4u : 0u)
                       : kind == 9 ? 4u : 0u;
    for (int32_t t = 0; t < n && ok && !d.err; ++t) {
      topic();
      if (kind == 3 || d.err) continue;
      int32_t np;
      if (!arraylen(d, &np)) {
        ok = false;
        break;
      }
      if (esz) {
        const uint64_t need = static_cast<uint64_t>(np) * esz;
        if (d.len - d.pos < need) {
          d.pos = d.len;
          d.err = true;
        } else {
          d.pos += static_cast<uint32_t>(need);
        }
      } else if (kind == 0) {
        for (int32_t p = 0; p < np; ++p) {
          R::skip(d, 4);  // partition
          const int32_t mss = static_cast<int32_t>(R::be(d, 4));
          if (d.err) break;
          if (read_message_set(d, mss, version, crc_tab, comp) == kMsErr) {
            ok = false;
            break;
          }
        }
      } else {  // 8
        for (int32_t p = 0; p < np && !d.err; ++p) {
          R::skip(d, 4 + 8 + (version == 1 ? 8 : 0));
          R::str(d, &a, &b);
        }
      }
    }
    if (kind == 3 && version >= 4) R::skip(d, 1);
    if (!ok || d.err) return L7M_VERDICT_PARSE_ERROR;
    if (kind == 10) {
      // ConsumerMetadataReq: GetTopics() is nil and ruleMatches -> true.
      first = first_in(v, spans[kKafkaKinds + kidx], 0, kNone, kind, false, version, false, kNone, gmask);
    } else if (ntop == 0) {
      first = first_in(v, spans[kKafkaKinds + kidx], 0, kNone, kind, false, version, true, cid, gmask);
    } else {
      const uint64_t tr0 = kProf ? __builtin_amdgcn_s_memtime() : 0;
      if constexpr (kProf && kLds) prof[1] += tr0 - prof[0];
      // The parked topics' home-slot heads (hash, meta, first rule) are
      // fetched together, so the lookups of a request cost one dependent
      // L2 round trip instead of one per topic; the second pass compares
      // names against the slots' inline prefixes (same cache line).
      uint32_t hs[kTopicQ];
      u32x4 hd[kTopicQ];
#pragma unroll
      for (uint32_t r = 0; r < kTopicQ; ++r) {
        hs[r] = 0;
        hd[r] = u32x4{0u, 0u, 0u, 0u};
        if (r < nq && maxf != kNone) {
          const uint32_t toff = tq[64 * r];
          const uint32_t tlen = (static_cast<uint32_t>(rec[toff - 2]) << 8) | rec[toff - 1];
          if (tlen && tlen <= kMaxTopicLen && v.n_slots) {
            hs[r] = load_name<kLds>(rec + toff, tlen).hash;
            hd[r] = reinterpret_cast<const u32x4*>(v.slots + (hs[r] & (v.n_slots - 1)))[0];
          }
        }
      }
#pragma unroll
      for (uint32_t r = 0; r < kTopicQ; ++r) {
        if (r < nq && maxf != kNone) {
          uint32_t f = kNone;
          if (hs[r] && hd[r].x != 0) {
            const uint32_t toff = tq[64 * r];
            const uint32_t tlen = (static_cast<uint32_t>(rec[toff - 2]) << 8) | rec[toff - 1];
            const uint32_t at = hs[r] & (v.n_slots - 1);
            KafkaTopicSlot sl;
            sl.hash = hd[r].x;
            sl.meta = hd[r].y;
            sl.r0 = hd[r].z;
            sl.r0_client = hd[r].w;
            const u32x4 pf = reinterpret_cast<const u32x4*>(v.slots + at)[1];
            sl.pfx[0] = pf.x;
            sl.pfx[1] = pf.y;
            sl.pfx[2] = pf.z;
            sl.pfx[3] = pf.w;
            const Name nm = load_name<kLds, false>(rec + toff, tlen);
            f = probe_topic(v, sl, hs[r], nm, rec + toff, tlen, kok, kind, version, cid, gmask);
          }
          maxf = f > maxf ? f : maxf;
        }
      }
      const uint32_t j = first_in(v, spans[kidx], 0, maxf, kind, false, version, true, cid, gmask);
      first = j < maxf ? j : maxf;
      if constexpr (kProf && kLds) prof[2] += __builtin_amdgcn_s_memtime() - tr0;
    }
  }
  return first == kNone ? L7M_VERDICT_DENY : static_cast<int32_t>(first);
}

__device__ __forceinline__ void count_slot(unsigned long long* __restrict__ hits, uint32_t slot, bool active) {
  uint64_t todo = __ballot(active);
  const uint32_t lane = __lane_id();
  while (todo) {
    const uint32_t leader = __builtin_ctzll(todo);
    const uint32_t key = __shfl(slot, leader);
    const uint64_t same = __ballot(active && slot == key) & todo;
    if (lane == leader) atomicAdd(hits + key, static_cast<unsigned long long>(__popcll(same)));
    todo &= ~same;
  }
}

constexpr uint32_t kKWaves = 16;
constexpr uint32_t kKBlock = 64 * kKWaves;
constexpr uint32_t kKMaxStage = 6144;
constexpr uint32_t kKCopyIters = kKMaxStage / 1024;  // 16-byte loads per lane
constexpr uint32_t kKLdsBytes = 160 * 1024;
constexpr uint32_t kKMaxLdsCounters = 16384;
constexpr uint32_t kSpanLds = (4 * kKafkaKinds + 3) & ~3u;  // words
constexpr uint32_t kKindOkLds = (2 * kKafkaKinds + 3) & ~3u;  // words
constexpr uint32_t kMaxCliLdsBytes = 8192;  // client table copied to LDS up to this size

__device__ __forceinline__ uint64_t shfl64(uint64_t x, uint32_t src) {
  const uint32_t lo = __shfl(static_cast<uint32_t>(x), src);
  const uint32_t hi = __shfl(static_cast<uint32_t>(x >> 32), src);
  return (static_cast<uint64_t>(hi) << 32) | lo;
}

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

enum KHitMode { kKNoHits = 0, kKLdsHits = 1, kKGlobalHits = 2 };

// Persistent layout as the HTTP kernel: one 1024-thread workgroup per CU,
// each wave consumes its contiguous share of the batch in tiles of <= 64
// records copied HBM -> the wave's LDS stage (coalesced 16-byte loads, the
// next tile's bytes in flight while this one is decoded); a record outside
// its tile window is decoded from HBM.
// kAblate (diagnostics only, L7M_FLAG_DIAG_*): 1 = stage records, no
// decoding; 2 = decode without table lookups.
// kGroups: the program's rules belong to several L7DataMap entries, so each
// request's source identity selects the rules that apply (else all do).
// One workgroup's share (`part` of `nparts`) of a batch: the grid of
// kafka_eval_kernel, or the single workgroup of kafka_resident_kernel, which
// keeps the LDS tables of the previous batch when the program is the same
// (load_tables false).
template <int kHits, int kAblate, bool kCliLds, bool kGroups>
__device__ __forceinline__ void kafka_eval_body(const uint32_t* __restrict__ prog, const uint8_t* __restrict__ arena,
                                                uint64_t arena_bytes, const uint64_t* __restrict__ offs, uint64_t n,
                                                int32_t* __restrict__ verdicts,
                                                unsigned long long* __restrict__ hits, uint32_t stage,
                                                uint32_t* __restrict__ crecs, uint32_t* qhdr, uint32_t qcap,
                                                const uint32_t* __restrict__ ids, bool load_tables, uint32_t part,
                                                uint32_t nparts, uint32_t wave_index, uint32_t wave_count) {
  extern __shared__ __align__(16) uint32_t ksmem[];
  uint64_t prof[5] = {0, 0, 0, 0, 0};  // (kProf diagnostic builds)
  const KafkaHeader& h = *reinterpret_cast<const KafkaHeader*>(prog);
  const uint32_t tid = threadIdx.x, lane = tid & 63u, wv = tid >> 6;
  const uint32_t n_ctr = h.n_rules + 2;
  // LDS: crc | spans | kind_ok | client table (kCliLds) | counters (kKLdsHits) | topic columns | stages
  uint32_t* crc_tab = ksmem;
  Span* spans = reinterpret_cast<Span*>(ksmem + 256);
  uint64_t* kind_ok = reinterpret_cast<uint64_t*>(ksmem + 256 + kSpanLds);
  uint32_t* cli = ksmem + 256 + kSpanLds + kKindOkLds;
  const uint32_t cli_words = kCliLds ? h.n_clients * (sizeof(KafkaClientSlot) / 4) : 0u;
  uint32_t* ctr = cli + cli_words;
  uint16_t* tq = reinterpret_cast<uint16_t*>(ctr + (kHits == kKLdsHits ? ((n_ctr + 3u) & ~3u) : 0u));
  uint8_t* stg = reinterpret_cast<uint8_t*>(tq + kKWaves * 64 * kTopicQ) + wv * (stage + 16u);
  tq += wv * 64 * kTopicQ + lane;
  static_assert(offsetof(KafkaHeader, all_by_kind) == offsetof(KafkaHeader, notopic_by_kind) + 8 * kKafkaKinds,
                "span arrays are adjacent");
  if (load_tables) {
    if (kCliLds)
      for (uint32_t i = tid; i < cli_words; i += kKBlock) cli[i] = prog[h.off_clients + i];
    for (uint32_t i = tid; i < 2 * kKafkaKinds; i += kKBlock) ksmem[256 + kSpanLds + i] = prog[h.off_kind_ok + i];
    for (uint32_t i = tid; i < 256; i += kKBlock) crc_tab[i] = prog[h.off_crc + i];
    for (uint32_t i = tid; i < 4 * kKafkaKinds; i += kKBlock)
      ksmem[256 + i] = prog[offsetof(KafkaHeader, notopic_by_kind) / 4 + i];
  }
  if (kHits == kKLdsHits)
    for (uint32_t i = tid; i < n_ctr; i += kKBlock) ctr[i] = 0;
  __syncthreads();
  KView v;
  v.prog = prog;
  v.rules = reinterpret_cast<const KafkaRuleDesc*>(prog + h.off_rules);
  v.slots = reinterpret_cast<const KafkaTopicSlot*>(prog + h.off_slots);
  v.ext = reinterpret_cast<const KafkaTopicExt*>(prog + h.off_ext);
  v.kind_ok = kind_ok;
  v.clients = reinterpret_cast<const KafkaClientSlot*>(kCliLds ? cli : prog + h.off_clients);
  v.n_clients = kAblate == 2 ? 0 : h.n_clients;
  v.pool = prog + h.off_pool;
  v.strings = reinterpret_cast<const uint8_t*>(prog + h.off_strings);
  v.n_slots = kAblate == 2 ? 0 : h.n_slots;

  const uint64_t gw = wave_index;  // this wave's share of the batch: wave wave_index of wave_count
  const uint64_t nw = wave_count;
  const uint64_t end = n * (gw + 1) / nw;
  struct Tile {
    uint64_t cur, o, onext, base;
    uint32_t k, bytes, take;
  };
  auto load_offs = [&](uint64_t cur, uint64_t* o, uint64_t* onext) {
    *o = 0;
    *onext = 0;
    if (cur < end && lane < end - cur) {
      *o = offs[cur + lane];
      *onext = cur + lane + 1 < n ? offs[cur + lane + 1] : arena_bytes;
    }
  };
  auto plan = [&](uint64_t cur, uint64_t o, uint64_t onext) -> Tile {
    Tile t;
    t.cur = cur;
    t.o = o;
    t.onext = onext;
    if (cur >= end) {
      t.base = 0;
      t.k = t.bytes = t.take = 0;
      return t;
    }
    const uint64_t m = end - cur < 64 ? end - cur : 64;
    const uint64_t o0 = shfl64(o, 0);
    t.base = o0 & ~15ull;
    const bool ok = lane < m && (o & 3) == 0 && o >= o0 && onext >= o && onext <= arena_bytes &&
                    onext - t.base <= stage;
    const uint64_t okm = __ballot(ok);
    t.k = okm == ~0ull ? 64u : static_cast<uint32_t>(__builtin_ctzll(~okm));
    t.bytes = t.k ? static_cast<uint32_t>(shfl64(onext, t.k - 1) - t.base) : 0u;
    t.take = t.k ? t.k : 1u;
    return t;
  };
  // Register staging: the next tile's bytes are loaded into VGPRs at the top
  // of the iteration and written to the stage at the top of the next one.
  // (LDS-DMA staging issued after the lookups measured slower here: 4.30 vs
  // 4.22 ms, profiles/r03/ab_round3.md: the decode alone does not cover the
  // HBM latency.)
  u32x4 buf[kKCopyIters];
  auto issue_bytes = [&](const Tile& t) {
    const u32x4* src = reinterpret_cast<const u32x4*>(arena + t.base);
#pragma unroll
    for (uint32_t it = 0; it < kKCopyIters; ++it) {
      const uint32_t q = it * 64u + lane;
      if (q * 16u < t.bytes) buf[it] = __builtin_nontemporal_load(src + q);
    }
  };
  uint64_t o1, n1, o2, n2;
  load_offs(n * gw / nw, &o1, &n1);
  Tile t = plan(n * gw / nw, o1, n1);
  issue_bytes(t);
  load_offs(t.cur + t.take, &o2, &n2);
  while (t.cur < end) {
#pragma unroll
    for (uint32_t it = 0; it < kKCopyIters; ++it) {
      const uint32_t q = it * 64u + lane;
      if (q * 16u < t.bytes) reinterpret_cast<u32x4*>(stg)[q] = buf[it];
    }
    wave_sync();
    const Tile t2 = plan(t.cur + t.take, o2, n2);
    issue_bytes(t2);
    load_offs(t2.cur + t2.take, &o2, &n2);

    const uint64_t o = t.o, onext = t.onext;
    int32_t verdict = 0;
    const uint64_t te0 = kProf ? __builtin_amdgcn_s_memtime() : 0;
    // GetRelevantRules (pkg/policy/l4.go:110-129): the L7DataMap entries whose
    // rules apply to this request's source identity
    uint64_t gmask = ~0ull;
    if (kGroups && lane < t.take) {
      const KafkaIdSlot* it = reinterpret_cast<const KafkaIdSlot*>(prog + h.off_ids);
      gmask = (static_cast<uint64_t>(it[0].mask_hi) << 32) | it[0].mask_lo;
      const uint32_t id = ids ? ids[t.cur + lane] : 0u;
      for (uint32_t at = kafka_id_hash(id) & (h.n_id_slots - 1); id; at = (at + 1) & (h.n_id_slots - 1)) {
        const KafkaIdSlot e = it[1 + at];
        if (e.identity == 0) break;  // not listed: the reference's nil identity
        if (e.identity == id) {
          gmask = (static_cast<uint64_t>(e.mask_hi) << 32) | e.mask_lo;
          break;
        }
      }
    }
    if (lane < t.take) {
      bool done = false, comp = false;
      if (lane < t.k && onext - o >= 4) {
        const uint8_t* rec = stg + (o - t.base);
        const uint32_t msize = (static_cast<uint32_t>(rec[0]) << 24) | (static_cast<uint32_t>(rec[1]) << 16) |
                               (static_cast<uint32_t>(rec[2]) << 8) | rec[3];
        if (kAblate == 1) {
          verdict = static_cast<int32_t>(msize & 1u) - 1;
          done = true;
        } else if (msize < 0x7ffffff0u && ((4ull + msize + 3) & ~3ull) <= onext - o) {
          verdict = eval_kafka<true>(v, spans, rec, onext - o, crc_tab, tq, gmask, comp, prof);
          done = true;
        }
      }
      if (!done) {  // outside the staged window: decode from HBM
        const bool inb = (o & 3) == 0 && o + 4 <= arena_bytes;
        verdict = inb ? eval_kafka<false>(v, spans, arena + o, arena_bytes - o, crc_tab, tq, gmask, comp, prof)
                      : L7M_VERDICT_PARSE_ERROR;
      }
      if (comp && verdict != L7M_VERDICT_PARSE_ERROR) {  // queue the request for the second pass
        const uint32_t at = atomicAdd(qhdr, 1u);
        if (at < qcap) crecs[at] = static_cast<uint32_t>(t.cur + lane);
        else verdict = L7M_VERDICT_UNSUPPORTED;
      }
      verdicts[t.cur + lane] = verdict;
    }
    if constexpr (kProf) prof[4] += __builtin_amdgcn_s_memtime() - te0;
    if (kHits != kKNoHits) {
      uint32_t slot = kNone;
      if (lane < t.take) slot = verdict >= 0 ? static_cast<uint32_t>(verdict) + 2 : (verdict == -1 ? 0u : 1u);
      if (kHits == kKLdsHits) {
        if (slot != kNone) atomicAdd(ctr + slot, 1u);
      } else {
        count_slot(hits, slot, slot != kNone);
      }
    }
    wave_sync();  // the stage is overwritten by the next tile
    t = t2;
  }
  if (kProf && part == 0 && wv == 0) {
    for (int k = 0; k < 5; ++k)
      for (uint32_t m = 1; m < 64; m <<= 1) {
        const uint64_t o2 = shfl64(prof[k], lane ^ m);
        prof[k] = o2 > prof[k] ? o2 : prof[k];
      }
    if (lane == 0)
      printf("L7M_PROF decode %llu client %llu rounds %llu eval %llu\n", (unsigned long long)prof[1],
             (unsigned long long)prof[3], (unsigned long long)prof[2], (unsigned long long)prof[4]);
  }
  if (kHits == kKLdsHits) {
    __syncthreads();
    for (uint32_t i = tid; i < n_ctr; i += kKBlock)
      if (ctr[i]) atomicAdd(hits + i, static_cast<unsigned long long>(ctr[i]));
  }
}

template <int kHits, int kAblate, bool kCliLds, bool kGroups>
__global__ __launch_bounds__(kKBlock) void kafka_eval_kernel(const uint32_t* __restrict__ prog,
                                                             const uint8_t* __restrict__ arena, uint64_t arena_bytes,
                                                             const uint64_t* __restrict__ offs, uint64_t n,
                                                             int32_t* __restrict__ verdicts,
                                                             unsigned long long* __restrict__ hits, uint32_t stage,
                                                             uint32_t* __restrict__ crecs, uint32_t* qhdr,
                                                             uint32_t qcap, const uint32_t* __restrict__ ids) {
  kafka_eval_body<kHits, kAblate, kCliLds, kGroups>(prog, arena, arena_bytes, offs, n, verdicts, hits, stage, crecs,
                                                    qhdr, qcap, ids, true, blockIdx.x, gridDim.x,
                                                    blockIdx.x * kKWaves + (threadIdx.x >> 6), gridDim.x * kKWaves);
}

__device__ __forceinline__ uint64_t uniform64(uint64_t v) {  // uniform: in SGPRs
  const uint32_t lo = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v));
  const uint32_t hi = __builtin_amdgcn_readfirstlane(static_cast<uint32_t>(v >> 32));
  return (static_cast<uint64_t>(hi) << 32) | lo;
}
__device__ __forceinline__ void resident_exit(ResidentBox* box) {
  if (threadIdx.x == 0) __hip_atomic_store(&box->exited, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t resident_load(const uint64_t* p) {
  return uniform64(__hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
}

// Resident Kafka evaluator for the batcher's small batches (l7m_batch.cc):
// ONE workgroup stays on the GPU and polls a mailbox in pinned host memory
// (ResidentBox, l7m_device.h), so a batch costs no kernel launch, no
// completion signal and no LDS table load (kept while the program is the
// same).  Per round: wait until post_seq reaches the next sequence number,
// read every posted slot (one per wave group), evaluate them together with
// the kafka_eval_kernel code, publish done_seq.  Exit (every wave takes the
// same branch after a barrier): quit set by the host, a slot for another
// instantiation (the host relaunches the right one), or kResidentIdleTicks
// of s_memrealtime without work, so the workgroup drains by itself when its
// process ends.  Memory: mailbox fields are read and written with relaxed
// system-scope atomics; per round one thread invalidates the L1 / L2 before
// the records are read and one writes the L2 back after every thread's
// verdict stores have been acknowledged.  Requests with compressed message sets
// need the codec pass (kafka_codec_kernel): the resident workgroup has no
// queue (capacity 0), counts them, and reports the batch back (slot.result
// = 1) so the host evaluates that batch with the normal launches.
template <bool kCliLds, bool kGroups>
__global__ __launch_bounds__(kKBlock) void kafka_resident_kernel(ResidentBox* box, uint64_t seq, uint32_t* qhdr) {
  extern __shared__ __align__(16) uint32_t ksmem[];
  const uint32_t tid = threadIdx.x, wv = tid >> 6;
  // broadcast: [0] decision, [1] detection time, [2] post_seq seen, [4 + 16 b ...] slot b
  uint64_t* bc = reinterpret_cast<uint64_t*>(ksmem + kKLdsBytes / 4 - kResidentLdsWords);
  const uint32_t* cur = nullptr;
  uint64_t cur_gen = 0, rounds = resident_load(&box->rounds);
  const uint64_t my_kind = kResidentKafka | (kCliLds ? 1u : 0u) | (kGroups ? 2u : 0u);
  for (;;) {
    if (tid == 0) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      uint64_t act = 0, ps = 0;
      for (uint32_t it = 1;; ++it) {  // one host-memory read per poll; quit and the idle limit every 64th
        ps = resident_load(&box->post_seq);
        if (ps >= seq) {
          act = 1;
          break;
        }
        if (!(it & 63) && (resident_load(&box->quit) || __builtin_amdgcn_s_memrealtime() - t0 > kResidentIdleTicks))
          break;
      }
      bc[0] = act;
      bc[1] = __builtin_amdgcn_s_memrealtime();
      bc[2] = ps;
      if (act) __atomic_thread_fence(__ATOMIC_ACQUIRE);  // one L1 / L2 invalidation per round: its records
    }
    __syncthreads();
    const uint64_t act = bc[0];
    const uint32_t pend = static_cast<uint32_t>(
        act ? (bc[2] - seq + 1 < kResidentRound ? bc[2] - seq + 1 : kResidentRound) : 0);
    if (tid < 16 * pend)  // every posted slot in one round trip
      bc[4 + tid] = __hip_atomic_load(reinterpret_cast<const uint64_t*>(&box->slots[(seq + tid / 16) % kResidentSlots]) +
                                          (tid & 15u),
                                      __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __syncthreads();
    if (!act) return resident_exit(box);
    const ResidentSlot* rs = reinterpret_cast<const ResidentSlot*>(bc + 4);
    if (uniform64(rs[0].kind) != my_kind) return resident_exit(box);  // another instantiation: the host relaunches
    const uint64_t gen = uniform64(rs[0].gen), prog0 = uniform64(rs[0].prog);
    uint32_t nb = 1;
    while (nb < pend && rs[nb].kind == rs[0].kind && rs[nb].gen == gen && rs[nb].prog == prog0) ++nb;
    nb = __builtin_amdgcn_readfirstlane(nb);
    const uint32_t b = wv % nb, wi = wv / nb, wc = (kKWaves - b + nb - 1) / nb;
    const ResidentSlot& sl = rs[b];
    const uint32_t* prog = reinterpret_cast<const uint32_t*>(prog0);
    const uint8_t* arena = reinterpret_cast<const uint8_t*>(uniform64(sl.arena));
    const uint64_t* offs = reinterpret_cast<const uint64_t*>(uniform64(sl.offs));
    int32_t* verdicts = reinterpret_cast<int32_t*>(uniform64(sl.verdicts));
    const uint32_t* ids = reinterpret_cast<const uint32_t*>(uniform64(sl.ids));
    const uint64_t arena_bytes = uniform64(sl.arena_bytes), n = uniform64(sl.n);
    const uint32_t stage = static_cast<uint32_t>(uniform64(rs[0].stage));
    const uint64_t t_read = __builtin_amdgcn_s_memrealtime();
    kafka_eval_body<kKNoHits, 0, kCliLds, kGroups>(prog, arena, arena_bytes, offs, n, verdicts, nullptr, stage,
                                                   nullptr, qhdr, 0, ids, prog != cur || gen != cur_gen, 0, 1, wi, wc);
    cur = prog;
    cur_gen = gen;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      const uint64_t t_body = __builtin_amdgcn_s_memrealtime();
      __threadfence_system();  // one L2 write-back per round: the verdicts, then done_seq
      const uint64_t t_sync = __builtin_amdgcn_s_memrealtime();
      const uint64_t st[4] = {bc[1], t_read, t_body, t_sync};
      // a compressed set anywhere in the round: its batches go to the normal launches
      const uint32_t queued = __hip_atomic_load(qhdr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(qhdr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (uint32_t q = 0; q < nb; ++q) {
        ResidentSlot* slp = &box->slots[(seq + q) % kResidentSlots];
        for (int k = 0; k < 4; ++k)
          __hip_atomic_store(&slp->stamp[k], st[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&slp->result, queued ? 1ull : 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
      __hip_atomic_store(&box->rounds, ++rounds, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&box->done_seq, seq + nb - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    seq += nb;
    __syncthreads();  // bc is rewritten by the next round
  }
}

template <int kHits, int kAblate = 0, bool kCliLds = false, bool kGroups = false>
static hipError_t launch_k(dim3 grid, size_t lds, hipStream_t stream, const uint32_t* dprog, const uint8_t* arena,
                           uint64_t arena_bytes, const uint64_t* offs, uint64_t n, int32_t* verdicts,
                           unsigned long long* hits, uint32_t stage, const KafkaCodecQueue& cq, const uint32_t* ids) {
  const hipError_t e =
      set_lds_attr_once(reinterpret_cast<const void*>(kafka_eval_kernel<kHits, kAblate, kCliLds, kGroups>), kKLdsBytes);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((kafka_eval_kernel<kHits, kAblate, kCliLds, kGroups>), grid, dim3(kKBlock), lds, stream, dprog, arena,
                     arena_bytes, offs, n, verdicts, hits, stage, cq.recs, cq.qhdr, cq.cap, ids);
  return hipGetLastError();
}

}  // namespace

// Record stage of a Kafka workgroup (what the LDS leaves after the tables),
// `reserve` bytes kept at the end.
static size_t kafka_stage(const KafkaHeader& h, int mode, bool cli_lds, size_t reserve) {
  const uint32_t n_ctr = h.n_rules + 2;
  const size_t cli_words = static_cast<size_t>(h.n_clients) * (sizeof(KafkaClientSlot) / 4);
  const size_t fixed = 4u * (256u + kSpanLds + kKindOkLds + (cli_lds ? cli_words : 0u) +
                             (mode == kKLdsHits ? ((n_ctr + 3u) & ~3u) : 0u)) +
                       2u * kKWaves * 64 * kTopicQ;
  size_t stage = (kKLdsBytes - reserve - fixed) / kKWaves - 16u;
  stage &= ~size_t(15);
  return stage > kKMaxStage ? kKMaxStage : stage;
}

bool kafka_resident_ok(const KafkaHeader& h, int* kind, uint32_t* stage) {
  const size_t cli_words = static_cast<size_t>(h.n_clients) * (sizeof(KafkaClientSlot) / 4);
  const bool cli_lds = cli_words && cli_words * 4 <= kMaxCliLdsBytes;
  const size_t st = kafka_stage(h, kKNoHits, cli_lds, 4u * kResidentLdsWords);
  if (st < 1024) return false;
  *kind = static_cast<int>(kResidentKafka | (cli_lds ? 1u : 0u) | (h.n_id_slots ? 2u : 0u));
  *stage = static_cast<uint32_t>(st);
  return true;
}

hipError_t launch_kafka_resident(ResidentBox* dbox, uint64_t first_seq, int kind, uint32_t* qhdr,
                                 hipStream_t stream) {
#define L7M_KRES(C, G)                                                                                        \
  {                                                                                                          \
    const hipError_t e = set_lds_attr_once(reinterpret_cast<const void*>(kafka_resident_kernel<C, G>), kKLdsBytes); \
    if (e != hipSuccess) return e;                                                                           \
    hipLaunchKernelGGL((kafka_resident_kernel<C, G>), dim3(1), dim3(kKBlock), kKLdsBytes, stream, dbox, first_seq, \
                       qhdr);                                                                                \
    return hipGetLastError();                                                                                \
  }
  switch (kind & 3) {
    case 0: L7M_KRES(false, false)
    case 1: L7M_KRES(true, false)
    case 2: L7M_KRES(false, true)
    default: L7M_KRES(true, true)
  }
#undef L7M_KRES
}

hipError_t launch_kafka(const uint32_t* dprog, const KafkaHeader& h, const uint8_t* arena, uint64_t arena_bytes,
                        const uint64_t* offs, uint64_t n, int32_t* verdicts, unsigned long long* hits,
                        hipStream_t stream, int num_cus, uint32_t flags, const KafkaCodecQueue& cq,
                        const uint32_t* ids) {
  if (n == 0) return hipSuccess;
  const uint32_t n_ctr = h.n_rules + 2;
  const int mode = !hits ? kKNoHits : (n_ctr <= kKMaxLdsCounters ? kKLdsHits : kKGlobalHits);
  const size_t cli_words = static_cast<size_t>(h.n_clients) * (sizeof(KafkaClientSlot) / 4);
  const bool cli_lds = cli_words && cli_words * 4 <= kMaxCliLdsBytes;
  const size_t fixed = 4u * (256u + kSpanLds + kKindOkLds + (cli_lds ? cli_words : 0u) +
                             (mode == kKLdsHits ? ((n_ctr + 3u) & ~3u) : 0u)) +
                       2u * kKWaves * 64 * kTopicQ;
  const size_t stage = kafka_stage(h, mode, cli_lds, 0);
  const size_t lds = fixed + kKWaves * (stage + 16u);
  uint64_t blocks = static_cast<uint64_t>(num_cus > 0 ? num_cus : 256);
  const uint64_t want = (n + 2 * kKBlock - 1) / (2 * kKBlock);
  if (want < blocks) blocks = want;
  const dim3 grid(static_cast<uint32_t>(blocks));
  const uint32_t st = static_cast<uint32_t>(stage);
  if (flags & (L7M_FLAG_DIAG_COPY_ONLY | L7M_FLAG_DIAG_WALK_ONLY)) {
    if (flags & L7M_FLAG_DIAG_COPY_ONLY)
      return launch_k<kKNoHits, 1>(grid, lds, stream, dprog, arena, arena_bytes, offs, n, verdicts, hits, st, cq, ids);
    return launch_k<kKNoHits, 2>(grid, lds, stream, dprog, arena, arena_bytes, offs, n, verdicts, hits, st, cq, ids);
  }
#define L7M_KAFKA_LAUNCH(M, C, G) \
  return launch_k<M, 0, C, G>(grid, lds, stream, dprog, arena, arena_bytes, offs, n, verdicts, hits, st, cq, ids)
#define L7M_KAFKA_LAUNCH_G(M, C)        \
  {                                     \
    if (groups) L7M_KAFKA_LAUNCH(M, C, true); \
    L7M_KAFKA_LAUNCH(M, C, false);      \
  }
  const bool groups = h.n_id_slots != 0;
  if (cli_lds) {
    if (mode == kKNoHits) L7M_KAFKA_LAUNCH_G(kKNoHits, true);
    if (mode == kKLdsHits) L7M_KAFKA_LAUNCH_G(kKLdsHits, true);
    L7M_KAFKA_LAUNCH_G(kKGlobalHits, true);
  }
  if (mode == kKNoHits) L7M_KAFKA_LAUNCH_G(kKNoHits, false);
  if (mode == kKLdsHits) L7M_KAFKA_LAUNCH_G(kKLdsHits, false);
  L7M_KAFKA_LAUNCH_G(kKGlobalHits, false);
#undef L7M_KAFKA_LAUNCH_G
#undef L7M_KAFKA_LAUNCH
}

namespace {

// Second pass over the requests the first pass queued (ProduceReqs holding
// gzip / snappy messages): one worker per workgroup (lane 0; decoding is a
// serial bit stream), each with its own slab for decoded sets, re-reads the
// request with every compressed value decoded (kc_check_produce).  A request
// the reference's ReadRequest would fail becomes -2, moving its count from
// the verdict's counter slot to slot 1; -3 where the slab or nesting limit
// was reached.
__global__ __launch_bounds__(64) void kafka_codec_kernel(const uint32_t* __restrict__ prog,
                                                         const uint8_t* __restrict__ arena,
                                                         const uint64_t* __restrict__ offs, uint64_t n_recs,
                                                         uint64_t arena_bytes, const uint32_t* __restrict__ recs,
                                                         uint32_t* qhdr, uint32_t qcap, int32_t* verdicts,
                                                         unsigned long long* hits, uint8_t* slabs,
                                                         uint64_t slab_bytes) {
  if (threadIdx.x != 0) return;
  const KafkaHeader& h = *reinterpret_cast<const KafkaHeader*>(prog);
  const uint32_t* crc_tab = prog + h.off_crc;
  uint8_t* slab = slabs + static_cast<uint64_t>(blockIdx.x) * slab_bytes;
  const uint32_t pushed = __hip_atomic_load(qhdr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t n = pushed < qcap ? pushed : qcap;
  KcInflateScratch s;
  for (uint32_t i = atomicAdd(qhdr + 1, 1u); i < n; i = atomicAdd(qhdr + 1, 1u)) {
    const uint32_t ri = recs[i];
    if (ri >= n_recs) continue;
    const uint64_t o = offs[ri];
    // the first pass decoded this record in bounds: 4 + size bytes at o
    const uint8_t* rec = arena + o;
    const uint32_t len = 4u + ((static_cast<uint32_t>(rec[0]) << 24) | (static_cast<uint32_t>(rec[1]) << 16) |
                               (static_cast<uint32_t>(rec[2]) << 8) | rec[3]);
    if (o + len > arena_bytes) continue;
    const int rc = kc_check_produce(rec, len, slab, static_cast<uint32_t>(slab_bytes), crc_tab, s);
    if (rc == kCodecOk) continue;
    const int32_t v = verdicts[ri];  // this request's only writer after the first pass
    const int32_t nv = rc == kCodecErr ? L7M_VERDICT_PARSE_ERROR : L7M_VERDICT_UNSUPPORTED;
    verdicts[ri] = nv;
    if (hits) {
      atomicAdd(hits + (v >= 0 ? static_cast<uint32_t>(v) + 2u : 0u), ~0ull);  // -1
      atomicAdd(hits + 1, 1ull);  // -2 and -3 share slot 1
    }
  }
  // The last worker to finish resets the queue header for the next launch on
  // this queue (which waits for this kernel): no memset per launch.
  __threadfence();
  if (atomicAdd(qhdr + 2, 1u) == gridDim.x - 1) {
    __hip_atomic_store(qhdr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(qhdr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(qhdr + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

}  // namespace

hipError_t launch_kafka_codec(const uint32_t* dprog, const uint8_t* arena, uint64_t arena_bytes, const uint64_t* offs,
                              uint64_t n, int32_t* verdicts, unsigned long long* hits, hipStream_t stream,
                              const KafkaCodecQueue& cq) {
  if (!cq.cap || !cq.workers || !n) return hipSuccess;
  hipLaunchKernelGGL(kafka_codec_kernel, dim3(cq.workers), dim3(64), 0, stream, dprog, arena, offs, n, arena_bytes,
                     cq.recs, cq.qhdr, cq.cap, verdicts, hits, cq.slabs, cq.slab_bytes);
  return hipGetLastError();
}

}  // namespace l7m
