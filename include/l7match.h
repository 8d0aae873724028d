/*
 * l7match.h — C ABI of libl7match.so, the MI355X-native batched L7 policy
 * evaluator for Cilium's L7 rule model (PortRuleHTTP / PortRuleKafka).
 *
 * This is the drop-in boundary.  Each entry point replaces one reference
 * interface (all paths relative to the uniberg/cilium tree):
 *
 *   l7m_compile_http   replaces the rule-import half of the HTTP path:
 *                      getHTTPRule  pkg/envoy/server.go:261-320  (PortRuleHTTP ->
 *                      HeaderMatcher list) followed by the std::regex construction
 *                      in Envoy's HeaderData (envoy/cilium_network_policy.h:52-66,
 *                      policy instantiation envoy/cilium_network_policy.cc:63-65).
 *                      A regex that std::regex rejects makes the call fail
 *                      (L7M_EINVAL_REGEX) exactly where Envoy would NACK the
 *                      policy; the caller keeps its previous handle.
 *   l7m_compile_kafka  replaces PortRuleKafka.Sanitize
 *                      (pkg/policy/api/rule_validation.go:190-233) applied to the
 *                      rule slice handed to MatchesRule (pkg/kafka/policy.go:200).
 *   l7m_compile_http_policies
 *                      the rule import of whole NPDS NetworkPolicy resources
 *                      (envoy/cilium/npds.proto:32-118) into Envoy's
 *                      NetworkPolicyMap (envoy/cilium_network_policy.cc:42-108,
 *                      PolicyInstance / PortNetworkPolicy construction
 *                      envoy/cilium_network_policy.h:40-208): per endpoint policy
 *                      name, ingress and egress per-port rule sets.
 *   l7m_eval           replaces, for a batch of N requests,
 *                        HTTP : NetworkPolicyMap::Allowed
 *                               envoy/cilium_network_policy.h:223-237 (-> :198-203,
 *                               :169-192, :128-146, :90-108, :68-71)
 *                        Kafka: kafka.ReadRequest pkg/kafka/request.go:186-229 +
 *                               (*RequestMessage).MatchesRule pkg/kafka/policy.go:200-225
 *                      The reference returns a bare bool per request; this ABI
 *                      returns an int32 verdict per request (see L7M_VERDICT_*):
 *                      -1 deny, i >= 0 allow decided by rule i (input order).
 *   l7m_eval_device    the same on buffers already resident in HBM, enqueued on a
 *                      caller-provided HIP stream (no host synchronisation).
 *
 * Conventions: every int-returning function returns L7M_OK (0) or a negative
 * L7M_E* code.  When err != NULL and errlen > 0 a NUL-terminated message is
 * written on failure.  Handles are immutable after compile and reference
 * counted; l7m_eval / l7m_eval_device are reentrant and may be called
 * concurrently from many threads on the same handle (each call uses its own
 * stream and scratch), mirroring Envoy's lock-free per-worker read path.
 *
 * Nothing in this header depends on HIP or torch types: streams are passed
 * as void* (hipStream_t), device buffers as void*.
 */
#ifndef L7MATCH_H
#define L7MATCH_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define L7M_ABI_VERSION 4

/* ---- status codes ------------------------------------------------------ */
#define L7M_OK 0
#define L7M_EINVAL (-1)         /* bad argument (NULL pointer, bad size)          */
#define L7M_EINVAL_REGEX (-2)   /* std::regex would throw: Envoy NACKs the policy */
#define L7M_EINVAL_RULE (-3)    /* Sanitize() error / getHTTPRule sort panic      */
#define L7M_EUNSUPPORTED (-4)   /* valid regex outside the compiled subset        */
#define L7M_ENOMEM (-5)         /* host or device allocation failed               */
#define L7M_EDEVICE (-6)        /* HIP runtime error / no device                  */
#define L7M_ETOOBIG (-7)        /* rule set exceeds a compile-time limit          */

/* ---- verdicts (int32 per request) --------------------------------------- */
#define L7M_VERDICT_DENY (-1)         /* no rule allows the request               */
#define L7M_VERDICT_PARSE_ERROR (-2)  /* Kafka: ReadRequest would return an error  */
#define L7M_VERDICT_UNSUPPORTED (-3)  /* Kafka: a gzip/snappy message set past the second
                                        pass's limits (nesting depth 8, slab, queue).
                                        HTTP: a rule with a back-reference / look-around
                                        matcher (slow path, regex_vm.h) ran past the
                                        executor's second-tier limits before any
                                        earlier rule decided the request: more than
                                        1 MiB of backtracking stack (262144 words),
                                        which std::regex_match's recursion turns into
                                        more than 8 MiB of native stack (>= 8 native
                                        bytes per executor byte, measured >= 12 on
                                        every family in tests/test_slow_tiers_cpu.py):
                                        it overflows an Envoy worker's default thread
                                        stack there; or more than 2^25 backtracking
                                        steps (exponential patterns the reference
                                        spends seconds on)                          */
#define L7M_VERDICT_ALLOW_NO_L7 (0x7fffffff) /* HTTP rule list empty: port has no L7
                                        rules, Envoy allows (cilium_network_policy.h:129-135) */
#define L7M_VERDICT_ALLOW_NO_PORT_POLICY (0x7ffffffe) /* no per-port policy for the
                                        request's port, not even port 0: Envoy allows
                                        (cilium_network_policy.h:187-191) */

/* ---- dialects ------------------------------------------------------------ */
#define L7M_DIALECT_ENVOY_ECMA_FULL 0 /* std::regex ECMAScript, regex_match (full)  */
#define L7M_DIALECT_RE2_SEARCH 1      /* Go regexp MatchString: RE2, unanchored     */

#define L7M_PROTO_HTTP 1
#define L7M_PROTO_KAFKA 2

typedef struct l7m_ruleset l7m_ruleset; /* opaque */

/* Verbatim api.PortRuleHTTP (pkg/policy/api/http.go:26-58).  NULL or "" = unset.
 * remote_ids: allowed_remotes_ of the PortNetworkPolicyRule this HTTP rule
 * belongs to (envoy/cilium_network_policy.h:90-97, NPDS remote_policies);
 * n_remote_ids == 0 means any remote identity.  A request is allowed by rule i
 * iff its remote_id is in the set AND every matcher of the rule holds. */
typedef struct {
  const char* path;
  const char* method;
  const char* host;
  const char* const* headers; /* "Name: value" (literal) or "Name" (presence) */
  uint32_t n_headers;
  uint32_t n_remote_ids;
  const uint32_t* remote_ids;
} l7m_http_rule;

/* ---- NPDS network policies (the full NetworkPolicyMap::Allowed boundary) --
 * PortNetworkPolicyRule (npds.proto:78-95; cilium_network_policy.h:76-112):
 * remote identities (empty = any) and, when has_http_rules != 0, the OR of its
 * HTTP rules (each an AND of getHTTPRule matchers; the rules' own remote_ids
 * must be empty).  has_http_rules == 0 = no L7 predicate: any request from an
 * allowed remote matches.  has_http_rules with n_http_rules == 0 violates
 * HttpNetworkPolicyRules.http_rules min_items = 1 (L7M_EINVAL_RULE). */
typedef struct {
  const uint32_t* remote_ids;
  uint32_t n_remote_ids;
  uint32_t has_http_rules;
  const l7m_http_rule* http_rules;
  size_t n_http_rules;
} l7m_port_rule;

#define L7M_L4_TCP 0 /* envoy SocketAddress.Protocol: only TCP policies are installed */
#define L7M_L4_UDP 1

/* PortNetworkPolicy (npds.proto:58-76): port 0 = every port.  A port may
 * appear once per direction (else L7M_EINVAL_RULE, Envoy's "Duplicate port
 * number"); non-TCP entries are skipped as Envoy does
 * (cilium_network_policy.h:154-166). */
typedef struct {
  uint32_t port;
  uint32_t protocol; /* L7M_L4_* */
  const l7m_port_rule* rules;
  size_t n_rules;
} l7m_port_policy;

/* NetworkPolicy (npds.proto:32-56) of one endpoint, keyed by name. */
typedef struct {
  const char* name;
  const l7m_port_policy* ingress;
  size_t n_ingress;
  const l7m_port_policy* egress;
  size_t n_egress;
} l7m_network_policy;

/* Where a verdict's rule index comes from (l7m_ruleset_rule_origin).  The
 * index space of l7m_compile_http_policies is the policies' HTTP rules
 * flattened in this order: policies as given; ingress, then egress; port
 * entries as given except that the port-0 entry of a direction comes last
 * (so the smallest matching index is the exact-port match Envoy checks first,
 * cilium_network_policy.h:169-186); port rules as given; a port rule with
 * has_http_rules == 0 contributes one matcher-less pseudo rule
 * (http_rule = -1), else one index per HTTP rule. */
typedef struct {
  uint32_t policy;    /* index into the compiled policies               */
  uint32_t ingress;   /* 1 ingress, 0 egress                            */
  uint32_t port;      /* PortNetworkPolicy.port (0 = wildcard)          */
  uint32_t port_rule; /* index into that PortNetworkPolicy's rules      */
  int32_t http_rule;  /* index into the port rule's http_rules, or -1   */
  uint32_t reserved;
} l7m_rule_origin;

/* Verbatim api.PortRuleKafka (pkg/policy/api/kafka.go:26-106).  NULL or "" = unset. */
typedef struct {
  const char* role;
  const char* api_key;
  const char* api_version;
  const char* client_id;
  const char* topic;
} l7m_kafka_rule;

/* The Kafka redirect's L7DataMap (pkg/policy/l4.go:110-129 GetRelevantRules):
 * one entry per endpoint selector with that selector's PortRuleKafka rules.
 * `wildcard` marks api.WildcardEndpointSelector, whose rules apply to every
 * source; the others apply to the source identities whose labels the
 * selector matches, listed per identity in an l7m_identity_selectors
 * table; the control plane evaluates selector.Matches(labels).  At most 64
 * entries. */
typedef struct {
  const l7m_kafka_rule* rules;
  size_t n_rules;
  uint32_t wildcard;
  uint32_t reserved;
} l7m_kafka_selector_rules;

typedef struct {
  uint32_t identity;          /* numeric security identity (!= 0)                 */
  uint32_t reserved;
  const uint32_t* selectors;  /* indices of the L7DataMap entries that select it  */
  size_t n_selectors;
} l7m_identity_selectors;

typedef struct {
  uint32_t struct_size;     /* sizeof(l7m_opts); 0 = use defaults               */
  uint32_t dialect;         /* L7M_DIALECT_*                                    */
  uint32_t max_dfa_states;  /* per DFA group before splitting (0 = default)     */
  uint32_t flags;           /* reserved, 0                                      */
  uint64_t max_table_bytes; /* per DFA group before splitting (0 = default)     */
  uint32_t lds_budget_bytes;/* DFA slot tables kept in LDS per workgroup
                               (0 = default 64 KiB); the rest is walked from HBM */
  uint32_t reserved;
} l7m_opts;

typedef struct {
  uint32_t proto;           /* L7M_PROTO_*                                       */
  uint32_t n_rules;
  uint32_t n_fields;        /* HTTP: distinct header fields referenced          */
  uint32_t n_dfas;          /* HTTP: DFA groups (incl. the header-name DFA)     */
  uint64_t total_dfa_states;
  uint64_t program_bytes;   /* size of the device program blob                  */
  uint32_t n_counters;      /* length of rule_hits arrays = n_rules + 2         */
  uint32_t reserved;
} l7m_ruleset_info;

/* ---- rule compilation (cold path) ---------------------------------------- */
int l7m_compile_http(const l7m_http_rule* rules, size_t n, const l7m_opts* opts,
                     l7m_ruleset** out, char* err, size_t errlen);
int l7m_compile_kafka(const l7m_kafka_rule* rules, size_t n, const l7m_opts* opts,
                      l7m_ruleset** out, char* err, size_t errlen);
/* canAccess with GetRelevantRules (pkg/proxy/kafka.go:116-152): a request
 * from source identity s is decided by MatchesRule over the rules of the
 * entries that select s (none when s == 0 or s is not listed: the reference's
 * nil identity) followed by the wildcard entries' rules; no such rule ->
 * deny.  Verdict indices number the rules entry by entry in `map` order.
 * The source identities travel beside the arena (l7m_eval_ids);
 * l7m_compile_kafka(rules, n) is the map of one wildcard entry. */
int l7m_compile_kafka_map(const l7m_kafka_selector_rules* map, size_t n_entries,
                          const l7m_identity_selectors* identities, size_t n_identities,
                          const l7m_opts* opts, l7m_ruleset** out, char* err, size_t errlen);
/* A NetworkPolicyMap of n endpoint policies.  A request names its policy by
 * index in the record (l7m_ruleset_policy_index; 0xffff = a name the map does
 * not hold -> deny, cilium_network_policy.h:231-235); its direction and dport
 * select the per-port rule sets (exact port, then port 0, then allow).
 * l7m_compile_http(rules, n) is the one-policy map whose every port and
 * direction use `rules`. */
int l7m_compile_http_policies(const l7m_network_policy* policies, size_t n, const l7m_opts* opts,
                              l7m_ruleset** out, char* err, size_t errlen);
/* Index of an endpoint policy name in the record's policy field, or -1. */
int l7m_ruleset_policy_index(const l7m_ruleset* rs, const char* name);
/* Origin of verdict index `rule` (L7M_EINVAL if out of range). */
int l7m_ruleset_rule_origin(const l7m_ruleset* rs, uint32_t rule, l7m_rule_origin* out);
void l7m_retain(l7m_ruleset* rs);
void l7m_release(l7m_ruleset* rs);
int l7m_ruleset_get_info(const l7m_ruleset* rs, l7m_ruleset_info* out);
/* Copy of the packed device program (for inspection / tests).  *len receives
 * the size; when buf is NULL only the size is returned. */
int l7m_ruleset_program(const l7m_ruleset* rs, void* buf, size_t* len);

/* getHTTPRule translation of one rule (pkg/envoy/server.go:261-320), sorted as
 * SortHeaderMatchers (pkg/envoy/sort.go:205-250).  Writes up to cap matchers;
 * returns the number of matchers (>= 0) or a negative status.  kind: 0 regex,
 * 1 literal value, 2 presence (Envoy HeaderMatchType Regex/Value/Present). Name
 * and value pointers stay valid until the next call on the same thread. */
typedef struct {
  const char* name;  /* as in the NPDS HeaderMatcher (not lower-cased)           */
  const char* value;
  uint32_t kind;
  uint32_t has_regex_flag; /* HeaderMatcher.Regex != nil                        */
} l7m_header_matcher;
int l7m_http_translate(const l7m_http_rule* rule, l7m_header_matcher* out, size_t cap,
                       char* err, size_t errlen);

/* ---- request arena --------------------------------------------------------
 * A batch is a byte arena holding N records plus an array of N uint64 byte
 * offsets (each record 4-byte aligned).
 *
 * HTTP record (little endian), L7M_HTTP_REC_FIXED bytes of fixed header:
 *   u32 rec_len        bytes of this record, unpadded (>= 20 + 4*n_hdr)
 *   u32 remote_id      source security identity (Envoy remote_id)
 *   u16 dport          destination port
 *   u8  flags          L7M_HTTP_F_*
 *   u8  n_hdr          number of regular headers
 *   u16 method_len, u16 path_len, u16 authority_len, u16 policy
 *                      policy: endpoint policy index (l7m_ruleset_policy_index),
 *                      0xffff = unknown endpoint policy (deny)
 *   n_hdr x { u16 name_len, u16 value_len }           header directory
 *   method | path | authority | name0 | value0 | name1 | value1 | ...
 * Header names must already be lower case (Envoy's codec lower-cases them);
 * the first occurrence of a name is the one matched (HeaderMap::get).
 *
 * Kafka record: the request exactly as proto.ReadReq returns it
 * (vendor/github.com/optiopay/kafka/proto/messages.go:124-165): big-endian
 * int32 size followed by size bytes; record length = 4 + size.
 */
#define L7M_HTTP_REC_FIXED 20
#define L7M_HTTP_F_METHOD 0x01
#define L7M_HTTP_F_PATH 0x02
#define L7M_HTTP_F_AUTHORITY 0x04
#define L7M_HTTP_F_INGRESS 0x08

typedef struct {
  const char* method;    /* NULL = absent */
  const char* path;      /* NULL = absent */
  const char* authority; /* NULL = absent */
  const char* const* header_names;  /* lower-cased by the packer */
  const char* const* header_values;
  uint32_t n_headers;
  uint32_t remote_id;
  uint16_t dport;
  uint16_t ingress;
  uint32_t policy;  /* endpoint policy index (0 for l7m_compile_http rule sets) */
} l7m_http_request;
#define L7M_POLICY_UNKNOWN 0xffffu

/* Bytes one request occupies in the arena (4-byte padded); 0 if not encodable. */
size_t l7m_http_record_size(const l7m_http_request* req);
/* Pack n requests; writes offsets[i]; returns bytes used or 0 on overflow. */
size_t l7m_pack_http(const l7m_http_request* reqs, size_t n, uint8_t* arena, size_t cap,
                     uint64_t* offsets);

/* ---- evaluation flags ------------------------------------------------------
 * 0 for normal use.  The DIAG flags select profiling ablations of the HTTP
 * kernel whose verdicts are NOT valid (used by bench.py --diag).  HTTP
 * programs with more than 8 value automata, RE2-dialect search automata or
 * slow-path rules have no ablation build: the call returns L7M_EDEVICE. */
#define L7M_FLAG_DIAG_WALK_ONLY 0x40000000u  /* stop after the DFA walks       */
#define L7M_FLAG_DIAG_COPY_ONLY 0x80000000u  /* stop after staging/validation  */

/* ---- evaluation (hot path) ----------------------------------------------
 * verdicts: int32[n].  rule_hits: NULL or uint64[n_rules + 2], ACCUMULATED
 * (not cleared): [0] denies, [1] parse errors + unsupported, [2 + i] requests
 * allowed by rule i.  flags: 0 (or L7M_FLAG_DIAG_* for profiling).
 */
int l7m_eval(const l7m_ruleset* rs, const uint8_t* arena, size_t arena_bytes,
             const uint64_t* rec_offsets, size_t n, int32_t* verdicts, uint64_t* rule_hits,
             uint32_t flags);

/* l7m_eval with the source identity of every request (u32 per request; the
 * redirect's srcIdentity, pkg/proxy/kafka.go:245).  Kafka rule sets only;
 * src_identities == NULL is every request from identity 0.  HTTP records
 * carry their remote identity themselves: L7M_EINVAL for HTTP rule sets. */
int l7m_eval_ids(const l7m_ruleset* rs, const uint8_t* arena, size_t arena_bytes,
                 const uint64_t* rec_offsets, size_t n, const uint32_t* src_identities,
                 int32_t* verdicts, uint64_t* rule_hits, uint32_t flags);

/* Device-resident variant: all pointers are device pointers on the current HIP
 * device; the work is enqueued on `hip_stream` (NULL = default stream) and the
 * call returns without synchronising.  d_arena must be 16-byte aligned and
 * readable up to round_up(arena_bytes, 16) (records are streamed with aligned
 * 16-byte loads); L7M_EINVAL otherwise. */
int l7m_eval_device(const l7m_ruleset* rs, const void* d_arena, size_t arena_bytes,
                    const void* d_rec_offsets, size_t n, void* d_verdicts, void* d_rule_hits,
                    void* hip_stream, uint32_t flags);
/* ... with device-resident source identities (see l7m_eval_ids). */
int l7m_eval_device_ids(const l7m_ruleset* rs, const void* d_arena, size_t arena_bytes,
                        const void* d_rec_offsets, size_t n, const void* d_src_identities,
                        void* d_verdicts, void* d_rule_hits, void* hip_stream, uint32_t flags);

/* ---- several GPUs from one process ----------------
 * Requests are independent, so a batch is cut into contiguous byte-balanced
 * shards, one per device, evaluated concurrently (one HIP stream per device,
 * the program replicated on each), and the per-rule counters are summed with
 * ONE RCCL all-reduce (ncclAllReduce, uint64 sum) over a single-process
 * communicator of the devices (ncclCommInitAll).  This is the in-library
 * form of bench.py's process-per-GPU sharding, for a caller that is one
 * process: cilium-agent's Kafka proxy calling canAccess
 * (pkg/proxy/kafka.go:116-152) through cgo, or one Envoy filter instance.
 * A device may appear more than once (several shards on one GPU); RCCL needs
 * distinct devices, so such sets (and L7M_MULTI_NO_RCCL=1) sum the counters
 * on the host instead.  Verdicts and counters equal one l7m_eval over the
 * whole batch.  Calls on one device set are serialised; distinct sets run
 * concurrently. */
typedef struct l7m_multi l7m_multi;
int l7m_multi_create(const int* devices, uint32_t n_devices, l7m_multi** out);
void l7m_multi_destroy(l7m_multi* m);
/* 1 when the set's counters are reduced by RCCL, 0 when on the host. */
int l7m_multi_uses_rccl(const l7m_multi* m);
/* Byte-balanced contiguous shards of a packed batch: bounds[0..parts] record
 * indices (bounds[0] = 0, bounds[parts] = n); shard k = [bounds[k],
 * bounds[k+1]) holds the records whose arena bytes are closest to k / parts
 * of the total (cilium_amd/dist.py byte_balanced_bounds).  Offsets must
 * ascend (what every packer produces): L7M_EINVAL otherwise. */
int l7m_shard_bounds(const uint64_t* rec_offsets, size_t n, size_t arena_bytes, uint32_t parts,
                     uint64_t* bounds);
/* l7m_eval_ids over the device set: host arena cut by l7m_shard_bounds,
 * each shard copied to its device, verdicts gathered, counters reduced. */
int l7m_multi_eval(l7m_multi* m, const l7m_ruleset* rs, const uint8_t* arena, size_t arena_bytes,
                   const uint64_t* rec_offsets, size_t n, const uint32_t* src_identities,
                   int32_t* verdicts, uint64_t* rule_hits, uint32_t flags);
/* Device-resident shards (HBM): shard k lives on device k of the set (its
 * pointers are device pointers there; rec_offsets relative to its arena).
 * Synchronous: returns after every device's kernels and the counter
 * all-reduce; rule_hits (host, n_rules + 2) accumulates the job's sum.
 * The set evaluates on its own (non-blocking) streams and takes no caller
 * stream: the shards' contents must be complete on their devices when this
 * is called (synchronise the stream or device that produced them first, e.g.
 * hipStreamSynchronize / torch.cuda.synchronize()); nothing orders the
 * kernels after a producer still in flight. */
typedef struct {
  const void* arena;
  size_t arena_bytes;
  const void* rec_offsets;
  size_t n;
  const void* src_identities; /* Kafka L7DataMap rule sets, or NULL */
  void* verdicts;
} l7m_shard;
int l7m_multi_eval_device(l7m_multi* m, const l7m_ruleset* rs, const l7m_shard* shards,
                          uint64_t* rule_hits, uint32_t flags);

/* ---- batching front-end (the call-site shape of the reference) ------------
 * canAccess (pkg/proxy/kafka.go:116-152) and AccessFilter::decodeHeaders
 * (envoy/cilium_l7policy.cc:126-186) decide one request per call on the
 * connection's goroutine / worker thread.  l7m_batcher keeps that blocking
 * per-request call: any number of threads call l7m_batcher_eval; their
 * records share one evaluation, flushed when max_batch requests are pending
 * (or the batch's arena is full) or the first has waited max_delay_us, while
 * the next batch fills.  Callers reserve their slot with one atomic
 * compare-and-swap (no lock); batches live in pinned, device-mapped host
 * memory that the kernels read and write in place (no copies); up to
 * in_flight batches are evaluated at once, each flusher on its own stream,
 * polling for completion; callers spin briefly, then sleep.  Destroying a
 * batcher with calls in flight is safe: pending batches are still decided,
 * later calls get L7M_EINVAL, and the memory is freed after the last caller
 * has returned.
 * l7m_batcher_set_ruleset swaps the rules for later batches (the
 * Redirect.updateRules policy update, pkg/proxy/redirect.go:68-74). */
typedef struct l7m_batcher l7m_batcher;
typedef struct {
  uint32_t struct_size;  /* sizeof(l7m_batcher_opts); 0 = defaults          */
  uint32_t max_batch;    /* requests per evaluation (0 = 65536)             */
  uint32_t max_delay_us; /* longest wait of a batch's first request (0 = 200) */
  int32_t device;        /* HIP device the batches run on                   */
  uint32_t in_flight;    /* batches evaluated concurrently (0 = 4, max 8)   */
  uint32_t eager;        /* 1: a free flusher takes the pending requests at
                            once (batch size follows the load; max_delay_us
                            unused); 0: wait for max_batch / max_delay_us  */
} l7m_batcher_opts;
int l7m_batcher_create(l7m_ruleset* rs, const l7m_batcher_opts* opts, l7m_batcher** out);
int l7m_batcher_set_ruleset(l7m_batcher* b, l7m_ruleset* rs);
/* One request (a record as in the arena); blocks until its batch is decided. */
int l7m_batcher_eval(l7m_batcher* b, const uint8_t* record, size_t len, int32_t* verdict);
/* ... from source identity src_identity (canAccess's srcIdentity; Kafka rule
 * sets compiled from an L7DataMap, see l7m_eval_ids; ignored for HTTP). */
int l7m_batcher_eval_from(l7m_batcher* b, const uint8_t* record, size_t len, uint32_t src_identity,
                          int32_t* verdict);
int l7m_batcher_eval_http(l7m_batcher* b, const l7m_http_request* req, int32_t* verdict);
int l7m_batcher_stats(l7m_batcher* b, uint64_t* batches, uint64_t* requests);
/* Where a batch's time goes (means since creation): fill = first request
 * appended -> batch closed by a flusher; launch = closed -> kernels enqueued
 * (l7m_eval_device on the batch's pinned, device-mapped buffers: records read
 * and verdicts written in place); gpu = enqueued -> completion observed by the
 * flusher (event polling); wake = completion -> the caller has its verdict
 * (mean per request). */
typedef struct {
  uint64_t batches, requests;
  double fill_us, launch_us, gpu_us, wake_us;
  /* batches served by the resident workgroup, and its mean time per batch
   * reading the slot (incl. cache invalidation), evaluating, and writing the
   * verdicts back (device clock) */
  uint64_t resident_batches, resident_rounds; /* rounds: one or more batches evaluated together */
  double resident_read_us, resident_eval_us, resident_sync_us;
} l7m_batcher_profile;
int l7m_batcher_get_profile(l7m_batcher* b, l7m_batcher_profile* out);
void l7m_batcher_destroy(l7m_batcher* b);

/* ---- verdict side effects (host; for requests the GPU decided) ------------
 * l7m_http_deny_body: the 403 body AccessFilter sends on deny: the configured
 * denied_403_body, "Access denied" when empty, CRLF-terminated
 * (envoy/cilium_l7policy.cc:89-95, 169-181).  Returns its length; writes up
 * to cap-1 bytes + NUL.
 * l7m_kafka_deny_response: the bytes handleRequest enqueues for a denied
 * Kafka request, CreateResponse(ErrTopicAuthorizationFailed)
 * (pkg/proxy/kafka.go:245-259, pkg/kafka/request.go:158-182,
 * pkg/kafka/response.go) as optiopay's Resp.Bytes(version): every topic /
 * partition of the request with error 29.  *out_len = the response size
 * (L7M_ENOMEM when cap is smaller); L7M_EUNSUPPORTED for kinds ReadRequest
 * leaves untyped ("unsupported request API key"); L7M_EINVAL if the request
 * does not decode.
 * l7m_proxy_stats_add: per-endpoint proxy counters of a batch
 * (Endpoint.UpdateProxyStatistics, pkg/endpoint/endpoint.go:2099-2122):
 * received, forwarded (allowed), denied, error (ReadRequest failed /
 * unsupported). */
typedef struct {
  uint64_t received, forwarded, denied, error;
} l7m_proxy_stats;
size_t l7m_http_deny_body(const char* configured, char* out, size_t cap);
int l7m_kafka_deny_response(const uint8_t* req, size_t len, uint8_t* out, size_t cap, size_t* out_len);
int l7m_proxy_stats_add(const int32_t* verdicts, size_t n, l7m_proxy_stats* stats);

/* Per-endpoint proxy statistics keyed as the endpoint keeps them
 * (Endpoint.UpdateProxyStatistics(l7Protocol, port, ingress, request,
 * verdict), pkg/endpoint/endpoint.go:2060-2122): one entry per (protocol,
 * port, direction, request/response).  l7m_proxy_stats_update counts each
 * request of a decided batch once, as the reference's call sites do:
 *   HTTP  - port and direction from each record (the access-log entry's
 *           DestinationEndpoint.Port / is_ingress, pkg/envoy/
 *           accesslog_server.go:165-169); `port`, `ingress` unused;
 *   Kafka - the redirect's port and direction (`port`, `ingress`); port 0
 *           is not counted, nor a request ReadRequest rejected (the proxy
 *           closes the connection) (pkg/proxy/kafka.go:213-229, 349-354).
 * Verdicts: allowed -> forwarded, L7M_VERDICT_DENY -> denied, others ->
 * error; a denied Kafka request of a kind ReadRequest leaves untyped counts
 * as error (its deny response cannot be built, pkg/proxy/kafka.go:246-252,
 * pkg/kafka/request.go:174-175).  The records are read for both protocols
 * (arena / rec_offsets required).  Thread-safe.  l7m_proxy_stats_get copies up to cap entries in key
 * order and returns the number of entries. */
typedef struct l7m_proxy_stats_table l7m_proxy_stats_table;
typedef struct {
  uint32_t proto;    /* L7M_PROTO_HTTP ("http") / L7M_PROTO_KAFKA ("kafka") */
  uint16_t port;
  uint8_t ingress;
  uint8_t request;   /* 1: Statistics.Requests (verdicts are request-side)  */
  l7m_proxy_stats stats;
} l7m_proxy_stats_entry;
l7m_proxy_stats_table* l7m_proxy_stats_table_create(void);
void l7m_proxy_stats_table_destroy(l7m_proxy_stats_table* t);
int l7m_proxy_stats_update(l7m_proxy_stats_table* t, uint32_t proto, const uint8_t* arena, size_t arena_bytes,
                           const uint64_t* rec_offsets, const int32_t* verdicts, size_t n, uint16_t port,
                           int ingress);
size_t l7m_proxy_stats_get(l7m_proxy_stats_table* t, l7m_proxy_stats_entry* out, size_t cap);

/* ---- access-log records of a decided batch ---------------------------------
 * HTTP: the HttpLogEntry protobuf (envoy/cilium/accesslog.proto) Envoy's
 * filter sends over the access-log socket for each request
 * (AccessLog::Entry::InitFromRequest / UpdateFromResponse / AccessLog::Log,
 * envoy/accesslog.cc:59-170; AccessFilter::decodeHeaders / encodeHeaders,
 * envoy/cilium_l7policy.cc:166-191): EntryType Request for an allowed request,
 * Denied with status 403 for a denied one; timestamp, http_protocol,
 * policy_name, source_security_id (ingress: the record's remote identity,
 * egress: opts->local_identity), addresses (when given), scheme (the
 * x-forwarded-proto header), host / path / method, the other headers in
 * request order, is_ingress.  Messages are written back to back into out;
 * entry_offs[i] .. entry_offs[i+1] is request i's message (n + 1 entries;
 * empty for records that do not parse).  Returns the total size (out == NULL:
 * the size needed; L7M_ENOMEM when cap is too small). */
typedef struct {
  uint32_t struct_size;          /* sizeof(l7m_access_log_opts); 0 = defaults */
  uint32_t http_protocol;        /* accesslog.proto Protocol: 0 HTTP10, 1 HTTP11 (default), 2 HTTP2 */
  uint64_t timestamp_ns;         /* RequestInfo::startTime of the batch's requests */
  const char* policy_name;       /* the filter's policy_name */
  uint32_t local_identity;       /* egress: the local (source) endpoint's identity */
  uint32_t reserved;
  const char* source_address;    /* NULL: unset */
  const char* destination_address;
} l7m_access_log_opts;
int64_t l7m_http_access_log(const uint8_t* arena, size_t arena_bytes, const uint64_t* rec_offsets, size_t n,
                            const int32_t* verdicts, const l7m_access_log_opts* opts, uint8_t* out, size_t cap,
                            uint64_t* entry_offs);
/* Kafka: the proxy's log records (kafkaLogRecord.log, pkg/proxy/kafka.go
 * :168-230; LogRecordKafka, pkg/proxy/accesslog/record.go:220-241): one
 * record per topic of GetTopics() (none for requests without topics), verdict
 * Forwarded / ErrorCode 0 for allowed requests, Denied / 29
 * (ErrTopicAuthorizationFailed) for denied ones; requests ReadRequest rejects
 * log nothing.  Topic names point into the arena.  Returns the number of
 * records (out == NULL: the number needed; L7M_ENOMEM when cap is too small).
 * l7m_kafka_api_key_name: apiKeyToString (pkg/proxy/kafka.go:161-166). */
typedef struct {
  uint64_t request;        /* index in the batch */
  uint32_t verdict;        /* accesslog.FlowVerdict: 0 Forwarded, 1 Denied, 2 Error */
  int32_t error_code;      /* Kafka.ErrorCode */
  int16_t api_key;
  int16_t api_version;
  int32_t correlation_id;
  uint64_t topic_off;      /* Kafka.Topic.Topic = arena[topic_off, topic_off + topic_len) */
  uint32_t topic_len;
  uint32_t pad;
} l7m_kafka_log_record;
int64_t l7m_kafka_access_log(const uint8_t* arena, size_t arena_bytes, const uint64_t* rec_offsets, size_t n,
                             const int32_t* verdicts, l7m_kafka_log_record* out, size_t cap);
size_t l7m_kafka_api_key_name(int16_t api_key, char* out, size_t cap);

/* Pinned host memory helpers (cgo may not retain Go pointers across calls).
 * l7m_eval on an arena in pinned, device-mapped memory whose padded range
 * [arena, arena + arena_bytes + 64) lies inside one such allocation (16-byte
 * aligned) runs the kernels on it in place over PCIe, with no staging copy
 * (zero-copy; L7M_ZERO_COPY=0 in the environment disables it); other arenas
 * are copied.  The 64 bytes past arena_bytes are readable slack only: the
 * kernels may read them but never use their contents as record data (the
 * copying path zero-fills them, the zero-copy path leaves them as they are).  l7m_host_mapped(p, bytes) = 1 when [p, p + bytes) qualifies. */
int l7m_alloc_pinned(size_t bytes, void** out);
void l7m_free_pinned(void* p);
int l7m_host_mapped(const void* p, size_t bytes);

/* Library / device information. */
int l7m_abi_version(void);
int l7m_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* L7MATCH_H */
