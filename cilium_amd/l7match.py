"""Python binding of libl7match.so — the MI355X batched L7 policy evaluator.

This module is a thin ctypes layer over the C ABI declared in
``include/l7match.h`` (the same entry points a cgo shim would bind, see
INTEGRATION.md).  It mirrors the reference's rule-import types
(``api.PortRuleHTTP`` pkg/policy/api/http.go:26-58, ``api.PortRuleKafka``
pkg/policy/api/kafka.go:26-106) and its verdict calls
(``NetworkPolicyMap::Allowed`` envoy/cilium_network_policy.h:223,
``(*RequestMessage).MatchesRule`` pkg/kafka/policy.go:200), batched.

There is no CPU evaluation path: every verdict is computed by the HIP kernels
in libl7match.so.  If the library is missing, importing this module fails.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass, field
from typing import Iterable, List, Optional, Sequence, Tuple

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# L7M_LIB: alternative in-tree build of the same ABI (kernel experiments).
LIB_PATH = os.environ.get("L7M_LIB") or os.path.join(_HERE, "libl7match.so")

L7M_OK = 0
L7M_EINVAL = -1
L7M_EINVAL_REGEX = -2
L7M_EINVAL_RULE = -3
L7M_EUNSUPPORTED = -4
L7M_ENOMEM = -5
L7M_EDEVICE = -6
L7M_ETOOBIG = -7

VERDICT_DENY = -1
VERDICT_PARSE_ERROR = -2
VERDICT_UNSUPPORTED = -3
VERDICT_ALLOW_NO_L7 = 0x7FFFFFFF
VERDICT_ALLOW_NO_PORT_POLICY = 0x7FFFFFFE
POLICY_UNKNOWN = 0xFFFF
L4_TCP, L4_UDP = 0, 1

DIALECT_ENVOY_ECMA_FULL = 0
DIALECT_RE2_SEARCH = 1

FLAG_DIAG_WALK_ONLY = 0x40000000  # profiling ablations: verdicts NOT valid
FLAG_DIAG_COPY_ONLY = 0x80000000

PROTO_HTTP = 1
PROTO_KAFKA = 2

HTTP_REC_FIXED = 20
F_METHOD, F_PATH, F_AUTHORITY, F_INGRESS = 1, 2, 4, 8

# Every symbol include/l7match.h declares (checked by
# tests/test_http_cpu.py::test_library_exports_every_header_symbol).
EXPORTED_SYMBOLS = (
    "l7m_compile_http", "l7m_compile_kafka", "l7m_retain", "l7m_release",
    "l7m_ruleset_get_info", "l7m_ruleset_program", "l7m_http_translate",
    "l7m_http_record_size", "l7m_pack_http", "l7m_eval", "l7m_eval_device",
    "l7m_alloc_pinned", "l7m_free_pinned", "l7m_host_mapped", "l7m_abi_version", "l7m_device_count",
    "l7m_compile_http_policies", "l7m_ruleset_policy_index", "l7m_ruleset_rule_origin",
    "l7m_batcher_create", "l7m_batcher_set_ruleset", "l7m_batcher_eval", "l7m_batcher_eval_http",
    "l7m_batcher_stats", "l7m_batcher_destroy", "l7m_http_deny_body", "l7m_kafka_deny_response",
    "l7m_proxy_stats_add", "l7m_compile_kafka_map", "l7m_eval_ids", "l7m_eval_device_ids",
    "l7m_batcher_eval_from", "l7m_proxy_stats_table_create", "l7m_proxy_stats_table_destroy",
    "l7m_proxy_stats_update", "l7m_proxy_stats_get", "l7m_http_access_log", "l7m_kafka_access_log",
    "l7m_kafka_api_key_name", "l7m_batcher_get_profile",
    "l7m_multi_create", "l7m_multi_destroy", "l7m_multi_uses_rccl", "l7m_shard_bounds", "l7m_multi_eval",
    "l7m_multi_eval_device",
)


class L7Error(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"l7match error {code}: {msg}")
        self.code = code


class _HttpRule(ctypes.Structure):
    _fields_ = [("path", ctypes.c_char_p), ("method", ctypes.c_char_p), ("host", ctypes.c_char_p),
                ("headers", ctypes.POINTER(ctypes.c_char_p)), ("n_headers", ctypes.c_uint32),
                ("n_remote_ids", ctypes.c_uint32), ("remote_ids", ctypes.POINTER(ctypes.c_uint32))]


class _KafkaRule(ctypes.Structure):
    _fields_ = [("role", ctypes.c_char_p), ("api_key", ctypes.c_char_p),
                ("api_version", ctypes.c_char_p), ("client_id", ctypes.c_char_p),
                ("topic", ctypes.c_char_p)]


class _KafkaSelectorRules(ctypes.Structure):
    _fields_ = [("rules", ctypes.POINTER(_KafkaRule)), ("n_rules", ctypes.c_size_t),
                ("wildcard", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


class _IdentitySelectors(ctypes.Structure):
    _fields_ = [("identity", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("selectors", ctypes.POINTER(ctypes.c_uint32)), ("n_selectors", ctypes.c_size_t)]


class _Opts(ctypes.Structure):
    _fields_ = [("struct_size", ctypes.c_uint32), ("dialect", ctypes.c_uint32),
                ("max_dfa_states", ctypes.c_uint32), ("flags", ctypes.c_uint32),
                ("max_table_bytes", ctypes.c_uint64), ("lds_budget_bytes", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32)]


class _Info(ctypes.Structure):
    _fields_ = [("proto", ctypes.c_uint32), ("n_rules", ctypes.c_uint32),
                ("n_fields", ctypes.c_uint32), ("n_dfas", ctypes.c_uint32),
                ("total_dfa_states", ctypes.c_uint64), ("program_bytes", ctypes.c_uint64),
                ("n_counters", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


class _Matcher(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("value", ctypes.c_char_p),
                ("kind", ctypes.c_uint32), ("has_regex_flag", ctypes.c_uint32)]


class _HttpReq(ctypes.Structure):
    _fields_ = [("method", ctypes.c_char_p), ("path", ctypes.c_char_p),
                ("authority", ctypes.c_char_p),
                ("header_names", ctypes.POINTER(ctypes.c_char_p)),
                ("header_values", ctypes.POINTER(ctypes.c_char_p)),
                ("n_headers", ctypes.c_uint32), ("remote_id", ctypes.c_uint32),
                ("dport", ctypes.c_uint16), ("ingress", ctypes.c_uint16), ("policy", ctypes.c_uint32)]


class _PortRule(ctypes.Structure):
    _fields_ = [("remote_ids", ctypes.POINTER(ctypes.c_uint32)), ("n_remote_ids", ctypes.c_uint32),
                ("has_http_rules", ctypes.c_uint32), ("http_rules", ctypes.POINTER(_HttpRule)),
                ("n_http_rules", ctypes.c_size_t)]


class _PortPolicy(ctypes.Structure):
    _fields_ = [("port", ctypes.c_uint32), ("protocol", ctypes.c_uint32),
                ("rules", ctypes.POINTER(_PortRule)), ("n_rules", ctypes.c_size_t)]


class _NetworkPolicy(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("ingress", ctypes.POINTER(_PortPolicy)), ("n_ingress", ctypes.c_size_t),
                ("egress", ctypes.POINTER(_PortPolicy)), ("n_egress", ctypes.c_size_t)]


class _BatcherProfile(ctypes.Structure):
    _fields_ = [("batches", ctypes.c_uint64), ("requests", ctypes.c_uint64), ("fill_us", ctypes.c_double),
                ("launch_us", ctypes.c_double), ("gpu_us", ctypes.c_double), ("wake_us", ctypes.c_double),
                ("resident_batches", ctypes.c_uint64), ("resident_rounds", ctypes.c_uint64),
                ("resident_read_us", ctypes.c_double),
                ("resident_eval_us", ctypes.c_double), ("resident_sync_us", ctypes.c_double)]


class _BatcherOpts(ctypes.Structure):
    _fields_ = [("struct_size", ctypes.c_uint32), ("max_batch", ctypes.c_uint32),
                ("max_delay_us", ctypes.c_uint32), ("device", ctypes.c_int32), ("in_flight", ctypes.c_uint32),
                ("eager", ctypes.c_uint32)]


class _AccessLogOpts(ctypes.Structure):
    _fields_ = [("struct_size", ctypes.c_uint32), ("http_protocol", ctypes.c_uint32),
                ("timestamp_ns", ctypes.c_uint64), ("policy_name", ctypes.c_char_p),
                ("local_identity", ctypes.c_uint32), ("reserved", ctypes.c_uint32),
                ("source_address", ctypes.c_char_p), ("destination_address", ctypes.c_char_p)]


class _KafkaLogRecord(ctypes.Structure):
    _fields_ = [("request", ctypes.c_uint64), ("verdict", ctypes.c_uint32), ("error_code", ctypes.c_int32),
                ("api_key", ctypes.c_int16), ("api_version", ctypes.c_int16), ("correlation_id", ctypes.c_int32),
                ("topic_off", ctypes.c_uint64), ("topic_len", ctypes.c_uint32), ("pad", ctypes.c_uint32)]


class _ProxyStats(ctypes.Structure):
    _fields_ = [("received", ctypes.c_uint64), ("forwarded", ctypes.c_uint64), ("denied", ctypes.c_uint64),
                ("error", ctypes.c_uint64)]


class _RuleOrigin(ctypes.Structure):
    _fields_ = [("policy", ctypes.c_uint32), ("ingress", ctypes.c_uint32), ("port", ctypes.c_uint32),
                ("port_rule", ctypes.c_uint32), ("http_rule", ctypes.c_int32), ("reserved", ctypes.c_uint32)]


def _load() -> ctypes.CDLL:
    # PyTorch-ROCm ships its own libamdhip64 (same SONAME).  If torch is
    # present, load it first so this process has ONE HIP runtime: our DT_NEEDED
    # then binds to torch's copy and device buffers/streams are shared.  (If
    # libl7match pulled /opt/rocm's copy first, torch would load a second
    # runtime and fail with "No HIP GPUs are available".)
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `make -C cilium_amd/csrc` "
                          "(there is no CPU fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    if os.environ.get("L7M_LIB"):
        # an experimental build (tools/build_variant.sh, an older round's
        # library for A/B timing) may lack newer entry points: bind what exists
        class _Tolerant:
            def __init__(self, lib):
                self.__dict__["_lib"] = lib

            def __getattr__(self, name):
                try:
                    return getattr(self._lib, name)
                except AttributeError:
                    return ctypes.CFUNCTYPE(None)()

            def __setattr__(self, name, value):
                setattr(self._lib, name, value)
        lib = _Tolerant(lib)
    P = ctypes.c_void_p
    sz = ctypes.c_size_t
    lib.l7m_compile_http.argtypes = [ctypes.POINTER(_HttpRule), sz, ctypes.POINTER(_Opts),
                                     ctypes.POINTER(P), ctypes.c_char_p, sz]
    lib.l7m_compile_kafka.argtypes = [ctypes.POINTER(_KafkaRule), sz, ctypes.POINTER(_Opts),
                                      ctypes.POINTER(P), ctypes.c_char_p, sz]
    lib.l7m_compile_kafka_map.argtypes = [ctypes.POINTER(_KafkaSelectorRules), sz,
                                          ctypes.POINTER(_IdentitySelectors), sz, ctypes.POINTER(_Opts),
                                          ctypes.POINTER(P), ctypes.c_char_p, sz]
    lib.l7m_eval_ids.argtypes = [P, P, sz, P, sz, P, P, P, ctypes.c_uint32]
    lib.l7m_eval_device_ids.argtypes = [P, P, sz, P, sz, P, P, P, P, ctypes.c_uint32]
    lib.l7m_compile_http_policies.argtypes = [ctypes.POINTER(_NetworkPolicy), sz, ctypes.POINTER(_Opts),
                                              ctypes.POINTER(P), ctypes.c_char_p, sz]
    lib.l7m_ruleset_policy_index.argtypes = [P, ctypes.c_char_p]
    lib.l7m_batcher_create.argtypes = [P, ctypes.POINTER(_BatcherOpts), ctypes.POINTER(P)]
    lib.l7m_batcher_set_ruleset.argtypes = [P, P]
    lib.l7m_batcher_eval.argtypes = [P, ctypes.c_char_p, sz, ctypes.POINTER(ctypes.c_int32)]
    lib.l7m_batcher_eval_from.argtypes = [P, ctypes.c_char_p, sz, ctypes.c_uint32, ctypes.POINTER(ctypes.c_int32)]
    lib.l7m_batcher_eval_http.argtypes = [P, ctypes.POINTER(_HttpReq), ctypes.POINTER(ctypes.c_int32)]
    lib.l7m_batcher_stats.argtypes = [P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
    lib.l7m_batcher_get_profile.argtypes = [P, ctypes.POINTER(_BatcherProfile)]
    lib.l7m_batcher_destroy.argtypes = [P]
    lib.l7m_batcher_destroy.restype = None
    lib.l7m_http_deny_body.argtypes = [ctypes.c_char_p, ctypes.c_char_p, sz]
    lib.l7m_http_deny_body.restype = sz
    lib.l7m_kafka_deny_response.argtypes = [ctypes.c_char_p, sz, P, sz, ctypes.POINTER(sz)]
    lib.l7m_proxy_stats_add.argtypes = [P, sz, ctypes.POINTER(_ProxyStats)]
    lib.l7m_proxy_stats_table_create.restype = P
    lib.l7m_proxy_stats_table_destroy.argtypes = [P]
    lib.l7m_proxy_stats_update.argtypes = [P, ctypes.c_uint32, P, sz, P, P, sz, ctypes.c_uint16, ctypes.c_int]
    lib.l7m_proxy_stats_get.argtypes = [P, P, sz]
    lib.l7m_proxy_stats_get.restype = sz
    lib.l7m_http_access_log.argtypes = [P, sz, P, sz, P, ctypes.POINTER(_AccessLogOpts), P, sz, P]
    lib.l7m_http_access_log.restype = ctypes.c_int64
    lib.l7m_kafka_access_log.argtypes = [P, sz, P, sz, P, P, sz]
    lib.l7m_kafka_access_log.restype = ctypes.c_int64
    lib.l7m_kafka_api_key_name.argtypes = [ctypes.c_int16, ctypes.c_char_p, sz]
    lib.l7m_kafka_api_key_name.restype = sz
    lib.l7m_ruleset_rule_origin.argtypes = [P, ctypes.c_uint32, ctypes.POINTER(_RuleOrigin)]
    lib.l7m_release.argtypes = [P]
    lib.l7m_release.restype = None
    lib.l7m_retain.argtypes = [P]
    lib.l7m_retain.restype = None
    lib.l7m_ruleset_get_info.argtypes = [P, ctypes.POINTER(_Info)]
    lib.l7m_ruleset_program.argtypes = [P, P, ctypes.POINTER(sz)]
    lib.l7m_http_translate.argtypes = [ctypes.POINTER(_HttpRule), ctypes.POINTER(_Matcher), sz,
                                       ctypes.c_char_p, sz]
    lib.l7m_http_record_size.argtypes = [ctypes.POINTER(_HttpReq)]
    lib.l7m_http_record_size.restype = sz
    lib.l7m_pack_http.argtypes = [ctypes.POINTER(_HttpReq), sz, P, sz, P]
    lib.l7m_pack_http.restype = sz
    lib.l7m_eval.argtypes = [P, P, sz, P, sz, P, P, ctypes.c_uint32]
    lib.l7m_eval_device.argtypes = [P, P, sz, P, sz, P, P, P, ctypes.c_uint32]
    lib.l7m_alloc_pinned.argtypes = [sz, ctypes.POINTER(P)]
    lib.l7m_host_mapped.argtypes = [P, sz]
    lib.l7m_free_pinned.argtypes = [P]
    lib.l7m_free_pinned.restype = None
    lib.l7m_multi_create.argtypes = [P, ctypes.c_uint32, ctypes.POINTER(P)]
    lib.l7m_multi_destroy.argtypes = [P]
    lib.l7m_multi_destroy.restype = None
    lib.l7m_multi_uses_rccl.argtypes = [P]
    lib.l7m_shard_bounds.argtypes = [P, sz, sz, ctypes.c_uint32, P]
    lib.l7m_multi_eval.argtypes = [P, P, P, sz, P, sz, P, P, P, ctypes.c_uint32]
    lib.l7m_multi_eval_device.argtypes = [P, P, P, P, ctypes.c_uint32]
    return lib


_lib = _load()


def lib() -> ctypes.CDLL:
    return _lib


def device_count() -> int:
    return int(_lib.l7m_device_count())


def kafka_available() -> bool:
    try:
        RuleSet.compile_kafka([])
        return True
    except L7Error as e:
        if e.code == L7M_EUNSUPPORTED:
            return False
        raise


def _b(s: Optional[str]) -> Optional[bytes]:
    if s is None:
        return None
    return s.encode("utf-8", "surrogateescape") if isinstance(s, str) else bytes(s)


# --------------------------------------------------------------------------
# Reference rule types
# --------------------------------------------------------------------------
@dataclass
class PortRuleHTTP:
    """api.PortRuleHTTP (pkg/policy/api/http.go:26-58). Empty string = unset."""
    Path: str = ""
    Method: str = ""
    Host: str = ""
    Headers: Sequence[str] = field(default_factory=list)
    # allowed_remotes_ of the enclosing PortNetworkPolicyRule (NPDS
    # remote_policies, envoy/cilium_network_policy.h:90-97); empty = any.
    RemoteIDs: Sequence[int] = field(default_factory=list)


@dataclass
class PortRuleKafka:
    """api.PortRuleKafka (pkg/policy/api/kafka.go:26-106). Empty string = unset."""
    Role: str = ""
    APIKey: str = ""
    APIVersion: str = ""
    ClientID: str = ""
    Topic: str = ""


@dataclass
class PortNetworkPolicyRule:
    """NPDS PortNetworkPolicyRule (envoy/cilium/npds.proto:78-95): remote
    identities (empty = any) and, if HttpRules is not None, their HTTP rules."""
    RemotePolicies: Sequence[int] = field(default_factory=list)
    HttpRules: Optional[Sequence[PortRuleHTTP]] = None


@dataclass
class PortNetworkPolicy:
    """NPDS PortNetworkPolicy (npds.proto:58-76); Port 0 = any port."""
    Port: int
    Rules: Sequence[PortNetworkPolicyRule] = field(default_factory=list)
    Protocol: int = 0  # L4_TCP


@dataclass
class NetworkPolicy:
    """NPDS NetworkPolicy (npds.proto:32-56) of one endpoint."""
    Name: str
    Ingress: Sequence[PortNetworkPolicy] = field(default_factory=list)
    Egress: Sequence[PortNetworkPolicy] = field(default_factory=list)


def _policies_struct(policies: Sequence[NetworkPolicy], keep: list):
    def port_policies(pps):
        arr = (_PortPolicy * max(1, len(pps)))()
        for k, pp in enumerate(pps):
            rules = (_PortRule * max(1, len(pp.Rules)))()
            for j, pr in enumerate(pp.Rules):
                rem = (ctypes.c_uint32 * max(1, len(pr.RemotePolicies)))(*list(pr.RemotePolicies))
                hr = list(pr.HttpRules) if pr.HttpRules is not None else []
                harr = (_HttpRule * max(1, len(hr)))(*[_http_rule_struct(r, keep) for r in hr])
                keep.extend([rem, harr])
                rules[j] = _PortRule(ctypes.cast(rem, ctypes.POINTER(ctypes.c_uint32)), len(pr.RemotePolicies),
                                     1 if pr.HttpRules is not None else 0,
                                     ctypes.cast(harr, ctypes.POINTER(_HttpRule)), len(hr))
            keep.append(rules)
            arr[k] = _PortPolicy(pp.Port, pp.Protocol, ctypes.cast(rules, ctypes.POINTER(_PortRule)), len(pp.Rules))
        keep.append(arr)
        return ctypes.cast(arr, ctypes.POINTER(_PortPolicy)), len(pps)

    out = (_NetworkPolicy * max(1, len(policies)))()
    for i, p in enumerate(policies):
        ing, ni = port_policies(p.Ingress)
        eg, ne = port_policies(p.Egress)
        out[i] = _NetworkPolicy(_b(p.Name), ing, ni, eg, ne)
    keep.append(out)
    return out


@dataclass
class HeaderMatcher:
    """envoy_api_v2_route.HeaderMatcher as emitted by getHTTPRule."""
    Name: str
    Value: str = ""
    Regex: Optional[bool] = None  # None = nil BoolValue

    @property
    def kind(self) -> str:
        return "present" if not self.Value else ("regex" if self.Regex else "value")


@dataclass
class HTTPRequest:
    """One HTTP request head as Envoy's HeaderMap presents it."""
    method: Optional[str] = "GET"
    path: Optional[str] = "/"
    authority: Optional[str] = None
    headers: Sequence[Tuple[str, str]] = ()
    remote_id: int = 0
    dport: int = 80
    ingress: bool = True
    policy: int = 0  # endpoint policy index (RuleSet.policy_index); POLICY_UNKNOWN = deny


def _http_rule_struct(r: PortRuleHTTP, keep: list) -> _HttpRule:
    hs = [_b(h) for h in r.Headers]
    arr = (ctypes.c_char_p * max(1, len(hs)))(*hs)
    rem = (ctypes.c_uint32 * max(1, len(r.RemoteIDs)))(*list(r.RemoteIDs))
    keep += [arr, rem]
    return _HttpRule(_b(r.Path) or None, _b(r.Method) or None, _b(r.Host) or None,
                     ctypes.cast(arr, ctypes.POINTER(ctypes.c_char_p)), len(hs),
                     len(r.RemoteIDs), ctypes.cast(rem, ctypes.POINTER(ctypes.c_uint32)))


def get_http_rule(r: PortRuleHTTP) -> List[HeaderMatcher]:
    """getHTTPRule (pkg/envoy/server.go:261-320) as computed by libl7match."""
    keep: list = []
    st = _http_rule_struct(r, keep)
    out = (_Matcher * 256)()
    err = ctypes.create_string_buffer(512)
    n = _lib.l7m_http_translate(ctypes.byref(st), out, 256, err, 512)
    if n < 0:
        raise L7Error(n, err.value.decode())
    res = []
    for i in range(n):
        m = out[i]
        res.append(HeaderMatcher(m.name.decode(), (m.value or b"").decode(),
                                 True if m.has_regex_flag else None))
    return res


# --------------------------------------------------------------------------
# Arena packing
# --------------------------------------------------------------------------
def pack_http(reqs: Sequence[HTTPRequest]) -> Tuple[np.ndarray, np.ndarray]:
    """Pack requests into (arena uint8[], offsets uint64[]) via l7m_pack_http."""
    keep: list = []
    arr = (_HttpReq * max(1, len(reqs)))()
    total = 0
    for i, q in enumerate(reqs):
        names = (ctypes.c_char_p * max(1, len(q.headers)))(*[_b(h[0]) for h in q.headers])
        vals = (ctypes.c_char_p * max(1, len(q.headers)))(*[_b(h[1]) for h in q.headers])
        keep += [names, vals]
        arr[i] = _HttpReq(_b(q.method), _b(q.path), _b(q.authority),
                          ctypes.cast(names, ctypes.POINTER(ctypes.c_char_p)),
                          ctypes.cast(vals, ctypes.POINTER(ctypes.c_char_p)),
                          len(q.headers), q.remote_id, q.dport, 1 if q.ingress else 0, q.policy)
        sz = _lib.l7m_http_record_size(ctypes.byref(arr[i]))
        if sz == 0:
            raise L7Error(L7M_EINVAL, f"request {i} is not encodable")
        total += sz
    arena = np.zeros(max(4, total), dtype=np.uint8)
    offs = np.zeros(len(reqs), dtype=np.uint64)
    if reqs:
        used = _lib.l7m_pack_http(arr, len(reqs), arena.ctypes.data, arena.nbytes, offs.ctypes.data)
        if used != total:
            raise L7Error(L7M_EINVAL, "pack failed")
    return arena, offs


def pack_records(records: Sequence[bytes]) -> Tuple[np.ndarray, np.ndarray]:
    """Pack pre-encoded records (e.g. Kafka wire requests), 4-byte aligned."""
    offs = np.zeros(len(records), dtype=np.uint64)
    total = 0
    for i, r in enumerate(records):
        offs[i] = total
        total += (len(r) + 3) & ~3
    arena = np.zeros(max(4, total), dtype=np.uint8)
    for i, r in enumerate(records):
        o = int(offs[i])
        arena[o:o + len(r)] = np.frombuffer(r, dtype=np.uint8)
    return arena, offs


# --------------------------------------------------------------------------
# Rule sets
# --------------------------------------------------------------------------
class RuleSet:
    """An immutable compiled rule set (refcounted handle in libl7match)."""

    def __init__(self, handle: int, proto: int):
        self._h = ctypes.c_void_p(handle)
        self.proto = proto
        info = _Info()
        _lib.l7m_ruleset_get_info(self._h, ctypes.byref(info))
        self.info = info

    def __del__(self, _release=_lib.l7m_release):  # bound early: module globals are gone at exit
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            _release(h)
            self._h = None

    @property
    def handle(self) -> ctypes.c_void_p:
        return self._h

    @property
    def n_rules(self) -> int:
        return int(self.info.n_rules)

    @property
    def n_counters(self) -> int:
        return int(self.info.n_counters)

    def program(self) -> np.ndarray:
        n = ctypes.c_size_t(0)
        _lib.l7m_ruleset_program(self._h, None, ctypes.byref(n))
        buf = np.zeros(n.value // 4, dtype=np.uint32)
        _lib.l7m_ruleset_program(self._h, buf.ctypes.data, ctypes.byref(n))
        return buf

    @staticmethod
    def _opts(dialect: int, max_dfa_states: int, max_table_bytes: int, lds_budget_bytes: int = 0) -> _Opts:
        return _Opts(ctypes.sizeof(_Opts), dialect, max_dfa_states, 0, max_table_bytes, lds_budget_bytes, 0)

    @classmethod
    def compile_http(cls, rules: Sequence[PortRuleHTTP], dialect: int = DIALECT_ENVOY_ECMA_FULL,
                     max_dfa_states: int = 0, max_table_bytes: int = 0,
                     lds_budget_bytes: int = 0) -> "RuleSet":
        keep: list = []
        arr = (_HttpRule * max(1, len(rules)))(*[_http_rule_struct(r, keep) for r in rules])
        out = ctypes.c_void_p()
        err = ctypes.create_string_buffer(1024)
        opts = cls._opts(dialect, max_dfa_states, max_table_bytes, lds_budget_bytes)
        rc = _lib.l7m_compile_http(arr, len(rules), ctypes.byref(opts), ctypes.byref(out), err, 1024)
        if rc != L7M_OK:
            raise L7Error(rc, err.value.decode(errors="replace"))
        return cls(out.value, PROTO_HTTP)

    @classmethod
    def compile_http_policies(cls, policies: Sequence[NetworkPolicy], dialect: int = DIALECT_ENVOY_ECMA_FULL,
                              lds_budget_bytes: int = 0) -> "RuleSet":
        """A NetworkPolicyMap of NPDS NetworkPolicy resources (l7m_compile_http_policies)."""
        keep: list = []
        arr = _policies_struct(policies, keep)
        out = ctypes.c_void_p()
        err = ctypes.create_string_buffer(1024)
        opts = cls._opts(dialect, 0, 0, lds_budget_bytes)
        rc = _lib.l7m_compile_http_policies(arr, len(policies), ctypes.byref(opts), ctypes.byref(out), err, 1024)
        if rc != L7M_OK:
            raise L7Error(rc, err.value.decode(errors="replace"))
        return cls(out.value, PROTO_HTTP)

    def policy_index(self, name: str) -> int:
        """Record policy field for an endpoint policy name (POLICY_UNKNOWN if absent)."""
        i = _lib.l7m_ruleset_policy_index(self._h, _b(name))
        return POLICY_UNKNOWN if i < 0 else i

    def rule_origin(self, rule: int) -> Tuple[int, bool, int, int, int]:
        """(policy, ingress, port, port_rule, http_rule) of a verdict index."""
        o = _RuleOrigin()
        rc = _lib.l7m_ruleset_rule_origin(self._h, rule, ctypes.byref(o))
        if rc != L7M_OK:
            raise L7Error(rc, "rule index out of range")
        return (o.policy, bool(o.ingress), o.port, o.port_rule, o.http_rule)

    @staticmethod
    def _kafka_rules(rules: Sequence[PortRuleKafka]):
        return (_KafkaRule * max(1, len(rules)))(*[
            _KafkaRule(_b(r.Role) or None, _b(r.APIKey) or None, _b(r.APIVersion) or None,
                       _b(r.ClientID) or None, _b(r.Topic) or None) for r in rules])

    @classmethod
    def compile_kafka_map(cls, entries: Sequence[Tuple[Sequence[PortRuleKafka], bool]],
                          identities: Optional[dict] = None) -> "RuleSet":
        """The Kafka redirect's L7DataMap (pkg/policy/l4.go:110-129): entries =
        [(rules, is_wildcard_selector)], identities = {numeric identity:
        [indices of the entries whose selector matches its labels]}.  Evaluate
        with eval(..., identities=per-request source identities)."""
        keep = [cls._kafka_rules(r) for r, _ in entries]
        ents = (_KafkaSelectorRules * max(1, len(entries)))(*[
            _KafkaSelectorRules(keep[i], len(r), 1 if w else 0, 0) for i, (r, w) in enumerate(entries)])
        items = sorted((identities or {}).items())
        sels = [(ctypes.c_uint32 * max(1, len(v)))(*v) for _, v in items]
        ids = (_IdentitySelectors * max(1, len(items)))(*[
            _IdentitySelectors(k, 0, sels[i], len(v)) for i, (k, v) in enumerate(items)])
        out = ctypes.c_void_p()
        err = ctypes.create_string_buffer(1024)
        opts = cls._opts(0, 0, 0)
        rc = _lib.l7m_compile_kafka_map(ents, len(entries), ids, len(items), ctypes.byref(opts), ctypes.byref(out),
                                        err, 1024)
        if rc != L7M_OK:
            raise L7Error(rc, err.value.decode(errors="replace"))
        return cls(out.value, PROTO_KAFKA)

    @classmethod
    def compile_kafka(cls, rules: Sequence[PortRuleKafka]) -> "RuleSet":
        arr = cls._kafka_rules(rules)
        out = ctypes.c_void_p()
        err = ctypes.create_string_buffer(1024)
        opts = cls._opts(0, 0, 0)
        rc = _lib.l7m_compile_kafka(arr, len(rules), ctypes.byref(opts), ctypes.byref(out), err, 1024)
        if rc != L7M_OK:
            raise L7Error(rc, err.value.decode(errors="replace"))
        return cls(out.value, PROTO_KAFKA)

    # ---- evaluation -------------------------------------------------------
    def eval(self, arena: np.ndarray, offsets: np.ndarray, hits: Optional[np.ndarray] = None,
             identities: Optional[np.ndarray] = None) -> np.ndarray:
        """Host buffers -> int32 verdicts (H2D, kernel, D2H on the current device).
        identities: per-request source identity (Kafka rule sets, l7m_eval_ids)."""
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = offsets.shape[0]
        verdicts = np.empty(n, dtype=np.int32)
        hp = None
        if hits is not None:
            assert hits.dtype == np.uint64 and hits.shape[0] >= self.n_counters
            hp = hits.ctypes.data
        if identities is not None:
            identities = np.ascontiguousarray(identities, dtype=np.uint32)
            assert identities.shape[0] == n
            rc = _lib.l7m_eval_ids(self._h, arena.ctypes.data, arena.nbytes, offsets.ctypes.data, n,
                                   identities.ctypes.data, verdicts.ctypes.data, hp, 0)
        else:
            rc = _lib.l7m_eval(self._h, arena.ctypes.data, arena.nbytes, offsets.ctypes.data, n,
                               verdicts.ctypes.data, hp, 0)
        if rc != L7M_OK:
            raise L7Error(rc, "l7m_eval failed")
        return verdicts

    def eval_device(self, d_arena, arena_bytes: int, d_offsets, n: int, d_verdicts,
                    d_hits=None, stream=None, flags: int = 0) -> None:
        """Device pointers (ints or torch tensors) -> enqueue on `stream` (int handle)."""
        def ptr(x):
            if x is None:
                return None
            return x.data_ptr() if hasattr(x, "data_ptr") else int(x)
        rc = _lib.l7m_eval_device(self._h, ptr(d_arena), arena_bytes, ptr(d_offsets), n,
                                  ptr(d_verdicts), ptr(d_hits), stream, flags)
        if rc != L7M_OK:
            raise L7Error(rc, "l7m_eval_device failed")


class NetworkPolicyMap:
    """Batched mirror of Envoy's NetworkPolicyMap (envoy/cilium_network_policy.h
    :19-253): built from NPDS NetworkPolicy resources (or, as a shorthand, from
    one []PortRuleHTTP applied to every port and direction);
    Allowed(requests, policy_names) is NetworkPolicyMap::Allowed(policy_name,
    ingress, port, remote_id, headers) for a batch (h:223-237)."""

    def __init__(self, policies):
        policies = list(policies)
        if policies and isinstance(policies[0], PortRuleHTTP):
            self.ruleset = RuleSet.compile_http(policies)
        else:
            self.ruleset = RuleSet.compile_http_policies(policies)

    def verdicts(self, reqs: Sequence[HTTPRequest], policy_names: Optional[Sequence[str]] = None) -> np.ndarray:
        if policy_names is not None:
            idx = {n: self.ruleset.policy_index(n) for n in set(policy_names)}
            reqs = [HTTPRequest(q.method, q.path, q.authority, q.headers, q.remote_id, q.dport, q.ingress,
                                idx[n]) for q, n in zip(reqs, policy_names)]
        arena, offs = pack_http(reqs)
        return self.ruleset.eval(arena, offs)

    def Allowed(self, reqs: Sequence[HTTPRequest], policy_names: Optional[Sequence[str]] = None) -> np.ndarray:
        v = self.verdicts(reqs, policy_names)
        return (v >= 0)


class Batcher:
    """l7m_batcher: blocking per-request verdicts shared in GPU batches (the
    canAccess / decodeHeaders call shape, see include/l7match.h)."""

    def __init__(self, ruleset: "RuleSet", max_batch: int = 0, max_delay_us: int = 0, device: int = 0,
                 in_flight: int = 0, eager: bool = False):
        self.ruleset = ruleset
        opts = _BatcherOpts(ctypes.sizeof(_BatcherOpts), max_batch, max_delay_us, device, in_flight,
                            1 if eager else 0)
        h = ctypes.c_void_p()
        rc = _lib.l7m_batcher_create(ruleset.handle, ctypes.byref(opts), ctypes.byref(h))
        if rc != L7M_OK:
            raise L7Error(rc, "l7m_batcher_create failed")
        self._h = h

    def set_ruleset(self, ruleset: "RuleSet") -> None:
        self.ruleset = ruleset
        _lib.l7m_batcher_set_ruleset(self._h, ruleset.handle)

    def eval(self, record: bytes, src_identity: int = 0) -> int:
        v = ctypes.c_int32()
        rc = _lib.l7m_batcher_eval_from(self._h, record, len(record), src_identity, ctypes.byref(v))
        if rc != L7M_OK:
            raise L7Error(rc, "l7m_batcher_eval failed")
        return v.value

    def stats(self) -> Tuple[int, int]:
        b, r = ctypes.c_uint64(), ctypes.c_uint64()
        _lib.l7m_batcher_stats(self._h, ctypes.byref(b), ctypes.byref(r))
        return b.value, r.value

    def profile(self) -> dict:
        """Mean per-batch phases (l7m_batcher_get_profile), microseconds."""
        p = _BatcherProfile()
        _lib.l7m_batcher_get_profile(self._h, ctypes.byref(p))
        return {"batches": p.batches, "requests": p.requests, "fill_us": p.fill_us, "launch_us": p.launch_us,
                "gpu_us": p.gpu_us, "wake_us": p.wake_us, "resident_batches": p.resident_batches, "resident_rounds": p.resident_rounds,
                "resident_read_us": p.resident_read_us, "resident_eval_us": p.resident_eval_us,
                "resident_sync_us": p.resident_sync_us}

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.l7m_batcher_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


class _Shard(ctypes.Structure):
    _fields_ = [("arena", ctypes.c_void_p), ("arena_bytes", ctypes.c_size_t), ("rec_offsets", ctypes.c_void_p),
                ("n", ctypes.c_size_t), ("src_identities", ctypes.c_void_p), ("verdicts", ctypes.c_void_p)]


def shard_bounds(offsets: np.ndarray, arena_bytes: int, parts: int) -> np.ndarray:
    """l7m_shard_bounds: byte-balanced contiguous shards, bounds[0..parts]."""
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    out = np.zeros(parts + 1, dtype=np.uint64)
    rc = _lib.l7m_shard_bounds(offsets.ctypes.data, offsets.shape[0], int(arena_bytes), parts, out.ctypes.data)
    if rc != L7M_OK:
        raise L7Error(rc, "l7m_shard_bounds failed")
    return out


class DeviceSet:
    """l7m_multi: several GPUs from one process (include/l7match.h) -- byte-
    balanced shards, one stream per device, counters summed by one RCCL
    all-reduce over a single-process communicator (or on the host when a
    device repeats)."""

    def __init__(self, devices: Sequence[int]):
        arr = (ctypes.c_int * len(devices))(*devices)
        h = ctypes.c_void_p()
        rc = _lib.l7m_multi_create(arr, len(devices), ctypes.byref(h))
        if rc != L7M_OK:
            raise L7Error(rc, "l7m_multi_create failed")
        self._h = h
        self.devices = list(devices)

    @property
    def uses_rccl(self) -> bool:
        return bool(_lib.l7m_multi_uses_rccl(self._h))

    def eval(self, rs: "RuleSet", arena: np.ndarray, offsets: np.ndarray, hits: Optional[np.ndarray] = None,
             identities: Optional[np.ndarray] = None) -> np.ndarray:
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        n = offsets.shape[0]
        v = np.empty(n, dtype=np.int32)
        ids = None if identities is None else np.ascontiguousarray(identities, dtype=np.uint32)
        rc = _lib.l7m_multi_eval(self._h, rs.handle, arena.ctypes.data, arena.nbytes, offsets.ctypes.data, n,
                                 None if ids is None else ids.ctypes.data, v.ctypes.data,
                                 None if hits is None else hits.ctypes.data, 0)
        if rc != L7M_OK:
            raise L7Error(rc, "l7m_multi_eval failed")
        return v

    def eval_device(self, rs: "RuleSet", shards, hits: Optional[np.ndarray] = None, flags: int = 0) -> None:
        """shards: one (d_arena, arena_bytes, d_offsets, n, d_verdicts[, d_ids]) per device (device pointers
        as ints or objects with data_ptr())."""
        ptr = lambda x: None if x is None else (x.data_ptr() if hasattr(x, "data_ptr") else int(x))  # noqa: E731
        arr = (_Shard * len(shards))()
        for k, sh in enumerate(shards):
            a, ab, o, n, v = sh[:5]
            ids = sh[5] if len(sh) > 5 else None
            arr[k] = _Shard(ptr(a), ab, ptr(o), n, ptr(ids), ptr(v))
        rc = _lib.l7m_multi_eval_device(self._h, rs.handle, arr, None if hits is None else hits.ctypes.data, flags)
        if rc != L7M_OK:
            raise L7Error(rc, "l7m_multi_eval_device failed")

    def close(self) -> None:
        if getattr(self, "_h", None) is not None and self._h.value:
            _lib.l7m_multi_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


def http_deny_body(configured: str = "") -> bytes:
    """The 403 body AccessFilter sends on deny (envoy/cilium_l7policy.cc:89-95)."""
    n = _lib.l7m_http_deny_body(_b(configured) or None, None, 0)
    buf = ctypes.create_string_buffer(n + 1)
    _lib.l7m_http_deny_body(_b(configured) or None, buf, n + 1)
    return buf.raw[:n]


def kafka_deny_response(request: bytes) -> bytes:
    """CreateResponse(ErrTopicAuthorizationFailed) bytes for a denied request."""
    need = ctypes.c_size_t(0)
    rc = _lib.l7m_kafka_deny_response(request, len(request), None, 0, ctypes.byref(need))
    if rc not in (L7M_OK, L7M_ENOMEM):
        raise L7Error(rc, "l7m_kafka_deny_response failed")
    buf = ctypes.create_string_buffer(need.value)
    rc = _lib.l7m_kafka_deny_response(request, len(request), buf, need.value, ctypes.byref(need))
    if rc != L7M_OK:
        raise L7Error(rc, "l7m_kafka_deny_response failed")
    return buf.raw[:need.value]


def proxy_stats(verdicts: np.ndarray) -> dict:
    """Per-endpoint proxy counters of a batch of verdicts (l7m_proxy_stats_add)."""
    v = np.ascontiguousarray(verdicts, dtype=np.int32)
    st = _ProxyStats()
    _lib.l7m_proxy_stats_add(v.ctypes.data, v.shape[0], ctypes.byref(st))
    return {"received": st.received, "forwarded": st.forwarded, "denied": st.denied, "error": st.error}


class _ProxyStatsEntry(ctypes.Structure):
    _fields_ = [("proto", ctypes.c_uint32), ("port", ctypes.c_uint16), ("ingress", ctypes.c_uint8),
                ("request", ctypes.c_uint8), ("stats", _ProxyStats)]


class ProxyStatsTable:
    """Endpoint.proxyStatistics keyed by (protocol, port, ingress, request)
    (l7m_proxy_stats_table; pkg/endpoint/endpoint.go:2060-2122)."""

    def __init__(self):
        self._h = _lib.l7m_proxy_stats_table_create()

    def __del__(self, _free=_lib.l7m_proxy_stats_table_destroy):
        if getattr(self, "_h", None):
            _free(self._h)

    def update(self, proto: int, arena: np.ndarray, offsets: np.ndarray, verdicts: np.ndarray,
               port: int = 0, ingress: bool = True) -> None:
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        v = np.ascontiguousarray(verdicts, dtype=np.int32)
        rc = _lib.l7m_proxy_stats_update(self._h, proto, arena.ctypes.data, arena.nbytes, offsets.ctypes.data,
                                         v.ctypes.data, v.shape[0], port, 1 if ingress else 0)
        if rc != L7M_OK:
            raise L7Error(rc, "l7m_proxy_stats_update failed")

    def entries(self) -> dict:
        n = _lib.l7m_proxy_stats_get(self._h, None, 0)
        arr = (_ProxyStatsEntry * max(1, n))()
        _lib.l7m_proxy_stats_get(self._h, arr, n)
        name = {PROTO_HTTP: "http", PROTO_KAFKA: "kafka"}
        return {(name[e.proto], e.port, bool(e.ingress), bool(e.request)):
                {"received": e.stats.received, "forwarded": e.stats.forwarded, "denied": e.stats.denied,
                 "error": e.stats.error} for e in arr[:n]}


def http_access_log(arena: np.ndarray, offsets: np.ndarray, verdicts: np.ndarray, policy_name: str = "",
                    timestamp_ns: int = 0, http_protocol: int = 1, local_identity: int = 0,
                    source_address: str = None, destination_address: str = None) -> List[bytes]:
    """Serialized HttpLogEntry per request (l7m_http_access_log)."""
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    v = np.ascontiguousarray(verdicts, dtype=np.int32)
    n = v.shape[0]
    o = _AccessLogOpts(ctypes.sizeof(_AccessLogOpts), http_protocol, timestamp_ns, _b(policy_name), local_identity,
                       0, _b(source_address), _b(destination_address))
    eo = np.zeros(n + 1, dtype=np.uint64)
    need = _lib.l7m_http_access_log(arena.ctypes.data, arena.nbytes, offsets.ctypes.data, n, v.ctypes.data,
                                    ctypes.byref(o), None, 0, eo.ctypes.data)
    if need < 0:
        raise L7Error(int(need), "l7m_http_access_log failed")
    buf = ctypes.create_string_buffer(max(1, need))
    got = _lib.l7m_http_access_log(arena.ctypes.data, arena.nbytes, offsets.ctypes.data, n, v.ctypes.data,
                                   ctypes.byref(o), buf, need, eo.ctypes.data)
    if got != need:
        raise L7Error(L7M_EINVAL, "l7m_http_access_log size changed")
    raw = buf.raw
    return [raw[int(eo[i]):int(eo[i + 1])] for i in range(n)]


def kafka_access_log(arena: np.ndarray, offsets: np.ndarray, verdicts: np.ndarray) -> List[dict]:
    """The Kafka proxy's per-topic log records (l7m_kafka_access_log)."""
    arena = np.ascontiguousarray(arena, dtype=np.uint8)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    v = np.ascontiguousarray(verdicts, dtype=np.int32)
    n = _lib.l7m_kafka_access_log(arena.ctypes.data, arena.nbytes, offsets.ctypes.data, v.shape[0], v.ctypes.data,
                                  None, 0)
    if n < 0:
        raise L7Error(int(n), "l7m_kafka_access_log failed")
    arr = (_KafkaLogRecord * max(1, n))()
    _lib.l7m_kafka_access_log(arena.ctypes.data, arena.nbytes, offsets.ctypes.data, v.shape[0], v.ctypes.data,
                              arr, n)
    names = ["Forwarded", "Denied", "Error"]
    buf = arena.tobytes()
    return [{"request": r.request, "verdict": names[r.verdict], "error_code": r.error_code,
             "api_key": kafka_api_key_name(r.api_key), "api_version": r.api_version,
             "correlation_id": r.correlation_id,
             "topic": buf[r.topic_off:r.topic_off + r.topic_len].decode(errors="replace")} for r in arr[:n]]


def kafka_api_key_name(key: int) -> str:
    b = ctypes.create_string_buffer(64)
    _lib.l7m_kafka_api_key_name(key, b, 64)
    return b.value.decode()


def matches_rule(records: Sequence[bytes], rules: Sequence[PortRuleKafka]) -> np.ndarray:
    """Batched (*RequestMessage).MatchesRule (pkg/kafka/policy.go:200) over raw
    wire requests as proto.ReadReq returns them; returns int32 verdicts."""
    rs = RuleSet.compile_kafka(rules)
    arena, offs = pack_records(records)
    return rs.eval(arena, offs)
