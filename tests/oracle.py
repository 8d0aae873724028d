"""ctypes binding of the CPU oracle (oracle/liboracle.so).  TEST INFRASTRUCTURE
ONLY: used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
as the checker, never by the product path."""
import ctypes
import os
import subprocess

import numpy as np

from cilium_amd import l7match as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "liboracle.so")


def _load():
    if not os.path.exists(ORACLE_SO):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    lib = ctypes.CDLL(ORACLE_SO)
    P, sz = ctypes.c_void_p, ctypes.c_size_t
    lib.orc_http_new.argtypes = [ctypes.POINTER(L._HttpRule), sz, ctypes.POINTER(P), ctypes.c_char_p, sz]
    lib.orc_http_new_dialect.argtypes = [ctypes.POINTER(L._HttpRule), sz, ctypes.c_uint32, ctypes.POINTER(P),
                                         ctypes.c_char_p, sz]
    lib.orc_http_new_engine.argtypes = [ctypes.POINTER(L._HttpRule), sz, ctypes.c_uint32, ctypes.c_int,
                                        ctypes.POINTER(P), ctypes.c_char_p, sz]
    lib.orc_http_policies_new_engine.argtypes = [ctypes.POINTER(L._NetworkPolicy), sz, ctypes.c_uint32, ctypes.c_int,
                                                 ctypes.POINTER(P), ctypes.c_char_p, sz]
    lib.orc_nfa_match.argtypes = [ctypes.c_char_p, ctypes.c_char_p, sz, ctypes.c_int]
    lib.orc_http_eval.argtypes = [P, P, sz, P, sz, P, ctypes.c_int]
    lib.orc_http_free.argtypes = [P]
    lib.orc_http_set_prefilter.argtypes = [P, ctypes.c_int]
    lib.orc_http_policies_new.argtypes = [ctypes.POINTER(L._NetworkPolicy), sz, ctypes.c_uint32,
                                          ctypes.POINTER(P), ctypes.c_char_p, sz]
    lib.orc_http_policies_eval.argtypes = [P, P, sz, P, sz, P, ctypes.c_int]
    lib.orc_http_policies_free.argtypes = [P]
    lib.orc_kafka_new.argtypes = [ctypes.POINTER(L._KafkaRule), sz, ctypes.POINTER(P), ctypes.c_char_p, sz]
    lib.orc_kafka_eval.argtypes = [P, P, sz, P, sz, P, ctypes.c_int]
    lib.orc_kafka_free.argtypes = [P]
    lib.orc_snappy_decode.argtypes = [ctypes.c_char_p, sz, ctypes.c_char_p, sz, ctypes.POINTER(sz)]
    lib.orc_kafka_new_map.argtypes = [ctypes.POINTER(L._KafkaSelectorRules), sz, ctypes.POINTER(L._IdentitySelectors),
                                      sz, ctypes.POINTER(P), ctypes.c_char_p, sz]
    lib.orc_kafka_eval_ids.argtypes = [P, P, sz, P, sz, P, P, ctypes.c_int]
    lib.orc_regex_match.argtypes = [ctypes.c_char_p, ctypes.c_char_p, sz]
    lib.orc_regex_search.argtypes = [ctypes.c_char_p, ctypes.c_char_p, sz]
    lib.orc_http_eval_stack.argtypes = [P, P, sz, P, sz, P, P]
    lib.orc_regex_match_stack.argtypes = [ctypes.c_char_p, ctypes.c_char_p, sz, ctypes.POINTER(ctypes.c_uint64)]
    return lib


_lib = _load()


class OracleError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"oracle error {code}: {msg}")
        self.code = code


ENGINES = {"std": 0, "nfa": 1}


class HttpOracle:
    """engine="std": std::regex_match (the reference engine); engine="nfa":
    the Thompson-NFA / Pike-VM simulator (oracle/nfa.h), the long-input oracle
    for config 5 where the backtracker cannot finish or would overflow."""

    def __init__(self, rules, dialect=L.DIALECT_ENVOY_ECMA_FULL, engine="std", prefilter=True):
        """prefilter=False: every rule's matchers are evaluated per request, as
        Envoy does (bench.py's cpu_baseline); the default skips rules whose
        literal prefixes the request's values lack (same verdicts, faster)."""
        keep = []
        arr = (L._HttpRule * max(1, len(rules)))(*[L._http_rule_struct(r, keep) for r in rules])
        h = ctypes.c_void_p()
        err = ctypes.create_string_buffer(512)
        rc = _lib.orc_http_new_engine(arr, len(rules), dialect, ENGINES[engine], ctypes.byref(h), err, 512)
        if rc != 0:
            raise OracleError(rc, err.value.decode(errors="replace"))
        self._h = h
        _lib.orc_http_set_prefilter(h, 1 if prefilter else 0)

    def __del__(self, _free=_lib.orc_http_free):  # bound early: module globals are gone at exit
        if getattr(self, "_h", None) and self._h.value:
            _free(self._h)

    def eval(self, arena, offsets, threads=1):
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        v = np.empty(offsets.shape[0], dtype=np.int32)
        _lib.orc_http_eval(self._h, arena.ctypes.data, arena.nbytes, offsets.ctypes.data,
                           offsets.shape[0], v.ctypes.data, threads)
        return v

    def eval_stack(self, arena, offsets):
        """(verdicts, native stack bytes each request's evaluation touched):
        every request on a fresh thread with a 1 GiB reserved stack, so
        std::regex_match finishes where an 8 MiB thread would overflow."""
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        v = np.empty(offsets.shape[0], dtype=np.int32)
        used = np.empty(offsets.shape[0], dtype=np.uint64)
        _lib.orc_http_eval_stack(self._h, arena.ctypes.data, arena.nbytes, offsets.ctypes.data,
                                 offsets.shape[0], v.ctypes.data, used.ctypes.data)
        return v, used


# The default stack of a thread (ulimit -s: an Envoy worker's): std::regex_match
# overflows it (SIGSEGV, the Envoy process dies) past this much recursion.
ENVOY_THREAD_STACK = 8 << 20


class PolicyOracle:
    """NetworkPolicyMap restated (oracle/l7oracle.cc PolicyOracle)."""

    def __init__(self, policies, dialect=L.DIALECT_ENVOY_ECMA_FULL, engine="std"):
        keep = []
        arr = L._policies_struct(policies, keep)
        h = ctypes.c_void_p()
        err = ctypes.create_string_buffer(512)
        rc = _lib.orc_http_policies_new_engine(arr, len(policies), dialect, ENGINES[engine], ctypes.byref(h), err,
                                               512)
        if rc != 0:
            raise OracleError(rc, err.value.decode(errors="replace"))
        self._h = h

    def __del__(self, _free=_lib.orc_http_policies_free):
        if getattr(self, "_h", None) and self._h.value:
            _free(self._h)

    def eval(self, arena, offsets, threads=1):
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        v = np.empty(offsets.shape[0], dtype=np.int32)
        _lib.orc_http_policies_eval(self._h, arena.ctypes.data, arena.nbytes, offsets.ctypes.data,
                                    offsets.shape[0], v.ctypes.data, threads)
        return v


class KafkaOracle:
    def __init__(self, rules):
        arr = (L._KafkaRule * max(1, len(rules)))(*[
            L._KafkaRule(L._b(r.Role) or None, L._b(r.APIKey) or None, L._b(r.APIVersion) or None,
                         L._b(r.ClientID) or None, L._b(r.Topic) or None) for r in rules])
        h = ctypes.c_void_p()
        err = ctypes.create_string_buffer(512)
        rc = _lib.orc_kafka_new(arr, len(rules), ctypes.byref(h), err, 512)
        if rc != 0:
            raise OracleError(rc, err.value.decode(errors="replace"))
        self._h = h

    def __del__(self, _free=_lib.orc_kafka_free):
        if getattr(self, "_h", None) and self._h.value:
            _free(self._h)

    @classmethod
    def from_map(cls, entries, identities=None):
        """L7DataMap oracle: entries = [(rules, is_wildcard)], identities =
        {identity: [entry indices whose selector matches it]}."""
        self = cls.__new__(cls)
        keep = [L.RuleSet._kafka_rules(r) for r, _ in entries]
        ents = (L._KafkaSelectorRules * max(1, len(entries)))(*[
            L._KafkaSelectorRules(keep[i], len(r), 1 if w else 0, 0) for i, (r, w) in enumerate(entries)])
        items = sorted((identities or {}).items())
        sels = [(ctypes.c_uint32 * max(1, len(v)))(*v) for _, v in items]
        ids = (L._IdentitySelectors * max(1, len(items)))(*[
            L._IdentitySelectors(k, 0, sels[i], len(v)) for i, (k, v) in enumerate(items)])
        h = ctypes.c_void_p()
        err = ctypes.create_string_buffer(512)
        rc = _lib.orc_kafka_new_map(ents, len(entries), ids, len(items), ctypes.byref(h), err, 512)
        if rc != 0:
            raise OracleError(rc, err.value.decode(errors="replace"))
        self._h = h
        return self

    def eval(self, arena, offsets, threads=1, identities=None):
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        v = np.empty(offsets.shape[0], dtype=np.int32)
        if identities is None:
            _lib.orc_kafka_eval(self._h, arena.ctypes.data, arena.nbytes, offsets.ctypes.data,
                                offsets.shape[0], v.ctypes.data, threads)
        else:
            identities = np.ascontiguousarray(identities, dtype=np.uint32)
            _lib.orc_kafka_eval_ids(self._h, arena.ctypes.data, arena.nbytes, offsets.ctypes.data,
                                    offsets.shape[0], identities.ctypes.data, v.ctypes.data, threads)
        return v


def regex_match(pattern: str, value: bytes) -> int:
    """std::regex_match(value, std::regex(pattern, optimize)) -> 1/0, -1 if invalid."""
    return _lib.orc_regex_match(pattern.encode(), value, len(value))


def regex_match_stack(pattern: str, value: bytes):
    """(std::regex_match result 1/0/-1, native stack bytes it touched)."""
    used = ctypes.c_uint64(0)
    r = _lib.orc_regex_match_stack(pattern.encode(), value, len(value), ctypes.byref(used))
    return r, int(used.value)


def regex_search(pattern: str, value: bytes) -> int:
    """std::regex_search(value, std::regex(pattern, optimize)) -> 1/0, -1 if invalid."""
    return _lib.orc_regex_search(pattern.encode(), value, len(value))


def nfa_match(pattern: str, value: bytes, search: bool = False) -> int:
    """The oracle's NFA simulator (oracle/nfa.h): 1/0, -1 syntax error, -2 unsupported."""
    return _lib.orc_nfa_match(pattern.encode(), value, len(value), 1 if search else 0)


def snappy_decode(src: bytes, cap: int = 1 << 22):
    """proto/snappy.go snappyDecode restated (oracle/l7oracle.cc go_snappy):
    (0, decoded bytes), or (1, None) where the reference errors or panics."""
    out = ctypes.create_string_buffer(max(cap, 1))
    n = ctypes.c_size_t(0)
    rc = _lib.orc_snappy_decode(src, len(src), out, cap, ctypes.byref(n))
    return (rc, out.raw[:n.value] if rc == 0 else None)
