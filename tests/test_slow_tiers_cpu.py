"""The slow pass's stack bound (regex_vm.h kVmScratchWords2 = 1 MiB) against
the reference engine's own recursion: libstdc++'s std::regex_match (Envoy's
HeaderMatcher regexes, envoy/cilium_network_policy.h:52-71) keeps one native
frame per NFA state on the current path and overflows an Envoy worker's 8 MiB
thread stack.  For the HTTP slow path to report
L7M_VERDICT_UNSUPPORTED only where the reference itself would overflow, every
explicit-stack word the executor needs must cost the reference at least 8
native bytes (8 MiB / 1 MiB).  Measured here per pattern family: native bytes
touched by std::regex_match on a fresh measured stack (oracle
orc_regex_match_stack) vs the smallest scratch the executor (host build of
regex_vm.h) decides the same subject with."""
import ctypes

import numpy as np
import pytest

from cilium_amd import l7match as L
from oracle import ENVOY_THREAD_STACK, HttpOracle, regex_match_stack
from program_interp import _VM, VM_DEEP, VM_SCRATCH_WORDS, HttpProgram

FAMILIES = [
    ("/(a)(?:.)*\\1z", "/a", "b", "az"),
    ("/(a)(.)*\\1z", "/a", "b", "az"),
    ("/(a)(?:b|c)*\\1z", "/a", "b", "az"),
    ("/(a)(b|c)*\\1z", "/a", "b", "az"),
    ("/(a)(?:.)*?\\1z", "/a", "b", "az"),
    ("/(a)[^z]*\\1z", "/a", "b", "az"),
    ("/(a)(?:(?=b).)*\\1z", "/a", "b", "az"),
    ("/(a)(?:b+)*\\1z", "/a", "b", "az"),
    ("/(a)(?:(b)|(c))*\\1z", "/a", "b", "az"),
    ("/(a)(?:bb|b)*\\1z", "/a", "b", "az"),
    # (/(\\w+)/\\1(/.*)? is a forced capture since round 6: decided in the
    # first pass by byte compares, program.h DcapSpec, so it has no executor
    # program; a near-miss form with two references keeps one)
    ("/(\\w+)/\\1\\1(/.*)?", "/abc/abcabc/", "x", ""),
    ("/(a|bb)+-\\1", "/", "a", "-a"),
]


def _vm_program(pattern):
    """The slow-path program of a one-rule set's :path matcher."""
    P = HttpProgram(L.RuleSet.compile_http([L.PortRuleHTTP(Path=pattern)]).program())
    h = P.h
    so, sl = P.w[h["off_slow"]: h["off_slow"] + 2]
    assert sl == 1, "expected one slow matcher"
    off = P.w[h["off_pool"] + so + 1]
    return P.prog[off:]


def _words_needed(prog, subject):
    lo, hi = 64, 1 << 24  # hi decides
    assert _VM.vm_host_match(prog.ctypes.data, subject, len(subject), hi, 1 << 30) >= 0
    while hi - lo > 8:
        m = (lo + hi) // 2
        if _VM.vm_host_match(prog.ctypes.data, subject, len(subject), m, 1 << 30) == VM_DEEP:
            lo = m
        else:
            hi = m
    return hi


@pytest.mark.parametrize("pat,pre,c,post", FAMILIES)
def test_reference_stack_per_executor_word(pat, pre, c, post):
    prog = _vm_program(pat)
    ratios = []
    for n in (2000, 6000):
        s = (pre + c * n + post).encode()
        r, native = regex_match_stack(pat, s)
        assert r == 1
        ratios.append(native / (4.0 * _words_needed(prog, s)))
    # >= 8 native bytes per executor byte: a subject that needs more than the
    # 1 MiB second-tier stack needs more than 8 MiB in the reference
    assert min(ratios) >= ENVOY_THREAD_STACK / (4.0 * VM_SCRATCH_WORDS), (pat, ratios)


def test_interpreter_unsupported_only_where_reference_overflows():
    """The program interpreter (tier-2 limits, the GPU's final verdicts)
    decides every subject the reference decides on an 8 MiB stack, and the
    −3 it reports sits where the reference overflows."""
    rules = [L.PortRuleHTTP(Path="/(a)(?:.)*\\1z"), L.PortRuleHTTP(Path="/(a)(b|c)*\\1z"), L.PortRuleHTTP(Path="/.*")]
    reqs = [L.HTTPRequest("GET", "/a" + "b" * n + "az") for n in (10, 2000, 8000, 12000, 20000, 40000)]
    reqs += [L.HTTPRequest("GET", "/a" + "b" * n + "ay") for n in (100, 20000)]
    arena, offs = L.pack_http(reqs)
    rs = L.RuleSet.compile_http(rules)
    got = HttpProgram(rs.program()).eval(arena, offs)
    exp, used = HttpOracle(rules, prefilter=False).eval_stack(arena, offs)
    for i in range(len(reqs)):
        if used[i] <= ENVOY_THREAD_STACK:
            assert got[i] == exp[i], (i, int(got[i]), int(exp[i]), int(used[i]))
        if got[i] == L.VERDICT_UNSUPPORTED:
            assert used[i] > ENVOY_THREAD_STACK, (i, int(used[i]))
    assert got[:4].tolist() == [0, 0, 0, 0]
    assert got[-2:].tolist() == [2, 2]
