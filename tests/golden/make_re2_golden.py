"""Writes tests/golden/re2_search.json: golden vectors for the
L7M_DIALECT_RE2_SEARCH dialect (Go `regexp.MustCompile(p).MatchString(s)`).

No Go toolchain exists in this environment, so these vectors are
"RE2-semantics, not run against Go" (SURVEY.md §8(c)):

* `search` — expected values computed with Python `re.search` on bytes over
  the intersection grammar where Python `re` and RE2 agree: literals,
  escaped punctuation, `.`, `^ $`, `\\d \\w \\s` and their negations,
  bracket classes with ranges, groups, `(?:`, alternation, `* + ? {n} {n,}
  {n,m}` (never `{,n}`), non-greedy markers; subjects are printable ASCII
  without CR / LF / VT (Python's `$` before a final newline and its `\\s`
  including VT are the only behaviours that would differ there).
* `syntax` — compile outcomes taken from the RE2 / Go regexp syntax
  documentation (`regexp/syntax` package doc: nested repetition, repeat
  count limit 1000, `\\pN`, flag groups, `\\b`, back-references), each with
  the rule it exercises.

Run:  python tests/golden/make_re2_golden.py
"""
import json
import os
import random
import re

HERE = os.path.dirname(os.path.abspath(__file__))

HAND = [
    # (pattern, subject)
    ("/public/.*", b"/public/a"), ("/public/.*", b"/x/public/a"), ("/public/.*", b"/publi"),
    ("^/public/", b"/public/x"), ("^/public/", b"/x/public/"), ("\\.html$", b"/a/index.html"),
    ("\\.html$", b"/a/index.html?x"), ("^$", b""), ("^$", b"a"), ("", b""), ("", b"anything"),
    ("a|b", b"xxbxx"), ("^(a|b)$", b"ab"), ("x*", b"yyy"), ("x+", b"yyy"), ("GET|HEAD", b"GETX"),
    ("^(GET|HEAD)$", b"GETX"), ("[0-9]{3}", b"ab123cd"), ("^[0-9]{3}$", b"1234"), ("\\d+", b"v12"),
    ("\\D", b"123"), ("\\w+@\\w+", b"mail: a@b"), ("\\s", b"a b"), ("\\S", b"   "),
    ("[^a-z]", b"abc"), ("[^a-z]", b"abC"), ("a.c", b"abc"), ("a.c", b"ac"), ("(?:ab)+$", b"xababab"),
    ("ab??c", b"ac"), ("a{2,3}", b"a"), ("a{2,3}", b"aaaa"), ("a{2,}b", b"aaab"), ("^a{2}$", b"aaa"),
    ("[-a]", b"-"), ("[a-]", b"x-"), ("\\[x\\]", b"[x]"), ("\\$\\^", b"a$^b"),
    (".*REGEX.*", b"hostREGEXname"), ("^svc[0-9]+\\.ns\\.local$", b"svc12.ns.local"),
    ("^svc[0-9]+\\.ns\\.local$", b"svc12.ns.localx"), ("(users|orders|items)/[0-9]+", b"/svc1/v2/orders/77"),
    ("/v[0-9]+/", b"/svc/vx/"), ("^/api/[a-z]+/.*", b"/api/books/1"), ("b$|^a", b"cab"),
    ("(a|aa)*b", b"aaaaaaaaaaaaaaaaaaaaaaaac"), ("(a|aa)*b", b"aaab"), (".*(x|y).*(z|w).*q", b"..x..w..q"),
    (".*(x|y).*(z|w).*q", b"..x..w.."), ("(.{0,8}){1,8}foo", b"zzzzzzzzzzzzfoo"),
]

ALPHA = "abcxyz019/._-"


def rand_pattern(rng, depth=0):
    k = rng.randrange(10 if depth < 3 else 6)
    if k <= 2:
        return rng.choice(["a", "b", "c", "x", "0", "1", "/", "\\.", "\\-", "\\/"])
    if k == 3:
        return rng.choice([".", "\\d", "\\w", "\\D", "\\W", "\\s", "\\S"])
    if k == 4:
        lo = rng.choice("abx0")
        hi = chr(min(ord(lo) + rng.randrange(4), ord("z")))
        return "[" + ("^" if rng.random() < 0.3 else "") + lo + "-" + hi + rng.choice(["", "/", "."]) + "]"
    if k == 5:
        return rng.choice(["^", "$"]) if rng.random() < 0.3 else rng.choice(["ab", "xyz", "19"])
    if k == 6:
        return rand_pattern(rng, depth + 1) + rand_pattern(rng, depth + 1)
    if k == 7:
        return "(" + rand_pattern(rng, depth + 1) + "|" + rand_pattern(rng, depth + 1) + ")"
    if k == 8:
        return "(?:" + rand_pattern(rng, depth + 1) + ")"
    q = rng.choice(["*", "+", "?", "{2}", "{1,3}", "{2,}", "*?", "+?"])
    return "(" + rand_pattern(rng, depth + 1) + ")" + q


def rand_subject(rng):
    n = rng.randrange(0, 12)
    return "".join(rng.choice(ALPHA) for _ in range(n)).encode()


def main():
    rng = random.Random(0xE2)
    cases = [{"pattern": p, "subject": s.decode("latin-1"), "match": bool(re.search(p.encode(), s))}
             for p, s in HAND]
    seen = set()
    while len(cases) < len(HAND) + 400:
        p = rand_pattern(rng)
        if p in seen:
            continue
        seen.add(p)
        for _ in range(3):
            s = rand_subject(rng)
            cases.append({"pattern": p, "subject": s.decode("latin-1"), "match": bool(re.search(p.encode(), s))})
    syntax = [
        {"pattern": "a**", "status": "invalid", "rule": "invalid nested repetition operator"},
        {"pattern": "a+*", "status": "invalid", "rule": "invalid nested repetition operator"},
        {"pattern": "a{2}{3}", "status": "invalid", "rule": "invalid nested repetition operator"},
        {"pattern": "*a", "status": "invalid", "rule": "missing argument to repetition operator"},
        {"pattern": "(*)", "status": "invalid", "rule": "missing argument to repetition operator"},
        {"pattern": "a{1001}", "status": "invalid", "rule": "invalid repeat count (max 1000)"},
        {"pattern": "a{3,2}", "status": "invalid", "rule": "invalid repeat count"},
        {"pattern": "(a", "status": "invalid", "rule": "missing closing )"},
        {"pattern": "a)", "status": "invalid", "rule": "unexpected )"},
        {"pattern": "[a", "status": "invalid", "rule": "missing closing ]"},
        {"pattern": "[z-a]", "status": "invalid", "rule": "invalid character class range"},
        {"pattern": "\\1", "status": "invalid", "rule": "back-references are not supported"},
        {"pattern": "a\\", "status": "invalid", "rule": "trailing backslash"},
        {"pattern": "\\y", "status": "invalid", "rule": "invalid escape sequence"},
        {"pattern": "(?=a)", "status": "invalid_or_unsupported", "rule": "look-ahead is not RE2 syntax"},
        {"pattern": "a{,3}", "status": "ok", "rule": "{,n} is a literal in RE2", "subject": "a{,3}", "match": True},
        {"pattern": "a{,3}", "status": "ok", "rule": "{,n} is a literal in RE2", "subject": "aaa", "match": False},
        {"pattern": "x{", "status": "ok", "rule": "lone { is a literal", "subject": "x{", "match": True},
        {"pattern": "\\Qa.b\\E", "status": "ok", "rule": "\\Q...\\E quotes", "subject": "a.b", "match": True},
        {"pattern": "\\Qa.b\\E", "status": "ok", "rule": "\\Q...\\E quotes", "subject": "axb", "match": False},
        {"pattern": "\\x41\\x{42}", "status": "ok", "rule": "hex escapes", "subject": "zAB", "match": True},
        {"pattern": "\\101", "status": "ok", "rule": "octal escape", "subject": "A", "match": True},
        {"pattern": "[[:digit:]]+", "status": "ok", "rule": "POSIX class in brackets", "subject": "a7", "match": True},
        {"pattern": "(?P<n>ab)c", "status": "ok", "rule": "named group", "subject": "xabc", "match": True},
        {"pattern": "\\Aab\\z", "status": "ok", "rule": "\\A \\z text anchors", "subject": "ab", "match": True},
        {"pattern": "\\Aab\\z", "status": "ok", "rule": "\\A \\z text anchors", "subject": "abc", "match": False},
        {"pattern": "[]a]", "status": "ok", "rule": "] first in a class is a literal", "subject": "]", "match": True},
        {"pattern": "(?i)abc", "status": "unsupported", "rule": "flag groups"},
        {"pattern": "\\bfoo", "status": "unsupported", "rule": "word boundary"},
        {"pattern": "\\pL", "status": "unsupported", "rule": "Unicode classes"},
    ]
    with open(os.path.join(HERE, "re2_search.json"), "w") as f:
        json.dump({"source": "Python re.search (intersection grammar) and the RE2 syntax documentation; "
                             "RE2-semantics, not run against Go", "search": cases, "syntax": syntax}, f, indent=0)


if __name__ == "__main__":
    main()
