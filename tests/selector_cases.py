"""L7DataMap cases (pkg/policy/l4.go:110-129 GetRelevantRules under
kafkaRedirect.canAccess, pkg/proxy/kafka.go:116-152): a map of selector
entries, per-identity selector matches, and requests from mixed sources."""
import random

import numpy as np

from cilium_amd import l7match as L
from cilium_amd import workloads as W


def random_map(seed, n_entries=6, n_rules=1200, n_ids=40, n_wild=2):
    """Config-3 rules dealt over n_entries entries (the last n_wild of them
    wildcard selectors) and n_ids identities, each selected by a random
    subset of the non-wildcard entries (possibly none)."""
    rnd = random.Random(seed)
    rules = W.rules(3, n_rules=n_rules)
    cut = sorted(rnd.sample(range(1, n_rules), n_entries - 1))
    parts = [rules[a:b] for a, b in zip([0] + cut, cut + [n_rules])]
    entries = [(parts[g], g >= n_entries - n_wild) for g in range(n_entries)]
    sel = [g for g in range(n_entries) if g < n_entries - n_wild]
    ids = {}
    for k in range(n_ids):
        ident = 1000 + 7 * k
        ids[ident] = sorted(rnd.sample(sel, rnd.randrange(0, len(sel) + 1)))
    return entries, ids


def request_identities(seed, n, ids):
    """Per-request sources: listed identities, 0 (unresolved) and unlisted ones."""
    rnd = np.random.default_rng(seed)
    pool = np.array(sorted(ids) + [0, 0, 5, 999_999], dtype=np.uint32)
    return pool[rnd.integers(0, len(pool), n)]


def relevant_rules(entries, ids, identity):
    """GetRelevantRules' list for one source, in the reference's order: the
    selecting entries' rules, then the wildcard entries' rules (appended)."""
    sel = ids.get(identity, []) if identity else []
    out = []
    for g in sel:
        out += list(entries[g][0])
    for rules, wild in entries:
        if wild:
            out += list(rules)
    return out
