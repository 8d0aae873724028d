"""Shared NPDS policy-map cases (CPU interpreter tests and GPU parity tests).

The reference boundary is NetworkPolicyMap::Allowed(policy_name, ingress,
port, remote_id, headers) (envoy/cilium_network_policy.h:223-237): per
endpoint policy, per direction, the exact-port entry, then port 0, then
"no entry -> allow"; an entry without HTTP rules allows; an unknown endpoint
policy denies."""
import json
import os
import random

from cilium_amd import l7match as L

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "http_known_answers.json")


def _http(d):
    return L.PortRuleHTTP(Path=d.get("Path", ""), Method=d.get("Method", ""), Host=d.get("Host", ""),
                          Headers=d.get("Headers", []))


def npds(d):
    """JSON fixture form -> L.NetworkPolicy."""
    def pp(x):
        return L.PortNetworkPolicy(Port=x["Port"], Protocol=x.get("Protocol", L.L4_TCP), Rules=[
            L.PortNetworkPolicyRule(RemotePolicies=r.get("RemotePolicies", []),
                                    HttpRules=None if r.get("HttpRules") is None else [_http(h) for h in r["HttpRules"]])
            for r in x.get("Rules", [])])
    return L.NetworkPolicy(Name=d["Name"], Ingress=[pp(x) for x in d.get("Ingress", [])],
                           Egress=[pp(x) for x in d.get("Egress", [])])


def golden_npds():
    with open(GOLD) as f:
        return json.load(f)["npds_basic_policy"]


def basic_requests(g):
    """Ingress and egress known-answer requests of the integration test."""
    reqs, expect = [], []
    for key, ingress in (("ingress_cases", True), ("egress_cases", False)):
        for c in g[key]:
            reqs.append(L.HTTPRequest(c["method"], c["path"], c["authority"], remote_id=g["remote_id"],
                                      dport=g["dport"], ingress=ingress, policy=0))
            expect.append(c["allow"])
    return reqs, expect


_PATHS = ["/public/a", "/private/x", "/api/v1/users", "/admin", "/", "/public/b/c", "/health"]
_HOSTS = ["svc.local", "api.example", "h", "admin.local"]


def random_policies(seed, n_policies=3):
    """Random NPDS policies exercising every branch of PortNetworkPolicy /
    PortNetworkPolicyRules / PortNetworkPolicyRule::Matches."""
    rnd = random.Random(seed)

    def http_rule():
        r = L.PortRuleHTTP()
        k = rnd.randrange(6)
        if k == 0:
            r.Path = rnd.choice(["/public/.*", "/api/v[0-9]+/.*", "/admin", "/(health|ready)"])
        elif k == 1:
            r.Method = rnd.choice(["GET", "POST|PUT", "[A-Z]+"])
            r.Path = rnd.choice(["/public/.*", "/api/.*"])
        elif k == 2:
            r.Host = rnd.choice(["svc\\.local", ".*example", "admin\\..*"])
        elif k == 3:
            r.Headers = [rnd.choice(["x-token: abc", "x-debug", "x-tenant: t1"])]
        elif k == 4:
            r.Path = "/"
        return r

    def port_rule():
        rem = rnd.sample([1, 2, 3, 4], rnd.randrange(3))
        if rnd.random() < 0.2:
            return L.PortNetworkPolicyRule(RemotePolicies=rem, HttpRules=None)
        return L.PortNetworkPolicyRule(RemotePolicies=rem, HttpRules=[http_rule() for _ in range(rnd.randrange(1, 4))])

    def direction():
        ports = rnd.sample([0, 80, 443, 8080], rnd.randrange(0, 4))
        out = []
        for p in ports:
            k = rnd.random()
            if k < 0.15:
                rules = []  # empty PortNetworkPolicyRules: allow everything
            elif k < 0.3:
                rules = [L.PortNetworkPolicyRule(RemotePolicies=[1])]  # remote-only: no HTTP rules
            else:
                rules = [port_rule() for _ in range(rnd.randrange(1, 4))]
            out.append(L.PortNetworkPolicy(Port=p, Rules=rules))
        if rnd.random() < 0.3:
            out.append(L.PortNetworkPolicy(Port=9999, Protocol=L.L4_UDP,
                                           Rules=[L.PortNetworkPolicyRule(HttpRules=[http_rule()])]))
        return out

    return [L.NetworkPolicy(Name=f"ep-{seed}-{i}", Ingress=direction(), Egress=direction())
            for i in range(n_policies)]


def random_requests(seed, n, n_policies=3):
    rnd = random.Random(seed ^ 0x5EED)
    out = []
    for _ in range(n):
        hdrs = []
        if rnd.random() < 0.3:
            hdrs.append(("x-token", rnd.choice(["abc", "abd"])))
        if rnd.random() < 0.2:
            hdrs.append(("x-debug", "1"))
        if rnd.random() < 0.2:
            hdrs.append(("x-tenant", rnd.choice(["t1", "t2"])))
        pol = rnd.randrange(n_policies) if rnd.random() < 0.95 else L.POLICY_UNKNOWN
        out.append(L.HTTPRequest(rnd.choice(["GET", "POST", "PUT", "DELETE"]), rnd.choice(_PATHS),
                                 rnd.choice(_HOSTS + [None]), hdrs, remote_id=rnd.choice([1, 2, 3, 5]),
                                 dport=rnd.choice([80, 443, 8080, 9999, 0, 22]), ingress=rnd.random() < 0.5,
                                 policy=pol))
    return out
