"""Reentrancy through the C ABI: 8 host threads of a plain C program
(tests/cpp/abi_harness.c, no ctypes) call l7m_eval concurrently on ONE
compiled handle; every thread's verdicts equal the oracle's and the summed
per-rule counters equal threads x iterations x one evaluation's."""
import numpy as np
import pytest

from abi_files import run
from cilium_amd import l7match as L
from cilium_amd import workloads as W
from oracle import HttpOracle

pytestmark = pytest.mark.gpu


def test_eight_threads_one_handle_c_harness(gpu, tmp_path):
    rules = W.rules(2)
    arena, offs = W.requests(2, 3_000_000, 50_000)
    threads, iters = 8, 3
    p, res = run(str(tmp_path), rules, arena, offs, threads, iters)
    assert p.returncode == 0, p.stderr[-2000:]
    verd, hits = res
    exp = HttpOracle(rules).eval(arena, offs, threads=8)
    assert np.array_equal(verd, exp)
    one = np.zeros(len(rules) + 2, dtype=np.uint64)
    L.RuleSet.compile_http(rules).eval(arena, offs, one)
    assert np.array_equal(hits, one * threads * iters)


def test_batcher_call_site_c_harness(gpu, tmp_path):
    """The call-site shape through the C ABI: 8 threads decide requests one
    at a time with the blocking l7m_batcher_eval (canAccess / decodeHeaders),
    a policy update (l7m_batcher_set_ruleset) lands halfway, denied requests
    get the 403 body; verdicts equal the oracle's, requests share batches,
    and the proxy stats add up."""
    rules = W.rules(2)
    arena, offs = W.requests(2, 5_000_000, 6_000)
    p, res = run(str(tmp_path), rules, arena, offs, 8, 1, batcher=True)
    assert p.returncode == 0, p.stderr[-2000:]
    verd, st = res
    exp = HttpOracle(rules).eval(arena, offs, threads=8)
    assert np.array_equal(verd, exp)
    batches, requests, denied, forwarded = (int(x) for x in st)
    # Coalescing is a scheduling property, not a parity one: deadline batches
    # flush as soon as every free caller is in them (l7m_batch.cc run()), so
    # the mean batch size follows the box's timing.  What holds on any box:
    # every request was decided exactly once, and with 8 callers not every
    # batch was a singleton.  Batch sizes / latency are reported by bench.py.
    assert requests == len(offs) and 1 <= batches < requests
    assert denied == int((exp == L.VERDICT_DENY).sum()) and forwarded == int((exp >= 0).sum())


def test_pipelined_host_eval_large_batches(gpu):
    """Host batches of >= 128 MiB take the chunked two-stream pipeline of
    l7m_eval (H2D of chunk k+1 overlapping chunk k's kernel): verdicts and
    counters equal the device-resident evaluation, HTTP and Kafka, pinned or
    pageable host memory; an oracle sample pins the verdicts."""
    import torch
    for cfg, n in ((2, 1_500_000), (3, 2_200_000)):
        rules = W.rules(cfg)
        rs = L.RuleSet.compile_http(rules) if cfg == 2 else L.RuleSet.compile_kafka(rules)
        arena, offs = W.requests(cfg, 9_000_000, n)
        assert arena.nbytes >= (128 << 20), arena.nbytes  # the pipelined path
        h = np.zeros(rs.n_counters, dtype=np.uint64)
        v = rs.eval(arena, offs, h)
        pinned = torch.from_numpy(arena).pin_memory().numpy()
        h2 = np.zeros(rs.n_counters, dtype=np.uint64)
        assert np.array_equal(rs.eval(pinned, offs, h2), v) and np.array_equal(h, h2)
        dev = torch.device("cuda:0")
        da = torch.from_numpy(arena).to(dev)
        do = torch.from_numpy(offs.view(np.int64)).to(dev)
        dv = torch.empty(len(offs), dtype=torch.int32, device=dev)
        dh = torch.zeros(rs.n_counters, dtype=torch.int64, device=dev)
        rs.eval_device(da, arena.nbytes, do, len(offs), dv, dh, torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        assert np.array_equal(dv.cpu().numpy(), v)
        assert np.array_equal(dh.cpu().numpy().astype(np.uint64), h) and int(h.sum()) == n
        # oracle on records spread over every chunk
        from oracle import KafkaOracle
        keep = np.arange(0, n, 997)
        recs = [arena[int(offs[i]):int(offs[i + 1]) if i + 1 < n else arena.nbytes - 64].tobytes() for i in keep]
        a2, o2 = L.pack_records(recs)
        orc = HttpOracle(rules) if cfg == 2 else KafkaOracle(rules)
        assert np.array_equal(orc.eval(a2, o2, threads=16), v[keep])


def test_batcher_destroy_with_calls_in_flight(gpu):
    """l7m_batcher_destroy while 64 threads are blocked inside
    l7m_batcher_eval (a 60 s flush deadline would keep a pending batch
    waiting): the pending batch is still decided, every caller gets the
    oracle's verdict, destroy returns only after they have left (well before
    the deadline), and a later call is L7M_EINVAL."""
    import threading
    import time
    rules = W.rules(2)
    rs = L.RuleSet.compile_http(rules)
    arena, offs = W.requests(2, 11_000_000, 64)
    exp = HttpOracle(rules).eval(arena, offs, threads=8)
    recs = [arena[int(offs[i]):int(offs[i + 1]) if i + 1 < len(offs) else arena.nbytes - 64].tobytes()
            for i in range(len(offs))]
    for in_flight in (1, 3):
        b = L.Batcher(rs, max_batch=1 << 20, max_delay_us=60_000_000, in_flight=in_flight)
        got = np.full(len(recs), -100, dtype=np.int64)
        entered = [False] * len(recs)

        def worker(i):
            entered[i] = True
            got[i] = b.eval(recs[i])

        th = [threading.Thread(target=worker, args=(i,)) for i in range(len(recs))]
        t0 = time.perf_counter()
        for x in th:
            x.start()
        while not all(entered):
            time.sleep(0.001)
        time.sleep(0.2)
        b.close()  # flushes the pending batch now, not at the 2 s deadline
        for x in th:
            x.join()
        assert time.perf_counter() - t0 < 30.0  # not the 60 s deadline
        assert np.array_equal(got, exp)
        with pytest.raises(L.L7Error) as e:
            b.eval(recs[0])
        assert e.value.code == L.L7M_EINVAL


def test_batcher_idle_gap_and_rule_switches(gpu):
    """HTTP through the batcher with 8 threads calling concurrently: verdicts
    equal the oracle's across an idle gap, switches between programs of the
    4- and 8-register instantiations (7 value DFAs), one with back-references
    (slow-path second kernel) and back."""
    import threading
    import time
    import numpy as np
    from regex_ext_cases import REALISTIC, realistic_requests

    rng = np.random.default_rng(5)
    rules_a = W.rules(2)
    arena, offs = W.requests(2, 13_000_000, 400)
    recs_a = [arena[int(offs[i]):int(offs[i + 1]) if i + 1 < len(offs) else arena.nbytes - 64].tobytes()
              for i in range(len(offs))]
    exp_a = HttpOracle(rules_a).eval(arena, offs, threads=8)
    rules_b = [L.PortRuleHTTP(Path="/a/.*", Method="GET", Host="h[0-9]+\\.example",
                              Headers=["X-A: 1", "X-B: two", "X-C: 3"]),
               L.PortRuleHTTP(Path="/b/[a-z]+", Method="POST", Headers=["X-D: 4"])]
    reqs_b = []
    for i in range(300):
        hdr = [("x-a", "1"), ("x-b", "two"), ("x-c", "3")] if rng.random() < 0.7 else [("x-d", "4")]
        reqs_b.append(L.HTTPRequest(str(rng.choice(["GET", "POST"])), str(rng.choice(["/a/x", "/b/yz", "/b/9", "/c"])),
                                    str(rng.choice(["h1.example", "h22.example", "hx.example"])), hdr))
    ab, ob = L.pack_http(reqs_b)
    recs_b = [ab[int(ob[i]):int(ob[i + 1]) if i + 1 < len(ob) else ab.nbytes].tobytes() for i in range(len(ob))]
    exp_b = HttpOracle(rules_b).eval(ab, ob)
    ac, oc = L.pack_http(realistic_requests(rng, 300))
    recs_c = [ac[int(oc[i]):int(oc[i + 1]) if i + 1 < len(oc) else ac.nbytes].tobytes() for i in range(len(oc))]
    exp_c = HttpOracle(REALISTIC).eval(ac, oc)

    rs_a, rs_b, rs_c = (L.RuleSet.compile_http(r) for r in (rules_a, rules_b, REALISTIC))
    b = L.Batcher(rs_a, max_delay_us=100, in_flight=3)

    def run(recs, exp):
        got = np.full(len(recs), -100, dtype=np.int64)

        def worker(t):
            for i in range(t, len(recs), 8):
                got[i] = b.eval(recs[i])

        th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert np.array_equal(got, exp)

    run(recs_a, exp_a)
    time.sleep(0.06)  # the resident workgroup exits after 20 ms idle
    run(recs_a, exp_a)
    for rs, recs, exp in ((rs_b, recs_b, exp_b), (rs_c, recs_c, exp_c), (rs_a, recs_a, exp_a), (rs_b, recs_b, exp_b)):
        b.set_ruleset(rs)
        run(recs, exp)
    # every request was counted once (an empty batch closed from a stale
    # pointer used to be counted as a batch with a fill phase of ~10^6 us,
    # i.e. batches > what the requests could form); no wall-clock bound here
    p = b.profile()
    assert p["requests"] == 3 * len(recs_a) + 2 * len(recs_b) + len(recs_c)
    assert 1 <= p["batches"] <= p["requests"] and p["fill_us"] >= 0.0
    b.close()


def test_batcher_small_batches_both_staging_paths(gpu):
    """program.h L7M_SPEC_TILE: a batcher launch of <= 64 records whose bytes
    fit one record stage is taken whole by the first wave, which requests the
    batch's bytes before its offsets and alone signals completion; larger
    batches (more records, or more bytes than a stage) take the per-wave
    path, and a record longer than the stage is read from memory by its lane.
    Batches of 1 / 40 / 64 / 65 concurrent callers over records of ~80 B,
    ~200 B (40 fit a stage, 64 do not) and ~9 KB: every verdict equals the
    oracle's."""
    import threading
    rng = np.random.default_rng(11)
    rules = [L.PortRuleHTTP(Path="/a/[a-z]+", Method="GET", Headers=["X-Pad"]),
             L.PortRuleHTTP(Path="/b/[0-9]+", Method="POST"),
             L.PortRuleHTTP(Path="/c/.*", Host="h[0-9]\\.example")]
    rs = L.RuleSet.compile_http(rules)
    for pad in (0, 120, 9000):
        reqs = []
        for i in range(65):
            hdr = [("x-pad", "p" * (pad + int(rng.integers(0, 8))))] if pad or rng.random() < 0.5 else []
            reqs.append(L.HTTPRequest(str(rng.choice(["GET", "POST"])),
                                      str(rng.choice(["/a/xyz", "/b/123", "/c/q", "/b/x", "/d"])),
                                      str(rng.choice(["h1.example", "hx.example"])), hdr))
        ar, of = L.pack_http(reqs)
        recs = [ar[int(of[i]):int(of[i + 1]) if i + 1 < len(of) else ar.nbytes].tobytes() for i in range(len(of))]
        exp = HttpOracle(rules).eval(ar, of)
        for k in (1, 40, 64, 65):
            b = L.Batcher(rs, max_batch=64, max_delay_us=200_000, in_flight=2)
            got = np.full(k, -100, dtype=np.int64)
            go = threading.Barrier(k)

            def worker(i):
                go.wait()
                got[i] = b.eval(recs[i])

            th = [threading.Thread(target=worker, args=(i,)) for i in range(k)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            b.close()
            assert np.array_equal(got, exp[:k]), (pad, k)
