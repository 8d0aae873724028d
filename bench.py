"""bench.py — L7 verdicts/s (+ HBM roofline fraction) on BASELINE.json's
headline workload: config 2, 1k HTTP path/method/host/header regex rules,
64M synthetic requests per GPU, inputs resident in HBM.

One step = one l7m_eval_device pass over the rank's whole batch (+ the RCCL
all-reduce of the per-rule hit/deny counters when N > 1).  The job's batch is
one deterministic workload cut into contiguous byte-balanced shards
(dist.balanced_shard); each rank generates its own shard.
--scaling weak (default; config 4: strong): the job holds N x the per-GPU
request count; strong: the job holds the config's request count, whatever N.

At N = 1 the line also carries:
  cpu_baseline  the oracle (reference algorithm restated) on all host cores
                and on one, bounded sample (config 5: the NFA engine);
  e2e           the host drop-in path: l7m_eval on a pinned host arena
                (chunked H2D on two streams overlapped with the kernel, D2H
                of verdicts): PCIe-inclusive verdicts/s;
  batcher       per-request blocking calls (l7m_batcher_eval, the canAccess /
                decodeHeaders call shape) from 8 / 64 / 512 caller threads:
                verdicts/s and latency percentiles (cilium_amd/batcher_bench).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2] [--requests R]
N > 1: python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from cilium_amd import dist as D  # noqa: E402
from cilium_amd import l7match as L  # noqa: E402
from cilium_amd import workloads as W  # noqa: E402

METRIC = "L7 verdicts/sec (HTTP reqs, 1k rules) + achieved HBM GB/s vs peak"  # BASELINE.json
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--requests", type=int, default=0, help="requests per GPU (default: config's)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--no-hits", action="store_true", help="skip the per-rule counters (diagnostic)")
    ap.add_argument("--diag", choices=["walk", "copy"], default=None,
                    help="profiling ablation of the HTTP kernel (verdicts invalid)")
    ap.add_argument("--lds-budget", type=int, default=0, help="bytes of rule tables kept in LDS (0 = default)")
    ap.add_argument("--mixed-streams", type=int, choices=[1, 2], default=1,
                    help="config 4: HIP streams for the two kernels (1 = back to back on one stream)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default=None,
                    help="weak: N x per-GPU requests (default); strong: the config's batch split over N "
                         "(default for config 4, 'request batch sharded across 2/4/8')")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="process-group backend (nccl = RCCL; gloo: the N>1 code path on one GPU in tests)")
    ap.add_argument("--dump", default=None, help="write this rank's shard bounds + verdicts to DUMP.rank<r>.npz")
    ap.add_argument("--no-e2e", action="store_true", help="skip the pinned-host end-to-end leg")
    ap.add_argument("--no-batcher", action="store_true", help="skip the per-request batcher leg")
    ap.add_argument("--batcher-seconds", type=float, default=3.0)
    ap.add_argument("--no-parity", action="store_true", help="skip the oracle sample of the timed batch")
    ap.add_argument("--dialect", choices=["envoy", "re2"], default="envoy",
                    help="HTTP regex dialect: envoy = std::regex full match (the reference as deployed, default); "
                         "re2 = Go regexp MatchString (BASELINE.json's wording; RE2 semantics, not run against Go)")
    ap.add_argument("--parity-sample", type=int, default=200_000, help="requests of the timed batch checked")
    ap.add_argument("--single-process", action="store_true",
                    help="N GPUs from ONE process through the library's device set (l7m_multi_eval_device: byte-"
                         "balanced shards, one stream per GPU, RCCL counter all-reduce) instead of one process per GPU")
    ap.add_argument("--devices", default=None,
                    help="--single-process device list, e.g. 0,1,2,3 (default: 0..N-1; 0,0 = two shards on one GPU)")
    ap.add_argument("--extended", action="store_true",
                    help="config 2 with workloads.EXTENDED_RULES (\\b, look-ahead, back-references) in front of its "
                         "1000 rules: the slow pass (http_slow_kernel) decides the requests they may match")
    return ap.parse_args()


def host_cores():
    """CPUs this process may run on, the machine's count, and the cgroup CPU
    quota (cores) when one is set."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(per)
    except (OSError, ValueError):
        pass
    usable = aff if quota is None else max(1, min(aff, int(quota + 0.999)))
    return {"affinity": aff, "nproc": os.cpu_count(), "cgroup_quota_cores": quota, "usable": usable}


def cpu_baseline(cfg, rules, seconds, threads, dialect=L.DIALECT_ENVOY_ECMA_FULL, n_rules=None):
    """Oracle (the reference algorithm restated: per-request linear rule scan,
    std::regex_match per matcher; K4 coverage for Kafka) timed on the host on a
    bounded sample, on `threads` threads (all the host cores this process may
    use) and on one.  Config 5 uses the oracle's NFA engine (oracle/nfa.h):
    std::regex backtracks for seconds per request on the /f{i}/ family's
    long tails and overflows its stack on long subjects, so
    the unfiltered sample is timed with the linear-time engine."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import HttpOracle, KafkaOracle  # test infrastructure: cpu_baseline leg only
    proto = W.CONFIGS[cfg]["proto"]
    engine = "nfa" if cfg == 5 else "std"
    # the reference's per-request loop as Envoy runs it: every rule's matchers,
    # no prefilter (parity_leg uses the prefiltered scan)
    orc = (HttpOracle(rules, dialect=dialect, engine=engine, prefilter=False) if proto == L.PROTO_HTTP
           else KafkaOracle(rules))
    n0 = 20_000 if cfg != 5 else 16 * threads

    def sample(start, n):
        return W.requests(cfg, start, n, n_rules=n_rules or len(rules), threads=min(threads, 64))

    # calibrate on a small sample, then size the timed sample to ~`seconds`
    a, o = sample(10_000_000, n0)
    t = time.perf_counter()
    orc.eval(a, o, threads=threads)
    rate = len(o) / max(1e-6, time.perf_counter() - t)
    n = int(min(20_000_000, max(n0, rate * seconds)))
    a, o = sample(20_000_000, n)
    t = time.perf_counter()
    orc.eval(a, o, threads=threads)
    dt = time.perf_counter() - t
    # one core, on a prefix of the same sample sized to ~seconds/4
    n1 = int(min(len(o), max(min(len(o), n0 // 4), rate / threads * seconds / 4)))
    a1, o1 = sample(20_000_000, n1)
    t = time.perf_counter()
    orc.eval(a1, o1, threads=1)
    dt1 = time.perf_counter() - t
    hc = host_cores()
    what = ("oracle/l7oracle.cc with the NFA engine (oracle/nfa.h; linear rule scan, Pike-VM full match)"
            if engine == "nfa" else ("oracle/l7oracle.cc (std::regex_search linear rule scan, RE2 dialect)"
                                     if dialect == L.DIALECT_RE2_SEARCH else
                                     "oracle/l7oracle.cc (std::regex_match linear rule scan)")
            if proto == L.PROTO_HTTP else "oracle/l7oracle.cc (ReadRequest + MatchesRule)")
    return {"value": len(o) / dt, "unit": "verdicts/s", "cores": threads, "kind": "port",
            "single_thread_value": len(o1) / dt1, "cpu_model": cpu_model(), "host": hc,
            "sample": f"{len(o)} requests of config {cfg} (requests [20M, 20M+{n})), {dt:.1f} s, {what} "
                      f"on {threads} threads = every core this process can use (affinity {hc['affinity']} CPUs, "
                      f"nproc {hc['nproc']}, cgroup CPU quota {hc['cgroup_quota_cores']} cores); "
                      f"single_thread_value: the first {len(o1)} of them on 1 thread, {dt1:.1f} s"}


def parity_leg(cfg, rules, verdicts, lo, n, threads, n_sample=200_000, blocks=256, seed=None, n_rules=None,
               dialect=L.DIALECT_ENVOY_ECMA_FULL):
    """The timed batch's own verdicts against the oracle (test infrastructure,
    outside the timed region): `blocks` contiguous runs of requests spread
    evenly over this rank's shard [lo, lo + n), n_sample requests in all (the
    whole shard when it is smaller), regenerated on the host (request i
    depends only on (config, seed, i)) and evaluated by oracle/l7oracle.cc;
    config 5 with its NFA engine (std::regex cannot run its long subjects)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from oracle import HttpOracle, KafkaOracle  # test infrastructure: the checker
    gcfg = cfg
    proto = W.CONFIGS[gcfg]["proto"]
    engine = "nfa" if cfg == 5 else "std"
    t0 = time.perf_counter()
    orc = HttpOracle(rules, dialect=dialect, engine=engine) if proto == L.PROTO_HTTP else KafkaOracle(rules)
    if n <= n_sample:
        runs = [(0, n)]
    else:
        b = -(-n_sample // blocks)
        runs = [((n - b) * j // (blocks - 1), b) for j in range(blocks)]
    sampled = mism = 0
    first = None
    for start, cnt in runs:
        a, o = W.requests(gcfg, lo + start, cnt, seed=seed, n_rules=n_rules if n_rules else len(rules),
                          threads=min(threads, 16))
        exp = orc.eval(a, o, threads=threads)
        got = verdicts[start:start + cnt]
        bad = np.nonzero(got != exp)[0]
        if len(bad) and first is None:
            first = {"request": int(lo + start + bad[0]), "gpu": int(got[bad[0]]), "oracle": int(exp[bad[0]])}
        sampled += cnt
        mism += len(bad)
    return {"sampled": sampled, "mismatches": mism, "runs": len(runs), "first_mismatch": first,
            "oracle": f"oracle/l7oracle.cc ({'NFA engine' if engine == 'nfa' else 'std::regex' if proto == L.PROTO_HTTP else 'ReadRequest + MatchesRule'})",
            "sample": f"{len(runs)} evenly spaced runs of {runs[0][1]} requests over this rank's shard of the timed "
                      f"batch (last timed step's verdicts)", "seconds": time.perf_counter() - t0}


def e2e_leg(rs, arena_pinned, offs, n, passes=2):
    """PCIe-inclusive rate of the host drop-in path: l7m_eval on a pinned host
    arena (the library cuts it into ~64 MiB chunks and overlaps chunk k+1's
    H2D copy with chunk k's kernel on two streams, then copies the verdicts
    back).  Inputs start on the host, verdicts end on the host."""
    verd = np.empty(n, dtype=np.int32)
    rs.eval(arena_pinned, offs, None)  # warm: device buffers of this size
    t = time.perf_counter()
    for _ in range(passes):
        rs.eval(arena_pinned, offs, None)
    dt = (time.perf_counter() - t) / passes
    del verd
    zc = bool(L._lib.l7m_host_mapped(arena_pinned.ctypes.data, ((arena_pinned.nbytes + 64) & ~3)))
    return {"verdicts_per_s": n / dt, "ms_per_batch": dt * 1e3, "host_GBps": arena_pinned.nbytes / dt / 1e9,
            "requests": n, "passes": passes, "zero_copy": zc,
            "path": ("l7m_eval(pinned host arena): zero-copy, the kernel reads the device-mapped arena in place "
                     "over PCIe; offsets H2D, verdicts D2H") if zc else
                    ("l7m_eval(pinned host arena): 64 MiB chunks, H2D on 2 streams overlapped with the kernel, "
                     "D2H verdicts")}


def batcher_leg(cfg, seconds):
    """Per-request blocking calls through l7m_batcher (cilium_amd/batcher_bench,
    a plain C client): verdicts/s, latency percentiles and the per-batch
    phases (fill / launch / gpu / wake) at 8 caller threads and at one per
    usable core (more callers than cores measure the cgroup's CPU quota, not
    the batcher: each line reports the cgroup's throttling during its run),
    eager batching and deadline batching (max_delay 200 us)."""
    import subprocess
    exe = os.path.join(ROOT, "cilium_amd", "batcher_bench")
    usable = host_cores()["usable"]
    counts = sorted({8, max(8, usable)})
    out = []
    for eager in (1, 0):
        p = subprocess.run([exe, str(cfg), "1000000", str(seconds), str(eager)] + [str(c) for c in counts],
                           capture_output=True, text=True, timeout=120)
        if p.returncode != 0:
            return {"error": p.stderr[-500:]}
        out += [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    return out


def cpu_model():
    """The host CPU's model name (what `lscpu` prints), from /proc/cpuinfo."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def measured_traffic(cfg):
    """HBM bytes per launch from the committed rocprofv3 FETCH_SIZE/WRITE_SIZE
    passes (tools/traffic.py) of THIS kernel build (matched by the .so hash,
    or by the hashes of its device code, cilium_amd/codehash.py) on the
    default workload; None when no such measurement exists."""
    import glob
    import hashlib
    from cilium_amd.codehash import code_md5, kernel_md5
    with open(L.LIB_PATH, "rb") as f:
        md5 = hashlib.md5(f.read()).hexdigest()
    kmd5 = kernel_md5(L.LIB_PATH)
    cmd5 = code_md5(L.LIB_PATH)
    for path in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", f"traffic_cfg{cfg}.json")), reverse=True):
        with open(path) as f:
            t = json.load(f)
        if t.get("so_md5") == md5 or t.get("kernel_md5") == kmd5 or t.get("code_md5") == cmd5:
            return float(t["traffic_bytes"])
    return None


def emit(res):
    """Print the bench line, naming the device code it measured
    (cilium_amd/codehash.py code_md5: the md5 of the library's gfx950 code,
    stable across rebuilds of the same source -- the key that ties rocprof
    summaries and traffic files under profiles/ to a build)."""
    from cilium_amd.codehash import code_md5
    res["code_md5"] = code_md5(L.LIB_PATH)
    print(json.dumps(res), flush=True)


def log(msg):
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    ndev = torch.cuda.device_count()
    gpu = local % max(1, ndev)  # ranks beyond the visible GPUs share them (gloo tests)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group("gloo")
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    cfg = args.config
    scaling = args.scaling or ("strong" if cfg == 4 else "weak")
    if args.single_process:
        return run_single_process(args, scaling)
    if cfg == 4:
        return run_mixed(args, world, rank, dev, scaling)
    c = W.CONFIGS[cfg]
    threads = args.threads or max(1, min(16, len(os.sched_getaffinity(0)) // max(1, world)))
    n_job = (args.requests or c["n_requests"]) * (world if scaling == "weak" else 1)

    rules = W.rules(cfg)
    if args.extended:
        if cfg != 2:
            raise SystemExit("--extended applies to config 2")
        rules = list(W.EXTENDED_RULES) + rules  # requests still come from config 2's 1000-rule generator
    dialect = L.DIALECT_RE2_SEARCH if args.dialect == "re2" else L.DIALECT_ENVOY_ECMA_FULL
    if dialect != L.DIALECT_ENVOY_ECMA_FULL and c["proto"] != L.PROTO_HTTP:
        raise SystemExit("--dialect applies to HTTP configurations")
    rs = (L.RuleSet.compile_http(rules, dialect=dialect, lds_budget_bytes=args.lds_budget)
          if c["proto"] == L.PROTO_HTTP else L.RuleSet.compile_kafka(rules))

    # ---- rank's byte-balanced shard, generated deterministically, in HBM ----
    lo, hi = D.balanced_shard(cfg, n_job, world, rank, threads=threads,
                              device=dev if args.backend == "nccl" else None)
    per_gpu = hi - lo
    log(f"rank {rank}: compiled {len(rules)} rules; generating requests [{lo}, {hi}) of {n_job}")
    t0 = time.perf_counter()
    arena, offs = W.requests(cfg, lo, per_gpu, threads=threads)
    gen_s = time.perf_counter() - t0
    rec_bytes = arena.nbytes - 64  # W.requests: packed (4-byte padded) records + 64 B tail pad
    pinned = torch.from_numpy(arena).pin_memory()
    d_arena = torch.empty(arena.nbytes, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    d_arena.copy_(pinned, non_blocking=True)
    torch.cuda.synchronize()
    h2d_s = time.perf_counter() - t0
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    arena_nbytes = arena.nbytes
    keep_host = world == 1 and not args.no_e2e and not args.diag
    host_offs = offs if keep_host else None
    if not keep_host:
        del pinned
    del arena, offs
    d_verd = torch.empty(per_gpu, dtype=torch.int32, device=dev)
    d_hits = torch.zeros(rs.n_counters, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream()

    hits_arg = None if args.no_hits or args.diag else d_hits
    flags = {None: 0, "walk": L.FLAG_DIAG_WALK_ONLY, "copy": L.FLAG_DIAG_COPY_ONLY}[args.diag]

    def step():
        d_hits.zero_()
        rs.eval_device(d_arena, arena_nbytes, d_offs, per_gpu, d_verd, hits_arg, stream.cuda_stream, flags)
        D.allreduce_counters(d_hits)  # RCCL (backend "nccl") when world > 1

    log(f"rank {rank}: arena {arena_nbytes / 1e9:.2f} GB resident (gen {gen_s:.1f} s, h2d {h2d_s:.2f} s); warmup")
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kernel_ms = []
    for i in range(args.steps):
        d_hits.zero_()
        ev[i][0].record(stream)
        rs.eval_device(d_arena, arena_nbytes, d_offs, per_gpu, d_verd, hits_arg, stream.cuda_stream, flags)
        ev[i][1].record(stream)
        D.allreduce_counters(d_hits)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = [a.elapsed_time(b) for a, b in ev]
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev if args.backend == "nccl" else "cpu")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    if args.dump:
        np.savez(f"{args.dump}.rank{rank}.npz", lo=lo, hi=hi, verdicts=d_verd.cpu().numpy(),
                 hits=d_hits.cpu().numpy(), elapsed=elapsed)

    total_requests = n_job * args.steps
    value = total_requests / elapsed
    kavg = float(np.mean(kernel_ms)) / 1e3
    # algorithmic bytes per launch: records + u64 offset + i32 verdict per request (+ counters)
    alg_bytes = rec_bytes + 12 * per_gpu + 8 * rs.n_counters
    achieved = alg_bytes / kavg / 1e9
    # sanity: verdicts were produced for every request of every step
    hits_total = int(d_hits.sum().item())
    expect_hits = n_job

    if rank == 0:
        res = {
            "metric": (METRIC if cfg == 2 and dialect == L.DIALECT_ENVOY_ECMA_FULL and not args.extended else
                       f"L7 verdicts/sec ({c['name']}{', RE2 MatchString dialect' if dialect else ''}) + achieved "
                       f"HBM GB/s vs peak"),
            "value": value,
            "unit": "verdicts/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (deterministic generator libl7gen.so, SURVEY.md §8(d))",
            "config": {"workload": c["name"] + ("-re2" if dialect else "") + ("+extended10" if args.extended else ""),
                       "baseline_config": cfg,
                       "dialect": ("re2-search (Go regexp MatchString semantics; RE2 semantics, not run against Go)"
                                   if dialect else "envoy-ecma-full (std::regex_match, the reference as deployed)"),
                       "n_rules": len(rules),
                       "requests_per_gpu": per_gpu, "requests_total": n_job, "seed": hex(c["seed"]),
                       "mean_record_bytes": rec_bytes / per_gpu,
                       "parallelism": f"dp{world} (byte-balanced request shards, "
                                      f"{'RCCL' if args.backend == 'nccl' else 'gloo'} all-reduce of "
                                      f"{rs.n_counters} counters)",
                       "dfa_groups": int(rs.info.n_dfas), "dfa_states": int(rs.info.total_dfa_states)},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBPS,
                         "traffic": (measured_traffic(cfg) if not args.requests and not dialect and not args.extended
                                     else None),
                         "kernel_ms": kavg * 1e3, "algorithmic_bytes_per_launch": alg_bytes},
            "counters_ok": hits_total == expect_hits,
            "host": {"gen_s": gen_s, "h2d_GBps": arena_nbytes / h2d_s / 1e9},
        }
        tr = res["roofline"]["traffic"]
        # PMC HBM bytes per launch over the algorithmic bytes: > 1 = re-reads,
        # < 1 = bytes counted as algorithmic that the kernel never fetched
        res["roofline"]["traffic_over_algorithmic"] = tr / alg_bytes if tr else None
        log(f"timed {args.steps} steps: {elapsed:.3f} s; kernel {kavg * 1e3:.2f} ms")
        if not args.no_parity and not args.diag:
            log("parity sample (oracle, outside the timed region)")
            res["parity"] = parity_leg(cfg, rules, d_verd.cpu().numpy(), lo, per_gpu,
                                       args.threads or host_cores()["usable"], n_sample=args.parity_sample,
                                       dialect=dialect, n_rules=c["n_rules"])
            log(f"parity: {res['parity']['mismatches']} mismatches in {res['parity']['sampled']}")
        if keep_host:
            log("end-to-end (pinned host arena)")
            res["e2e"] = e2e_leg(rs, pinned.numpy(), host_offs, per_gpu)
            del pinned
        if (world == 1 and not args.no_batcher and not args.diag and cfg in (2, 3) and not args.requests and
                not dialect and not args.extended):
            log("batcher (per-request calls)")
            res["batcher"] = batcher_leg(cfg, args.batcher_seconds)
        if world == 1 and not args.no_cpu_baseline:
            log("cpu baseline")
            res["cpu_baseline"] = cpu_baseline(cfg, rules, args.cpu_baseline_seconds,
                                               args.threads or host_cores()["usable"], dialect=dialect,
                                               n_rules=c["n_rules"])
        emit(res)
    if world > 1:
        dist.destroy_process_group()


def run_single_process(args, scaling):
    """--single-process: the job on N GPUs from this one process through the
    library's device set (include/l7match.h l7m_multi_*): the batch is
    generated once, cut by l7m_shard_bounds into byte-balanced shards, each
    shard made resident on its GPU; a step is one l7m_multi_eval_device (all
    shards' kernels concurrently, one stream per GPU, then one RCCL
    all-reduce of the counters when the GPUs are distinct)."""
    cfg = args.config
    if cfg == 4:
        raise SystemExit("--single-process: configs 1, 2, 3, 5")
    c = W.CONFIGS[cfg]
    devs = [int(x) for x in args.devices.split(",")] if args.devices else list(range(args.gpus))
    N = len(devs)
    threads = args.threads or max(1, min(16, len(os.sched_getaffinity(0))))
    n_job = (args.requests or c["n_requests"]) * (N if scaling == "weak" else 1)
    rules = W.rules(cfg)
    rs = L.RuleSet.compile_http(rules) if c["proto"] == L.PROTO_HTTP else L.RuleSet.compile_kafka(rules)
    ds = L.DeviceSet(devs)
    log(f"single process, devices {devs} (RCCL counters: {ds.uses_rccl}); generating {n_job} requests")
    arena, offs = W.requests(cfg, 0, n_job, threads=threads)
    size = arena.nbytes - 64
    b = L.shard_bounds(offs, size, N)
    shards, verd = [], []
    for k, d in enumerate(devs):
        lo, hi = int(b[k]), int(b[k + 1])
        a0 = int(offs[lo]) if lo < n_job else size
        a1 = int(offs[hi]) if hi < n_job else size
        dv = torch.device("cuda", d)
        da = torch.zeros(((a1 - a0 + 64 + 15) // 16) * 16, dtype=torch.uint8, device=dv)
        da[:a1 - a0].copy_(torch.from_numpy(arena[a0:a1]))
        do = torch.from_numpy((offs[lo:hi] - np.uint64(a0)).view(np.int64)).to(dv)
        vv = torch.empty(hi - lo, dtype=torch.int32, device=dv)
        verd.append(vv)
        shards.append((da, a1 - a0, do, hi - lo, vv))
    rec_bytes = size
    del arena
    hits = np.zeros(rs.n_counters, dtype=np.uint64)
    for _ in range(args.warmup):
        ds.eval_device(rs, shards, hits)
    hits[:] = 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ds.eval_device(rs, shards, hits)
    elapsed = time.perf_counter() - t0
    got = np.concatenate([v.cpu().numpy() for v in verd])
    value = n_job * args.steps / elapsed
    alg = rec_bytes + 12 * n_job + 8 * rs.n_counters
    res = {
        "metric": (METRIC if cfg == 2 else f"L7 verdicts/sec ({c['name']}) + achieved HBM GB/s vs peak"),
        "value": value, "unit": "verdicts/s", "n_gpus": N, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": scaling,
        "vs_baseline": None, "dtype": "u8", "data": "synthetic (deterministic generator libl7gen.so, SURVEY.md §8(d))",
        "config": {"workload": c["name"], "baseline_config": cfg, "n_rules": len(rules), "requests_total": n_job,
                   "devices": devs, "shard_bounds": [int(x) for x in b],
                   "parallelism": f"single process, {N} shards (l7m_multi_eval_device, "
                                  f"{'RCCL all-reduce' if ds.uses_rccl else 'host sum'} of {rs.n_counters} counters)"},
        "roofline": {"bound": "hbm", "achieved": alg / (elapsed / args.steps) / 1e9, "peak": HBM_PEAK_GBPS * len(set(devs)),
                     "unit": "GB/s", "frac": alg / (elapsed / args.steps) / 1e9 / (HBM_PEAK_GBPS * len(set(devs))),
                     "traffic": None,
                     "note": "whole-step wall time (kernels + counter reduce); peak = distinct GPUs x 8 TB/s"},
        "counters_ok": int(hits.sum()) == n_job * args.steps,
    }
    if not args.no_parity:
        res["parity"] = parity_leg(cfg, rules, got, 0, n_job, threads, n_sample=args.parity_sample)
    emit(res)
    ds.close()


def run_mixed(args, world, rank, dev, scaling):
    """Config 4: 5k HTTP + 5k Kafka rules, 128M requests split by protocol tag
    (W.mixed_parts).  Strong scaling by default ("request batch sharded across
    2/4/8"): the job is the config's 128M requests and rank r evaluates its
    byte-balanced shard of each protocol's stream (--scaling weak: 128M per
    GPU).  Per
    step the two kernels run back to back on one HIP stream (default; each is
    a persistent kernel sized to the whole GPU whose waves own fixed shares of
    the batch, so running them concurrently on two streams only delays the
    workgroups that start late: --mixed-streams 2), then one RCCL all-reduce
    sums the concatenated (R_http+2) + (R_kafka+2) counters."""
    c = W.CONFIGS[4]
    threads = args.threads or max(1, min(16, len(os.sched_getaffinity(0)) // max(1, world)))
    per_gpu = args.requests or c["n_requests"]
    n_job_part = (per_gpu // 2) * (world if scaling == "weak" else 1)
    parts = []
    for proto, gcfg, seed, n_rules in W.mixed_parts(4):
        lo, hi = D.balanced_shard(gcfg, n_job_part, world, rank, threads=threads, seed=seed, n_rules=n_rules,
                                  device=dev if args.backend == "nccl" else None)
        rules = W.rules(gcfg, seed=seed, n_rules=n_rules)
        rs = (L.RuleSet.compile_http(rules, lds_budget_bytes=args.lds_budget) if proto == L.PROTO_HTTP
              else L.RuleSet.compile_kafka(rules))
        arena, offs = W.requests(gcfg, lo, hi - lo, seed=seed, n_rules=n_rules, threads=threads)
        d_arena = torch.from_numpy(arena).to(dev)
        d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
        parts.append(dict(proto=proto, gcfg=gcfg, rules=rules, rs=rs, n=hi - lo, lo=lo, seed=seed,
                          arena_nbytes=arena.nbytes, rec_bytes=arena.nbytes - 64, d_arena=d_arena,
                          d_offs=d_offs, d_verd=torch.empty(hi - lo, dtype=torch.int32, device=dev),
                          stream=(torch.cuda.Stream(device=dev) if args.mixed_streams == 2
                                  else torch.cuda.current_stream())))
        del arena, offs
        log(f"rank {rank}: part config {gcfg}: {len(rules)} rules, {hi - lo} requests")
    n_cnt = [p["rs"].n_counters for p in parts]
    d_hits = torch.zeros(sum(n_cnt), dtype=torch.int64, device=dev)
    hit_views = [d_hits[:n_cnt[0]], d_hits[n_cnt[0]:]]
    main_s = torch.cuda.current_stream()

    def step(ev=None):
        d_hits.zero_()
        start = torch.cuda.Event(enable_timing=True)
        start.record(main_s)
        ends = []
        for p, hv in zip(parts, hit_views):
            p["stream"].wait_event(start)
            p["rs"].eval_device(p["d_arena"], p["arena_nbytes"], p["d_offs"], p["n"], p["d_verd"],
                                None if args.no_hits else hv,
                                p["stream"].cuda_stream, 0)
            e = torch.cuda.Event(enable_timing=True)
            e.record(p["stream"])
            main_s.wait_event(e)
            ends.append(e)
        D.allreduce_counters(d_hits)
        if ev is not None:
            ev.append((start, ends))

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    evs = []
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(evs)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = [max(s.elapsed_time(e) for e in ends) for s, ends in evs]
    cdev = dev if args.backend == "nccl" else "cpu"
    t = torch.tensor([elapsed], dtype=torch.float64, device=cdev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())
    n_rank = sum(p["n"] for p in parts)
    n_job = torch.tensor([n_rank], dtype=torch.int64, device=cdev)
    if world > 1:
        dist.all_reduce(n_job)
    n_job = int(n_job.item())
    kavg = float(np.mean(kernel_ms)) / 1e3
    alg_bytes = sum(p["rec_bytes"] + 12 * p["n"] for p in parts) + 8 * sum(n_cnt)
    achieved = alg_bytes / kavg / 1e9
    counters_ok = None if args.no_hits else int(d_hits.sum().item()) == n_job
    if rank != 0:
        dist.destroy_process_group()
        return
    res = {
        "metric": f"L7 verdicts/sec ({c['name']}) + achieved HBM GB/s vs peak",
        "value": n_job * args.steps / elapsed,
        "unit": "verdicts/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": scaling,
        "vs_baseline": None, "dtype": "u8",
        "data": "synthetic (deterministic generator libl7gen.so, SURVEY.md §8(d))",
        "config": {"workload": c["name"], "baseline_config": 4, "n_rules": sum(len(p["rules"]) for p in parts),
                   "requests_per_gpu": n_rank, "requests_total": n_job, "seed": hex(c["seed"]),
                   "parts": [{"generator_config": p["gcfg"], "n_rules": len(p["rules"]), "requests_rank0": p["n"],
                              "mean_record_bytes": p["rec_bytes"] / max(1, p["n"])} for p in parts],
                   "parallelism": f"dp{world} (request-sharded per protocol, {args.mixed_streams} HIP stream(s), "
                                  f"RCCL all-reduce of {sum(n_cnt)} counters)"},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS, "traffic": None,
                     "kernel_ms": kavg * 1e3, "algorithmic_bytes_per_launch": alg_bytes,
                     "note": "both kernels, first start to last end, rank 0"},
        "counters_ok": counters_ok,
    }
    if not args.no_parity:
        log("parity sample (oracle, outside the timed region)")
        thr = args.threads or host_cores()["usable"]
        res["parity"] = [dict(parity_leg(p["gcfg"], p["rules"], p["d_verd"].cpu().numpy(), p["lo"], p["n"], thr,
                                         n_sample=args.parity_sample // 2, seed=p["seed"], n_rules=len(p["rules"])),
                              part_config=p["gcfg"]) for p in parts]
    if world == 1 and not args.no_cpu_baseline:
        threads = args.threads or host_cores()["usable"]
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from oracle import HttpOracle, KafkaOracle  # test infrastructure: cpu_baseline leg only
        n_tot, t_tot, samples = 0, 0.0, []
        for p in parts:
            orc = (HttpOracle(p["rules"], prefilter=False) if p["proto"] == L.PROTO_HTTP
                   else KafkaOracle(p["rules"]))
            a, o = W.requests(p["gcfg"], 10_000_000, 5_000, seed=p["seed"], n_rules=len(p["rules"]),
                              threads=threads)
            t1 = time.perf_counter()
            orc.eval(a, o, threads=threads)
            rate = 5_000 / max(1e-6, time.perf_counter() - t1)
            n = int(min(20_000_000, max(5_000, rate * args.cpu_baseline_seconds / 2)))
            a, o = W.requests(p["gcfg"], 20_000_000, n, seed=p["seed"], n_rules=len(p["rules"]), threads=threads)
            t1 = time.perf_counter()
            orc.eval(a, o, threads=threads)
            dt = time.perf_counter() - t1
            n_tot, t_tot = n_tot + n, t_tot + dt
            samples.append(f"{n} requests of part config {p['gcfg']} in {dt:.1f} s")
        # one core, on the first tenth of the last part's sample
        n1 = max(1, len(o) // 10)
        a1, o1 = W.requests(p["gcfg"], 20_000_000, n1, seed=p["seed"], n_rules=len(p["rules"]), threads=threads)
        t1 = time.perf_counter()
        orc.eval(a1, o1, threads=1)
        st_rate = n1 / (time.perf_counter() - t1)
        res["cpu_baseline"] = {"value": n_tot / t_tot, "unit": "verdicts/s", "cores": threads, "kind": "port",
                               "single_thread_value": st_rate, "cpu_model": cpu_model(),
                               "sample": "; ".join(samples) + f" (oracle/l7oracle.cc on {threads} threads); "
                                         f"single_thread_value: {n1} requests of part config {p['gcfg']} on 1 "
                                         f"thread"}
    emit(res)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
