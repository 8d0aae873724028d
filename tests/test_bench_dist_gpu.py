"""bench.py's own multi-GPU code path, executed: two ranks launched by
torch.distributed.run (the driver's launch line) on the one GPU of the box,
process group switched to gloo (--backend gloo; RCCL needs one GPU per rank).
Each rank takes its byte-balanced shard (dist.balanced_shard), runs the timed
steps with the counter all-reduce and the max-over-ranks time, and dumps its
shard bounds and verdicts; the concatenated verdicts must equal a one-rank run
of the same job, the reduced counters must sum to the job, and an oracle
sample pins the verdicts.  Weak scaling (config 2), strong scaling (config 3)
and the mixed config 4 (strong by default).  Multi-GPU scaling itself is
unmeasured on hardware until the driver's 8-GPU run."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from cilium_amd import l7match as L
from cilium_amd import workloads as W

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _bench(tmp, nproc, args, tag):
    dump = os.path.join(tmp, tag)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", os.path.join(ROOT, "bench.py"),
           "--gpus", str(nproc), "--backend", "gloo", "--no-cpu-baseline", "--no-e2e", "--no-batcher",
           "--steps", "3", "--warmup", "1", "--dump", dump] + args
    env = dict(os.environ, OMP_NUM_THREADS="4")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [x for x in p.stdout.splitlines() if x.startswith("{")]
    assert len(line) == 1, p.stdout[-2000:]
    res = json.loads(line[0])
    shards = [np.load(f"{dump}.rank{r}.npz") for r in range(nproc) if os.path.exists(f"{dump}.rank{r}.npz")]
    return res, shards


@pytest.mark.parametrize("cfg,scaling,per", [(2, "weak", 150_000), (3, "strong", 240_000)])
def test_bench_two_ranks_gloo_equals_one_rank(gpu, tmp_path, cfg, scaling, per):
    res2, sh2 = _bench(str(tmp_path), 2, ["--config", str(cfg), "--requests", str(per), "--scaling", scaling], "two")
    n_job = per * (2 if scaling == "weak" else 1)
    assert res2["n_gpus"] == 2 and res2["scaling"] == scaling and res2["config"]["requests_total"] == n_job
    assert res2["counters_ok"] is True and res2["value"] > 0
    assert sh2[0]["lo"] == 0 and sh2[0]["hi"] == sh2[1]["lo"] and sh2[1]["hi"] == n_job
    v2 = np.concatenate([s["verdicts"] for s in sh2])
    # the same job on one rank
    res1, sh1 = _bench(str(tmp_path), 1, ["--config", str(cfg), "--requests", str(n_job), "--scaling", "weak"], "one")
    assert np.array_equal(sh1[0]["verdicts"], v2)
    assert np.array_equal(sh2[0]["hits"], sh1[0]["hits"])  # all-reduced counters == one rank's
    # oracle on a strided sample of the job
    from oracle import HttpOracle, KafkaOracle
    rules = W.rules(cfg)
    idx = np.arange(0, n_job, 1499)
    recs = []
    for i in idx.tolist():
        a, o = W.requests(cfg, i, 1)
        recs.append(a[: a.nbytes - 64].tobytes())
    a2, o2 = L.pack_records(recs)
    orc = HttpOracle(rules) if cfg == 2 else KafkaOracle(rules)
    assert np.array_equal(orc.eval(a2, o2, threads=16), v2[idx])


def test_bench_mixed_config4_two_ranks_strong(gpu, tmp_path):
    res, _ = _bench(str(tmp_path), 2, ["--config", "4", "--requests", "400000"], "mixed")
    assert res["scaling"] == "strong" and res["n_gpus"] == 2
    assert res["config"]["requests_total"] == 400_000 and res["counters_ok"] is True
