"""Zero-copy probe (diagnostic, GPU box): the HTTP kernel reading a pinned HOST
arena directly over PCIe (no H2D copy), against the chunked-copy host path
(l7m_eval) and the HBM-resident kernel, on the same config-2 batch.

    python tools/zero_copy_probe.py [n_requests]

The arena comes from l7m_alloc_pinned (hipHostMalloc); its device address is
taken from hipHostGetDevicePointer, and the probe stops before any launch if
the runtime does not report one.  Verdicts of the three paths must agree."""
import ctypes
import json
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from cilium_amd import l7match as L  # noqa: E402
from cilium_amd import workloads as W  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16_000_000
    rs = L.RuleSet.compile_http(W.rules(2))
    size = W._gen.l7g_requests(2, W.CONFIGS[2]["seed"], 1000, 0, n, None, 0, None, 16)
    nbytes = size + 64
    hp = ctypes.c_void_p()
    assert L._lib.l7m_alloc_pinned(nbytes, ctypes.byref(hp)) == L.L7M_OK
    arena = np.ctypeslib.as_array((ctypes.c_uint8 * nbytes).from_address(hp.value))
    _, offs = W.requests(2, 0, n, out_arena=arena, threads=16)
    arena[size:] = 0
    hip = ctypes.CDLL("libamdhip64.so")
    dptr = ctypes.c_void_p()
    rc = hip.hipHostGetDevicePointer(ctypes.byref(dptr), hp, 0)
    if rc != 0 or not dptr.value:
        print(json.dumps({"error": f"hipHostGetDevicePointer rc={rc}: host arena not mapped; no launch"}))
        return 2
    dev = torch.device("cuda:0")
    d_offs = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_arena = torch.from_numpy(arena).to(dev)
    v_hbm = torch.empty(n, dtype=torch.int32, device=dev)
    v_zc = torch.empty(n, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    res = {"requests": n, "arena_bytes": size, "host_ptr_is_device_ptr": dptr.value == hp.value}

    def timed(fn, reps=5):
        fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    ms = timed(lambda: rs.eval_device(d_arena, size, d_offs, n, v_hbm, stream=s))
    res["hbm_resident"] = {"ms": ms, "GBps": size / ms / 1e6}
    ms = timed(lambda: rs.eval_device(dptr.value, size, d_offs, n, v_zc, stream=s))
    res["zero_copy_kernel"] = {"ms": ms, "GBps": size / ms / 1e6,
                               "note": "kernel reads the pinned host arena over PCIe; offsets resident"}
    res["zero_copy_matches_hbm"] = bool(torch.equal(v_hbm, v_zc))
    host_v = np.empty(n, dtype=np.int32)
    rs.eval(arena[:nbytes], offs, None)
    t = time.perf_counter()
    for _ in range(2):
        host_v = rs.eval(arena[:nbytes], offs, None)
    dt = (time.perf_counter() - t) / 2
    res["chunked_copy_l7m_eval"] = {"ms": dt * 1e3, "GBps": size / dt / 1e9}
    res["chunked_matches_hbm"] = bool(np.array_equal(host_v, v_hbm.cpu().numpy()))
    print(json.dumps(res))
    del d_arena
    L._lib.l7m_free_pinned(hp)
    return 0 if res["zero_copy_matches_hbm"] and res["chunked_matches_hbm"] else 1


if __name__ == "__main__":
    sys.exit(main())
