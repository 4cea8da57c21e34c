"""A/B of the software-pipelined bf16 A1 forward (diagnostic build): variant 0 (production,
attn_fwd_wave_pipe) against 16 (the earlier attn_fwd_wave_il, reads just in time), at the bench
shape (B=1, h=8, n=8448) and three more.  Graph-replayed us per call, variants alternated three
times, and a bitwise comparison of every output.  (The same pipelining of the A3 forward's chunk
body, then variant 37, measured level and was dropped: profiles/r05z_ab_fwd_pipe.txt.)

    TRANSMIL_HIP_LIB=<diag .so> python scripts/dev/fwd_pipe_ab.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.getcwd())
from transmil_deepgraft_amd import _lib                    # noqa: E402
from transmil_deepgraft_amd.engine import _p, _stream      # noqa: E402

L = _lib.lib()
dev = "cuda"


def timeit(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(reps):
            fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    gr.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


def ab(name, f, outs, variants):
    res = {}
    for var in variants:
        L.tm_debug_set_nys_variant(var)
        for o in outs:
            o.fill_(float("nan") if o.is_floating_point() else 0)
        f()
        torch.cuda.synchronize()
        res[var] = [o.clone() for o in outs]
    times = {v: [] for v in variants}
    for _ in range(3):
        for var in variants:
            L.tm_debug_set_nys_variant(var)
            times[var].append(timeit(f))
    L.tm_debug_set_nys_variant(0)
    same = all(torch.equal(a.view(torch.uint8), b.view(torch.uint8)) for a, b in zip(res[variants[0]], res[variants[1]]))
    print(f"{name}: " + "; ".join(f"variant {v} {min(t):.2f} us ({', '.join(f'{x:.2f}' for x in t)})" for v, t in times.items())
          + f"; bitwise equal {same}", flush=True)
    assert same


for B, nh, n in ((1, 8, 8448), (2, 8, 256), (1, 8, 4352), (3, 8, 1024)):
    nbh = B * nh
    g = torch.Generator(device="cpu").manual_seed(n + B)
    q = (torch.randn(nbh, n, 64, generator=g) * 0.6).to(torch.bfloat16).to(dev)
    v = (torch.randn(nbh, n, 64, generator=g) * 0.3).to(torch.bfloat16).to(dev)
    kl = (torch.randn(nbh, 256, 64, generator=g) * 0.6).to(torch.bfloat16).to(dev)
    y = (torch.randn(nbh, 256, 64, generator=g) * 0.3).to(torch.bfloat16).to(dev)
    wconv = torch.randn(nh, 33, device=dev) * 0.1
    merged = torch.empty(B, n, nh * 64, dtype=torch.bfloat16, device=dev)
    lse = torch.empty(nbh, n, device=dev)
    ab(f"A1 fwd B={B} n={n}", lambda: _lib.call("tm_nys_a1_fwd", 1, _p(q), _p(v), _p(kl), _p(y), _p(wconv), nbh, nh, n,
                                                _p(merged), _p(lse), _stream()), [merged, lse], (16, 0))
print("FWD_PIPE_OK")
