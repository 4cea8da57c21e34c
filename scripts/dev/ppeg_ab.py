"""A/B of the PPEG stencil's cells per thread (diagnostic build: variant 0 = 2 cells / 8 x 8 tiles,
variant 1 = 4 cells / 8 x 16 tiles, variant 2 = persistent 8 x 8 with the next window prefetched) at the bench shape (G = 91, D = 512): graph-replayed µs per
call for the forward and the backward (data gradient + weight gradient), outputs bitwise.

    TRANSMIL_HIP_LIB=<diag .so> python scripts/dev/ppeg_ab.py
"""
import ctypes as C
import os
import sys
import time

import torch

sys.path.insert(0, os.getcwd())
from transmil_deepgraft_amd import _lib                  # noqa: E402
from transmil_deepgraft_amd.engine import _p, _stream    # noqa: E402

L = _lib.lib()


def timeit(fn, reps=50):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


B, G, D = 1, 91, 512
S = 1 + G * G
dev = "cuda"
torch.manual_seed(0)
x = torch.randn(B, S, D, device=dev)
dy = torch.randn(B, S, D, device=dev)
w7, w5, w3 = (torch.randn(D, k * k, device=dev) * 0.1 for k in (7, 5, 3))
b7, b5, b3 = (torch.randn(D, device=dev) for _ in range(3))
wf = torch.empty(49 * D, device=dev)
bf = torch.empty(D, device=dev)
_lib.call("tm_ppeg_fold", _p(w7), _p(b7), _p(w5), _p(b5), _p(w3), _p(b3), D, _p(wf), _p(bf), _stream())
work = torch.empty(_lib.query("tm_ppeg_bwd_workspace", B, G, D) // 4, device=dev)
res = {}
for v in (0, 1, 2, 0, 1, 2):
    L.tm_debug_set_ppeg_variant(v)
    y = torch.empty_like(x)
    dx = torch.empty_like(x)
    g7, g5, g3 = (torch.empty(D, k * k, device=dev) for k in (7, 5, 3))
    gb7, gb5, gb3 = (torch.empty(D, device=dev) for _ in range(3))
    f = lambda: _lib.call("tm_ppeg_fwd", _p(x), B, G, D, _p(wf), _p(bf), _p(y), _stream())   # noqa: E731
    bwd = lambda: _lib.call("tm_ppeg_bwd", _p(x), _p(dy), B, G, D, _p(wf), _p(dx), _p(work), _p(g7),   # noqa: E731
                            _p(gb7), _p(g5), _p(gb5), _p(g3), _p(gb3), 0, None, 0, 0, C.c_float(0.0), C.c_uint64(0),
                            None, None, _stream())
    tf, tb = timeit(f), timeit(bwd)
    torch.cuda.synchronize()
    if v in res:
        res[v][0].append((tf, tb))
    else:
        res[v] = [[(tf, tb)], y.clone(), dx.clone(), g7.clone()]
L.tm_debug_set_ppeg_variant(0)
for v, (ts, y, dx, g7) in res.items():
    print(f"variant {v}: fwd " + " / ".join(f"{a:.2f}" for a, _ in ts) + " us   bwd " +
          " / ".join(f"{b:.2f}" for _, b in ts) + " us", flush=True)
for v in (1, 2):
    print(f"bitwise {v} vs 0: y", torch.equal(res[0][1], res[v][1]), " dx", torch.equal(res[0][2], res[v][2]),
          " dw7", torch.equal(res[0][3], res[v][3]))
