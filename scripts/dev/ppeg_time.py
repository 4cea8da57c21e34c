"""Time the PPEG stencil forward / backward (+ weight gradient) at the bench shape (G = 91, D = 512)."""
import sys, os, time
sys.path.insert(0, os.getcwd())
import ctypes as C
import torch
from transmil_deepgraft_amd import _lib
from transmil_deepgraft_amd.engine import _p, _stream


def timeit(fn, reps=50):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps): fn()
    torch.cuda.synchronize(); t = time.perf_counter(); g.replay(); torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6


B, G, D = 1, 91, 512
S = 1 + G * G
dev = "cuda"
x = torch.randn(B, S, D, device=dev)
dy = torch.randn(B, S, D, device=dev)
y = torch.empty_like(x)
dx = torch.empty_like(x)
w7, w5, w3 = (torch.randn(D, k * k, device=dev) * 0.1 for k in (7, 5, 3))
b7, b5, b3 = (torch.randn(D, device=dev) for _ in range(3))
wf = torch.empty(49 * D, device=dev)
bf = torch.empty(D, device=dev)
_lib.call("tm_ppeg_fold", _p(w7), _p(b7), _p(w5), _p(b5), _p(w3), _p(b3), D, _p(wf), _p(bf), _stream())
work = torch.empty(_lib.query("tm_ppeg_bwd_workspace", B, G, D) // 4, device=dev)
g7, g5, g3 = (torch.empty(D, k * k, device=dev) for k in (7, 5, 3))
gb7, gb5, gb3 = (torch.empty(D, device=dev) for _ in range(3))
f = lambda: _lib.call("tm_ppeg_fwd", _p(x), B, G, D, _p(wf), _p(bf), _p(y), _stream())
bwd = lambda: _lib.call("tm_ppeg_bwd", _p(x), _p(dy), B, G, D, _p(wf), _p(dx), _p(work), _p(g7), _p(gb7),
                        _p(g5), _p(gb5), _p(g3), _p(gb3), 0, None, 0, 0, C.c_float(0.0), C.c_uint64(0), None,
                        None, _stream())
mb = S * D * 4 * 2 / 1e6
tf, tb = timeit(f), timeit(bwd)
print(f"ppeg fwd {tf:6.2f} us ({mb / tf:5.2f} TB/s on {mb:.1f} MB)   bwd (data + weights) {tb:6.2f} us", flush=True)
