"""Ablations of the bf16 A1 forward (a1_fwd_bf16_kernel, diagnostic build) at the bench shape
(B=1, h=8, n=8448): graph-replayed µs per call of variant 0 (production), 11 (no conv MFMAs),
12 (no attention phase), 13 (prologue only), and the stamps of variant 19 (slots: 0 start,
1 keys / Y / band in LDS, 2 first attention phase, 3 window landed, 4 first conv, 5 first stores,
6 end; waves 0 and 3).

    TRANSMIL_HIP_LIB=<diag .so> python scripts/dev/a1_fwd_ablate.py
"""
import ctypes as C
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.getcwd())
from transmil_deepgraft_amd import _lib                    # noqa: E402
from transmil_deepgraft_amd.engine import _p, _stream      # noqa: E402

nh, n, B = 8, 8448, 1
nbh = B * nh
dev = "cuda"
g = torch.Generator(device="cpu").manual_seed(1)
q = (torch.randn(nbh, n, 64, generator=g) * 0.3).to(torch.bfloat16).to(dev)
v = (torch.randn(nbh, n, 64, generator=g) * 0.3).to(torch.bfloat16).to(dev)
kl = (torch.randn(nbh, 256, 64, generator=g) * 0.3).to(torch.bfloat16).to(dev)
y = (torch.randn(nbh, 256, 64, generator=g) * 0.3).to(torch.bfloat16).to(dev)
wconv = torch.randn(nh, 33, device=dev) * 0.1
merged = torch.empty(B, n, nh * 64, dtype=torch.bfloat16, device=dev)
lse = torch.empty(nbh, n, device=dev)
f = lambda: _lib.call("tm_nys_a1_fwd", 1, _p(q), _p(v), _p(kl), _p(y), _p(wconv), nbh, nh, n, _p(merged),   # noqa: E731
                      _p(lse), _stream())
L = _lib.lib()


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


for var in (0, 11, 12, 13, 0):
    L.tm_debug_set_nys_variant(var)
    print(f"variant {var}: {timeit(f):.2f} us", flush=True)
L.tm_debug_set_nys_variant(19)
f()
torch.cuda.synchronize()
L.tm_debug_set_nys_variant(0)
buf = (C.c_ulonglong * (512 * 8 * 8))()
_lib.call("tm_debug_a1_stamps", buf, 512 * 8 * 8)
a = np.frombuffer(buf, dtype=np.uint64).reshape(512, 8, 8)[:32 * nbh].astype(np.int64)
for w in (0, 3):
    st = a[:, w, :]
    d = np.diff(st, axis=1)
    print(f"  wave {w}: mean cycles per phase", [int(x) for x in d.mean(0)], " max", [int(x) for x in d.max(0)])
    print(f"     total mean {int((st[:, 6] - st[:, 0]).mean())} cycles; start spread {int(st[:, 0].max() - st[:, 0].min())}")
