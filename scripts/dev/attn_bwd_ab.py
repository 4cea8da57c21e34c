"""A/B of attention-backward variants (diagnostic build, nys variants) on the bench shapes: the A1
backward (tm_nys_a1_bwd_dqkv) and the fused A3 backward (tm_nys_a3_bwd_fused), 100 calls each per
variant, then graph-replayed us per call of each (variants in the order given, twice).  Under
`rocprofv3 --kernel-trace --stats` each variant is its own template instance, so the kernel stats
separate them.

    TRANSMIL_HIP_LIB=transmil_deepgraft_amd/libtransmil_hip_diag.so python scripts/dev/attn_bwd_ab.py 0 36
"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.getcwd())
os.environ.setdefault("TRANSMIL_HIP_LIB", os.path.join(os.getcwd(), "transmil_deepgraft_amd", "libtransmil_hip_diag.so"))
import torch                  # noqa: E402
from transmil_deepgraft_amd import _lib                    # noqa: E402
from transmil_deepgraft_amd.engine import _p, _stream      # noqa: E402

nh, n, B = 8, 8448, 1
nbh = B * nh
dev = "cuda"
g = torch.Generator(device="cpu").manual_seed(1)
r = lambda *s, sc=1.0: (torch.randn(*s, generator=g) * sc)
q = r(B, nh, n, 64, sc=0.3).to(torch.bfloat16).to(dev)
dmerged = r(B, n, nh * 64, sc=0.1).to(torch.bfloat16).to(dev)
kl = r(B, nh, 256, 64, sc=0.3).to(torch.bfloat16).to(dev)
y = r(B, nh, 256, 64, sc=0.3).to(torch.bfloat16).to(dev)
lse = torch.randn(nbh, n, device=dev) + 6
d1 = torch.randn(nbh, n, device=dev) * 0.01
dqkv = torch.empty(B, n, 3 * nh * 64, dtype=torch.bfloat16, device=dev)
work1 = torch.empty(_lib.query("tm_nys_a1_bwd_workspace", nbh, n, 256) // 4 + 16, device=dev)
dkl = torch.empty(nbh, 256, 64, device=dev)
dy = torch.empty(nbh, 256, 64, device=dev)
a1 = lambda: _lib.call("tm_nys_a1_bwd_dqkv", _p(q), _p(dmerged), _p(kl), _p(y), _p(lse), _p(d1), nbh, nh, n, _p(dqkv),
                       C.c_float(0.125), _p(work1), _p(dkl), _p(dy), None, _stream())
ql = r(nbh, 256, 64, sc=0.3).to(torch.bfloat16).to(dev)
dw = r(nbh, 256, 64, sc=0.1).to(torch.bfloat16).to(dev)
k = r(nbh, n, 64, sc=0.3).to(torch.bfloat16).to(dev)
v = r(nbh, n, 64).to(torch.bfloat16).to(dev)
lse3 = torch.randn(nbh, 256, device=dev) + 9
d3 = torch.randn(2, nbh, 256, device=dev) * 0.01
dql = torch.empty(nbh, 256, 64, device=dev)
work3 = torch.empty(_lib.query("tm_nys_a3_bwd_workspace", nbh, n) // 4 + 16, device=dev)
dvc = torch.randn(nbh, n, 64, device=dev) * 0.01
dkl3 = torch.randn(nbh, 256, 64, device=dev) * 0.01
a3 = lambda: _lib.call("tm_nys_a3_bwd_fused", _p(ql), _p(dw), _p(k), _p(v), _p(lse3), _p(d3), nbh, 8, n, _p(dvc),
                       0, n, _p(dkl3), _p(work3), _p(dql), _p(dqkv), None, _stream())
L = _lib.lib()
ref = None
for var in [int(x) for x in (sys.argv[1:] or ["0", "36"])]:
    L.tm_debug_set_nys_variant(var)
    for f in (a1, a3):
        for _ in range(100):
            f()
    torch.cuda.synchronize()
    out = (dqkv.float().clone(), dkl.clone(), dy.clone(), dql.clone())
    if ref is None:
        ref = out
    else:
        print(f"variant {var}: max |diff| vs first variant (dqkv, dkl, dy, dql):",
              [f"{(a - b).abs().max().item():.3e}" for a, b in zip(out, ref)], flush=True)


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


for rep in range(2):
    for var in [int(x) for x in (sys.argv[1:] or ["0", "36"])]:
        L.tm_debug_set_nys_variant(var)
        print(f"variant {var}: A1 bwd {timeit(a1):.2f} us, A3 bwd {timeit(a3):.2f} us", flush=True)
L.tm_debug_set_nys_variant(0)
print("done", flush=True)
