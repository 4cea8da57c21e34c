"""The step's GEMM shapes at M = 8448 rows per kernel variant of the diagnostic build
(0 ring 128x128 2-stage, 4 persistent ring, 6 3-stage ring, 7 big-tile 256x256 / 256x128)."""
import os, sys, time
sys.path.insert(0, os.getcwd())
os.environ.setdefault("TRANSMIL_HIP_LIB", os.path.join(os.getcwd(), "transmil_deepgraft_amd", "libtransmil_hip_diag.so"))
import torch
from transmil_deepgraft_amd import engine as E
from transmil_deepgraft_amd._lib import BF16, F32
from transmil_deepgraft_amd import _lib

def timeit(fn, reps=40):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps): fn()
    torch.cuda.synchronize(); t = time.perf_counter(); g.replay(); torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6

dev = "cuda"
variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,4,6,7").split(",")]
M = 8448
for name, N, K, bkn, cd in (("qkv", 1536, 512, 0, BF16), ("to_out", 512, 512, 0, F32), ("dmerged", 512, 512, 1, BF16),
                            ("dxn", 512, 1536, 1, BF16), ("fc1", 512, 1024, 0, F32)):
    A = (torch.randn(M, K, device=dev) * 0.1).to(torch.bfloat16)
    Bm = ((torch.randn(K, N, device=dev) if bkn else torch.randn(N, K, device=dev)) * 0.1).to(torch.bfloat16)
    Cm = torch.empty(M, N, device=dev, dtype=torch.float32 if cd == F32 else torch.bfloat16)
    ref = None
    line = []
    for v in variants:
        _lib.lib().tm_debug_set_variant(2, v)
        f = lambda: E.gemm(A, Bm, Cm, M, N, K, lda=K, ldb=N if bkn else K, ldc=N, b_kn=bkn, dtype=BF16, c_dtype=cd)
        f(); torch.cuda.synchronize()
        out = Cm.float().clone()
        if ref is None: ref = out
        err = ((out - ref).abs().max() / ref.abs().max()).item()
        t = timeit(f)
        line.append(f"v{v} {t:6.1f}us {2.0*M*N*K/t/1e6:5.0f}TF err{err:.0e}")
    print(f"{name:8s} N{N} K{K}: " + " | ".join(line), flush=True)
_lib.lib().tm_debug_set_variant(2, 0)
