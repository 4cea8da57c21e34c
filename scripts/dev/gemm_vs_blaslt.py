"""The step's dense GEMM shapes: the HIP ring GEMM against torch.mm (hipBLASLt) on the same
operands, each timed as 40 launches in one captured graph (what is reachable on this shape)."""
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import torch
from transmil_deepgraft_amd import engine as E
from transmil_deepgraft_amd._lib import BF16, F32


def timeit(fn, reps=40):
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


dev = "cuda"
M = 8448
for name, N, K, bkn, cd in (("qkv", 1536, 512, 0, BF16), ("to_out", 512, 512, 0, F32),
                            ("dmerged", 512, 512, 1, BF16), ("dxn", 512, 1536, 1, BF16),
                            ("fc1", 512, 512, 0, F32)):
    A = (torch.randn(M, K, device=dev) * 0.1).to(torch.bfloat16)
    Bm = ((torch.randn(K, N, device=dev) if bkn else torch.randn(N, K, device=dev)) * 0.1).to(torch.bfloat16)
    odt = torch.float32 if cd == F32 else torch.bfloat16
    Cm = torch.empty(M, N, device=dev, dtype=odt)
    t_ours = timeit(lambda: E.gemm(A, Bm, Cm, M, N, K, lda=K, ldb=N if bkn else K, ldc=N, b_kn=bkn,
                                   dtype=BF16, c_dtype=cd))
    Bt = Bm if bkn else Bm.t()
    if odt == torch.float32:
        fn = lambda: torch.mm(A, Bt, out_dtype=torch.float32)
    else:
        fn = lambda: torch.mm(A, Bt)
    t_lt = timeit(fn)
    fl = 2.0 * M * N * K
    print(f"{name:8s} M{M} N{N} K{K}: ours {t_ours:6.1f} us ({fl / t_ours / 1e6:5.0f} TF/s) | "
          f"hipBLASLt {t_lt:6.1f} us ({fl / t_lt / 1e6:5.0f} TF/s)", flush=True)
for Mw, Nw in ((1536, 512), (1024, 512), (512, 512)):
    dY = (torch.randn(M, Mw, device=dev) * 0.1).to(torch.bfloat16)
    X = (torch.randn(M, Nw, device=dev) * 0.1).to(torch.bfloat16)
    out = torch.empty(Mw, Nw, device=dev)
    pool = E.Pool(dev)
    t_ours = timeit(lambda: E.weight_grad(dY, X, out, Mw, Nw, M, ldy=Mw, ldx=Nw, dtype=BF16, work_pool=pool))
    t_lt = timeit(lambda: torch.mm(dY.t(), X, out_dtype=torch.float32))
    fl = 2.0 * M * Mw * Nw
    print(f"wgrad {Mw}x{Nw} K{M}: ours {t_ours:6.1f} us ({fl / t_ours / 1e6:5.0f} TF/s) | "
          f"hipBLASLt {t_lt:6.1f} us ({fl / t_lt / 1e6:5.0f} TF/s)", flush=True)
