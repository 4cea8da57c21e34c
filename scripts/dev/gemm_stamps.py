"""Per-workgroup timeline of the 2-stage ring GEMM (variant 8 stamps) on the step's shapes."""
import sys, os, ctypes
sys.path.insert(0, os.getcwd())
import numpy as np
import torch
from transmil_deepgraft_amd import engine as E
from transmil_deepgraft_amd._lib import BF16, F32
from transmil_deepgraft_amd import _lib

L = _lib.lib()
dev = "cuda"
for name, M, N, K, bkn, cd in (("out", 8448, 512, 512, 0, F32), ("dmerged", 8448, 512, 512, 1, BF16),
                               ("qkv", 8448, 1536, 512, 0, BF16), ("dxn", 8448, 512, 1536, 1, BF16),
                               ("fc1", 8192, 512, 1024, 0, F32), ("out8192", 8192, 512, 512, 0, F32)):
    A = (torch.randn(M, K, device=dev) * 0.1).to(torch.bfloat16)
    Bm = ((torch.randn(K, N, device=dev) if bkn else torch.randn(N, K, device=dev)) * 0.1).to(torch.bfloat16)
    Cm = torch.empty(M, N, device=dev, dtype=torch.float32 if cd == F32 else torch.bfloat16)
    L.tm_debug_set_variant(2, 8)
    for _ in range(4):
        E.gemm(A, Bm, Cm, M, N, K, lda=K, ldb=N if bkn else K, ldc=N, b_kn=bkn, dtype=BF16, c_dtype=cd)
    torch.cuda.synchronize()
    L.tm_debug_set_variant(2, 0)
    nb = ((M + 127) // 128) * ((N + 127) // 128)
    buf = (ctypes.c_ulonglong * (nb * 8))()
    assert L.tm_debug_gemm_stamps(buf, nb * 8) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 8).astype(np.int64)
    r0 = st[:, 0].min()
    end_us = (st[:, 7] - r0) / 100.0
    d = np.diff(st[:, 1:7], axis=1)
    def q(x): return "p10 %6.0f p50 %6.0f p90 %6.0f max %6.0f" % tuple(np.percentile(x, [10, 50, 90, 100]))
    print(f"{name} M{M} N{N} K{K}: {nb} WGs, span {end_us.max():.2f} us, end p50 {np.median(end_us):.2f} us", flush=True)
    for i, lab in enumerate(["first tile", "k-loop", "stage+sync", "epi issue", "store drain"]):
        print(f"   {lab:12s} cyc {q(d[:, i])}")
