"""dxn = dqkv W_qkv (M = 8448, N = 512, K = 1536 / 1024, b_kn) as the engine launches it (one
output, 160-row ring tiles) against split-K 2 / 3 on the 128 x 128 ring with bf16 slabs (two
workgroups per CU: the ring's k-loop is latency-paced per workgroup), in graph replay."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from transmil_deepgraft_amd import engine as E            # noqa: E402
from transmil_deepgraft_amd import _lib                   # noqa: E402
from transmil_deepgraft_amd._lib import BF16, F32, GemmArgs, EPI_SPLITK   # noqa: E402
sys.path.insert(0, os.path.join(os.getcwd(), "scripts"))
from microbench import timeit                              # noqa: E402

M, N, dev = 8448, 512, "cuda"
for K in (1536, 1024):
    A = (torch.randn(M, 1536, device=dev) * 0.1).to(torch.bfloat16)     # dqkv rows (ld 1536)
    W = (torch.randn(K, N, device=dev) * 0.05).to(torch.bfloat16)
    out = torch.empty(M, N, device=dev, dtype=torch.bfloat16)
    t0 = timeit(lambda: E.gemm(A, W, out, M, N, K, lda=1536, ldb=N, ldc=N, b_kn=1, dtype=BF16), 30)
    ref = (A[:, :K].float() @ W.float())
    print(f"K {K}: engine launch {t0:7.2f} us", flush=True)
    for s in (2, 3):
        kps = ((K + s - 1) // s + 63) // 64 * 64
        slab = torch.empty(s * M * N, device=dev, dtype=torch.bfloat16)
        g = GemmArgs()
        g.M, g.N, g.K = M, N, K
        g.lda, g.ldb, g.ldc = 1536, N, N
        g.a_trans, g.b_kn = 0, 1
        g.ab_dtype, g.c_dtype = BF16, F32
        g.splits, g.k_per_split = s, kps
        g.mode = EPI_SPLITK
        g.alpha = 1.0
        g.slab_bf16 = 1
        fn = lambda: _lib.call("tm_gemm", E._p(A), E._p(W), E._p(slab), C.byref(g), E._stream())
        t1 = timeit(fn, 30)
        got = slab.view(s, M, N).float().sum(0)
        err = ((got - ref).abs().max() / ref.abs().max()).item()
        print(f"K {K}: split-K {s} bf16 slabs {t1:7.2f} us (max rel err of the slab sum {err:.2e})", flush=True)
