"""Per-workgroup phases of the split-K weight-gradient ring GEMM (diagnostic build, gemm variant 8
stamps) at the step's shapes: dWo / dW_fc1 (512 x 512, K = 8448 / 8192) and dWqkv (1536 x 512,
K = 8448); also the same products with the operands stored k-contiguous (A = dY^T, B = X^T
materialised), to separate the k-row (a_trans / b_kn) image fill from the k-contiguous one.

    TRANSMIL_HIP_LIB=transmil_deepgraft_amd/libtransmil_hip_diag.so python scripts/dev/wgrad_stamps.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.getcwd())
from transmil_deepgraft_amd import _lib                      # noqa: E402
from transmil_deepgraft_amd import engine as E               # noqa: E402
from transmil_deepgraft_amd._lib import BF16, F32            # noqa: E402

L = _lib.lib()
dev = "cuda"
torch.manual_seed(0)


def run(name, fn, nb):
    L.tm_debug_set_variant(2, 8)
    for _ in range(4):
        fn()
    torch.cuda.synchronize()
    L.tm_debug_set_variant(2, 0)
    buf = (ctypes.c_ulonglong * (nb * 8))()
    assert L.tm_debug_gemm_stamps(buf, nb * 8) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 8).astype(np.int64)
    r0 = st[:, 0].min()
    start_us, end_us = (st[:, 0] - r0) / 100.0, (st[:, 7] - r0) / 100.0
    d = np.diff(st[:, 1:7], axis=1)
    q = lambda x: "p10 %6.0f p50 %6.0f p90 %6.0f max %6.0f" % tuple(np.percentile(x, [10, 50, 90, 100]))
    print(f"{name}: {nb} WGs, span {end_us.max():.2f} us, WG life p50 {np.median(end_us - start_us):.2f} us", flush=True)
    for i, lab in enumerate(["first tile", "k-loop", "stage+sync", "epi issue", "store drain"]):
        print(f"   {lab:12s} cyc {q(d[:, i])}")


for M, N, K in ((512, 512, 8448), (1536, 512, 8448)):
    dY = (torch.randn(K, M, device=dev) * 0.1).to(torch.bfloat16)
    X = torch.randn(K, N, device=dev).to(torch.bfloat16)
    tiles = (M // 128) * (N // 128)
    splits = max(1, min(16, E.cu_count() // tiles, (K + 255) // 256))
    kps = ((K + splits - 1) // splits + 63) // 64 * 64
    splits = (K + kps - 1) // kps
    slab = torch.empty(splits * M * N, device=dev)

    def args(a_trans, b_kn, lda, ldb):
        g = E.GemmArgs()
        g.M, g.N, g.K = M, N, K
        g.lda, g.ldb, g.ldc = lda, ldb, N
        g.a_trans, g.b_kn = a_trans, b_kn
        g.ab_dtype, g.c_dtype = BF16, F32
        g.splits, g.k_per_split = splits, kps
        g.mode = E.EPI_SPLITK
        g.alpha = 1.0
        return g
    g1 = args(1, 1, M, N)
    run(f"wgrad {M}x{N} K{K} k-rows (a_trans, b_kn), {splits} splits",
        lambda: _lib.call("tm_gemm", E._p(dY), E._p(X), E._p(slab), ctypes.byref(g1), E._stream()), tiles * splits)
    dYt, Xt = dY.t().contiguous(), X.t().contiguous()
    g2 = args(0, 0, K, K)
    run(f"wgrad {M}x{N} K{K} k-contiguous operands, {splits} splits",
        lambda: _lib.call("tm_gemm", E._p(dYt), E._p(Xt), E._p(slab), ctypes.byref(g2), E._stream()), tiles * splits)
