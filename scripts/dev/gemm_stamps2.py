"""Per-workgroup timeline of the 2-stage ring GEMM (diagnostic build, variant 8 stamps) on the step's
shapes WITH their real epilogues: QKV head-major scatter, to_out (fp32 + bias + dropout + residual +
row map), _fc1 (bias + GELU + pre-activation + row map), dmerged (plain bf16).

    TRANSMIL_HIP_LIB=transmil_deepgraft_amd/libtransmil_hip_diag.so python scripts/dev/gemm_stamps2.py

Prints, per shape: the launch span, the per-phase cycle percentiles (first tile landed, k-loop,
accumulator staging, epilogue issue, store drain) and how many workgroups were co-resident on a CU
(from the realtime stamps)."""
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
n, N, S, pad = 8448, 8192, 8282, 166
torch.manual_seed(0)
A512 = (torch.randn(n, 512, device=dev) * 0.1).to(torch.bfloat16)
W1536 = (torch.randn(1536, 512, device=dev) * 0.05).to(torch.bfloat16)
W512 = (torch.randn(512, 512, device=dev) * 0.05).to(torch.bfloat16)
bias = torch.randn(512, device=dev) * 0.1
resid = torch.randn(S, 512, device=dev)
seed_dev = torch.tensor([7], dtype=torch.int64, device=dev)
qkv_out = torch.empty(3, 8, n, 64, device=dev, dtype=torch.bfloat16)
out32 = torch.empty(S, 512, device=dev)
fc1_out = torch.empty(S, 512, device=dev)
pre = torch.empty(N, 512, device=dev)
pre_b = torch.empty(N, 512, device=dev, dtype=torch.bfloat16)
X8192 = (torch.randn(N, 512, device=dev) * 0.1).to(torch.bfloat16)
dm = torch.empty(n, 512, device=dev, dtype=torch.bfloat16)

cases = {
    "qkv": (lambda: E.gemm(A512, W1536, qkv_out, n, 1536, 512, lda=512, ldb=512, ldc=0, dtype=BF16,
                           qkv=(1, 8, 64, n, 0.125)), n, 1536),
    "to_out": (lambda: E.gemm(A512, W512, out32, n, 512, 512, lda=512, ldb=512, ldc=512, dtype=BF16, c_dtype=F32,
                              bias=bias, drop_p=0.1, seed=3, seed_ptr=seed_dev, resid=resid,
                              rowmap=(n, pad, S, 0, 0, 0)), n, 512),
    "to_out_nodrop": (lambda: E.gemm(A512, W512, out32, n, 512, 512, lda=512, ldb=512, ldc=512, dtype=BF16,
                                     c_dtype=F32, bias=bias, resid=resid, rowmap=(n, pad, S, 0, 0, 0)), n, 512),
    "fc1": (lambda: E.gemm(X8192, W512, fc1_out, N, 512, 512, lda=512, ldb=512, ldc=512, dtype=BF16, c_dtype=F32,
                           bias=bias, gelu=True, pre=pre, ld_pre=512, rowmap=(N, 0, S, 1, 89, 1 + N)), N, 512),
    "fc1_prebf16": (lambda: E.gemm(X8192, W512, fc1_out, N, 512, 512, lda=512, ldb=512, ldc=512, dtype=BF16,
                                   c_dtype=F32, bias=bias, gelu=True, pre=pre_b, ld_pre=512, pre_bf16=True,
                                   rowmap=(N, 0, S, 1, 89, 1 + N)), N, 512),
    "fc1_nogelu":(lambda: E.gemm(X8192, W512, fc1_out, N, 512, 512, lda=512, ldb=512, ldc=512, dtype=BF16,
                                  c_dtype=F32, bias=bias, pre=pre, ld_pre=512, rowmap=(N, 0, S, 1, 89, 1 + N)), N, 512),
    "fc1_nopre": (lambda: E.gemm(X8192, W512, fc1_out, N, 512, 512, lda=512, ldb=512, ldc=512, dtype=BF16,
                                 c_dtype=F32, bias=bias, gelu=True, rowmap=(N, 0, S, 1, 89, 1 + N)), N, 512),
    "fc1_plain": (lambda: E.gemm(X8192, W512, fc1_out, N, 512, 512, lda=512, ldb=512, ldc=512, dtype=BF16,
                                 c_dtype=F32, bias=bias, rowmap=(N, 0, S, 1, 89, 1 + N)), N, 512),
    "dmerged_128": (lambda: E.gemm(A512, W512, dm, n, 512, 512, lda=512, ldb=512, ldc=512, b_kn=1, dtype=BF16),
                    n, 512),
}
only = sys.argv[1:] or list(cases)
for name in only:
    fn, M, Ncol = cases[name]
    L.tm_debug_set_variant(2, 8)
    for _ in range(4):
        fn()
    torch.cuda.synchronize()
    L.tm_debug_set_variant(2, 0)
    nb = ((M + 127) // 128) * ((Ncol + 127) // 128)
    buf = (ctypes.c_ulonglong * (nb * 8))()
    assert L.tm_debug_gemm_stamps(buf, nb * 8) == 0
    st = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 8).astype(np.int64)
    r0 = st[:, 0].min()
    start_us = (st[:, 0] - r0) / 100.0
    end_us = (st[:, 7] - r0) / 100.0
    d = np.diff(st[:, 1:7], axis=1)
    # co-residency: how many workgroups were running at each workgroup's midpoint
    mid = (start_us + end_us) / 2
    conc = np.array([np.sum((start_us <= m) & (end_us >= m)) for m in mid])

    def q(x):
        return "p10 %6.0f p50 %6.0f p90 %6.0f max %6.0f" % tuple(np.percentile(x, [10, 50, 90, 100]))

    # clock from the stamps: shader cycles per realtime 100 MHz tick
    clk = np.median((st[:, 6] - st[:, 1]) / np.maximum(st[:, 7] - st[:, 0], 1)) * 0.1
    print(f"{name} M{M} N{Ncol} K512: {nb} WGs, span {end_us.max():.2f} us, WG life p50 "
          f"{np.median(end_us - start_us):.2f} us, start p50/max {np.median(start_us):.2f}/{start_us.max():.2f} us, "
          f"concurrent WGs p50 {np.median(conc):.0f}, clock ~{clk:.2f} GHz", flush=True)
    for i, lab in enumerate(["first tile", "k-loop", "stage+sync", "epi issue", "store drain"]):
        print(f"   {lab:12s} cyc {q(d[:, i])}")
