"""A/B of the persistent register-epilogue GEMM (gemm_pr_kernel, diagnostic variant 11) against the
production selection (variant 0) on the training step's GEMM shapes with their real epilogues:
mean time per call over 200 calls (HIP events around the loop) and the max abs difference of the
outputs (the same products in the same k order: expected bitwise equal).

    TRANSMIL_HIP_LIB=transmil_deepgraft_amd/libtransmil_hip_diag.so python scripts/dev/gemm_pr_ab.py
"""
import os
import sys

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
A1536 = (torch.randn(n, 1536, device=dev) * 0.1).to(torch.bfloat16)
W1536 = (torch.randn(1536, 512, device=dev) * 0.05).to(torch.bfloat16)
W512 = (torch.randn(512, 512, device=dev) * 0.05).to(torch.bfloat16)
bias = torch.randn(512, device=dev) * 0.1
resid = torch.randn(S, 512, device=dev)
seed_dev = torch.tensor([7], dtype=torch.int64, device=dev)
X8192 = (torch.randn(N, 512, device=dev) * 0.1).to(torch.bfloat16)


def mk(name):
    if name == "qkv":
        out = torch.empty(3, 8, n, 64, device=dev, dtype=torch.bfloat16)
        return out, lambda: E.gemm(A512, W1536, out, n, 1536, 512, lda=512, ldb=512, ldc=0, dtype=BF16,
                                   qkv=(1, 8, 64, n, 0.125))
    if name == "to_out":
        out = torch.zeros(S, 512, device=dev)
        return out, lambda: E.gemm(A512, W512, out, n, 512, 512, lda=512, ldb=512, ldc=512, dtype=BF16, c_dtype=F32,
                                   bias=bias, drop_p=0.1, seed=3, seed_ptr=seed_dev, resid=resid,
                                   rowmap=(n, pad, S, 0, 0, 0))
    if name == "fc1":
        out = torch.zeros(S, 512, device=dev)
        pre = torch.zeros(N, 512, device=dev)
        return (out, pre), lambda: E.gemm(X8192, W512, out, N, 512, 512, lda=512, ldb=512, ldc=512, dtype=BF16,
                                          c_dtype=F32, bias=bias, gelu=True, pre=pre, ld_pre=512,
                                          rowmap=(N, 0, S, 1, 89, 1 + N))
    if name == "dmerged":
        out = torch.empty(n, 512, device=dev, dtype=torch.bfloat16)
        return out, lambda: E.gemm(A512, W512, out, n, 512, 512, lda=512, ldb=512, ldc=512, b_kn=1, dtype=BF16)
    if name == "dxn":
        out = torch.empty(n, 512, device=dev, dtype=torch.bfloat16)
        return out, lambda: E.gemm(A1536, W1536, out, n, 512, 1536, lda=1536, ldb=512, ldc=512, b_kn=1, dtype=BF16)
    raise ValueError(name)


def run(name, variant, reps=200):
    L.tm_debug_set_variant(2, variant)
    out, fn = mk(name)
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    L.tm_debug_set_variant(2, 0)
    outs = out if isinstance(out, tuple) else (out,)
    if name in ("to_out", "fc1"):       # accumulate-free epilogues: one more clean call for the comparison
        for o in outs:
            o.zero_()
        L.tm_debug_set_variant(2, variant)
        fn()
        L.tm_debug_set_variant(2, 0)
    return s.elapsed_time(e) / reps * 1e3, [o.float().clone() for o in outs]


for name in (sys.argv[1:] or ["qkv", "to_out", "fc1", "dmerged", "dxn"]):
    t0, o0 = run(name, 0)
    t1, o1 = run(name, 11)
    t0b, _ = run(name, 0)
    t1b, _ = run(name, 11)
    diff = max((a - b).abs().max().item() for a, b in zip(o0, o1))
    print(f"{name:8s} production {t0:7.2f} / {t0b:7.2f} us   pr {t1:7.2f} / {t1b:7.2f} us   max|diff| {diff:.3e}",
          flush=True)
