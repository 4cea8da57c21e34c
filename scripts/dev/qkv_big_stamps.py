"""Per-workgroup phase stamps of the big-tile to_qkv GEMM (256 x 256 tiles, head-major scatter
epilogue; diagnostic build, variant 12) at the bench shape (M = 8448, N = 1536, K = 512).

    TRANSMIL_HIP_LIB=transmil_deepgraft_amd/libtransmil_hip_diag.so python scripts/dev/qkv_big_stamps.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.getcwd())
from transmil_deepgraft_amd import _lib                      # noqa: E402
from transmil_deepgraft_amd import engine as E               # noqa: E402
from transmil_deepgraft_amd._lib import BF16                 # noqa: E402
sys.path.insert(0, os.path.join(os.getcwd(), "scripts"))
from microbench import timeit                                 # noqa: E402

L = _lib.lib()
n, dev = 8448, "cuda"
torch.manual_seed(0)
A = (torch.randn(n, 512, device=dev) * 0.1).to(torch.bfloat16)
W = (torch.randn(1536, 512, device=dev) * 0.05).to(torch.bfloat16)
out = torch.empty(3, 8, n, 64, device=dev, dtype=torch.bfloat16)
fn = lambda: E.gemm(A, W, out, n, 1536, 512, lda=512, ldb=512, ldc=0, dtype=BF16, qkv=(1, 8, 64, n, 0.125))
print(f"big-tile QKV (product pick): {timeit(fn, 30):.2f} us per call (graph replay)", flush=True)
L.tm_debug_set_variant(2, 12)
for _ in range(4):
    fn()
torch.cuda.synchronize()
L.tm_debug_set_variant(2, 0)
nb = 6 * 33
buf = (ctypes.c_ulonglong * (nb * 8))()
assert L.tm_debug_gemm_stamps(buf, nb * 8) == 0
st = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 8).astype(np.int64)
r0 = st[:, 0].min()
start_us, end_us = (st[:, 0] - r0) / 100.0, (st[:, 7] - r0) / 100.0
d = np.diff(st[:, 1:7], axis=1)
clk = np.median((st[:, 6] - st[:, 1]) / np.maximum(st[:, 7] - st[:, 0], 1)) * 0.1


def q(x):
    return "p10 %6.0f p50 %6.0f p90 %6.0f max %6.0f" % tuple(np.percentile(x, [10, 50, 90, 100]))


print(f"{nb} WGs, span {end_us.max():.2f} us, WG life p50 {np.median(end_us - start_us):.2f} us, start p50/max "
      f"{np.median(start_us):.2f}/{start_us.max():.2f} us, clock ~{clk:.2f} GHz; 8 k-steps of 64 KB")
for i, lab in enumerate(["first tile", "k-loop", "loop->barrier", "epilogue", "store drain"]):
    print(f"   {lab:14s} cyc {q(d[:, i])}")
