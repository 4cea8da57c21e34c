"""Timing of the class-row layer's q-part products (dWq = s Aq^T Xs, G = s Aq Wq; B = 1, D = 512,
288 operand rows) in candidate forms, under `rocprofv3 --kernel-trace --stats`:
  bmm2   tm_bmm, both jobs in one launch (bf16x3, fp32 operands)   [the engine's form]
  bmmG / bmmW   each job alone
  gemmG  tm_gemm, bf16 operands, G (M 288, N 512, K 512)
  gemmW  tm_gemm split-K (weight_grad), bf16 operands, dWq (M 512, N 512, K 288)
100 calls each, then the max |difference| of the bf16 forms against bmm2.

    python scripts/dev/cls_q_products.py
"""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
from transmil_deepgraft_amd import engine as E                # noqa: E402
from transmil_deepgraft_amd._lib import BF16, F32             # noqa: E402

dev = "cuda"
D, R = 512, E.QROWS
torch.manual_seed(0)
Aq = torch.randn(R, D, device=dev) * 1e-3
Aq[257:] = 0
Xs = torch.randn(R, D, device=dev) * 5
Xs[257:] = 0
Wq = torch.randn(D, D, device=dev) * 0.05
G = torch.empty(R, D, device=dev)
dW = torch.empty(D, D, device=dev)
s = 0.125
pool = E.Pool(dev)
Aqb, Xsb, Wqb = Aq.to(torch.bfloat16), Xs.to(torch.bfloat16), Wq.to(torch.bfloat16)
G2 = torch.empty(R, D, device=dev)
dW2 = torch.empty(D, D, device=dev)
jg = E.bmm_job(Aq, 0, Wq, 0, G, R, D, D, alpha=s)
jw = E.bmm_job(Aq, 1, Xs, 0, dW, D, D, R, alpha=s)
forms = {
    "bmm2": lambda: E.bmm([jg, jw], 1, 1),
    "bmmG": lambda: E.bmm([jg], 1, 1),
    "bmmW": lambda: E.bmm([jw], 1, 1),
    "gemmG": lambda: E.gemm(Aqb, Wqb, G2, R, D, D, lda=D, ldb=D, ldc=D, b_kn=1, dtype=BF16, c_dtype=F32, alpha=s),
    "gemmW": lambda: E.weight_grad(Aqb, Xsb, dW2, D, D, R, ldy=D, ldx=D, dtype=BF16, work_pool=pool),
}
for name in (sys.argv[1:] or list(forms)):
    for _ in range(100):
        forms[name]()
    torch.cuda.synchronize()
    print(name, "done", flush=True)
E.bmm([jg, jw], 1, 1)
torch.cuda.synchronize()
print("gemmG vs bmm: rel", ((G2 - G).abs().max() / G.abs().max()).item())
print("gemmW vs bmm: rel", ((s * dW2 - dW).abs().max() / dW.abs().max()).item())
