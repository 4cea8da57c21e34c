"""Would one launch holding both backward products of to_qkv (dW_qkv split-K, dxn) beat the two
launches back to back?  Eager timing at the bench shape (n' = 8448): each alone, both serial on one
stream, and both on two streams at once (co-resident workgroups: 2 x 64 KB LDS fits a CU)."""
import os, sys, time
sys.path.insert(0, os.getcwd())
import torch
from transmil_deepgraft_amd import _lib
from transmil_deepgraft_amd._lib import BF16
from transmil_deepgraft_amd import engine as E
n, D = 8448, 512
dev = "cuda"
g = torch.Generator(device="cpu").manual_seed(0)
dqkv = (torch.randn(n, 3 * D, generator=g) * 0.1).to(torch.bfloat16).to(dev)
xn = torch.randn(n, D, generator=g).to(torch.bfloat16).to(dev)
w = (torch.randn(3 * D, D, generator=g) * 0.05).to(torch.bfloat16).to(dev)
dW = torch.empty(3 * D, D, device=dev)
dxn = torch.empty(n, D, dtype=torch.bfloat16, device=dev)
work = torch.empty(16 * 3 * D * D, device=dev)
pool = lambda numel: work[:numel]
def wg(): E.weight_grad(dqkv, xn, dW, 3 * D, D, n, ldy=3 * D, ldx=D, dtype=BF16, work_pool=pool)
def dx(): E.gemm(dqkv, w, dxn, n, D, 3 * D, lda=3 * D, ldb=D, ldc=D, b_kn=1, dtype=BF16)
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
def timeit(f, reps=200):
    for _ in range(10): f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps): f()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6
def serial():
    with torch.cuda.stream(s1):
        wg(); dx()
def both():
    ev = torch.cuda.Event()
    with torch.cuda.stream(s1):
        wg()
    with torch.cuda.stream(s2):
        dx()
    ev.record(s2); s1.wait_event(ev)
    s2.wait_stream(s1)
for name, f in (("dW_qkv (split-K + reduce)", lambda: [wg() for _ in (0,)]), ("dxn", dx), ("serial", serial), ("two streams", both)):
    with torch.cuda.stream(s1):
        us = timeit(f)
    print(f"{name:28s} {us:7.1f} us per call (eager, launch gaps included)", flush=True)
