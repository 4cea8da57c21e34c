"""Time hipBLASLt (torch.mm) on the weight-gradient shapes against the HIP split-K path."""
import sys, os, time
sys.path.insert(0, os.getcwd())
import torch
from transmil_deepgraft_amd import engine as E
from transmil_deepgraft_amd._lib import BF16

def timeit(fn, reps=50):
    for _ in range(5): fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps): fn()
    torch.cuda.synchronize(); t = time.perf_counter(); g.replay(); torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6

dev = "cuda"
n = 8448
for M, N in ((512, 512), (1536, 512)):
    dY = (torch.randn(n, M, device=dev) * 0.1).to(torch.bfloat16)
    X = torch.randn(n, N, device=dev).to(torch.bfloat16)
    out = torch.empty(M, N, device=dev)
    pool = E.Pool(dev)
    t_ours = timeit(lambda: E.weight_grad(dY, X, out, M, N, n, ldy=M, ldx=N, dtype=BF16, work_pool=pool))
    ref = dY.double().t() @ X.double()
    try:
        o2 = torch.mm(dY.t(), X, out_dtype=torch.float32)
        err = ((o2.double() - ref).norm() / ref.norm()).item()
        t_lt = timeit(lambda: torch.mm(dY.t(), X, out_dtype=torch.float32))
    except Exception as exc:
        err, t_lt = repr(exc)[:80], None
    o3 = torch.mm(dY.t(), X)
    err3 = ((o3.double() - ref).norm() / ref.norm()).item()
    t_bf = timeit(lambda: torch.mm(dY.t(), X))
    print(f"wgrad {M}x{N}xK{n}: ours {t_ours:.1f} us | mm(out_dtype=fp32) {t_lt} us err {err} | mm bf16 out {t_bf:.1f} us err {err3:.2e}")
