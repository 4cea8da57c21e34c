"""Time the step's dense GEMM shapes per kernel variant and row count (tail-effect probe)."""
import sys, os, time
sys.path.insert(0, os.getcwd())
import torch
from transmil_deepgraft_amd import engine as E
from transmil_deepgraft_amd._lib import BF16, F32
from transmil_deepgraft_amd import _lib

def timeit(fn, reps=40):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps): fn()
    torch.cuda.synchronize(); t = time.perf_counter(); g.replay(); torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e6

dev = "cuda"
shapes = [] if os.environ.get("WGRAD_ONLY") else [  # name, N, K, b_kn, out dtype
    ("qkv", 1536, 512, 0, BF16), ("out", 512, 512, 0, F32), ("dmerged", 512, 512, 1, BF16),
    ("dxn", 512, 1536, 1, BF16), ("fc1", 512, 1024, 0, F32)]
variants = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0,1,3").split(",")]
rows = [8192, 8282, 8448]
for name, N, K, bkn, cd in shapes:
    line = []
    for M in rows:
        A = (torch.randn(M, K, device=dev) * 0.1).to(torch.bfloat16)
        Bm = (torch.randn(K, N, device=dev) if bkn else torch.randn(N, K, device=dev)).to(torch.bfloat16) * 0.1
        Cm = torch.empty(M, N, device=dev, dtype=torch.float32 if cd == F32 else torch.bfloat16)
        for v in variants:
            _lib.lib().tm_debug_set_variant(2, v)
            t = timeit(lambda: E.gemm(A, Bm, Cm, M, N, K, lda=K, ldb=N if bkn else K, ldc=N, b_kn=bkn, dtype=BF16, c_dtype=cd))
            fl = 2.0 * M * N * K / t / 1e6
            line.append(f"M{M}/v{v} {t:6.1f}us {fl:5.0f}TF")
    print(f"{name:8s} N{N} K{K}: " + " | ".join(line), flush=True)
for M, N in ((512, 512), (1536, 512), (512, 1024)):
    line = []
    for K, v in [(k, v) for k in rows for v in variants]:
        _lib.lib().tm_debug_set_variant(2, v)
        dY = (torch.randn(K, M, device=dev) * 0.1).to(torch.bfloat16)
        X = torch.randn(K, N, device=dev).to(torch.bfloat16)
        out = torch.empty(M, N, device=dev)
        pool = E.Pool(dev)
        t = timeit(lambda: E.weight_grad(dY, X, out, M, N, K, ldy=M, ldx=N, dtype=BF16, work_pool=pool))
        line.append(f"K{K}/v{v} {t:6.1f}us {2.0*M*N*K/t/1e6:5.0f}TF")
    print(f"wgrad {M}x{N}: " + " | ".join(line), flush=True)
_lib.lib().tm_debug_set_variant(2, 0)
