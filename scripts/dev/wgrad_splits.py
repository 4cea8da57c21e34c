"""Weight-gradient GEMMs (split-K + deferred-free reduce) at the step's shapes with the engine's split
count and with twice as many splits (two workgroups per CU), in graph replay."""
import os, sys
sys.path.insert(0, os.getcwd())
import torch
from transmil_deepgraft_amd import engine as E
from transmil_deepgraft_amd._lib import BF16
sys.path.insert(0, os.path.join(os.getcwd(), "scripts"))
from microbench import timeit
n, dev = 8448, "cuda"
g = torch.Generator(device="cpu").manual_seed(0)
shapes = {"dWqkv L1 (1536x512xn)": (1536, 512, n, 1536), "dWqkv L2 (1024x512xn)": (1024, 512, n, 1536),
          "dWout (512x512xn)": (512, 512, n, 512), "dWfc1 (512x512x8192)": (512, 512, 8192, 512)}
for name, (M, N, K, ldy) in shapes.items():
    dY = (torch.randn(K, ldy, generator=g) * 0.1).to(torch.bfloat16).to(dev)
    X = (torch.randn(K, N, generator=g) * 0.1).to(torch.bfloat16).to(dev)
    out = torch.empty(M, N, device=dev)
    bias = torch.empty(M, device=dev) if M == 512 else None
    for cu in (256, 512, 768):
        E._CU[torch.cuda.current_device()] = cu
        pool = E.Pool(dev)
        f = lambda: E.weight_grad(dY, X, out, M, N, K, ldy=ldy, ldx=N, dtype=BF16, work_pool=pool, bias_out=bias)
        f(); torch.cuda.synchronize(); ref = out.clone() if cu == 256 else ref
        err = (out - ref).abs().max().item()
        print(f"{name:24s} splits for {cu} slots: {timeit(f, 30):8.2f} us  (max |diff| vs 256: {err:.2e})", flush=True)
    E._CU.clear()
