"""C5 encoder op variants on one box: strided 1x1 (subsample copy + GEMM vs MIOpen conv) and
3x3 conv + ReLU (two passes vs torch.miopen_convolution_relu); then the folded encoder forward."""
import sys, os, time
sys.path.insert(0, os.getcwd())
import torch
import torch.nn.functional as F


def timeit(fn, reps=10):
    for _ in range(2): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(reps): fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


dev, bf, cl = "cuda", torch.bfloat16, torch.channels_last
torch.backends.cudnn.benchmark = True
x = torch.randn(512, 256, 56, 56, device=dev, dtype=bf).contiguous(memory_format=cl)
w = (torch.randn(512, 256, 1, 1, device=dev, dtype=bf) * 0.05).contiguous(memory_format=cl)
b = torch.randn(512, device=dev, dtype=bf)


def gemm_strided():
    xs = x[:, :, ::2, ::2].contiguous(memory_format=cl)
    n, c, h, wd = xs.shape
    return torch.addmm(b, xs.permute(0, 2, 3, 1).reshape(-1, c), w.reshape(512, c).t())


print(f"1x1 stride 2 256->512 @56: copy+GEMM {timeit(gemm_strided):.2f} ms, "
      f"conv2d {timeit(lambda: F.conv2d(x, w, b, stride=2)):.2f} ms", flush=True)
y = torch.randn(512, 128, 56, 56, device=dev, dtype=bf).contiguous(memory_format=cl)
w3 = (torch.randn(128, 128, 3, 3, device=dev, dtype=bf) * 0.05).contiguous(memory_format=cl)
b3 = torch.randn(128, device=dev, dtype=bf)
a = timeit(lambda: F.relu(F.conv2d(y, w3, b3, padding=1)))
c = timeit(lambda: F.conv2d(y, w3, b3, padding=1))
try:
    m = timeit(lambda: torch.miopen_convolution_relu(y, w3, b3, [1, 1], [1, 1], [1, 1], 1))
    ok = (torch.miopen_convolution_relu(y, w3, b3, [1, 1], [1, 1], [1, 1], 1).float()
          - F.relu(F.conv2d(y, w3, b3, padding=1)).float()).abs().max().item()
except Exception as e:  # noqa: BLE001
    m, ok = float("nan"), repr(e)[:80]
print(f"3x3 128->128 @56: conv+relu {a:.2f} ms, conv only {c:.2f} ms, miopen_convolution_relu {m:.2f} ms "
      f"(max diff {ok})", flush=True)
from transmil_deepgraft_amd.encoder import RetCCLResNet50
enc = RetCCLResNet50().to(dev).eval()
tiles = torch.randn(1024, 3, 224, 224, device=dev)
with torch.no_grad():
    t = timeit(lambda: enc(tiles), reps=3)
print(f"folded encoder forward: {t:.1f} ms per 1024 tiles ({1024 / t * 1e3:.0f} tiles/s)", flush=True)
