"""The eval encoder's 3x3 / stem convolutions with their folded-BN bias + ReLU: MIOpen convolution
then the in-place HIP bias + ReLU pass (encoder._bias_act_, the current form) against
torch.miopen_convolution_relu (MIOpen's fused conv + bias + activation), channels-last bf16,
1024-tile pieces, MIOpen find on.  Prints ms per call of each form and the max |difference|.

    python scripts/dev/c5_conv_relu.py [tiles]
"""
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.getcwd())
from transmil_deepgraft_amd import encoder as enc      # noqa: E402

torch.backends.cudnn.benchmark = True
dev = "cuda"
T = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
# (cin, cout, hw_in, k, stride, pad)
shapes = [(3, 64, 224, 7, 2, 3), (64, 64, 56, 3, 1, 1), (128, 128, 56, 3, 2, 1), (128, 128, 28, 3, 1, 1),
          (256, 256, 28, 3, 2, 1), (256, 256, 14, 3, 1, 1), (512, 512, 14, 3, 2, 1), (512, 512, 7, 3, 1, 1)]


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


torch.manual_seed(0)
for cin, cout, hw, k, s, p in shapes:
    x = torch.randn(T, cin, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, k, k, device=dev) * (2.0 / (cin * k * k)) ** 0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=torch.channels_last)
    b = torch.randn(cout, device=dev).to(torch.bfloat16)
    a = lambda: enc._bias_act_(F.conv2d(x, w, None, s, p), b)
    f = lambda: torch.miopen_convolution_relu(x, w, b, (s, s), (p, p), (1, 1), 1)
    try:
        ya, yf = a(), f()
        diff = (ya.float() - yf.float()).abs().max().item()
        ta, tf = timed(a), timed(f)
        print(f"cin {cin:4d} cout {cout:4d} hw {hw:3d} k{k} s{s}: conv + bias_act {ta:7.2f} ms | miopen_conv_relu "
              f"{tf:7.2f} ms | max|diff| {diff:.3e} | out cl {yf.is_contiguous(memory_format=torch.channels_last)}",
              flush=True)
    except Exception as e:   # noqa: BLE001
        print(f"cin {cin} cout {cout} hw {hw}: {type(e).__name__}: {str(e)[:200]}", flush=True)
