"""Time tm_stem_conv_pool alone (1024 tiles of 3 x 224 x 224 bf16, NCHW) against the library stem
(MIOpen conv + tm_bias_relu_maxpool), HIP events over 20 calls each.

    python scripts/dev/stem_time.py [tiles]
"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.getcwd())
import transmil_deepgraft_amd.encoder as E          # noqa: E402

torch.backends.cudnn.benchmark = True
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
x = torch.randn(n, 3, 224, 224, device="cuda").to(torch.bfloat16)
w = (torch.randn(64, 3, 7, 7, device="cuda") * 0.1).to(torch.bfloat16)
b = (torch.randn(64, device="cuda") * 0.1).to(torch.bfloat16)
wp = E._pack_stem(w)
wcl = w.contiguous(memory_format=torch.channels_last)
xcl = x.contiguous(memory_format=torch.channels_last)


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


t_f = timeit(lambda: E._stem_conv_pool(x, wp, b))
t_fcl = timeit(lambda: E._stem_conv_pool(xcl, wp, b))
t_lib = timeit(lambda: E._stem_pool_(F.conv2d(xcl, wcl, None, stride=2, padding=3), b))
byt = x.numel() * 2 + n * 64 * 56 * 56 * 2
fl = 2.0 * n * 112 * 112 * 64 * 147
print(f"{n} tiles: fused NCHW {t_f:.3f} ms ({byt / t_f / 1e6:.0f} GB/s, {fl / t_f / 1e9:.0f} TF/s), "
      f"fused NHWC {t_fcl:.3f} ms, library conv + pool {t_lib:.3f} ms")
