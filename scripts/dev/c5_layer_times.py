"""Per-op time of the C5 eval encoder (bf16, BN folded, channels-last) on one bag piece: every 1x1
GEMM (tm_conv1x1), library 3x3 / stem convolution, bias + ReLU pass and the stem pool, each
bracketed by HIP events on the current stream, with its algorithmic bytes and flops -> GB/s, TF/s.

    python scripts/dev/c5_layer_times.py [tiles=1024] [reps=3]
"""
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.getcwd())
import transmil_deepgraft_amd.encoder as E          # noqa: E402

tiles = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
torch.backends.cudnn.benchmark = True
dev = torch.device("cuda", 0)
torch.manual_seed(0)
enc = E.retccl_resnet50(chunk=tiles).to(dev).set_compute_dtype(torch.bfloat16).eval()
x = torch.randn(tiles, 3, 224, 224, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)

recs = []
on = [False]


def wrap(name, fn, cost):
    def f(*a, **k):
        if not on[0]:
            return fn(*a, **k)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        out = fn(*a, **k)
        e.record()
        recs.append((name, s, e) + cost(out, *a, **k))
        return out
    return f


def c1x1(out, x, w, b, relu, residual=None):
    n, c, h, wd = x.shape
    rows, co = n * h * wd, w.shape[0]
    byt = 2 * (rows * c + rows * co * (2 if residual is not None else 1) + co * c)
    return (f"1x1 {c}->{co} rows {rows}{' +res' if residual is not None else ''}", byt, 2.0 * rows * c * co)


def conv(out, x, w, b=None, stride=1, padding=0):
    n, c, h, wd = x.shape
    _, co, ho, wo = out.shape
    k = w.shape[2]
    byt = 2 * (x.numel() + out.numel() + w.numel())
    return (f"{k}x{k}/{stride} {c}->{co} {h}x{wd}", byt, 2.0 * n * ho * wo * co * c * k * k)


def bias_act(out, y, b, relu=True):
    return (f"bias_act {tuple(y.shape[1:])}", 4 * y.numel(), 0.0)


def stem_pool(out, y, b):
    return (f"stem bias+relu+pool {tuple(y.shape[1:])}", 2 * (y.numel() + out.numel()), 0.0)


E._conv1x1_gemm = wrap("gemm", E._conv1x1_gemm, c1x1)
E._lib_conv2d = wrap("conv", E._lib_conv2d, conv)
E._bias_act_ = wrap("bias_act", E._bias_act_, bias_act)
E._stem_pool_ = wrap("pool", E._stem_pool_, stem_pool)

with torch.no_grad():
    enc(x)                                  # fold, MIOpen find, conv1x1 tuning
    enc(x)
    torch.cuda.synchronize()
    agg = defaultdict(lambda: [0.0, 0, 0.0, 0])
    tot = []
    for r in range(reps):
        recs.clear()
        on[0] = True
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        enc(x)
        e.record()
        on[0] = False
        torch.cuda.synchronize()
        tot.append(s.elapsed_time(e))
        for i, (kind, a, b, label, byt, fl) in enumerate(recs):
            k = (i, kind, label)
            agg[k][0] += a.elapsed_time(b) / reps
            agg[k][1] = byt
            agg[k][2] = fl
    cat = defaultdict(float)
    print(f"# {tiles} tiles, eval bf16 channels-last, mean of {reps} forwards: total {sum(tot) / reps:.2f} ms "
          f"({tiles / (sum(tot) / reps) * 1e3:.0f} tiles/s)")
    print(f"{'#':>3} {'op':52s} {'ms':>8} {'GB/s':>8} {'TF/s':>8}")
    for (i, kind, label), (ms, byt, fl, _) in sorted(agg.items()):
        cat[kind] += ms
        print(f"{i:3d} {label:52s} {ms:8.3f} {byt / ms / 1e6:8.0f} {fl / ms / 1e9:8.1f}")
    print("# by kind (ms): " + ", ".join(f"{k} {v:.2f}" for k, v in sorted(cat.items(), key=lambda t: -t[1])),
          f"; other {sum(tot) / reps - sum(cat.values()):.2f}")
