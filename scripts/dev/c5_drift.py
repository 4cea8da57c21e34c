"""C5 one-pass drift diagnosis ("What's weak" 5): round 4's fp32 test found the features of
a 4096-tile bag run as ONE library batch differing from the 512-tile piecewise run by up to 3.35e-3
(per-tile relative L2).  This script re-runs the eval path of that tree (commit e545b33:
F.conv2d stem + ReLU + max_pool2d, torch.addmm 1x1 convolutions, F.conv2d 3x3, add + ReLU; fp32,
channels-last) both ways and reports, op by op, how the one-pass output differs from the piecewise one
on the SAME input (each op isolated), per tile, split at the tile where the op's largest tensor crosses
2^31 elements -- an index-width defect shows as a jump at that tile, an algorithm choice (MIOpen /
BLAS picking another kernel for the larger batch) as a spread over every tile.  Then both full chains
against the fp64 oracle (oracle/encoder_ref.py) on tiles either side of the boundary.

    python scripts/dev/c5_drift.py [--tiles 4096] [--chunk 512] > gpurun_out/c5_drift.json

Diagnostic only (it deliberately hands the libraries > 2^31-element tensors, the configuration the
round-4 fp32 test ran to completion; the product encoder refuses them, encoder._lib_guard)."""
import argparse
import json
import os
import sys
import time

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

LIM = 2 ** 31


def per_tile_err(a, b):
    d = (a - b).flatten(1).double().norm(dim=1)
    n = b.flatten(1).double().norm(dim=1).clamp_min(1e-30)
    return (d / n).cpu()


def summarise(name, a, b, numel_per_tile, boundary_elems=LIM):
    e = per_tile_err(a, b)
    t0 = -(-boundary_elems // numel_per_tile)       # first tile whose elements start past 2^31
    lo, hi = e[:t0], e[t0:]
    return dict(op=name, per_tile_elems=numel_per_tile, boundary_tile=int(t0) if t0 < len(e) else None,
                max=float(e.max()), argmax=int(e.argmax()), mean=float(e.mean()),
                exact_tiles=int((e == 0).sum()),
                max_below=float(lo.max()) if len(lo) else None, max_above=float(hi.max()) if len(hi) else None,
                mean_below=float(lo.mean()) if len(lo) else None, mean_above=float(hi.mean()) if len(hi) else None)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", type=int, default=4096)
    ap.add_argument("--chunk", type=int, default=512)
    ap.add_argument("--ref-tiles", default="0,1,2000,2674,2675,3000,4000,4095")
    a = ap.parse_args()
    from golden_util import deterministic_encoder_params_
    from transmil_deepgraft_amd.encoder import retccl_resnet50
    torch.backends.cudnn.allow_tf32 = False
    torch.backends.cuda.matmul.allow_tf32 = False
    dev = torch.device("cuda")
    enc = retccl_resnet50()
    deterministic_encoder_params_(enc, 2021)
    enc = enc.set_compute_dtype(torch.float32).eval().to(dev)
    sd_cpu = {k: v.detach().cpu() for k, v in enc.state_dict().items()}
    enc._fold_all()
    f = enc._folded
    g = torch.Generator(device=dev).manual_seed(4096)
    tiles = torch.randn(1, a.tiles, 3, 224, 224, device=dev, generator=g)[0]
    cl = torch.channels_last
    x0 = tiles.contiguous(memory_format=cl)
    N, ch = a.tiles, a.chunk

    def pieces(fn, *xs):
        return torch.cat([fn(*[t[s:s + ch] for t in xs]) for s in range(0, N, ch)]).contiguous(memory_format=cl)

    def conv(x, w, b, stride=1, padding=0):
        return F.conv2d(x, w, b, stride=stride, padding=padding).contiguous(memory_format=cl)

    def c1x1(x, w, b, relu, stride=1):       # the e545b33 1x1 path: one addmm over [n*h*w, c] rows
        if stride != 1:
            x = x[:, :, ::stride, ::stride].contiguous(memory_format=cl)
        n, c, h, wd = x.shape
        X = x.permute(0, 2, 3, 1).reshape(n * h * wd, c)
        W = w.reshape(w.shape[0], c).t()
        Y = torch._addmm_activation(b, X, W) if relu else torch.addmm(b, X, W)
        return Y.view(n, h, wd, -1).permute(0, 3, 1, 2)

    ops = []
    t_start = time.time()

    def step(name, fn, *xs):
        """one op on the piecewise chain's current tensors: one pass vs pieces, compared per tile"""
        with torch.no_grad():
            one = fn(*xs)
            pw = pieces(fn, *xs)
        torch.cuda.synchronize()
        per = max([one[:1].numel()] + [t[:1].numel() for t in xs])
        ops.append(summarise(name, one, pw, per))
        print(f"# {name}: max {ops[-1]['max']:.3e} below {ops[-1]['max_below']} above {ops[-1]['max_above']} "
              f"({time.time() - t_start:.0f} s)", file=sys.stderr, flush=True)
        del one
        return pw

    w, b = f["stem"]
    x = step("stem conv 7x7/2 (+bias)", lambda t: conv(t, w, b, 2, 3), x0)
    x = step("relu", lambda t: F.relu(t), x)
    x = step("max_pool 3/2", lambda t: F.max_pool2d(t, 3, 2, 1).contiguous(memory_format=cl), x)
    for bi, ((w1, b1), (w2, b2, s2), (w3, b3), d) in enumerate(f["blocks"]):
        y = step(f"block{bi} conv1 1x1 addmm+relu", lambda t: c1x1(t, w1, b1, True), x)
        y = step(f"block{bi} conv2 3x3 (+bias)+relu", lambda t: F.relu(conv(t, w2, b2, s2, 1)), y)
        y = step(f"block{bi} conv3 1x1 addmm", lambda t: c1x1(t, w3, b3, False), y)
        if d is not None:
            idt = step(f"block{bi} downsample 1x1 addmm", lambda t: c1x1(t, d[0], d[1], False, d[2][0]), x)
        else:
            idt = x
        # add + ReLU (e545b33: tm_add_relu; torch here -- elementwise, no reduction order)
        x = step(f"block{bi} add+relu", lambda u, v: F.relu(u + v), y, idt)
        del y, idt
    feats_pw = torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
    del x

    # the whole one-pass chain (each op on the one-pass chain's own tensors)
    with torch.no_grad():
        x = F.max_pool2d(F.relu(conv(x0, w, b, 2, 3)), 3, 2, 1).contiguous(memory_format=cl)
        for (w1, b1), (w2, b2, s2), (w3, b3), d in f["blocks"]:
            y = c1x1(x, w1, b1, True)
            y = F.relu(conv(y, w2, b2, s2, 1))
            y = c1x1(y, w3, b3, False)
            idt = x if d is None else c1x1(x, d[0], d[1], False, d[2][0])
            x = F.relu(y + idt).contiguous(memory_format=cl)
        feats_one = torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
    torch.cuda.synchronize()
    chain = per_tile_err(feats_one, feats_pw)
    from oracle.encoder_ref import features
    idx = [int(t) for t in a.ref_tiles.split(",") if int(t) < N]
    ref = features(tiles[idx].cpu(), sd_cpu)
    e_one = per_tile_err(feats_one[idx].cpu(), ref)
    e_pw = per_tile_err(feats_pw[idx].cpu(), ref)
    out = dict(tiles=N, chunk=ch, ops=ops,
               chain_one_vs_pieces=dict(max=float(chain.max()), argmax=int(chain.argmax()), mean=float(chain.mean()),
                                        max_below_2675=float(chain[:2675].max()),
                                        max_above_2675=float(chain[2675:].max()) if N > 2675 else None),
               vs_fp64={str(t): dict(one_pass=float(e_one[i]), pieces=float(e_pw[i])) for i, t in enumerate(idx)},
               torch=torch.__version__, seconds=round(time.time() - t_start, 1))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
