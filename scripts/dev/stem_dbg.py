import os, sys, torch
import torch.nn.functional as F
sys.path.insert(0, os.getcwd())
import transmil_deepgraft_amd.encoder as E
g = torch.Generator(device="cpu").manual_seed(1)
for (h, w) in [(64, 64), (224, 224)]:
    x = torch.randn(1, 3, h, w, generator=g).to(torch.bfloat16).cuda()
    wt = (torch.randn(64, 3, 7, 7, generator=g) * 0.1).to(torch.bfloat16).cuda()
    b = (torch.randn(64, generator=g) * 0.1).to(torch.bfloat16).cuda()
    ref = F.max_pool2d(F.relu(F.conv2d(x.float(), wt.float(), b.float(), stride=2, padding=3)), 3, 2, 1)
    out = E._stem_conv_pool(x, E._pack_stem(wt), b).float()
    bad = (out - ref).abs() > ref.abs() * 2 ** -8 + 1e-5
    print(h, w, "bad", bad.sum().item(), "of", bad.numel())
    idx = bad.nonzero()
    if len(idx):
        print("channels", sorted(set(idx[:, 1].tolist()))[:40])
        print("rows", sorted(set(idx[:, 2].tolist()))[:40])
        print("cols", sorted(set(idx[:, 3].tolist()))[:40])
        i = idx[0].tolist()
        print("first", i, out[tuple(i)].item(), ref[tuple(i)].item())
