"""test_c5_full_bag_4096_tiles's bitwise check in isolation: bf16 eval encoder over a 4096-tile bag
in one call (512-tile pieces inside) vs 8 calls of 512 tiles; prints which tiles differ.

    [TM_STEM_FUSED=0] [TM_CONV1X1_TUNE=0] python scripts/dev/c5_whole_vs_chunks.py
"""
import os
import sys

import torch

sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
from test_encoder import _encoder                    # noqa: E402

enc = _encoder(torch.bfloat16).cuda()
g = torch.Generator(device="cuda").manual_seed(4096)
tiles = torch.randn(1, 4096, 3, 224, 224, device="cuda", generator=g)
torch.backends.cudnn.deterministic = os.environ.get("DET", "0") == "1"
reps = int(os.environ.get("REPS", "1"))
with torch.no_grad():
    whole = enc(tiles[0])
    outs = [torch.cat([enc(tiles[0, s:s + 512]) for s in range(0, 4096, 512)])]
    outs += [enc(tiles[0]) for _ in range(reps)]
torch.cuda.synchronize()
msg = []
for i, o in enumerate(outs):
    bad = (whole != o).any(dim=1).nonzero().flatten().tolist()
    msg.append(f"{'chunks' if i == 0 else 'whole#%d' % i}: {len(bad)} {bad[:6]}")
print(f"stem_fused={os.environ.get('TM_STEM_FUSED', '1')} tune={os.environ.get('TM_CONV1X1_TUNE', '1')} "
      f"det={torch.backends.cudnn.deterministic}: differing tiles vs the first whole run -- " + "; ".join(msg))
