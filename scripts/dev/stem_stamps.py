"""Phase stamps of tm_stem_conv_pool (diagnostic build, variant 1): per workgroup of the first 4096,
shader-clock cycles from start to staged / k loop done / conv tile stored / pool stores issued,
and the realtime (100 MHz) span -> how many workgroups overlap per CU.

    TRANSMIL_HIP_LIB=transmil_deepgraft_amd/libtransmil_hip_diag.so python scripts/dev/stem_stamps.py
"""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.getcwd())
from transmil_deepgraft_amd import _lib                  # noqa: E402
import transmil_deepgraft_amd.encoder as E               # noqa: E402

L = _lib.lib()
n = 1024
x = torch.randn(n, 3, 224, 224, device="cuda").to(torch.bfloat16)
w = (torch.randn(64, 3, 7, 7, device="cuda") * 0.1).to(torch.bfloat16)
b = (torch.randn(64, device="cuda") * 0.1).to(torch.bfloat16)
wp = E._pack_stem(w)
for _ in range(3):
    E._stem_conv_pool(x, wp, b)
L.tm_debug_set_stem_variant(1)
E._stem_conv_pool(x, wp, b)
torch.cuda.synchronize()
L.tm_debug_set_stem_variant(0)
buf = (C.c_ulonglong * (4096 * 8))()
assert L.tm_debug_stem_stamps(buf, 4096 * 8) == 0
a = np.frombuffer(buf, dtype=np.uint64).reshape(4096, 8).astype(np.int64)
a = a[a[:, 0] != 0]
d = a[:, 2:6] - a[:, 1:2]
ph = np.diff(np.concatenate([np.zeros((len(a), 1), np.int64), d], axis=1), axis=1)
print("cycles per phase (median / p90): staged, k loop, conv tile, pool")
for i, nm in enumerate(["staged", "k loop", "conv tile", "pool"]):
    print(f"  {nm:10s} {np.median(ph[:, i]):8.0f} {np.percentile(ph[:, i], 90):8.0f}")
rt = a[:, 6] - a[:, 0]
print(f"realtime span per workgroup: median {np.median(rt) * 10:.0f} ns; first-4096 window "
      f"{(a[:, 6].max() - a[:, 0].min()) * 10 / 1000:.1f} us")
