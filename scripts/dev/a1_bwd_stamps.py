"""Per-phase s_memtime stamps of the bf16 A1 backward (attn_bwd_bf16_kernel<A1, 8>) at the bench shape
(diagnostic build; nys variant 33: slots 0 start, 1 loads issued, 2 operands staged, 3 after query
chunk 0, 4 after chunk 3, 5 after the query walk, 6 end (slab epilogue done); variant 34: inside
query chunk 2: 0 chunk start, 1 S / dP / dV / dK done, 2 after barrier 1, 3 after the dS write +
barrier 2, 4 dQ MFMAs + partials, 5 after barrier 3, 6 dq stored).  Prints mean / max cycle deltas
over workgroups for waves 0 and 4, and the eager time per call of the plain kernel.

    TRANSMIL_HIP_LIB=transmil_deepgraft_amd/libtransmil_hip_diag.so python scripts/dev/a1_bwd_stamps.py
"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.getcwd())
os.environ.setdefault("TRANSMIL_HIP_LIB", os.path.join(os.getcwd(), "transmil_deepgraft_amd", "libtransmil_hip_diag.so"))
import numpy as np            # noqa: E402
import torch                  # noqa: E402
from transmil_deepgraft_amd import _lib                    # noqa: E402
from transmil_deepgraft_amd.engine import _p, _stream      # noqa: E402

nh, n, B = 8, 8448, 1
nbh = B * nh
dev = "cuda"
g = torch.Generator(device="cpu").manual_seed(1)
q = (torch.randn(B, nh, n, 64, generator=g) * 0.3).to(torch.bfloat16).to(dev)
dmerged = (torch.randn(B, n, nh * 64, generator=g) * 0.1).to(torch.bfloat16).to(dev)
kl = (torch.randn(B, nh, 256, 64, generator=g) * 0.3).to(torch.bfloat16).to(dev)
y = (torch.randn(B, nh, 256, 64, generator=g) * 0.3).to(torch.bfloat16).to(dev)
lse = torch.randn(nbh, n, device=dev) + 6
d1 = torch.randn(nbh, n, device=dev) * 0.01
dqkv = torch.empty(B, n, 3 * nh * 64, dtype=torch.bfloat16, device=dev)
work = torch.empty(_lib.query("tm_nys_a1_bwd_workspace", nbh, n, 256) // 4 + 16, device=dev)
dkl = torch.empty(nbh, 256, 64, device=dev)
dy = torch.empty(nbh, 256, 64, device=dev)
f = lambda: _lib.call("tm_nys_a1_bwd_dqkv", _p(q), _p(dmerged), _p(kl), _p(y), _p(lse), _p(d1), nbh, nh, n, _p(dqkv),
                      C.c_float(0.125), _p(work), _p(dkl), _p(dy), None, _stream())
L = _lib.lib()
for var in [0] + [int(x) for x in (sys.argv[1:] or ["33", "34"])]:
    L.tm_debug_set_nys_variant(var)
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(50):
        f()
    torch.cuda.synchronize()
    print(f"variant {var}: {(time.perf_counter() - t) / 50 * 1e6:.1f} us per call (eager, incl. the two slab reduces)",
          flush=True)
    if var not in (33, 34):
        continue
    nblk = 32 * nbh
    buf = (C.c_ulonglong * (512 * 8 * 8))()
    _lib.call("tm_debug_a1_stamps", buf, 512 * 8 * 8)
    a = np.frombuffer(buf, dtype=np.uint64).reshape(512, 8, 8)[:nblk].astype(np.int64)
    for w in (0, 4):
        st = a[:, w, :]
        d = np.diff(st, axis=1)
        print(f"  wave {w}: mean cycles per phase", [int(x) for x in d.mean(0)], " max", [int(x) for x in d.max(0)])
        print(f"     total mean {int((st[:, 6] - st[:, 0]).mean())} cycles; start spread {int(st[:, 0].max() - st[:, 0].min())}")
L.tm_debug_set_nys_variant(0)
