"""Per-phase s_memtime stamps of the bf16 A3 forward (a3_fwd_v2_kernel) at the bench shape
(diagnostic build, variant 32): slots 0 start, 1 chunk-0 loads + query fragments issued, 2 chunk 0
staged, 3 chunk 0 computed, 4 chunk 1 staged, 5 key loop done, 6 partials stored (waitcnt 0).
Prints mean / max cycle deltas over workgroups for each wave."""
import ctypes as C, os, sys, time
sys.path.insert(0, os.getcwd())
os.environ.setdefault("TRANSMIL_HIP_LIB", os.path.join(os.getcwd(), "transmil_deepgraft_amd", "libtransmil_hip_diag.so"))
import numpy as np
import torch
from transmil_deepgraft_amd import _lib
from transmil_deepgraft_amd._lib import BF16
from transmil_deepgraft_amd.engine import _p, _stream
nbh, n = 8, 8448
dev = "cuda"
g = torch.Generator(device="cpu").manual_seed(1)
ql = (torch.randn(nbh, 256, 64, generator=g) * 0.3).to(dev)
k = (torch.randn(nbh, n, 64, generator=g) * 0.3).to(torch.bfloat16).to(dev)
v = torch.randn(nbh, n, 64, generator=g).to(torch.bfloat16).to(dev)
work = torch.empty(_lib.query("tm_nys_a3_workspace", nbh, n) // 4 + 16, device=dev)
f = lambda: _lib.call("tm_nys_a3_fwd", BF16, _p(ql), _p(k), _p(v), nbh, n, _p(work), _p(None), _p(None), _stream())
if os.environ.get("A3_SIM2", "0") == "1":   # the bench's form: the fused A2 rows (tm_nys_a3_fwd_sim2)
    kl = (torch.randn(nbh, 256, 64, generator=g) * 0.3).to(dev)
    a2 = torch.empty(nbh, 256, 256, device=dev)
    a2s = torch.empty(nbh, 256, 256, device=dev)
    f = lambda: _lib.call("tm_nys_a3_fwd_sim2", _p(ql), _p(kl), _p(k), _p(v), nbh, n, _p(work), _p(a2), _p(a2s),
                          _stream())
STV = 32
for var in (0, STV):
    _lib.lib().tm_debug_set_variant(1, var)
    for _ in range(3): f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(50): f()
    torch.cuda.synchronize()
    print(f"variant {var}: {(time.perf_counter() - t) / 50 * 1e6:.1f} us per call (eager)", flush=True)
P = _lib.query("tm_nys_a3_partials", nbh, n)
nblk = P * nbh
buf = (C.c_ulonglong * (512 * 8 * 8))()
_lib.call("tm_debug_a1_stamps", buf, 512 * 8 * 8)
a = np.frombuffer(buf, dtype=np.uint64).reshape(512, 8, 8)[:nblk].astype(np.int64)
for w in range(8):
    st = a[:, w, :7]
    d = np.diff(st, axis=1)
    print(f"wave {w}: mean cycles per phase", [int(x) for x in d.mean(0)], " max", [int(x) for x in d.max(0)])
    if os.environ.get("A3_SIM2", "0") == "1":
        print(f"   A2 tail: key loop done -> k~ staged {int((a[:, w, 7] - a[:, w, 5]).mean())}, k~ staged -> end "
              f"{int((a[:, w, 6] - a[:, w, 7]).mean())} cycles (means)")
    print(f"   total mean {int((st[:, 6] - st[:, 0]).mean())} cycles; start spread {int(st[:, 0].max() - st[:, 0].min())}"
          f"; end spread {int(st[:, 6].max() - st[:, 6].min())}; first start to last end {int(st[:, 6].max() - st[:, 0].min())}")
_lib.lib().tm_debug_set_variant(1, 0)
