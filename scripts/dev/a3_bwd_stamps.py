"""Per-phase (A3_STAMPS=31: slots 0 chunk start, 1 S/dP/dV/dK done, 2 after barrier 1, 3 after the dS
write + barrier 2, 4 dQ done, 5 after barrier 3, 6 dq~ partial stored) s_memtime stamps of the bf16 A3 backward at the bench shape (diagnostic build, variant 30):
slots 0 start, 1 loads issued, 2 operands staged, 3 after query chunk 0, 4 after chunk 3, 5 after
the query walk, 6 end (key-side epilogue done).  Prints mean / max cycle deltas over workgroups (wave 0)."""
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
ql = (torch.randn(nbh, 256, 64, generator=g) * 0.3).to(torch.bfloat16).to(dev)
dw = (torch.randn(nbh, 256, 64, generator=g) * 0.1).to(torch.bfloat16).to(dev)
k = (torch.randn(nbh, n, 64, generator=g) * 0.3).to(torch.bfloat16).to(dev)
v = torch.randn(nbh, n, 64, generator=g).to(torch.bfloat16).to(dev)
lse = torch.randn(nbh, 256, device=dev) + 9
d = torch.randn(2, nbh, 256, device=dev) * 0.01
dk = torch.empty(nbh, n, 64, device=dev)
dv = torch.zeros(nbh, n, 64, device=dev)
dql = torch.empty(nbh, 256, 64, device=dev)
work = torch.empty(_lib.query("tm_nys_a3_bwd_workspace", nbh, n) // 4 + 16, device=dev)
dvc = torch.randn(nbh, n, 64, device=dev) * 0.01
dkl = torch.randn(nbh, 256, 64, device=dev) * 0.01
dqkv = torch.empty(1, n, 3 * 512, dtype=torch.bfloat16, device=dev)
if os.environ.get("A3_FUSED", "1") == "1":   # the bench's form: bf16 k / v rows of dqkv straight from the kernel
    f = lambda: _lib.call("tm_nys_a3_bwd_fused", _p(ql), _p(dw), _p(k), _p(v), _p(lse), _p(d), nbh, 8, n, _p(dvc),
                          0, n, _p(dkl), _p(work), _p(dql), _p(dqkv), None, _stream())
else:
    f = lambda: _lib.call("tm_nys_a3_bwd", BF16, _p(ql), _p(dw), _p(k), _p(v), _p(lse), _p(d), nbh, 8, n, _p(dk),
                          _p(dv), _p(work), _p(dql), 0, None, _stream())
STV = int(os.environ.get("A3_STAMPS", "30"))   # 30: phases; 31: inside query chunk 2
for var in (0, STV):
    _lib.lib().tm_debug_set_variant(1, var)
    for _ in range(3): f()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(50): f()
    torch.cuda.synchronize()
    print(f"variant {var}: {(time.perf_counter() - t) / 50 * 1e6:.1f} us per call (eager, incl. the dq~ reduce)", flush=True)
nblk = 32 * nbh
buf = (C.c_ulonglong * (512 * 8 * 8))()
_lib.call("tm_debug_a1_stamps", buf, 512 * 8 * 8)
a = np.frombuffer(buf, dtype=np.uint64).reshape(512, 8, 8)[:nblk].astype(np.int64)
for w in (0, 4):
    st = a[:, w, :]
    d = np.diff(st, axis=1)
    print(f"wave {w}: mean cycles per phase", [int(x) for x in d.mean(0)], " max", [int(x) for x in d.max(0)])
    print(f"   total mean {int((st[:, 6] - st[:, 0]).mean())} cycles; start spread {int(st[:, 0].max() - st[:, 0].min())}")
_lib.lib().tm_debug_set_variant(1, 0)
