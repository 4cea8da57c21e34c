"""A3 forward with and without the fused A2 rows, and the standalone A2 kernel, in graph replay
(diagnostic timing; bench shape nbh 8, n' 8448)."""
import os, sys
sys.path.insert(0, os.getcwd())
import torch
from transmil_deepgraft_amd import _lib
from transmil_deepgraft_amd._lib import BF16
from transmil_deepgraft_amd.engine import _p, _stream
sys.path.insert(0, os.path.join(os.getcwd(), "scripts"))
from microbench import timeit
nbh, n, dev = 8, 8448, "cuda"
g = torch.Generator(device="cpu").manual_seed(1)
ql = (torch.randn(nbh, 256, 64, generator=g) * 0.3).to(dev)
kl = (torch.randn(nbh, 256, 64, generator=g) * 0.3).to(dev)
k = (torch.randn(nbh, n, 64, generator=g) * 0.3).to(torch.bfloat16).to(dev)
v = torch.randn(nbh, n, 64, generator=g).to(torch.bfloat16).to(dev)
work = torch.empty(_lib.query("tm_nys_a3_workspace", nbh, n) // 4 + 16, device=dev)
a2 = torch.empty(nbh, 256, 256, device=dev)
a2s = torch.empty(nbh, 256, 256, device=dev)
cases = {
    "a3_fwd + A2 rows (bench form)": lambda: _lib.call("tm_nys_a3_fwd_sim2", _p(ql), _p(kl), _p(k), _p(v), nbh, n,
                                                       _p(work), _p(a2), _p(a2s), _stream()),
    "a3_fwd partials only": lambda: _lib.call("tm_nys_a3_fwd", BF16, _p(ql), _p(k), _p(v), nbh, n, _p(work), None,
                                              None, _stream()),
    "A2 split kernel alone": lambda: _lib.call("tm_nys_sim2_softmax_split", _p(ql), _p(kl), nbh, _p(a2), _p(a2s),
                                               _stream()),
}
for name, fn in cases.items():
    print(f"{name:40s} {timeit(fn, 50):8.2f} us", flush=True)
