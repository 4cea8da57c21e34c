"""PPEG backward (data stencil + weight gradient + reduce) per wgrad tiles-per-block WT (diagnostic build)."""
import os, sys
sys.path.insert(0, os.getcwd())
os.environ.setdefault("TRANSMIL_HIP_LIB", os.path.join(os.getcwd(), "transmil_deepgraft_amd", "libtransmil_hip_diag.so"))
import runpy
import torch
from transmil_deepgraft_amd import _lib
ns = {}
src = open("scripts/dev/ppeg_time.py").read().split("mb = S * D")[0]
exec(src, ns)
ref = None
for wt in (4, 2, 1, 3, 6, 12):
    _lib.lib().tm_debug_set_ppeg_wt(wt)
    ns["bwd"](); torch.cuda.synchronize()
    g = ns["g7"].clone()
    if ref is None: ref = g
    err = ((g - ref).abs().max() / ref.abs().max()).item()
    print(f"WT {wt:2d}: bwd {ns['timeit'](ns['bwd']):6.2f} us  (dw7 vs WT 4: {err:.1e})", flush=True)
_lib.lib().tm_debug_set_ppeg_wt(0)
