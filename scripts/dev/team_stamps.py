"""Per-level timeline of the persistent pseudo-inverse chain (pinv_team_kernel, diagnostic build variant 8):
for every ticket the claim / operands-ready / done times (s_memrealtime, 100 MHz) and the stage
stamps (s_memtime cycles) of its four consumer waves."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ.setdefault("TRANSMIL_HIP_LIB", os.path.join(ROOT, "transmil_deepgraft_amd", "libtransmil_hip_diag.so"))
from transmil_deepgraft_amd import _lib  # noqa: E402
from transmil_deepgraft_amd import engine as E  # noqa: E402

L = _lib.lib()
L.tm_debug_set_split_variant(8)   # the persistent kernel (diagnostic build only)
dev = "cuda"
nbh = 8
X = torch.softmax(torch.randn(nbh, 256, 256, device=dev), -1)
Xs = torch.empty(2 * nbh * 65536, dtype=torch.bfloat16, device=dev)
_lib.call("tm_split_f32", E._p(X), E._p(Xs), nbh * 65536, E._stream())
saved = torch.empty(_lib.query("tm_pinv_split_saved_floats", nbh, 6), device=dev)
work = torch.zeros(_lib.query("tm_pinv_bwd_split_workspace_floats", nbh), device=dev)
out = torch.empty(nbh, 256, 256, device=dev)
buf = torch.zeros(8 * 512 * 40 + 16384, dtype=torch.int64, device=dev)


def run(direction):
    if direction == "fwd":
        _lib.call("tm_pinv_fwd_split", E._p(X), E._p(Xs), nbh, 6, E._p(saved), E._stream())
    else:
        _lib.call("tm_pinv_bwd_split", E._p(X), E._p(Xs), nbh, 6, E._p(saved), E._p(work), 1, E._p(out), E._stream())


teams = {}
for direction in ("fwd", "bwd"):
    for rep in range(4):
        run("fwd")
        torch.cuda.synchronize()
        if direction == "bwd":
            work[:nbh * 65536].normal_(0, 1e-3)
        buf.zero_()
        L.tm_debug_set_split_stamps(C.c_void_p(buf.data_ptr()))
        run(direction)
        L.tm_debug_set_split_stamps(None)
        torch.cuda.synchronize()
    off = 256 * 32 if direction == "fwd" else 0    # the forward's L1 launch stamps come first
    a = buf.cpu().numpy()[off:off + 8 * 512 * 40].reshape(8 * 512, 40)
    a = a[a[:, 34] > 0]
    teams[direction] = a.copy()
    t0 = a[:, 32].min()
    lev = a[:, 36]
    print(f"{direction}: {len(a)} tile-jobs, span {(a[:, 34].max() - t0) / 100:.2f} us")
    prev_end = t0
    for lv in range(int(lev.max()) + 1):
        s = a[lev == lv]
        if len(s) == 0:
            continue
        ready, end = s[:, 33], s[:, 34]
        st = s[:, :32].reshape(-1, 4, 8)
        d = np.diff(st[:, :, 1:7].astype(np.int64), axis=2)   # setup, wait c0, chunk0, chunks1+, epilogue
        med = [int(np.median(d[:, :, i])) for i in range(5)]
        print(f"  level {lv:2d} ({len(s):3d} tiles): ready p50 {(np.median(ready) - prev_end) / 100:5.2f} us after the "
              f"previous level's last done; tile span p50 {np.median(end - ready) / 100:5.2f} max "
              f"{(end - ready).max() / 100:5.2f} us; level done +{(end.max() - prev_end) / 100:5.2f} us | cycles "
              f"setup {med[0]} waitc0 {med[1]} chunk0 {med[2]} chunks1+ {med[3]} epi {med[4]}")
        prev_end = end.max()


print("per team (XCD): median over teams of the gap between a level's last done and the next level's first ready,")
print("and of the level span (first ready -> last done)")
for direction, a in teams.items():
    nl = int(a[:, 36].max()) + 1
    gaps, spans = np.zeros((8, nl)), np.zeros((8, nl))
    for x in range(8):
        b = a[a[:, 35] == x]
        prev = None
        for lv in range(nl):
            s_ = b[b[:, 36] == lv]
            if len(s_) == 0:
                continue
            spans[x, lv] = (s_[:, 34].max() - s_[:, 33].min()) / 100
            gaps[x, lv] = (s_[:, 33].min() - prev) / 100 if prev is not None else np.nan
            prev = s_[:, 34].max()
    print(direction, "gap  ", " ".join(f"{v:5.2f}" for v in np.nanmedian(gaps, axis=0)))
    print(direction, "span ", " ".join(f"{v:5.2f}" for v in np.median(spans, axis=0)))
