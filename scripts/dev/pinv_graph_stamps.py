"""Phase stamps of the split pseudo-inverse chain (pinv_split.hip) under hipGraph REPLAY, as the bench
runs it: the forward chain (tm_pinv_fwd_split: 14 launches) and the backward
chain (tm_pinv_bwd_split: 24 stage launches + the apply launch), each captured once with the
diagnostic build's stamp buffer armed, replayed 6 times; the last replay's stamps are read.

Per stage launch, from the consumer waves' stamps (pinv_split.hip stage_tile ts[0..7]):
  start   first workgroup's s_memrealtime (100 MHz) - previous launch's last end = the boundary
  span    last end - first start
  setup   ts1 -> ts2   (epilogue-operand loads issued, fragment addresses)
  fill0   ts2 -> ts3   (first chunk landed: the operand fill latency)
  chunk0  ts3 -> ts4   (first chunk's MFMAs)
  rest    ts4 -> ts5   (remaining chunks: fill-paced k-walk)
  epi     ts5 -> ts6   (accumulator staging, epilogue arithmetic, output stores issued)
in shader cycles (s_memtime; converted to us with the measured cycles per realtime tick).

    python scripts/dev/pinv_graph_stamps.py [--nbh 8]     (diagnostic build: make -C transmil_deepgraft_amd/csrc diag)
"""
import argparse
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

ITERS = 6


def fwd_wgs(nbh):
    t16 = 16 * nbh
    out = [2 * t16]                                   # L1: S = X X^T (+ the abs-sum job, unstamped)
    for lvl in range(2 * ITERS + 1):
        if lvl == 2 * ITERS:
            nj = 1
        else:
            k = lvl >> 1
            nj = (2 if k >= 1 else 1) if lvl % 2 == 0 else (2 if k + 1 < ITERS else 1)
        out.append(nj * t16)
    return out


def bwd_wgs(nbh):
    t16 = 16 * nbh
    return [(1 if (lvl & 3) == 2 else 2) * t16 for lvl in range(4 * ITERS)]


def analyse(buf, wgs, title, ratio=None):
    a = buf.cpu().numpy().astype(np.int64)
    off, prev_end = 0, None
    rows = []
    for li, nwg in enumerate(wgs):
        seg = a[off:off + nwg * 32].reshape(nwg, 4, 8)
        off += nwg * 32
        seg = seg[seg[:, 0, 7] > 0]
        rt0, rt1 = seg[:, :, 0].min(), seg[:, :, 7].max()
        d = np.diff(seg[:, :, 1:7], axis=2)          # [wg, wave, 5] shader cycles
        med = [float(np.median(d[:, :, i])) for i in range(5)]
        if ratio is None:
            r = (seg[:, :, 6] - seg[:, :, 1]) / np.maximum(seg[:, :, 7] - seg[:, :, 0], 1)
            ratio = float(np.median(r))               # shader cycles per 10 ns realtime tick
        gap = (rt0 - prev_end) / 100.0 if prev_end is not None else float("nan")
        rows.append(dict(launch=li, wgs=int(nwg), gap_us=gap, span_us=(rt1 - rt0) / 100.0,
                         start_spread_us=(seg[:, :, 0].max() - rt0) / 100.0,
                         **{n: m / ratio / 100.0 for n, m in zip(("setup", "fill0", "chunk0", "rest", "epi"), med)}))
        prev_end = rt1
    print(f"== {title}: {len(wgs)} stage launches, {ratio * 100:.0f} shader cycles per us")
    print(f"{'launch':>6} {'wgs':>4} {'gap':>6} {'span':>6} {'spread':>6} {'setup':>6} {'fill0':>6} {'chunk0':>6} "
          f"{'rest':>6} {'epi':>6}   (us; phases = medians over consumer waves)")
    for r in rows:
        print(f"{r['launch']:>6} {r['wgs']:>4} {r['gap_us']:6.2f} {r['span_us']:6.2f} {r['start_spread_us']:6.2f} "
              f"{r['setup']:6.2f} {r['fill0']:6.2f} {r['chunk0']:6.2f} {r['rest']:6.2f} {r['epi']:6.2f}")
    tot = {k: sum(r[k] for r in rows if not np.isnan(r[k])) for k in ("gap_us", "span_us")}
    print(f"   sum of gaps {tot['gap_us']:.1f} us, sum of spans {tot['span_us']:.1f} us")
    return rows, ratio


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nbh", type=int, default=8)
    ap.add_argument("--ab", default="", help="comma list of diagnostic split variants to A/B by graph replay "
                                             "(e.g. 0,6: 6 = write-through epilogue stores)")
    ap.add_argument("--variant", type=int, default=0, help="split variant of the stamped run")
    args = ap.parse_args()
    dev, nbh = "cuda", args.nbh
    st = E._stream
    torch.manual_seed(0)
    X = torch.softmax(torch.randn(nbh, 256, 256, device=dev) * 3, -1)
    Xs = torch.empty(2 * nbh * 65536, dtype=torch.bfloat16, device=dev)
    _lib.call("tm_split_f32", E._p(X), E._p(Xs), nbh * 65536, st())
    saved = torch.empty(_lib.query("tm_pinv_split_saved_floats", nbh, ITERS), device=dev)
    work = torch.zeros(_lib.query("tm_pinv_bwd_split_workspace_floats", nbh), device=dev)
    out = torch.empty(nbh, 256, 256, device=dev)
    dz = torch.randn(nbh, 256, 256, device=dev) * 1e-3
    dzs = torch.empty(2 * nbh * 65536, dtype=torch.bfloat16, device=dev)
    _lib.call("tm_split_f32", E._p(dz), E._p(dzs), nbh * 65536, st())
    L = _lib.lib()

    def fwd():
        _lib.call("tm_pinv_fwd_split", E._p(X), E._p(Xs), nbh, ITERS, E._p(saved), st())

    def bwd():
        work[:nbh * 65536].view(torch.bfloat16).copy_(dzs)
        _lib.call("tm_pinv_bwd_split", E._p(X), E._p(Xs), nbh, ITERS, E._p(saved), E._p(work), 1, E._p(out), st())

    fwd()
    bwd()
    torch.cuda.synchronize()
    if args.ab:
        vs = [int(v) for v in args.ab.split(",")]
        graphs = {}
        for v in vs:
            L.tm_debug_set_split_variant(v)
            for nm, fn in (("fwd", fwd), ("bwd", bwd)):
                fn()
                torch.cuda.synchronize()
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    fn()
                graphs[v, nm] = g
        L.tm_debug_set_split_variant(0)
        res = {k: [] for k in graphs}
        for rnd in range(7):          # interleaved rounds, 20 replays each
            for k, g in graphs.items():
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(20):
                    g.replay()
                e.record()
                torch.cuda.synchronize()
                res[k].append(s.elapsed_time(e) * 1e3 / 20)
        for k, xs in res.items():
            print(f"A/B variant {k[0]} {k[1]}: median {np.median(xs):.2f} us  (min {min(xs):.2f})")
    L.tm_debug_set_split_variant(args.variant)
    results = {}
    ratio = None
    for name, fn, wgs in (("forward chain (tm_pinv_fwd_split)", fwd, fwd_wgs(nbh)),
                          ("backward chain (tm_pinv_bwd_split)", bwd, bwd_wgs(nbh))):
        buf = torch.zeros(sum(wgs) * 32 + 64, dtype=torch.int64, device=dev)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            fwd()                    # the saved forward state both graphs read
            fn()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        g_plain, g_st = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.graph(g_plain):
            fn()
        L.tm_debug_set_split_stamps(C.c_void_p(buf.data_ptr()))
        try:
            with torch.cuda.graph(g_st):
                fn()
        finally:
            L.tm_debug_set_split_stamps(None)
        # whole-chain event timing of the graph without / with stamps (median of 9 replays)
        def ev(g):
            ts = []
            for _ in range(9):
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                g.replay()
                e.record()
                torch.cuda.synchronize()
                ts.append(s.elapsed_time(e) * 1e3)
            return float(np.median(ts))
        t_plain, t_st = ev(g_plain), ev(g_st)
        buf.zero_()
        for _ in range(6):
            g_st.replay()
        torch.cuda.synchronize()
        rows, ratio = analyse(buf, wgs, name, ratio)
        print(f"   graph replay: {t_plain:.1f} us without stamps, {t_st:.1f} us with stamps "
              f"({t_plain / len(wgs):.2f} us per stage launch incl. the apply launch share)")
        results[name] = dict(rows=rows, graph_us=t_plain, graph_stamped_us=t_st)
    import json
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "pinv_graph_stamps.json"), "w") as f:
        json.dump(results, f, indent=1)


if __name__ == "__main__":
    main()
