"""Benchmark: TransMIL training-step throughput (slides/sec, fwd+bwd) on MI355X.

BASELINE.json metric: "slides/sec (fwd+bwd) at N=8192 patches, d=512; 1/2/4/8 MI355X".
Workload (configs[1]): TransMIL_feat 2-class, one synthetic bag of N=8192 x 512
features per GPU per step, bf16 MFMA operands (fp32 softmax / LayerNorm /
pseudo-inverse / residual stream / master weights).

One step = forward (train mode, dropout 0.7 active) -> CrossEntropy(one-hot)
-> backward -> gradient all-reduce over ranks (RCCL, N > 1) -> Lookahead(RAdam)
optimizer step -> zero_grad.  Bags are resident in HBM before timing starts.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n 8192]
    torchrun --nproc-per-node N bench.py --gpus N ...     (one process per GPU)

Prints ONE JSON line on rank 0.  Extra objects:
  roofline      -- the dominant kernel's achieved rate: by default the pseudo-inverse
                   forward chain (tm_pinv_fwd_split: 14 launches of pinv_stage_kernel, the
                   largest share of the step in profiles/r02_*_kernel_summary.txt), its
                   algorithmic flops / the HIP-event span of the call on its stream
  gemm_roofline -- the dense projections (to_qkv, to_out, _fc1 and their backward products): per call
                   site and layer, 2 M N K / the same probe's event span, against the dense bf16 peak
  hbm_roofline  -- the HBM-bound NystromAttention / PPEG / LayerNorm kernels (north_star: >= 50 %
                   of HBM roofline): per call site and layer, algorithmic bytes (every compulsory
                   tensor read or written once) / the HIP-event span of the
                   launch in eager probe steps after the timed region (a GPU spin queued ahead, the
                   span of an empty event pair subtracted), against 8 TB/s
  cpu_baseline  -- the fp32 CPU oracle (oracle/transmil_ref.py, logits path) on a
                   bounded sample of the same workload, rank 0 only: median of 5 steps after
                   2 warm-ups at 8 threads (code/train.py:93) and at the box's CPU share
  cpu_baseline_as_written -- the same oracle as the reference is written: every TransLayer also
                   forms the [B, h, n', n'] return_attn product (code/models/TransMIL.py:47)
  optimizer_ms  -- the Lookahead(RAdam) step alone (inside the timed step too)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
import types

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
BF16_PEAK_TFS = 2500.0       # dense bf16 MFMA spec
F32_MATRIX_PEAK_TFS = 157.3  # v_mfma_f32_32x32x2_f32 = the fp32 vector rate (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)   # 20 warm-up, >= 200 timed steps
    ap.add_argument("--warmup", type=int, default=20)
    # --n-patches: the same option under a name torch.distributed.run does not take for its own
    # (it reads a bare --n after the script name as an ambiguous abbreviation of --nnodes / --nproc...)
    ap.add_argument("--n", "--n-patches", dest="n", type=int, default=8192, help="patches per bag")
    ap.add_argument("--classes", type=int, default=2)
    ap.add_argument("--features", type=int, default=512, choices=[512, 2048],
                    help="in_features: 512 (Linear+GELU _fc1, the metric's config) or 2048 (the RCC "
                         "_fc1 branch on RetCCL-width features, config C5 without its encoder)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--accumulate", type=int, default=1,
                    help="accumulate_grad_batches K (code/train.py:199 uses 10 under DDP): a timed step is one "
                         "micro-batch; every K-th one all-reduces and steps the optimizer (C4's every-10-steps row)")
    ap.add_argument("--probe", default="pinv_fwd", help="call site timed for the roofline object")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--eager", action="store_true", help="launch every kernel from Python instead of "
                    "replaying the captured hipGraph of the whole step")
    ap.add_argument("--cpu-steps", type=int, default=5, help="timed CPU steps per thread count (median)")
    ap.add_argument("--no-cpu-as-written", action="store_true",
                    help="skip the CPU oracle timed as the reference is written (the n'xn' return_attn product)")
    ap.add_argument("--no-hbm-probe", action="store_true", help="skip the per-kernel HBM roofline list")
    return ap.parse_args()


def roofline_model(site, n_patches, dtype_bytes):
    """Algorithmic bytes / flops of ONE call of `site`."""
    import math
    G = math.ceil(math.sqrt(n_patches))
    S = G * G + 1
    n = (S + 255) // 256 * 256
    heads, dh, m = 8, 64, 256
    t = dtype_bytes
    if site == "pinv_fwd":
        # 24 products of 256^3 per head (S = X X^T, then per iteration R, T5, P', Z; App. A eq. 7);
        # bytes: every chain matrix read / written once as split bf16 planes (4 B per element)
        mat = heads * m * m * 4
        flops = 24 * heads * 2 * m ** 3
        byts = mat * (1 + 1 + 3 + 6 * 5 + 5 * 5 + 4)   # X; S; A_0 out; B_k/A_k in+out; F
        return dict(bytes=byts, flops=flops, peak_tfs=F32_MATRIX_PEAK_TFS, units=14,
                    note="fp32-class products as bf16 hi/lo x3 on the bf16 MFMA; units = launches per call")
    if site == "pinv_bwd":
        # the adjoint of the chain (pinv_split.hip bwd_level_job), per iteration 8 products of 256^3 per
        # head in 4 launches (dT5, dZa | dP, dT3 | dP += dT3 P^T + P^T dT3 | dX, G; the last one also
        # the c-gradient dot of G0 with X^T), then the apply launch (Z_0 = X^T / c terms + the A2
        # softmax backward); bytes: every operand / addend read and every output written once per
        # level as split bf16 planes (4 B per element; dX fp32): 14 matrices read + 7 written per
        # iteration, X (fp32, the dot), then X, G, dX in + out (apply)
        mat = heads * m * m * 4
        flops = 6 * 8 * heads * 2 * m ** 3
        byts = mat * (6 * (14 + 7) + 1 + 4)
        return dict(bytes=byts, flops=flops, peak_tfs=F32_MATRIX_PEAK_TFS, units=25,
                    note="fp32-class products as bf16 hi/lo x3 on the bf16 MFMA; 24 pinv_stage_kernel launches "
                         "(the last with the c-gradient dot) + pinv_apply_bwd_kernel per call; units = launches per call")
    if site == "a1_fwd":
        # read q, v (conv) [n, 512] T; write merged [n, 512] T + lse [8, n] fp32; landmarks/Y fp32
        byts = 3 * n * 512 * t + heads * n * 4 + 2 * heads * m * dh * 4
        flops = 2 * 2 * heads * n * m * dh + 2 * 33 * heads * n * dh
        return dict(bytes=byts, flops=flops)
    if site == "qkv_gemm":
        byts = n * 512 * t + 1536 * 512 * t + 3 * n * 512 * t
        flops = 2 * n * 512 * 1536
        return dict(bytes=byts, flops=flops)
    if site == "a3_fwd":
        byts = 2 * n * 512 * t + heads * m * dh * 4 * 2
        flops = 2 * 2 * heads * m * n * dh
        return dict(bytes=byts, flops=flops)
    raise ValueError(site)


HBM_SITES = ("ln_fwd", "landmarks", "a3_fwd", "a1_fwd", "ppeg_fwd", "ppeg_bwd", "conv_bwd", "a1_bwd", "a3_bwd")

# the dense d_model projections (code/models/TransMIL.py:26-34 to_qkv / to_out, :128-133 _fc1) and
# their backward products, in bf16 mode: site -> (layers in call order, shape(n', N patches, layer) ->
# (M, N, K, algorithmic HBM bytes), what).  The shapes are the ones the engine launches
# (tests/test_interface.py::test_gemm_sites_match_the_engine_launches records them): layer 2's
# backward (the class-row layer) runs the k / v part of to_qkv only (K = 2D; its q part goes through
# tm_cls_q_rows' two small products, engine.CLS_Q_ROWS); layer 2 has no dense to_out GEMMs.
# Bytes: every operand read once and every final output written once (bf16 T = 2 B operands, fp32
# residual stream and weight gradients; split-K slabs are not algorithmic).
_D, _T = 512, 2


def _S(N):
    import math
    G = math.ceil(math.sqrt(N))
    return G * G + 1


def _qkv_k(layer):
    from transmil_deepgraft_amd import engine
    return 2 * _D if (layer == 2 and engine.CLS_Q_ROWS) else 3 * _D


GEMM_SITES = {
    "fc1_gemm": ((0,), lambda n, N, L: (N, _D, 512, N * 512 * _T + _D * 512 * _T + _D * 4 + (_S(N) - 1) * _D * 4
                                        + N * _D * _T),
                 "_fc1 Linear + GELU (+ grid-pad rows): x, W in; H0 (fp32), pre-activation (T) out"),
    "qkv_gemm": ((1, 2), lambda n, N, L: (n, 3 * _D, _D, n * _D * _T + 3 * _D * _D * _T + 3 * n * _D * _T),
                 "to_qkv (+ head-major scatter, q scale): xn, W in; q, k, v out"),
    "out_gemm": ((1,), lambda n, N, L: (n, _D, _D, n * _D * _T + _D * _D * _T + 2 * _S(N) * _D * 4),
                 "to_out + bias + dropout + residual: merged, W, H in; H' (fp32) out"),
    "wgrad_out": ((1,), lambda n, N, L: (_D, _D, n, 2 * n * _D * _T + (_D * _D + _D) * 4),
                  "dW_out split-K (+ bias gradient): dout, merged in; dW, db (fp32) out"),
    "dmerged_gemm": ((1,), lambda n, N, L: (n, _D, _D, 2 * n * _D * _T + _D * _D * _T),
                     "dmerged = dout W_out"),
    "wgrad_qkv": ((2, 1), lambda n, N, L: (_qkv_k(L), _D, n, n * _qkv_k(L) * _T + n * _D * _T + _qkv_k(L) * _D * 4),
                  "dW_qkv split-K (layer 2: the k / v rows): dqkv, xn in; dW (fp32) out"),
    "dxn_gemm": ((2, 1), lambda n, N, L: (n, _D, _qkv_k(L), n * _qkv_k(L) * _T + _qkv_k(L) * _D * _T + n * _D * _T),
                 "dxn = dqkv W_qkv (layer 2: K = 2D)"),
    "wgrad_fc1": ((0,), lambda n, N, L: (_D, 512, N, N * _D * _T + N * 512 * _T + (_D * 512 + _D) * 4),
                  "dW_fc1 split-K (+ bias gradient): dpre, x in; dW, db (fp32) out"),
}


def hbm_model(n_patches, dtype_bytes, d=512, heads=8, m=256, dh=64):
    """Algorithmic HBM bytes of one launch of each HBM-bound call site (bf16 mode: T = 2 B),
    by (site, layer): every compulsory tensor read or written once.  G = ceil(sqrt(N)),
    S = G^2 + 1 tokens, n' = S rounded up to 256."""
    import math
    G = math.ceil(math.sqrt(n_patches))
    S = G * G + 1
    n = (S + 255) // 256 * 256
    t, f4 = dtype_bytes, 4
    lm = heads * m * dh                              # one [h, 256, 64] landmark-sized tensor
    ln = S * d * f4 + n * d * t + 2 * S * f4         # H (fp32) in, xn (T, pad rows included) out, mean / rstd
    landmarks = 2 * n * d * t + 2 * lm * (f4 + t)    # q, k in; q~, k~ out (fp32 + T copies)
    a3f = 2 * n * d * t + lm * f4 + lm * f4 + heads * m * f4   # k, v, q~ in; W, lse3 out
    if t == 2:   # bf16: the same launch writes A2 (fp32 + split bf16 planes) from q~, k~ (tm_nys_a3_fwd_sim2)
        a3f += lm * f4 + heads * m * m * (f4 + 2 * t)
    a1f = 2 * n * d * t + 2 * lm * t + n * d * t + heads * n * f4   # q, v, k~, Y in; merged, lse1 out
    ppf = 2 * S * d * f4                             # H1 in, H2 out (fp32 residual stream)
    ppb = 3 * S * d * f4 + n * d * t                 # H1, dH in; dH1 out; layer 1's padded dropout gradient out
    cvb = 4 * n * d * t + heads * n * f4   # dmerged, merged, v in; dv (in T, round 6), D1 out
    # q, dO in (T); lse1, D1 in; k~, Y (T) in; dq out (T: the precision dqkv carries); dk~, dY out (fp32)
    a1b = 2 * n * d * t + 2 * heads * n * f4 + 2 * lm * t + n * d * t + 2 * lm * f4
    a3b_small = 2 * lm * t + 2 * heads * m * f4 + lm * f4 + lm * f4   # q~, dW in, lse3, D3, dk~ in, dq~3 out
    a3b_l2 = 2 * n * d * t + 2 * n * d * t + a3b_small                # k, v in; dk, dv (into dqkv) out
    a3b_l1 = a3b_l2 + n * d * f4                                      # + the conv path's fp32 dv in
    return {
        ("ln_fwd", 1): ("ln_fwd_kernel", ln), ("ln_fwd", 2): ("ln_fwd_kernel", ln),
        ("landmarks", 1): ("landmarks_kernel", landmarks), ("landmarks", 2): ("landmarks_kernel", landmarks),
        # the key-split kernel; its partials' combine runs inside the pseudo-inverse chain's last launch
        ("a3_fwd", 1): ("a3_fwd_v2_kernel<0, 4> (+ A2 rows; combine inside pinv F launch)", a3f),
        ("a3_fwd", 2): ("a3_fwd_v2_kernel<0, 4> (+ A2 rows; combine inside pinv F launch)", a3f),
        ("a1_fwd", 1): ("a1_fwd_bf16_kernel", a1f),
        ("ppeg_fwd", 0): ("ppeg_stencil_kernel<false>", ppf),
        # (the weight-gradient slab sums ride in the deferred multi_reduce flush that follows)
        ("ppeg_bwd", 0): ("ppeg_bwd_kernel (weight gradient + dx stencil, one launch)", ppb),
        ("conv_bwd", 1): ("conv_bwd_mfma_kernel", cvb),
        # the kernel alone; its dk~ / dY partial slabs are summed in the deferred flush that follows
        ("a1_bwd", 1): ("attn_bwd_bf16_kernel<1, 8> (dk~ / dY slab sums in the deferred flush)", a1b),
        ("a3_bwd", 2): ("attn_bwd_bf16_kernel<0, 9> (fused dk / dv epilogue)", a3b_l2),
        ("a3_bwd", 1): ("attn_bwd_bf16_kernel<0, 9> (fused dk / dv epilogue)", a3b_l1),
    }


# layer of the k-th call of a site within one step (forward: layer 1 then 2; backward: 2 then 1)
SITE_LAYERS = {"ln_fwd": (1, 2), "landmarks": (1, 2), "a3_fwd": (1, 2), "a1_fwd": (1,), "ppeg_fwd": (0,),
               "ppeg_bwd": (0,), "conv_bwd": (1,), "a1_bwd": (1,), "a3_bwd": (2, 1)}


def probe_site_times(engine, run_step, steps, sites):
    """Eager probe steps with every site in ``sites`` timed: a GPU spin queued ahead of each probed
    launch so its events bracket the kernel, the span of an empty event pair recorded just before it
    subtracted.  Returns site -> [ms per call, in call order over the steps]."""
    engine.probe.target = set(sites)
    engine.probe.spin_cycles = 2_000_000
    engine.probe.events.clear()
    engine.probe.names.clear()
    for i in range(steps):
        run_step(i)
    torch.cuda.synchronize()
    engine.probe.target = None
    engine.probe.spin_cycles = 0
    per = {}
    for name, ev in zip(engine.probe.names, engine.probe.events):
        s, e, zs, ze = ev
        per.setdefault(name, []).append(s.elapsed_time(e) - zs.elapsed_time(ze))
    return per


def gemm_roofline(per, n_patches):
    """The dense projections against their roofline: a site's time floor is
    max(flops / dense bf16 peak, algorithmic bytes / HBM peak); ``frac`` = that floor / the probe's
    median event span per call site and layer, ``bound`` says which term sets the floor (the
    to_out and _fc1 epilogues move more bytes than their flops need).  The split-K products' slab
    sums run in the deferred flush, not in this span."""
    import math
    G = math.ceil(math.sqrt(n_patches))
    n = (G * G + 1 + 255) // 256 * 256
    out = []
    for site, (layers, shape, what) in GEMM_SITES.items():
        xs = per.get(site, [])
        if not xs or len(xs) % len(layers):
            continue
        for k, layer in enumerate(layers):
            M, N, K, byts = shape(n, n_patches, layer)
            flops = 2 * M * N * K
            v = sorted(xs[k::len(layers)])
            ms = v[len(v) // 2]
            sec = ms / 1e3
            tf, tb = flops / (BF16_PEAK_TFS * 1e12), byts / (HBM_PEAK_GBS * 1e9)
            out.append(dict(site=site, layer=layer, what=what, M=M, N=N, K=K, flops=flops, algorithmic_bytes=byts,
                            us=round(ms * 1e3, 2), achieved_tfs=round(flops / sec / 1e12, 1),
                            achieved_gbs=round(byts / sec / 1e9, 1), bound="mfma" if tf >= tb else "hbm",
                            frac_mfma=round(tf / sec, 4), frac_hbm=round(tb / sec, 4), frac=round(max(tf, tb) / sec, 4)))
    return out


def hbm_roofline(per, n_patches, dtype_bytes):
    """HBM-bound sites: algorithmic bytes / the probe's median event span, against 8 TB/s."""
    model = hbm_model(n_patches, dtype_bytes)
    out = []
    for site in HBM_SITES:
        xs = per.get(site, [])
        layers = SITE_LAYERS[site]
        if not xs or len(xs) % len(layers):
            continue
        for k, layer in enumerate(layers):
            if (site, layer) not in model:
                continue
            ms = sorted(xs[k::len(layers)])[len(xs[k::len(layers)]) // 2]   # median over the probe steps
            kname, byts = model[(site, layer)]
            gbs = byts / (ms / 1e3) / 1e9
            tr = measured_traffic(f"{site}:{layer}" if len(layers) > 1 else site, n_patches,
                                  "bf16" if dtype_bytes == 2 else "fp32")
            out.append(dict(site=site, layer=layer, kernel=kname, algorithmic_bytes=byts, us=round(ms * 1e3, 2),
                            achieved_gbs=round(gbs, 1), frac=round(gbs / HBM_PEAK_GBS, 4), traffic=tr))
    return out


def measured_traffic(site, n_patches, dtype):
    """HBM bytes per launch of `site` from the committed rocprofv3 PMC passes
    (profiles/traffic.json, written by scripts/gpu_pmc_bench.sh + scripts/traffic_json.py):
    FETCH_SIZE (doubled for the gfx950 half-count) + WRITE_SIZE.  None when that file does not
    hold a measurement of this call site at this workload."""
    path = os.path.join(ROOT, "profiles", "traffic.json")
    try:
        rec = json.load(open(path))["sites"][site]
    except (OSError, KeyError, ValueError):
        return None
    if rec.get("n") != n_patches or rec.get("dtype") != dtype:
        return None
    return rec.get("traffic_bytes")


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or "unknown"


def cpu_baseline(n_patches, ncls, steps, feat=512, as_written=False, threads=None):
    """fp32 CPU oracle on this host: fwd + CE + bwd + RAdam, train mode, median of `steps` steps
    after 2 warm-ups, at 8 threads (code/train.py:93) and at the box's CPU share (16; the
    machine's physical cores belong to other jobs).  Logits path (no unused n'xn' product)
    unless `as_written`."""
    import statistics
    from oracle.transmil_ref import TransMIL as RefTransMIL, TransLayer
    share = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    counts = sorted(threads) if threads else sorted({8, max(1, min(share, os.cpu_count() or 1))})
    TransLayer.compute_attn = as_written
    torch.manual_seed(0)
    model = RefTransMIL(ncls, feat, 512).train()
    opt = torch.optim.RAdam(model.parameters(), lr=2e-4)
    x = torch.rand(1, n_patches, feat)
    y = torch.tensor([1])
    lossf = torch.nn.CrossEntropyLoss()

    def step():
        logits = model(x)
        loss = lossf(logits, torch.nn.functional.one_hot(y, ncls).float())
        loss.backward()
        opt.step()
        opt.zero_grad(set_to_none=True)

    by = {}
    try:
        for th in counts:
            torch.set_num_threads(th)
            for _ in range(2):
                step()
            ts = []
            for _ in range(steps):
                t0 = time.perf_counter()
                step()
                ts.append(time.perf_counter() - t0)
            by[th] = 1.0 / statistics.median(ts)
    finally:
        TransLayer.compute_attn = True
    best = max(by, key=by.get)
    variant = "as written (n'xn' return_attn product)" if as_written else "logits path"
    return dict(value=by[best], unit="slides/sec", cores=best, kind="port",
                by_threads={str(k): round(v, 4) for k, v in by.items()}, cpu_model=_cpu_model(),
                sample=f"median of {steps} fwd+CE+bwd+RAdam steps after 2 warm-ups per thread count, 1 bag "
                       f"N={n_patches}x{feat}, fp32, train mode, {variant}, torch.set_num_threads in {counts}")


def make_step(task, opt, allreduce, bags, labels, K, warmup, eager=False):
    """The timed step over the resident bags: ``step(i)`` runs micro-batch i (bag i % len(bags)).

    K = 1: fwd + CE + bwd + all-reduce + optimizer, one captured hipGraph per bag.  K > 1
    (accumulate_grad_batches, Lightning's semantics as TransMILTask.optimization_step): micro-batch
    i is "first" (i % K == 0: loss / K, gradients written), "mid" (added) or "last" ((i + 1) % K == 0:
    added, all-reduced, optimizer step), one captured graph per (bag, phase).  Warm-up: warmup * K
    eager micro-batches (at least 2 K) on a side stream before the captures, then every captured
    graph replayed once (micro-batches 0 .. len(bags) * K - 1).  Returns a namespace with ``step``,
    ``body(x, y, phase)``, ``load(i)``, ``graph`` (None when eager) and ``warm_micro`` = (eager
    warm-up micro-batches, warm-up replays)."""
    static_x = torch.empty_like(bags[0])
    static_y = torch.empty_like(labels[0])

    def body(x=None, y=None, phase="last"):
        """phase: "first" / "mid" micro-batch of an accumulation window (no all-reduce, no step;
        first writes the gradients, mid adds), "last" (adds, all-reduces, steps; K = 1: the step)."""
        loss = task.training_step((static_x if x is None else x, static_y if y is None else y, None))
        allreduce.sync = phase == "last"
        task.backward(loss / K if K > 1 else loss)
        if phase == "last":
            allreduce()
            opt.step()

    def phase_of(i):
        return "last" if (i + 1) % K == 0 else ("first" if i % K == 0 else "mid")

    def load(i):
        static_x.copy_(bags[i % len(bags)])
        static_y.copy_(labels[i % len(bags)])

    graph = None
    if eager:
        def step(i):
            load(i)
            body(phase=phase_of(i))
            if phase_of(i) == "last":
                opt.zero_grad(set_to_none=True)
        for i in range(warmup * K):
            step(i)
    else:
        # warm up on a side stream, then capture fwd + CE + bwd + all-reduce + optimizer as ONE hipGraph
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for i in range(max(warmup, 2) * K):
                load(i)
                body(phase=phase_of(i))
                if phase_of(i) == "last":
                    opt.zero_grad(set_to_none=True)
        torch.cuda.current_stream().wait_stream(side)
        # one captured step per resident bag (reading that bag in place: no copy into a static
        # input inside the timed region), all on one memory pool -- they never run at once
        pool = torch.cuda.graph_pool_handle()
        graphs = {}
        phases = ["last"] if K == 1 else (["first", "mid", "last"] if K > 2 else ["first", "last"])
        for j in range(len(bags)):
            opt.zero_grad(set_to_none=True)   # the first capture takes the first-micro-batch (=) path,
            for ph in phases:                 # the ones after it the accumulating (+=) path
                gj = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gj, pool=pool):
                    body(bags[j], labels[j], phase=ph)
                graphs[j, ph] = gj
        graph = graphs[0, "last"]

        def step(i):
            graphs[i % len(bags), phase_of(i)].replay()

        # every captured graph replayed once before the timed region (untimed warm-up, real steps):
        # a graph's first replay pays one-time work (the executable's upload, first-touch of its
        # pool), which a short timed run (the driver's --steps 20) must not carry.  len(bags) * K
        # micro-batches = every (bag, phase) graph, ending on an accumulation boundary.
        for i in range(len(bags) * K):
            step(i)
        torch.cuda.synchronize()
    return types.SimpleNamespace(step=step, body=body, load=load, graph=graph, phase_of=phase_of,
                                 warm_micro=(max(warmup, 2) * K, 0 if eager else len(bags) * K))


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # TM_BENCH_BACKEND=gloo: a rehearsal of the N > 1 control flow on fewer GPUs than ranks (ranks
    # share devices round-robin; gloo all-reduces the CUDA buckets; use with --eager, gloo does not
    # capture).  The measured path is RCCL ("nccl"), one rank per GPU.
    backend = os.environ.get("TM_BENCH_BACKEND", "nccl")
    if backend != "nccl":
        local = local % max(torch.cuda.device_count(), 1)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from transmil_deepgraft_amd.models import TransMIL
    from transmil_deepgraft_amd.interface import TransMILTask, GradAllReduce
    from transmil_deepgraft_amd import engine

    torch.manual_seed(1234)  # same random-init weights on every rank
    model = TransMIL(args.classes, args.features, 512).to(dev).train()
    model.set_compute_dtype(torch.bfloat16 if args.dtype == "bf16" else torch.float32)
    task = TransMILTask(model)
    opt = task.configure_optimizers()[0][0]
    allreduce = GradAllReduce(model.parameters(), model=model)   # grads = views of a 2-part bucket

    g = torch.Generator(device=dev).manual_seed(2021 + rank)
    bags = [torch.rand(1, args.n, args.features, device=dev, generator=g) for _ in range(4)]
    labels = [torch.randint(0, args.classes, (1,), device=dev, generator=g) for _ in range(4)]
    K = max(1, args.accumulate)
    st = make_step(task, opt, allreduce, bags, labels, K, args.warmup, eager=args.eager)
    body, load, step, graph = st.body, st.load, st.step, st.graph

    # the roofline call site, and the pseudo-inverse backward beside the forward chain
    probe_sites = {args.probe, "pinv_bwd"} if args.probe == "pinv_fwd" else {args.probe}
    if args.eager:
        engine.probe.target = probe_sites
        engine.probe.events.clear()
        engine.probe.names.clear()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    kernel_ms_samples = []
    overhead_samples = []
    span_samples = []
    for i in range(args.steps):
        step(i)
        if (i + 1) % 50 == 0 and rank == 0:
            print(f"# step {i + 1}/{args.steps}", file=sys.stderr, flush=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    engine.probe.target = None
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = t.item()
    if graph is not None:
        # after the timed region: the same step captured once more with external HIP events
        # around the probed launches (graph event-record nodes on the kernel's stream), replayed
        # three times; the events hold each replay's timestamps.  The timed graph has no probes.
        try:
            pgraph = torch.cuda.CUDAGraph()
            engine.probe.target, engine.probe.external = probe_sites, True
            engine.probe.events.clear()
            with torch.cuda.graph(pgraph):
                body()
            engine.probe.target, engine.probe.external = None, False
            for i in range(3):
                load(i)
                pgraph.replay()
                torch.cuda.synchronize()
                kernel_ms_samples += [(nm, s.elapsed_time(e)) for nm, (s, e) in zip(engine.probe.names, engine.probe.events)]
                engine.probe.names.clear()
        except Exception as exc:  # noqa: BLE001 - event timing inside graphs unsupported: probe eagerly
            print(f"# graph event probe unavailable ({exc}); eager probe", file=sys.stderr)
            engine.probe.target, engine.probe.external = None, False
            kernel_ms_samples = []
        if not kernel_ms_samples:
            # after the timed region: three eager steps with the probed launch queued behind
            # a GPU spin (engine._Probe.spin_cycles), so its events bracket the kernel itself
            engine.probe.target = probe_sites
            engine.probe.spin_cycles = 2_000_000
            engine.probe.events.clear()
            engine.probe.names.clear()
            for i in range(3):
                load(i)
                body()
            torch.cuda.synchronize()
            engine.probe.target = None
            engine.probe.spin_cycles = 0
            # launch span minus the span of an empty event pair recorded just before it
            evs = list(zip(engine.probe.names, engine.probe.events))
            kernel_ms_samples = [(nm, s.elapsed_time(e) - zs.elapsed_time(ze)) for nm, (s, e, zs, ze) in evs]
            overhead_samples = [(nm, zs.elapsed_time(ze)) for nm, (_, _, zs, ze) in evs]
            span_samples = [(nm, s.elapsed_time(e)) for nm, (s, e, _, _) in evs]
    if graph is None:
        kernel_ms_samples = [(nm, s.elapsed_time(e)) for nm, (s, e) in zip(engine.probe.names, engine.probe.events)]

    def site_mean(samples, site):
        xs = [v for nm, v in samples if nm == site]
        return sum(xs) / len(xs) if xs else None

    hbm = gemms = None
    if not args.no_hbm_probe and args.features == 512:
        # every rank runs the probe steps: each step's gradient all-reduce is a collective, so a
        # rank-0-only probe would leave rank 0 waiting in it at N > 1 (rank 0 reports the result)
        def probe_step(i):
            load(i)
            body()
        per = probe_site_times(engine, probe_step, 3, set(HBM_SITES) | set(GEMM_SITES))
        hbm = hbm_roofline(per, args.n, 2 if args.dtype == "bf16" else 4)
        gemms = gemm_roofline(per, args.n) if args.dtype == "bf16" else None

    # the optimizer step alone (it is also inside every timed step): a graph of opt.step()
    # replayed 20 times between two events (after the timed region; it advances the state)
    opt_ms = None
    if graph is not None:
        try:
            og = torch.cuda.CUDAGraph()
            with torch.cuda.graph(og):
                opt.step()
            s_ev, e_ev = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            og.replay()
            s_ev.record()
            for _ in range(20):
                og.replay()
            e_ev.record()
            torch.cuda.synchronize()
            opt_ms = s_ev.elapsed_time(e_ev) / 20
        except Exception as exc:  # noqa: BLE001
            print(f"# optimizer timing unavailable ({exc})", file=sys.stderr)

    def roofline_obj(site):
        kernel_ms = site_mean(kernel_ms_samples, site)
        if kernel_ms is None:
            return None
        tb = 2 if args.dtype == "bf16" else 4
        rm = roofline_model(site, args.n, tb)
        sec = kernel_ms / 1e3
        ach_bw = rm["bytes"] / sec / 1e9
        ach_fl = rm["flops"] / sec / 1e12
        peak_fl = rm.get("peak_tfs", BF16_PEAK_TFS if args.dtype == "bf16" else F32_MATRIX_PEAK_TFS)
        hbm_bound = rm["flops"] / rm["bytes"] < peak_fl * 1e12 / (HBM_PEAK_GBS * 1e9)
        roof = (dict(bound="hbm", achieved=round(ach_bw, 1), peak=HBM_PEAK_GBS, unit="GB/s",
                     frac=round(ach_bw / HBM_PEAK_GBS, 4), traffic=measured_traffic(site, args.n, args.dtype))
                if hbm_bound else
                dict(bound="mfma", achieved=round(ach_fl, 2), peak=peak_fl, unit="TFLOP/s",
                     frac=round(ach_fl / peak_fl, 4), traffic=measured_traffic(site, args.n, args.dtype)))
        if overhead_samples:
            roof.update(event_span_ms=round(site_mean(span_samples, site), 5),
                        event_pair_overhead_ms=round(site_mean(overhead_samples, site), 5))
        kname = {"pinv_fwd": "pinv_stage_kernel x14 (tm_pinv_fwd_split_a3)",
                 "pinv_bwd": "pinv_stage_kernel x24 + pinv_apply_bwd_kernel (tm_pinv_bwd_split)"}.get(site, site)
        roof.update(kernel=kname, kernel_ms=round(kernel_ms, 5),
                    samples=sum(1 for nm, _ in kernel_ms_samples if nm == site),
                    algorithmic_bytes=rm["bytes"], algorithmic_flops=rm["flops"])
        if "units" in rm:
            roof.update(launches_per_call=rm["units"], ms_per_launch=round(kernel_ms / rm["units"], 5),
                        note=rm["note"])
        return roof

    if rank == 0:
        slides = args.steps * world
        roof = roofline_obj(args.probe)
        base_metric = "slides/sec (fwd+bwd) at N=8192 patches, d=512"
        if args.features == 512:
            metric = base_metric if args.n == 8192 else f"slides/sec (fwd+bwd) at N={args.n} patches, d=512"
        else:
            metric = f"slides/sec (fwd+bwd) at N={args.n} patches, in_features={args.features}"
        out = {
            "metric": metric,
            "value": round(slides / elapsed, 3),
            "unit": "slides/sec",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.dtype,
            "data": "synthetic (torch.rand bags resident in HBM, random-init weights)",
            "config": {"workload": f"TransMIL_feat {args.classes}-class, 1 bag N={args.n}x{args.features} per GPU, "
                                   "train step fwd+CE+bwd+allreduce+Lookahead(RAdam)",
                       "execution": "eager" if args.eager else "hipGraph replay of the whole step (one graph per resident bag)",
                       "global_batch": world, "seq_len": args.n, "parallelism": f"dp{world}",
                       "accumulate_grad_batches": K},
            "roofline": roof,
            "roofline_pinv_bwd": roofline_obj("pinv_bwd") if args.probe == "pinv_fwd" else None,
            "hbm_roofline": hbm,
            "gemm_roofline": gemms,
            "optimizer_ms": round(opt_ms, 5) if opt_ms is not None else None,
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(args.n, args.classes, args.cpu_steps, args.features)
            if not args.no_cpu_as_written:
                out["cpu_baseline_as_written"] = cpu_baseline(args.n, args.classes, 2, args.features, as_written=True,
                                                              threads=(out["cpu_baseline"]["cores"],))
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()      # rank 0's CPU baselines / print done before any rank tears down
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
