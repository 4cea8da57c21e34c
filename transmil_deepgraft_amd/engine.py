"""Host-side orchestration of the TransMIL hot path on the HIP kernels.

This is the MI355X replacement for the torch op sequence of
``TransMIL.forward`` (code/models/TransMIL.py:167-211) and its autograd
backward.  Every arithmetic step is one of the C-ABI entry points of
``libtransmil_hip.so``; PyTorch only allocates device memory and supplies the
stream.  There is no fallback: without the library this module raises.

Shapes (B bags of N patches, D = 512 = 8 heads x 64):
    G = ceil(sqrt(N)), add = G*G - N, S = G*G + 1        (grid pad + class token, :177-186)
    n = ceil(S / 256) * 256, pad = n - S, l = n / 256    (NystromAttention front pad, App. A eq. 1)
Buffers:
    H*  [B*S, D] fp32 residual stream;  xn [B, n, D] T (LN output, pad rows 0)
    qkv [3, B*8, n, 64] T;  merged [B, n, D] T
``T`` is bf16 (bench mode) or fp32 (parity mode).
"""
from __future__ import annotations

import ctypes as C
import math
import os
from dataclasses import dataclass

import torch

from . import _lib
from ._lib import BF16, F32, EPI_PLAIN, EPI_QKV, EPI_SPLITK, GemmArgs, BmmJob

NL = 256        # landmarks
DH = 64         # dim_head
TAPS = 33       # residual conv
PINV_ITERS = 6
LN_EPS = 1e-5
QROWS = NL + 32  # rows per bag of tm_cls_q_rows' operands (landmarks, class row, zero rows to 32 | rows)
# bf16 class-row layer: the q part of to_qkv's backward as two small products (TM_CLS_Q_ROWS=0: the
# dense q block of dqkv, for A/B runs and the equivalence test)
CLS_Q_ROWS = os.environ.get("TM_CLS_Q_ROWS", "1") != "0"


class _Probe:
    """Optional HIP-event timing of named call sites (bench.py's roofline legs).

    ``target``: one site name, or a set of names.  Events are recorded on the current stream --
    the stream the kernel is launched on -- so their difference is that launch's duration;
    ``names[i]`` is the site of ``events[i]``."""

    def __init__(self):
        self.target = None
        self.events = []
        self.names = []
        # > 0: a GPU spin of this many cycles is queued ahead of the start event, so the host
        # has already submitted the kernel when the event fires and the pair times the kernel,
        # not the host's launch latency (used only outside any timed region or graph capture)
        self.spin_cycles = 0
        # True while capturing a probe graph: external events become graph event-record nodes
        self.external = False

    def __call__(self, name):
        return _ProbeCtx(self, name)

    def on(self, name):
        t = self.target
        return t is not None and (name == t if isinstance(t, str) else name in t)


class _ProbeCtx:
    def __init__(self, probe, name):
        self.p, self.name = probe, name

    def __enter__(self):
        self.active = self.p.on(self.name)
        if self.active:
            self.z = None
            if self.p.spin_cycles > 0:
                torch.cuda._sleep(self.p.spin_cycles)
                # an empty event pair first: its span is the pair's own overhead
                self.z = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                self.z[0].record()
                self.z[1].record()
            self.s = torch.cuda.Event(enable_timing=True, external=self.p.external)
            self.e = torch.cuda.Event(enable_timing=True, external=self.p.external)
            self.s.record()
        return self

    def __exit__(self, *exc):
        if self.active:
            self.e.record()
            self.p.events.append((self.s, self.e) if self.z is None else (self.s, self.e, *self.z))
            self.p.names.append(self.name)
        return False


probe = _Probe()


def _p(t):
    return C.c_void_p(t.data_ptr()) if t is not None else C.c_void_p(0)


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)
_cur_device = getattr(torch._C, "_cuda_getDevice", None)


def _stream():
    """The current HIP stream of the current device as a C pointer (capture-aware: inside a graph
    capture it is the capturing stream).  The raw accessor skips building a torch Stream object
    (~10 us per call in the eager step's host path; the public API is the fallback)."""
    if _raw_stream is not None and _cur_device is not None:
        return C.c_void_p(_raw_stream(_cur_device()))
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


@dataclass
class Geometry:
    B: int
    N: int
    F: int
    D: int
    heads: int

    def __post_init__(self):
        self.G = int(math.ceil(math.sqrt(self.N)))
        self.add = self.G * self.G - self.N
        self.S = self.G * self.G + 1
        self.n = ((self.S + NL - 1) // NL) * NL
        self.pad = self.n - self.S
        self.l = self.n // NL
        self.nbh = self.B * self.heads


# ----------------------------------------------------------------------------- GEMM helpers
def gemm(A, B, Cout, M, N, K, *, lda, ldb, ldc, a_trans=0, b_kn=0, dtype=BF16, c_dtype=None,
         alpha=1.0, bias=None, gelu=False, pre=None, ld_pre=0, drop_p=0.0, seed=0, seed_ptr=None, resid=None,
         accumulate=False, rowmap=None, qkv=None, splits=1, k_per_split=None, pre_bf16=False):
    g = GemmArgs()
    g.M, g.N, g.K = M, N, K
    g.lda, g.ldb, g.ldc = lda, ldb, ldc
    g.a_trans, g.b_kn = a_trans, b_kn
    g.ab_dtype = dtype
    g.c_dtype = dtype if c_dtype is None else c_dtype
    g.splits = splits
    bk = 64 if dtype == BF16 else 32
    if k_per_split is None:
        k_per_split = ((K + splits - 1) // splits + bk - 1) // bk * bk
    g.k_per_split = max(k_per_split, 1)
    g.mode = EPI_PLAIN
    g.alpha = alpha
    g.bias = _p(bias)
    g.gelu = int(gelu)
    g.pre = _p(pre)
    g.ld_pre = ld_pre
    g.pre_bf16 = int(pre_bf16)
    g.drop_p = drop_p
    g.drop_scale = 1.0 / (1.0 - drop_p) if drop_p > 0 else 1.0
    g.seed = seed
    g.seed_ptr = _p(seed_ptr)
    g.resid = _p(resid)
    g.accumulate = int(accumulate)
    if rowmap is not None:
        g.grp_in, g.skip, g.grp_out, g.out_off, g.dup_n, g.dup_off = rowmap
    if qkv is not None:
        g.mode = EPI_QKV
        g.nbags, g.nh, g.dh, g.seq, g.qscale = qkv
    _lib.call("tm_gemm", _p(A), _p(B), _p(Cout), C.byref(g), _stream())


_CU = {}


def cu_count():
    """Compute units of the current device (the schedules size grids to one workgroup per CU;
    256 on MI355X, also the value without a GPU)."""
    dev = torch.cuda.current_device() if torch.cuda.is_available() else -1
    if dev not in _CU:
        _CU[dev] = torch.cuda.get_device_properties(dev).multi_processor_count if dev >= 0 else 256
    return _CU[dev]


# A/B knobs (scripts/dev/ab_env.sh only; defaults are the measured choices): workgroup slots the
# split-K weight gradients size their splits for (0: one per CU), and the LayerNorm backward's rows
# per block
_WGRAD_SLOTS = int(os.environ.get("TM_WGRAD_SLOTS", "0"))
_LN_BWD_RPB = int(os.environ.get("TM_LN_BWD_RPB", "16"))


def weight_grad(dY, X, out, M, N, K, *, ldy, ldx, dtype, work_pool, bias_out=None, slab_bf16=None):
    """out[M,N] (fp32) = sum_k dY[k, m] X[k, n]  (split-K, deterministic).  ``bias_out`` [M]: also
    the bias gradient sum_k dY[k, m] -- in bf16 mode summed by the weight-gradient kernel itself
    while it stages dY (tm_gemm_args.colsum), else one tm_colsum pass.  ``slab_bf16`` (default: the
    bf16 mode): the split partials are stored bf16 (half the slab bytes written and read back by the
    flush, which sums them in fp32 in split order); False keeps fp32 slabs."""
    tiles = ((M + 127) // 128) * ((N + 127) // 128)
    slots = _WGRAD_SLOTS or cu_count()
    splits = max(1, min(16, slots // max(tiles, 1), (K + 255) // 256))   # <= one workgroup per CU
    if splits == 1:
        gemm(dY, X, out, M, N, K, lda=ldy, ldb=ldx, ldc=N, a_trans=1, b_kn=1, dtype=dtype, c_dtype=F32)
        if bias_out is not None:
            colsum(dY, K, M, ldy, dtype, bias_out, work_pool)
        return
    bk = 64 if dtype == BF16 else 32
    kps = ((K + splits - 1) // splits + bk - 1) // bk * bk
    splits = (K + kps - 1) // kps
    # bf16 mode: bf16 split slabs (each split's partial rounded once, summed in fp32 by the flush)
    sb16 = dtype == BF16 if slab_bf16 is None else bool(slab_bf16) and dtype == BF16
    slab = work_pool(splits * M * N, torch.bfloat16) if sb16 else work_pool(splits * M * N)
    g = GemmArgs()
    g.M, g.N, g.K = M, N, K
    g.lda, g.ldb, g.ldc = ldy, ldx, N
    g.a_trans, g.b_kn = 1, 1
    g.ab_dtype, g.c_dtype = dtype, F32
    g.splits, g.k_per_split = splits, kps
    g.mode = EPI_SPLITK
    g.alpha = 1.0
    g.slab_bf16 = int(sb16)
    fuse = bias_out is not None and dtype == BF16 and K % 64 == 0 and M % 8 == 0 and N % 8 == 0
    cs = work_pool(splits * M) if fuse else None
    if fuse:
        g.colsum = cs.data_ptr()
    _lib.call("tm_gemm", _p(dY), _p(X), _p(slab), C.byref(g), _stream())
    _lib.call("tm_splitk_reduce_bf16" if sb16 else "tm_splitk_reduce", _p(slab), _p(out), splits, M * N,
              C.c_float(1.0), 0, _rq(), _stream())
    if fuse:
        _lib.call("tm_splitk_reduce", _p(cs), _p(bias_out), splits, M, C.c_float(1.0), 0, _rq(), _stream())
    elif bias_out is not None:
        colsum(dY, K, M, ldy, dtype, bias_out, work_pool)


def colsum(X, rows, cols, ld, dtype, out, work_pool, accumulate=False):
    rpc = 256
    nchunk = (rows + rpc - 1) // rpc
    work = work_pool(nchunk * cols)
    _lib.call("tm_colsum", _p(X), dtype, rows, cols, ld, rpc, _p(work), _p(out), int(accumulate), _rq(), _stream())


def bmm_job(A, ta, B, tb, Cout, M, N, K, alpha=1.0, diag=0.0, E1=None, e1=0.0, E2=None, e2=0.0, Ct=None,
            ct_mode=0, ct_plane=0):
    j = BmmJob()
    j.A, j.B = A.data_ptr(), B.data_ptr()
    j.ta, j.tb = ta, tb
    j.lda = M if ta else K
    j.ldb = K if tb else N
    j.sa, j.sb = M * K, K * N
    j.A2 = j.B2 = None
    j.E1 = E1.data_ptr() if E1 is not None else None
    j.e1 = e1
    j.E2 = E2.data_ptr() if E2 is not None else None
    j.e2 = e2
    j.alpha, j.diag = alpha, diag
    j.C = Cout.data_ptr()
    j.ldc, j.sc = N, M * N
    j.M, j.N, j.K = M, N, K
    j.Ct = Ct.data_ptr() if Ct is not None else None
    j.ct_mode, j.ct_plane = (ct_mode, ct_plane) if Ct is not None else (0, 0)
    return j


def bmm(jobs, nbatch, prec=0):
    """prec 0: exact fp32 MFMA (parity mode); 1: bf16x3 split (bench mode)."""
    arr = (BmmJob * len(jobs))(*jobs)
    _lib.call("tm_bmm", arr, len(jobs), nbatch, prec, _stream())


class Pool:
    """Scratch allocator for one forward or backward call (torch caching allocator underneath).
    Buffers allocated while reductions are deferred are held until the pool dies (their
    slabs are read by the later flush launch)."""

    def __init__(self, device):
        self.device = device
        self.hold = []

    def __call__(self, numel, dtype=torch.float32):
        t = torch.empty(int(numel), dtype=dtype, device=self.device)
        if getattr(_TLS, "deferring", False):
            self.hold.append(t)
        return t


class ReduceQueue:
    """A caller-owned ``tm_reduce_queue`` (include/transmil_hip.h): the host-side list of
    parameter-gradient slab sums a backward defers to one ``tm_reduce_flush`` launch.  The library
    keeps no deferral state; each backward call owns one of these, so engines on different
    threads / streams never share entries."""

    def __init__(self):
        h = _lib.lib().tm_reduce_queue_create()
        if not h:
            raise RuntimeError(f"tm_reduce_queue_create failed: {_lib.last_error()}")
        self.handle = C.c_void_p(h)

    def pending(self) -> int:
        return int(_lib.lib().tm_reduce_queue_pending(self.handle))

    def flush(self):
        _lib.call("tm_reduce_flush", self.handle, _stream())

    def close(self):
        if self.handle is not None:
            _lib.lib().tm_reduce_queue_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# per-thread binding of the queue the current backward call owns (reduce_scope) and whether the
# call sites inside a ``defer_reductions`` block pass it (else NULL: reduce now)
import threading as _threading  # noqa: E402
_TLS = _threading.local()


class reduce_scope:
    """Bind a fresh ReduceQueue to this thread for one backward call; anything still queued at
    exit is flushed on the current stream, then the queue is destroyed."""

    def __enter__(self):
        self.prev = getattr(_TLS, "queue", None)
        self.q = ReduceQueue()
        _TLS.queue = self.q
        return self.q

    def __exit__(self, *exc):
        try:
            if exc[0] is None and self.q.pending() > 0:
                self.q.flush()
        finally:
            _TLS.queue = self.prev
            self.q.close()
        return False


def _rq():
    """The tm_reduce_queue* argument of a call site: the bound queue inside defer_reductions()."""
    q = getattr(_TLS, "queue", None)
    if q is not None and getattr(_TLS, "deferring", False):
        return q.handle
    return C.c_void_p(0)


class defer_reductions:
    """Queue the parameter-gradient slab sums issued inside the block in the thread's bound
    ReduceQueue; they run as ONE launch at the next ``flush_reductions()``.  Outside a
    ``reduce_scope`` the sums run immediately (nothing to defer into)."""

    def __enter__(self):
        self.prev = getattr(_TLS, "deferring", False)
        _TLS.deferring = getattr(_TLS, "queue", None) is not None
        return self

    def __exit__(self, *exc):
        _TLS.deferring = self.prev
        return False


def flush_reductions():
    q = getattr(_TLS, "queue", None)
    if q is not None:
        q.flush()


# ----------------------------------------------------------------------------- NystromAttention core
def nystrom_core_forward(qkv, geo: Geometry, wconv, tdtype, dt_code, pool, cls_row=None):
    """App. A eq. 4-9 on q, k, v [3, B*h, n, 64] -> merged [B, n, h*64] (T) + saved state.
    ``cls_row``: only that row of merged (and of the A1 log-sum-exp) is computed (clsrow.hip)."""
    n, nbh, nh = geo.n, geo.nbh, geo.heads
    q, k, v = qkv[0], qkv[1], qkv[2]
    st = _stream()
    ql = pool(nbh * NL * DH).view(nbh, NL, DH)
    kl = pool(nbh * NL * DH).view(nbh, NL, DH)
    ql_t = pool(nbh * NL * DH, tdtype).view(nbh, NL, DH)
    kl_t = pool(nbh * NL * DH, tdtype).view(nbh, NL, DH)
    with probe("landmarks"):
        _lib.call("tm_nys_landmarks", dt_code, _p(q), _p(k), nbh, n, _p(ql), _p(kl), _p(ql_t), _p(kl_t), st)
    a2 = pool(nbh * NL * NL).view(nbh, NL, NL)
    w = pool(nbh * NL * DH).view(nbh, NL, DH)
    lse3 = pool(nbh * NL)
    work = pool(_lib.query("tm_nys_a3_workspace", nbh, n) // 4)
    # (measured: running A3 V on a second stream beside the pseudo-inverse chain slowed
    #  the step -- the chain's launches then wait for CUs -- so the path stays serial; in bench
    #  mode the partials' combine runs inside the chain's last launch, on the CUs it leaves idle)
    prec = 1 if dt_code == BF16 else 0
    a2s = None
    if prec:
        # bench mode: the key-split A3 forward also writes A2 (+ its split bf16 hi/lo planes, the
        # operands of the pseudo-inverse chain, pinv_split.hip); the partials' combine runs in the
        # chain's last launch
        a2s = pool(nbh * NL * NL)   # hi + lo bf16 planes = one fp32 matrix's bytes
        with probe("a3_fwd"):
            _lib.call("tm_nys_a3_fwd_sim2", _p(ql), _p(kl), _p(k), _p(v), nbh, n, _p(work), _p(a2), _p(a2s), st)
    else:
        with probe("a3_fwd"):
            _lib.call("tm_nys_a3_fwd", dt_code, _p(ql), _p(k), _p(v), nbh, n, _p(work), _p(w), _p(lse3), st)
    if prec:
        saved = pool(_lib.query("tm_pinv_split_saved_floats", nbh, PINV_ITERS))
        with probe("pinv_fwd"):
            _lib.call("tm_pinv_fwd_split_a3", _p(a2), _p(a2s), nbh, PINV_ITERS, _p(saved), _p(work),
                      _lib.query("tm_nys_a3_partials", nbh, n), _p(w), _p(lse3), st)
        z = saved[:nbh * NL * NL].view(nbh, NL, NL)
    else:
        saved = pool(_lib.query("tm_pinv_saved_floats", nbh, PINV_ITERS))
        _lib.call("tm_nys_sim2_softmax", _p(ql), _p(kl), nbh, _p(a2), st)
        _lib.call("tm_pinv_fwd", _p(a2), nbh, PINV_ITERS, prec, _p(saved), st)
        z = saved[PINV_ITERS * nbh * NL * NL:(PINV_ITERS + 1) * nbh * NL * NL].view(nbh, NL, NL)
    y = pool(nbh * NL * DH).view(nbh, NL, DH)
    if dt_code == BF16:     # Y and its bf16 operand copy from the same launch
        y_t = pool(nbh * NL * DH, tdtype)
        bmm([bmm_job(z, 0, w, 0, y, NL, DH, NL, Ct=y_t, ct_mode=1)], nbh, prec)
    else:
        bmm([bmm_job(z, 0, w, 0, y, NL, DH, NL)], nbh, prec)
        y_t = y
    merged = pool(geo.B * n * nh * DH, tdtype).view(geo.B, n, nh * DH)
    lse1 = pool(nbh * n)
    if cls_row is not None:
        _lib.call("tm_cls_a1_row_fwd", dt_code, _p(q), _p(v), _p(kl_t), _p(y_t), _p(wconv), nbh, nh, n, cls_row,
                  _p(merged), _p(lse1), st)
    else:
        with probe("a1_fwd"):
            _lib.call("tm_nys_a1_fwd", dt_code, _p(q), _p(v), _p(kl_t), _p(y_t), _p(wconv), nbh, nh, n, _p(merged),
                      _p(lse1), st)
    state = dict(ql=ql, kl=kl, ql_t=ql_t, kl_t=kl_t, a2=a2, a2s=a2s, pinv=saved, z=z, w=w, lse3=lse3, y=y,
                 y_t=y_t, lse1=lse1)
    return merged, state


def nystrom_core_backward(dmerged, merged, qkv, state, geo: Geometry, wconv, tdtype, dt_code, pool,
                          dwconv_out, scale, cls_row=None, xn=None):
    """Backward of nystrom_core_forward: returns (dqkv [B, n, 3*h*64] (T), qrows); writes dwconv_out.
    ``cls_row``: dmerged is [B, h*64], the only non-zero row (``cls_row``) of the dense gradient.
    ``xn`` (bf16 class-row layer): the q block of dqkv is NOT written; qrows = (Aq, Xs), the
    operands of the q part's two small products (tm_cls_q_rows), else qrows = None."""
    n, nbh, nh = geo.n, geo.nbh, geo.heads
    q, k, v = qkv[0], qkv[1], qkv[2]
    st = _stream()
    mat = nbh * NL * NL
    prec = 1 if dt_code == BF16 else 0
    y_t = state["y_t"]
    dk = pool(nbh * n * DH)
    dkl = pool(nbh * NL * DH).view(nbh, NL, DH)
    dy = pool(nbh * NL * DH).view(nbh, NL, DH)
    dqkv_early = None
    fused = state["a2s"] is not None     # bf16 mode: the A3 backward writes the final k / v parts
    if cls_row is not None:
        # one non-zero query row: dq row, rank-1 dk~ / dY, the conv33 dv window (clsrow.hip); the
        # bf16 consumers read only that row / window, the fp32 path reads dense zero-filled buffers
        alloc = pool if fused else (lambda numel: torch.zeros(numel, dtype=torch.float32, device=q.device))
        dq = alloc(nbh * n * DH)
        dv = pool(nbh * n * DH, tdtype) if fused else alloc(nbh * n * DH)   # dv in T (the fused A3 reads bf16)
        _lib.call("tm_cls_a1_row_bwd", dt_code, _p(dmerged), _p(q), _p(v), _p(state["kl_t"]), _p(y_t),
                  _p(state["lse1"]), _p(wconv), geo.B, nh, n, cls_row, _p(dq), _p(dkl), _p(dy), _p(dv),
                  _p(dwconv_out), st)
    else:
        # conv33 backward + D1
        # bf16 mode: dq goes straight into the q part of dqkv as bf16 (tm_nys_a1_bwd_dqkv); the
        # landmark term is added there in place at the end (tm_nys_assemble_q_slab_inplace)
        dqkv_early = pool(geo.B * n * 3 * nh * DH, tdtype).view(geo.B, n, 3 * nh * DH) if fused else None
        dq = None if fused else pool(nbh * n * DH)
        dv = pool(nbh * n * DH, tdtype)      # the conv backward's dv in T (bf16 mode: read once by the fused A3)
        d1 = pool(nbh * n)
        with defer_reductions(), probe("conv_bwd"):
            work = pool(_lib.query("tm_nys_conv_bwd_workspace", geo.B, nh, n) // 4)
            _lib.call("tm_nys_conv_bwd", dt_code, _p(dmerged), _p(merged), _p(v), _p(wconv), nbh, nh, n, _p(dv),
                      _p(d1), _p(work), _p(dwconv_out), _rq(), st)
        # A1 product backward: dq (complete), dkl, dY
        qpw = 256 if n % 256 == 0 else 32
        work = pool(_lib.query("tm_nys_a1_bwd_workspace", nbh, n, qpw) // 4)
        with defer_reductions():     # its dk~ and dY slab sums as one launch
            with probe("a1_bwd"):
                if fused:
                    _lib.call("tm_nys_a1_bwd_dqkv", _p(q), _p(dmerged), _p(state["kl_t"]), _p(y_t), _p(state["lse1"]),
                              _p(d1), nbh, nh, n, _p(dqkv_early), C.c_float(scale), _p(work), _p(dkl), _p(dy), _rq(), st)
                else:
                    _lib.call("tm_nys_a1_bwd", dt_code, _p(q), _p(dmerged), _p(state["kl_t"]), _p(y_t),
                              _p(state["lse1"]), _p(d1), nbh, nh, n, qpw, _p(dq), _p(work), _p(dkl), _p(dy), 0, _rq(),
                              st)
        flush_reductions()
    # Y = Z W
    dz = pool(mat).view(nbh, NL, NL)
    dw = pool(nbh * NL * DH).view(nbh, NL, DH)
    pwork = None
    if state["a2s"] is not None:
        # the split bf16 hi / lo planes of dZ (work[0] of tm_pinv_bwd_split) from the same launch
        pwork = pool(_lib.query("tm_pinv_bwd_split_workspace_floats", nbh))
        dz_job = bmm_job(dy, 0, state["w"], 1, dz, NL, NL, DH, Ct=pwork, ct_mode=2, ct_plane=mat)
    else:
        dz_job = bmm_job(dy, 0, state["w"], 1, dz, NL, NL, DH)
    # dW = Z^T dY with, from the same launch, its T copy (the A3 backward's dO) and D3 =
    # rowsum(dW o W) as the two 32-column partials the A3 backward sums
    d3 = pool(2 * nbh * NL)
    if dt_code == BF16:
        dw_t = pool(nbh * NL * DH, tdtype)
        dw_job = bmm_job(state["z"], 1, dy, 0, dw, NL, DH, NL, Ct=dw_t, ct_mode=1)
    else:
        dw_t = dw
        dw_job = bmm_job(state["z"], 1, dy, 0, dw, NL, DH, NL)
    dw_job.Rd, dw_job.Rw = d3.data_ptr(), state["w"].data_ptr()
    bmm([dz_job, dw_job], nbh, prec)
    dql3 = pool(nbh * NL * DH).view(nbh, NL, DH)
    work3 = pool(_lib.query("tm_nys_a3_bwd_workspace", nbh, n) // 4)
    if not fused:
        # A3 product backward: dk (=), dv (+=), dql3 (=)
        with probe("a3_bwd"):
            _lib.call("tm_nys_a3_bwd", dt_code, _p(state["ql_t"]), _p(dw_t), _p(k), _p(v), _p(state["lse3"]),
                      _p(d3), nbh, nh, n, _p(dk), _p(dv), _p(work3), _p(dql3), 0, _rq(), st)
    # pseudo-inverse backward -> dA2, then softmax backward
    ds2 = pool(mat).view(nbh, NL, NL)
    if state["a2s"] is not None:
        # split operands; the softmax backward is fused into the chain's last launch
        with probe("pinv_bwd"):
            _lib.call("tm_pinv_bwd_split", _p(state["a2"]), _p(state["a2s"]), nbh, PINV_ITERS, _p(state["pinv"]),
                      _p(pwork), 1, _p(ds2), st)
    else:
        da2 = pool(mat).view(nbh, NL, NL)
        pwork = pool(_lib.query("tm_pinv_bwd_workspace_floats", nbh))
        _lib.call("tm_pinv_bwd", _p(state["a2"]), nbh, PINV_ITERS, prec, _p(state["pinv"]), _p(dz), _p(pwork),
                  _p(da2), st)
        _lib.call("tm_softmax_bwd_rows256", _p(state["a2"]), _p(da2), _p(ds2), nbh * NL, st)
    dql = pool(nbh * NL * DH).view(nbh, NL, DH)
    dqkv = None if cls_row is None and fused else pool(geo.B * n * 3 * nh * DH, tdtype).view(geo.B, n, 3 * nh * DH)
    if dqkv is None:
        dqkv = dqkv_early
    if fused:
        # dq~ (landmark path, without the A3 part) and the final dk~ (+= the A1 part) first; the
        # fused A3 backward then writes k / v of dqkv and dq~3; assemble_q writes q
        bmm([bmm_job(ds2, 0, state["kl"], 0, dql, NL, DH, NL),
             bmm_job(ds2, 1, state["ql"], 0, dkl, NL, DH, NL, E1=dkl, e1=1.0)], nbh, prec)
        with probe("a3_bwd"):
            lo, hi = (0, n) if cls_row is None else (max(cls_row - 16, 0), min(cls_row + 17, n))
            # dql = NULL: the dq~3 partial slab stays in work3; assemble_q_slab sums it in place
            _lib.call("tm_nys_a3_bwd_fused", _p(state["ql_t"]), _p(dw_t), _p(k), _p(v), _p(state["lse3"]), _p(d3),
                      nbh, nh, n, _p(dv), lo, hi, _p(dkl), _p(work3), None, _p(dqkv), _rq(), st)
        slabs = _lib.query("tm_nys_a3_bwd_slabs", nbh, n)
        if cls_row is None:
            _lib.call("tm_nys_assemble_q_slab_inplace", _p(dql), _p(work3), slabs, geo.B, nh, n, C.c_float(scale),
                      _p(dqkv), st)
        elif xn is not None:
            qr = pool(2 * geo.B * QROWS * nh * DH)
            Aq, Xs = qr[:geo.B * QROWS * nh * DH].view(geo.B, QROWS, nh * DH), qr[geo.B * QROWS * nh * DH:].view(
                geo.B, QROWS, nh * DH)
            with probe("cls_q_rows"):
                _lib.call("tm_cls_q_rows", _p(dql), _p(work3), slabs, _p(dq), _p(xn), geo.B, nh, n, cls_row, _p(Aq),
                          _p(Xs), st)
            return dqkv, (Aq, Xs)
        else:
            _lib.call("tm_nys_assemble_q_slab", dt_code, _p(dq), cls_row, _p(dql), _p(work3), slabs, geo.B, nh, n,
                      C.c_float(scale), _p(dqkv), st)
        return dqkv, None
    bmm([bmm_job(ds2, 0, state["kl"], 0, dql, NL, DH, NL, E1=dql3, e1=1.0),
         bmm_job(ds2, 1, state["ql"], 0, dkl, NL, DH, NL, E1=dkl, e1=1.0)], nbh, prec)
    _lib.call("tm_nys_assemble_dqkv", dt_code, _p(dq), _p(dql), _p(dk), _p(dkl), _p(dv), geo.B, nh, n,
              C.c_float(scale), _p(dqkv), st)
    return dqkv, None


# ----------------------------------------------------------------------------- TransLayer
def translayer_forward(H, geo: Geometry, prm, tdtype, dt_code, pool, drop_p, seed, seed_dev=None, cls_only=False):
    """H [B*S, D] fp32 -> H + NystromAttention(LN(H)) (code/models/TransMIL.py:45-57).

    ``cls_only`` (the last layer, whose output the logits read only at the class token,
    :201-203): the attention output, to_out and the residual add are computed for the class
    rows b*S only; the other output rows are left unwritten."""
    B, S, n, D, pad = geo.B, geo.S, geo.n, geo.D, geo.pad
    st = _stream()
    xn = pool(B * n * D, tdtype).view(B, n, D)
    mean = pool(B * S)
    rstd = pool(B * S)
    with probe("ln_fwd"):
        _lib.call("tm_layernorm_fwd", _p(H), _p(prm["norm_w"]), _p(prm["norm_b"]), C.c_float(LN_EPS), B * S, D,
                  S, n, pad, dt_code, _p(xn), _p(mean), _p(rstd), st)
    qkv = pool(3 * geo.nbh * n * DH, tdtype).view(3, geo.nbh, n, DH)
    with probe("qkv_gemm"):
        gemm(xn, prm["wqkv"], qkv, B * n, 3 * D, D, lda=D, ldb=D, ldc=0, dtype=dt_code,
             qkv=(B, geo.heads, DH, n, DH ** -0.5))
    merged, state = nystrom_core_forward(qkv, geo, prm["wconv"], tdtype, dt_code, pool,
                                         cls_row=pad if cls_only else None)
    Hout = pool(B * S * D).view(B * S, D)
    if cls_only:
        _lib.call("tm_cls_out_fwd", dt_code, _p(merged), _p(prm["wo"]), _p(prm["bo"]), _p(H), B, n, pad, S, D,
                  C.c_float(drop_p), C.c_uint64(seed), _p(seed_dev), _p(Hout), st)
    else:
        with probe("out_gemm"):
            gemm(merged, prm["wo"], Hout, B * n, D, D, lda=D, ldb=D, ldc=D, dtype=dt_code, c_dtype=F32,
                 bias=prm["bo"], drop_p=drop_p, seed=seed, seed_ptr=seed_dev, resid=H, rowmap=(n, pad, S, 0, 0, 0))
    saved = dict(xn=xn, mean=mean, rstd=rstd, qkv=qkv, merged=merged, core=state, seed=seed, seed_dev=seed_dev,
                 drop_p=drop_p, cls_only=cls_only)
    return Hout, saved


def translayer_backward(dH, H_in, saved, geo: Geometry, prm, grads, tdtype, dt_code, pool, dout=None, head=None):
    """dH [B*S, D] fp32 (gradient of the layer output) is turned IN PLACE into the
    gradient of the layer input.  Parameter gradients go to ``grads``.  ``dout``: the padded
    to_out-dropout gradient, already written by the producer of dH (tm_ppeg_bwd).  ``head``: the
    tm_cls_head_out_bwd head arguments (class-row layer only): dH's class row is then computed
    by that launch from the CE head instead of read."""
    B, S, n, D, pad = geo.B, geo.S, geo.n, geo.D, geo.pad
    st = _stream()
    if saved["cls_only"]:
        # dH is zero outside the class rows: dropout, dWo, dbo and dmerged on those rows only
        dmerged = pool(B * D, tdtype).view(B, D)
        if head is not None:
            _lib.call("tm_cls_head_out_bwd", dt_code, *head, _p(dH), _p(saved["merged"]), _p(prm["wo"]), n, pad, S,
                      D, C.c_float(saved["drop_p"]), C.c_uint64(saved["seed"]), _p(saved["seed_dev"]),
                      _p(grads["wo"]), _p(grads["bo"]), _p(dmerged), st)
        else:
            _lib.call("tm_cls_out_bwd", dt_code, _p(dH), _p(saved["merged"]), _p(prm["wo"]), B, n, pad, S, D,
                      C.c_float(saved["drop_p"]), C.c_uint64(saved["seed"]), _p(saved["seed_dev"]), _p(grads["wo"]),
                      _p(grads["bo"]), _p(dmerged), st)
    else:
        if dout is None:
            dout = pool(B * n * D, tdtype).view(B, n, D)
            _lib.call("tm_dropout_bwd_pad", dt_code, _p(dH), B, S, n, pad, D, C.c_float(saved["drop_p"]),
                      C.c_uint64(saved["seed"]), _p(saved["seed_dev"]), _p(dout), st)
        # to_out: dWo = dout^T merged ; dbo = colsum(dout) ; dmerged = dout Wo
        with defer_reductions(), probe("wgrad_out"):
            weight_grad(dout, saved["merged"], grads["wo"], D, D, B * n, ldy=D, ldx=D, dtype=dt_code,
                        work_pool=pool, bias_out=grads["bo"])
        dmerged = pool(B * n * D, tdtype).view(B, n, D)
        with probe("dmerged_gemm"):
            gemm(dout, prm["wo"], dmerged, B * n, D, D, lda=D, ldb=D, ldc=D, b_kn=1, dtype=dt_code)
    # bf16 class-row layer: q reaches the loss only through its landmark means and the class row, so
    # the q part of to_qkv's backward runs as two small products on tm_cls_q_rows' operands
    qrows_on = (CLS_Q_ROWS and saved["cls_only"] and dt_code == BF16 and saved["core"]["a2s"] is not None
                and "wqkv_f32" in prm)
    dqkv, qrows = nystrom_core_backward(dmerged, saved["merged"], saved["qkv"], saved["core"], geo, prm["wconv"],
                                        tdtype, dt_code, pool, grads["wconv"], DH ** -0.5,
                                        cls_row=pad if saved["cls_only"] else None,
                                        xn=saved["xn"] if qrows_on else None)
    dxn = pool(B * n * D, tdtype).view(B, n, D)
    rpb = _LN_BWD_RPB   # LN backward rows per block: 16 = 4 rows per wave, one ahead in flight (partials via the
                        # deferred reduce; 4 / 8 / 32 measured slower or level, profiles/r06w_*, r06x_*)
    if qrows is None:
        # to_qkv: dWqkv = dqkv^T xn ; dxn = dqkv Wqkv
        with defer_reductions(), probe("wgrad_qkv"):
            weight_grad(dqkv, saved["xn"], grads["wqkv"], 3 * D, D, B * n, ldy=3 * D, ldx=D, dtype=dt_code,
                        work_pool=pool)
        with probe("dxn_gemm"):
            gemm(dqkv, prm["wqkv"], dxn, B * n, D, 3 * D, lda=3 * D, ldb=D, ldc=D, b_kn=1, dtype=dt_code)
        # LayerNorm backward, accumulated into dH (residual branch already there)
        with defer_reductions():
            work = pool(_lib.query("tm_layernorm_bwd_workspace", B * S, D, rpb) // 4)
            _lib.call("tm_layernorm_bwd", _p(dxn), dt_code, _p(H_in), _p(prm["norm_w"]), _p(saved["mean"]),
                      _p(saved["rstd"]), B * S, D, S, n, pad, rpb, int(saved["cls_only"]), _p(dH), _p(work),
                      _p(grads["norm_w"]),
                      _p(grads["norm_b"]), _rq(), st)
        return
    # k / v parts: dW_kv = dqkv_kv^T xn, dxn = dqkv_kv W_kv (K = 2D instead of 3D)
    dkv = dqkv.view(B * n, 3 * D)[:, D:]
    with defer_reductions(), probe("wgrad_qkv"):
        weight_grad(dkv, saved["xn"], grads["wqkv"][D:], 2 * D, D, B * n, ldy=3 * D, ldx=D, dtype=dt_code,
                    work_pool=pool)
    with probe("dxn_gemm"):
        gemm(dkv, prm["wqkv"][D:], dxn, B * n, D, 2 * D, lda=3 * D, ldb=D, ldc=D, b_kn=1, dtype=dt_code)
    # q part: dWq = scale Aq^T Xs ; G = scale Aq Wq (its rows added to dxn by segment in the LN backward)
    Aq, Xs = qrows
    scale = DH ** -0.5
    wq = prm["wqkv_f32"][:D]
    gwq = grads["wqkv"][:D]
    G = pool(B * QROWS * D).view(B, QROWS, D)
    with probe("cls_q_products"):
        jobs = [bmm_job(Aq.view(B * QROWS, D), 0, wq, 0, G.view(B * QROWS, D), B * QROWS, D, D, alpha=scale),
                bmm_job(Aq[0], 1, Xs[0], 0, gwq, D, D, QROWS, alpha=scale)]
        bmm(jobs, 1, 1)
        for b in range(1, B):   # K <= 512 per product: one bag at a time, accumulated
            bmm([bmm_job(Aq[b], 1, Xs[b], 0, gwq, D, D, QROWS, alpha=scale, E1=gwq, e1=1.0)], 1, 1)
    with defer_reductions():
        work = pool(_lib.query("tm_layernorm_bwd_workspace", B * S, D, rpb) // 4)
        _lib.call("tm_layernorm_bwd_seg", _p(dxn), dt_code, _p(H_in), _p(prm["norm_w"]), _p(saved["mean"]),
                  _p(saved["rstd"]), B * S, D, S, n, pad, rpb, int(saved["cls_only"]), _p(G), n // NL, NL, QROWS,
                  _p(dH), _p(work), _p(grads["norm_w"]), _p(grads["norm_b"]), _rq(), st)


# ----------------------------------------------------------------------------- whole model
# _fc1 layouts the fused engine runs: the parameter prefix of the Linear whose GELU output is
# grid-padded (``main``) and the optional Linear + GELU + LayerNorm stage before it (``inner``)
FC1_PLAIN = {"main": "_fc1.0", "inner": None}                                  # TransMIL.py:128-133
FC1_RCC2048 = {"main": "_fc1.3", "inner": ("_fc1.0", "_fc1.2")}               # TransMIL.py:100-111
# input already embedded to D (the 768 _fc1 branch run by ops, TransMIL.py:122-126; CTMIL's conv
# stack, CTMIL.py:137-141): grid pad + class token only, and the backward returns dL/dx
FC1_EMBED = {"main": None, "inner": None}


class TransMILEngine:
    """Fused TransMIL forward / backward, heads = 8, dim_head = 64, 256 landmarks.

    ``fc1``: FC1_PLAIN (``in_features -> Linear+GELU``, code/models/TransMIL.py:128-133) or
    FC1_RCC2048 (``Linear(2048,1024)+GELU+LayerNorm(1024)+Linear(1024,512)+GELU``, :100-111).
    ``head``: parameter prefix of the class-token Linear (``_fc`` in TransMIL :155, ``_fc2`` in
    code/models/MDMIL.py:73).
    ``cls_only``: layer 2's attention output / to_out forward and backward on the class rows only
    (the logits read nothing else of it; clsrow.hip).  False runs them dense (same results)."""

    def __init__(self, dtype: torch.dtype = torch.bfloat16, fc1=None, head="_fc", cls_only=True):
        if dtype not in (torch.bfloat16, torch.float32):
            raise ValueError("compute dtype must be torch.bfloat16 or torch.float32")
        self.tdtype = dtype
        self.dt_code = BF16 if dtype == torch.bfloat16 else F32
        self.fc1 = FC1_PLAIN if fc1 is None else fc1
        self.head = head
        self.cls_only = cls_only
        _lib.lib()

    def _cast(self, w, pool):
        if self.dt_code == F32:
            return w.contiguous()
        out = pool(w.numel(), self.tdtype)
        _lib.call("tm_cast_f32", self.dt_code, _p(w.contiguous()), _p(out), w.numel(), _stream())
        return out.view(w.shape)

    def _cast_many(self, ws, pool):
        """T copies of several fp32 weights in one launch (fp32 mode: the weights themselves)."""
        ws = [w.contiguous() for w in ws]
        if self.dt_code == F32:
            return ws
        tab = _lib.CastTable()
        tab.count = len(ws)
        outs = []
        off = 0
        for i, w in enumerate(ws):
            o = pool(w.numel(), self.tdtype).view(w.shape)
            tab.src[i], tab.dst[i], tab.offset[i] = w.data_ptr(), o.data_ptr(), off
            off += w.numel()
            outs.append(o)
        tab.offset[len(ws)] = off
        _lib.call("tm_cast_f32_many", self.dt_code, C.byref(tab), _stream())
        return outs

    def prepare(self, params, pool, x2d=None, counter=None, seed_out=None, cls_rows=None):
        """fp32 master parameters -> the per-call operand set (T copies of the GEMM weights and,
        when given, of the bag ``x2d``), the folded PPEG kernel, and the dropout counter
        advanced into ``seed_out`` and (``cls_rows = (H, B, S)``) the class-token rows -- all in ONE
        launch (tm_step_prepare)."""
        D = params["norm.weight"].shape[0]
        p = {"D": D}
        main, inner = self.fc1["main"], self.fc1["inner"]
        ws = [params["layer1.attn.to_qkv.weight"], params["layer1.attn.to_out.0.weight"],
              params["layer2.attn.to_qkv.weight"], params["layer2.attn.to_out.0.weight"]]
        if main is not None:
            ws.append(params[main + ".weight"])
        if inner is not None:
            ws.append(params[inner[0] + ".weight"])
        tab = _lib.CastTable()
        if self.dt_code == F32:
            outs = [w.contiguous() for w in ws]
            p["xt"] = None if x2d is None else x2d.contiguous()
        else:
            # the preparation launch casts whole 4-element pieces: a bag whose B*N*F is not a
            # multiple of 4 (odd in_features) is cast by its own launch instead
            x_in_table = x2d is not None and x2d.numel() % 4 == 0
            srcs = [w.contiguous() for w in ws] + ([x2d.contiguous()] if x_in_table else [])
            outs, off = [], 0
            for i, w in enumerate(srcs):
                o = pool(w.numel(), self.tdtype).view(w.shape)
                tab.src[i], tab.dst[i], tab.offset[i] = w.data_ptr(), o.data_ptr(), off
                off += w.numel()
                outs.append(o)
            tab.count = len(srcs)
            tab.offset[len(srcs)] = off
            if x_in_table:
                p["xt"] = outs.pop()
            else:
                p["xt"] = None if x2d is None else self._cast(x2d, pool)
        wqkv1, wo1, wqkv2, wo2 = outs[:4]
        if main is not None:
            p["w1"] = outs[4]
            p["b1"] = params[main + ".bias"]
        if inner is not None:
            p["w0"], p["b0"] = outs[5], params[inner[0] + ".bias"]   # inner implies main
            p["ln0_w"], p["ln0_b"] = params[inner[1] + ".weight"], params[inner[1] + ".bias"]
        p["cls"] = params["cls_token"]
        for li, (wqkv, wo) in ((1, (wqkv1, wo1)), (2, (wqkv2, wo2))):
            pre = f"layer{li}."
            p[li] = {
                "norm_w": params[pre + "norm.weight"], "norm_b": params[pre + "norm.bias"],
                "wqkv": wqkv,
                "wqkv_f32": params[pre + "attn.to_qkv.weight"].contiguous(),
                "wo": wo,
                "bo": params[pre + "attn.to_out.0.bias"],
                "wconv": params[pre + "attn.res_conv.weight"].contiguous(),
            }
        wfold = pool(D * 49)
        bfold = pool(D)
        _lib.call("tm_step_prepare", self.dt_code, C.byref(tab), _p(params["pos_layer.proj.weight"]),
                  _p(params["pos_layer.proj.bias"]), _p(params["pos_layer.proj1.weight"]),
                  _p(params["pos_layer.proj1.bias"]), _p(params["pos_layer.proj2.weight"]),
                  _p(params["pos_layer.proj2.bias"]), D, _p(wfold), _p(bfold), _p(counter), _p(seed_out),
                  _p(params["cls_token"] if cls_rows else None), _p(cls_rows[0] if cls_rows else None),
                  cls_rows[1] if cls_rows else 0, cls_rows[2] if cls_rows else 0, _stream())
        p["wfold"], p["bfold"] = wfold, bfold
        p["norm_w"], p["norm_b"] = params["norm.weight"], params["norm.bias"]
        p["fc_w"], p["fc_b"] = params[self.head + ".weight"], params[self.head + ".bias"]
        return p

    def forward(self, x, params, drop_p=0.0, seeds=(0x1F123BB5, 0x2A9F4C61), seed_dev=None, counter=None, ce=None):
        """x [B, N, F] fp32 (on the GPU) -> logits [B, C] fp32 and the saved context.

        ``ce = (label int64 [B], class_stats int32 [C, 2] or None)``: the training step's
        CrossEntropyLoss(logits, one_hot(label)) with Y_prob / Y_hat in the head's launch
        (tm_head_ce_fwd); ctx["ce"] = (label, prob, loss, yhat) and backward(gloss=...) takes
        the loss gradient straight into the head backward (tm_head_ce_bwd).

        Dropout (train mode) hashes (row, col) with a per-layer seed; with ``seed_dev``
        (a 1-element int64 device tensor) the seed is read on the device, so a
        captured hipGraph draws a fresh mask every replay; with ``counter`` as well, the
        preparation launch first advances the counter and writes it into ``seed_dev``."""
        dev = x.device
        pool = Pool(dev)
        B, N, F = x.shape
        D = params["norm.weight"].shape[0]
        heads = params["layer1.attn.res_conv.weight"].shape[0]
        if D != heads * DH:
            raise NotImplementedError(f"HIP NystromAttention needs dim_head == 64 (D={D}, heads={heads})")
        geo = Geometry(B, N, F, D, heads)
        H0 = pool(B * geo.S * D).view(B * geo.S, D)
        prm = self.prepare(params, pool, None if self.fc1["main"] is None else x.reshape(B * N, F),
                           counter=counter if seed_dev is not None else None, seed_out=seed_dev,
                           cls_rows=(H0, B, geo.S))
        st = _stream()
        xt = prm["xt"]
        inner = None
        if self.fc1["inner"] is not None:
            # inner stage: y0 = GELU(x W0^T + b0) (fp32, pre-activation kept), then LayerNorm -> T,
            # the operand of the main Linear (code/models/TransMIL.py:101-110)
            Fm = prm["w0"].shape[0]
            y0 = pool(B * N * Fm).view(B * N, Fm)
            pre0 = pool(B * N * Fm).view(B * N, Fm)
            gemm(xt, prm["w0"], y0, B * N, Fm, F, lda=F, ldb=F, ldc=Fm, dtype=self.dt_code, c_dtype=F32,
                 bias=prm["b0"], gelu=True, pre=pre0, ld_pre=Fm)
            xln = pool(B * N * Fm, self.tdtype).view(B * N, Fm)
            mean0, rstd0 = pool(B * N), pool(B * N)
            _lib.call("tm_layernorm_fwd", _p(y0), _p(prm["ln0_w"]), _p(prm["ln0_b"]), C.c_float(LN_EPS), B * N, Fm,
                      N, N, 0, self.dt_code, _p(xln), _p(mean0), _p(rstd0), st)
            inner = dict(xt=xt, y0=y0, pre0=pre0, mean0=mean0, rstd0=rstd0, F=F)
            xt, F = xln, Fm
        # _fc1: Linear + GELU, grid pad (duplicate the first `add` rows); the class-token rows
        # were written by the preparation launch
        if self.fc1["main"] is None:
            if F != D:
                raise ValueError(f"pre-embedded input must be [B, N, {D}], got F={F}")
            pre = None
            H0v, xe = H0.view(B, geo.S, D), x.reshape(B, N, D)
            H0v[:, 1:N + 1].copy_(xe)
            if geo.add:
                H0v[:, N + 1:].copy_(xe[:, :geo.add])
        else:
            # the pre-activation for the GELU backward, in T: bf16 in the bf16 step (half the bytes of the
            # fp32 store and of its read-back; the GELU derivative's input then carries bf16 precision,
            # as the _fc1 operands themselves do), fp32 in the parity mode
            pre = pool(B * N * D, self.tdtype).view(B * N, D)
            with probe("fc1_gemm"):
                gemm(xt, prm["w1"], H0, B * N, D, F, lda=F, ldb=F, ldc=D, dtype=self.dt_code, c_dtype=F32,
                     bias=prm["b1"], gelu=True, pre=pre, ld_pre=D, rowmap=(N, 0, geo.S, 1, geo.add, 1 + N),
                     pre_bf16=self.dt_code == BF16)
        H1, s1 = translayer_forward(H0, geo, prm[1], self.tdtype, self.dt_code, pool, drop_p, seeds[0], seed_dev)
        H2 = pool(B * geo.S * D).view(B * geo.S, D)
        with probe("ppeg_fwd"):
            _lib.call("tm_ppeg_fwd", _p(H1), B, geo.G, D, _p(prm["wfold"]), _p(prm["bfold"]), _p(H2), st)
        # layer 2: the head reads its output only at the class rows (code/models/TransMIL.py:201-203)
        H3, s2 = translayer_forward(H2, geo, prm[2], self.tdtype, self.dt_code, pool, drop_p, seeds[1], seed_dev,
                                    cls_only=self.cls_only)
        Ccls = prm["fc_w"].shape[0]
        logits = torch.empty(B, Ccls, dtype=torch.float32, device=dev)
        xhat = pool(B * D)
        hrstd = pool(B)
        ce_out = None
        if ce is None:
            _lib.call("tm_head_fwd", _p(H3), B, geo.S, D, _p(prm["norm_w"]), _p(prm["norm_b"]), C.c_float(LN_EPS),
                      _p(prm["fc_w"]), _p(prm["fc_b"]), Ccls, _p(logits), _p(xhat), _p(hrstd), st)
        else:
            label, stats = ce
            loss = torch.empty((), dtype=torch.float32, device=dev)
            prob = torch.empty(B, Ccls, dtype=torch.float32, device=dev)
            yhat = torch.empty(B, dtype=torch.int64, device=dev)
            _lib.call("tm_head_ce_fwd", _p(H3), B, geo.S, D, _p(prm["norm_w"]), _p(prm["norm_b"]),
                      C.c_float(LN_EPS), _p(prm["fc_w"]), _p(prm["fc_b"]), Ccls, _p(label), _p(logits), _p(xhat),
                      _p(hrstd), _p(loss), _p(prob), _p(yhat), _p(stats), st)
            ce_out = (label, prob, loss, yhat)
        ctx = dict(geo=geo, prm=prm, xt=xt, pre=pre, H0=H0, H1=H1, H2=H2, s1=s1, s2=s2, xhat=xhat, hrstd=hrstd,
                   inner=inner, ce=ce_out)
        return logits, ctx

    def backward(self, dlogits, ctx, params, out=None, ready=None, gloss=None, parts=2):
        """Returns a dict name -> fp32 gradient with the reference parameter names.  The deferred
        parameter-gradient sums go into a ReduceQueue owned by this call (reentrant across
        threads / streams)."""
        with reduce_scope():
            return self._backward(dlogits, ctx, params, out, ready, gloss, parts)

    def _backward(self, dlogits, ctx, params, out=None, ready=None, gloss=None, parts=2):
        """Body of ``backward``.

        ``gloss``: the gradient of the forward's fused loss (``ce``; a 0-d device tensor); then
        ``dlogits`` is the gradient reaching the logits from other uses, or None.

        ``out``: name -> preallocated fp32 tensor to write each gradient into (the views of a
        ``GradBucket``); ``ready(part)``: called once the head, norm, layer2 and PPEG gradients
        are final (part 0, before layer1's backward is enqueued) and at the end (the last part), so
        a bucketed all-reduce of part 0 overlaps layer1 / _fc1 backward.  ``parts = 3`` (the bucket
        of a world > 1 run, ``TransMIL.grad_bucket_parts(split_layer1=True)``): layer1's gradients
        are flushed and ``ready(1)`` is called as soon as layer1's backward is enqueued, so their
        all-reduce overlaps the _fc1 backward; ``ready(2)`` (class token, _fc1) at the end."""
        geo, prm = ctx["geo"], ctx["prm"]
        dev = ctx["H0"].device
        pool = Pool(dev)
        B, N, F, D, S = geo.B, geo.N, geo.F, geo.D, geo.S
        st = _stream()
        g = out if out is not None else {name: torch.empty_like(p, dtype=torch.float32)
                                         for name, p in params.items()}
        Ccls = prm["fc_w"].shape[0]
        # layer 2 on the class rows reads dL/dH3 only there (its LayerNorm backward writes the rest)
        dH = (torch.empty if self.cls_only else torch.zeros)(B * S, D, dtype=torch.float32, device=dev)
        head = None
        if gloss is not None and dlogits is None and self.cls_only and B == 1 and Ccls <= 4 and D == 512:
            # the head + CE backward rides in layer 2's class-row to_out backward launch
            gls = gloss.float().contiguous()
            ctx["_gloss"] = gls     # keep the scalar alive until the launch is enqueued
            head = (_p(ctx["ce"][1]), _p(ctx["ce"][0]), _p(gls), Ccls, _p(ctx["xhat"]), _p(ctx["hrstd"]),
                    _p(prm["norm_w"]), _p(prm["norm_b"]), _p(prm["fc_w"]), _p(g[self.head + ".weight"]),
                    _p(g[self.head + ".bias"]), _p(g["norm.weight"]), _p(g["norm.bias"]))
        elif gloss is not None:
            label, prob = ctx["ce"][0], ctx["ce"][1]
            scratch = None if (B == 1 and Ccls <= 4) else pool(B * Ccls)
            dl_in = None if dlogits is None else dlogits.float().contiguous()
            _lib.call("tm_head_ce_bwd", _p(prob), _p(label), _p(gloss.float().contiguous()), _p(dl_in), B, Ccls, S,
                      D, _p(ctx["xhat"]), _p(ctx["hrstd"]), _p(prm["norm_w"]), _p(prm["norm_b"]), _p(prm["fc_w"]),
                      _p(g[self.head + ".weight"]), _p(g[self.head + ".bias"]), _p(g["norm.weight"]),
                      _p(g["norm.bias"]), _p(dH), _p(scratch), st)
        else:
            _lib.call("tm_head_bwd", _p(dlogits.contiguous()), B, Ccls, S, D, _p(ctx["xhat"]), _p(ctx["hrstd"]),
                      _p(prm["norm_w"]), _p(prm["norm_b"]), _p(prm["fc_w"]), _p(g[self.head + ".weight"]),
                      _p(g[self.head + ".bias"]),
                      _p(g["norm.weight"]), _p(g["norm.bias"]), _p(dH), st)
        dout1 = None
        for li, Hin, saved in ((2, ctx["H2"], ctx["s2"]), (1, ctx["H0"], ctx["s1"])):
            pre = f"layer{li}."
            gl = {"wo": g[pre + "attn.to_out.0.weight"], "bo": g[pre + "attn.to_out.0.bias"],
                  "wqkv": g[pre + "attn.to_qkv.weight"], "wconv": g[pre + "attn.res_conv.weight"],
                  "norm_w": g[pre + "norm.weight"], "norm_b": g[pre + "norm.bias"]}
            translayer_backward(dH, Hin, saved, geo, prm[li], gl, self.tdtype, self.dt_code, pool, dout=dout1,
                                head=head if li == 2 else None)
            if li == 2:
                dH1 = pool(B * S * D).view(B * S, D)
                work = pool(_lib.query("tm_ppeg_bwd_workspace", B, geo.G, D) // 4)
                # the stencil also writes layer 1's padded to_out-dropout gradient (its first step)
                s1 = ctx["s1"]
                dout1 = pool(B * geo.n * D, self.tdtype).view(B, geo.n, D)
                with probe("ppeg_bwd"), defer_reductions():
                    _lib.call("tm_ppeg_bwd", _p(ctx["H1"]), _p(dH), B, geo.G, D, _p(prm["wfold"]), _p(dH1),
                              _p(work), _p(g["pos_layer.proj.weight"]), _p(g["pos_layer.proj.bias"]),
                              _p(g["pos_layer.proj1.weight"]), _p(g["pos_layer.proj1.bias"]),
                              _p(g["pos_layer.proj2.weight"]), _p(g["pos_layer.proj2.bias"]), self.dt_code,
                              _p(dout1), geo.n, geo.pad, C.c_float(s1["drop_p"]), C.c_uint64(s1["seed"]),
                              _p(s1["seed_dev"]), _rq(), st)
                dH = dH1
                flush_reductions()     # head, norm, layer2 and PPEG parameter gradients final
                if ready is not None:
                    ready(0)
            elif ready is not None and parts >= 3 and self.fc1["main"] is not None:
                flush_reductions()     # layer1's parameter gradients final: part 1 goes now
                ready(1)
        if self.fc1["main"] is None:
            # pre-embedded input: dL/dx = the token rows + the duplicated pad rows folded back
            dHv = dH.view(B, S, D)
            dx = dHv[:, 1:N + 1].clone()
            if geo.add:
                dx[:, :geo.add] += dHv[:, N + 1:]
            torch.sum(dHv[:, 0], dim=0, out=g["cls_token"].view(D))
            g["__dx__"] = dx
            flush_reductions()
            if ready is not None:
                ready(1)
            return g
        # _fc1 backward (GELU + grid-pad fold) and the class token
        dpre = pool(B * N * D, self.tdtype).view(B * N, D)
        _lib.call("tm_fc1_gelu_bwd", self.dt_code, _p(dH), _p(ctx["pre"]), B, N, S, geo.add, D, _p(dpre),
                  _p(g["cls_token"]), st)
        main, inner = self.fc1["main"], ctx["inner"]
        Fx = F if inner is None else prm["w0"].shape[0]
        with defer_reductions(), probe("wgrad_fc1"):
            weight_grad(dpre, ctx["xt"], g[main + ".weight"], D, Fx, B * N, ldy=D, ldx=Fx, dtype=self.dt_code,
                        work_pool=pool, bias_out=g[main + ".bias"])
        if inner is not None:
            # d LN-out = dpre W1 ; LayerNorm backward ; GELU backward ; W0 / b0 gradients
            w0n, lnn = self.fc1["inner"]
            Fm, Fin = Fx, inner["F"]
            dxln = pool(B * N * Fm).view(B * N, Fm)
            gemm(dpre, prm["w1"], dxln, B * N, Fm, D, lda=D, ldb=Fm, ldc=Fm, b_kn=1, dtype=self.dt_code, c_dtype=F32)
            dy0 = torch.zeros(B * N, Fm, dtype=torch.float32, device=dev)
            rpb = 64
            work = pool(_lib.query("tm_layernorm_bwd_workspace", B * N, Fm, rpb) // 4)
            _lib.call("tm_layernorm_bwd", _p(dxln), F32, _p(inner["y0"]), _p(prm["ln0_w"]), _p(inner["mean0"]),
                      _p(inner["rstd0"]), B * N, Fm, N, N, 0, rpb, 0, _p(dy0), _p(work), _p(g[lnn + ".weight"]),
                      _p(g[lnn + ".bias"]), _rq(), st)
            dpre0 = pool(B * N * Fm, self.tdtype).view(B * N, Fm)
            _lib.call("tm_gelu_bwd", self.dt_code, _p(dy0), _p(inner["pre0"]), B * N * Fm, _p(dpre0), st)
            weight_grad(dpre0, inner["xt"], g[w0n + ".weight"], Fm, Fin, B * N, ldy=Fm, ldx=Fin, dtype=self.dt_code,
                        work_pool=pool, bias_out=g[w0n + ".bias"])
        flush_reductions()
        if ready is not None:
            ready(parts - 1 if parts >= 3 else 1)
        return g


# ----------------------------------------------------------------------------- standalone NystromAttention
class NystromEngine:
    """``nystrom_attention.NystromAttention.forward(x)`` (no mask) on the HIP kernels:
    front pad, to_qkv, core, to_out (+ Dropout), keep the last n rows (App. A eq. 1-10)."""

    def __init__(self, dtype: torch.dtype = torch.bfloat16):
        self.tdtype = dtype
        self.dt_code = BF16 if dtype == torch.bfloat16 else F32
        _lib.lib()

    def _cast(self, w, pool):
        if self.dt_code == F32:
            return w.contiguous()
        out = pool(w.numel(), self.tdtype)
        _lib.call("tm_cast_f32", self.dt_code, _p(w.contiguous()), _p(out), w.numel(), _stream())
        return out.view(w.shape)

    def forward(self, x, wqkv, wo, bo, wconv, heads, drop_p=0.0, seed=0, seed_dev=None):
        B, S, D = x.shape
        pool = Pool(x.device)
        geo = Geometry(B, max(S - 1, 1), D, D, heads)
        geo.S = S
        geo.n = ((S + NL - 1) // NL) * NL
        geo.pad = geo.n - S
        geo.l = geo.n // NL
        n, pad = geo.n, geo.pad
        xc = x.reshape(B * S, D).contiguous()
        xp = pool(B * n * D, self.tdtype).view(B, n, D)
        _lib.call("tm_pad_rows", self.dt_code, _p(xc), B, S, n, pad, D, _p(xp), _stream())
        wqkv_t, wo_t = self._cast(wqkv, pool), self._cast(wo, pool)
        qkv = pool(3 * geo.nbh * n * DH, self.tdtype).view(3, geo.nbh, n, DH)
        gemm(xp, wqkv_t, qkv, B * n, 3 * D, D, lda=D, ldb=D, ldc=0, dtype=self.dt_code,
             qkv=(B, heads, DH, n, DH ** -0.5))
        merged, state = nystrom_core_forward(qkv, geo, wconv.contiguous(), self.tdtype, self.dt_code, pool)
        out = torch.empty(B, S, D, dtype=torch.float32, device=x.device)
        gemm(merged, wo_t, out, B * n, D, D, lda=D, ldb=D, ldc=D, dtype=self.dt_code, c_dtype=F32,
             bias=bo, drop_p=drop_p, seed=seed, seed_ptr=seed_dev, rowmap=(n, pad, S, 0, 0, 0))
        ctx = dict(geo=geo, xp=xp, qkv=qkv, merged=merged, core=state, wqkv_t=wqkv_t, wo_t=wo_t,
                   wconv=wconv.contiguous(), drop_p=drop_p, seed=seed, seed_dev=seed_dev)
        return out, ctx

    def backward(self, dout, ctx):
        with reduce_scope():
            return self._backward(dout, ctx)

    def _backward(self, dout, ctx):
        geo = ctx["geo"]
        B, S, D, n, pad = geo.B, geo.S, geo.D, geo.n, geo.pad
        pool = Pool(dout.device)
        st = _stream()
        dpad = pool(B * n * D, self.tdtype).view(B, n, D)
        _lib.call("tm_dropout_bwd_pad", self.dt_code, _p(dout.contiguous()), B, S, n, pad, D,
                  C.c_float(ctx["drop_p"]), C.c_uint64(ctx["seed"]), _p(ctx["seed_dev"]), _p(dpad), st)
        dwo = torch.empty(D, D, dtype=torch.float32, device=dout.device)
        dbo = torch.empty(D, dtype=torch.float32, device=dout.device)
        weight_grad(dpad, ctx["merged"], dwo, D, D, B * n, ldy=D, ldx=D, dtype=self.dt_code, work_pool=pool,
                    bias_out=dbo)
        dmerged = pool(B * n * D, self.tdtype).view(B, n, D)
        gemm(dpad, ctx["wo_t"], dmerged, B * n, D, D, lda=D, ldb=D, ldc=D, b_kn=1, dtype=self.dt_code)
        dwconv = torch.empty_like(ctx["wconv"], dtype=torch.float32)
        dqkv, _ = nystrom_core_backward(dmerged, ctx["merged"], ctx["qkv"], ctx["core"], geo, ctx["wconv"],
                                        self.tdtype, self.dt_code, pool, dwconv, DH ** -0.5)
        dwqkv = torch.empty(3 * D, D, dtype=torch.float32, device=dout.device)
        weight_grad(dqkv, ctx["xp"], dwqkv, 3 * D, D, B * n, ldy=3 * D, ldx=D, dtype=self.dt_code, work_pool=pool)
        dx = torch.empty(B, S, D, dtype=torch.float32, device=dout.device)
        gemm(dqkv, ctx["wqkv_t"], dx, B * n, D, 3 * D, lda=3 * D, ldb=D, ldc=D, b_kn=1, dtype=self.dt_code,
             c_dtype=F32, rowmap=(n, pad, S, 0, 0, 0))
        flush_reductions()      # the res_conv weight gradient queued by nystrom_core_backward
        return dx, dwqkv, dwo, dbo, dwconv
