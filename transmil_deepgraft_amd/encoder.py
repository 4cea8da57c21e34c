"""On-GPU RetCCL ResNet-50 tile encoder for the image path (BASELINE config 5).

Replaces ``ModelInterface``'s ``backbone == 'retccl'`` feature extractor
(code/models/model_interface.py:237-247: ``ResNet.resnet50(num_classes=128, mlp=False,
two_branch=False, normlinear=True)``, checkpoint loaded with ``strict=False``, every parameter
frozen, ``fc = Identity``) and the image branch of ``ModelInterface.forward`` (:300-316:
``[B, bag, 3, 224, 224] -> [B*bag, 3, 224, 224] -> model_ft -> [B, bag, 2048] -> model``).

Same module / parameter / buffer names as code/models/ResNet.py (ResNet :130-277, Bottleneck
:75-117, resnet50 :309), so a RetCCL checkpoint loads unchanged.  MI355X-first execution:

* channels-last bf16 activations (``compute_dtype``), PyTorch-ROCm (MIOpen) convolutions --
  the encoder is frozen and outside the hand-written NystromAttention/PPEG path;
* in eval mode every BatchNorm is folded into its convolution once (weights rescaled, bias
  added) -- no separate normalisation passes -- and every 1x1 convolution (36 of the 53) runs
  as a hipBLASLt GEMM over the channels-last [n*h*w, c] rows (csrc/conv1x1.hip) whose epilogue
  adds the bias, the residual (conv3) and applies the ReLU; the 3x3 convolutions' bias + ReLU is
  one in-place HIP pass (tm_bias_act);
* in train mode the BatchNorms use batch statistics and update the running statistics, as the
  reference's frozen-but-train-mode encoder does under Lightning: each one statistics pass + one
  apply pass fused with its ReLU (bn3 with the residual), csrc/bn_train.hip, convolutions without
  bias (1x1 through the same hipBLASLt GEMM); with autograd on (unfrozen parameters) the modules
  run as written;
* in eval mode tiles go through in chunks (``chunk`` tiles, default 512; per-tile math, so the
  chunking is exact) so the activation peak stays a few GB whatever the bag size; in train mode
  the bag is held as pieces of ``train_pieces(N, chunk)`` tiles while every BatchNorm's statistics
  span the whole batch (tens of GB for a 4096-tile bag, well inside one GPU's HBM); the
  [B*bag, 2048] features stay on the device for the fused TransMIL engine (no host round trip);
* no library kernel is ever handed a tensor of 2 GiB or more (``_lib_guard``; a whole 4096-tile
  bag is 3.3 G elements at the stem output, and MIOpen's implicit-GEMM NHWC kernels wrap 32-bit
  offsets there: wrong outputs measured, see LIB_MAX_BYTES): every path runs on pieces of at most
  ``max_tiles_per_call()`` tiles or refuses the call.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class Bottleneck(nn.Module):
    """1x1 -> 3x3 (stride) -> 1x1 x4 with BN after each, residual + ReLU (ResNet.py:75-117)."""

    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, momentum_bn=0.1):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes, momentum=momentum_bn)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes, momentum=momentum_bn)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4, momentum=momentum_bn)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        idt = self.downsample(x) if self.downsample is not None else x
        return self.relu(out + idt)


def _fold(conv: nn.Conv2d, bn: nn.BatchNorm2d, dtype, cl=True):
    """conv followed by eval-mode BN as one conv: (w * g / sqrt(v + eps), b - m * g / sqrt(v + eps))."""
    s = bn.weight.detach().double() / torch.sqrt(bn.running_var.double() + bn.eps)
    w = (conv.weight.detach().double() * s[:, None, None, None]).to(dtype)
    b = (bn.bias.detach().double() - bn.running_mean.double() * s).to(dtype)
    return w.contiguous(memory_format=torch.channels_last if cl else torch.contiguous_format), b


def _dtype_code(t):
    from ._lib import BF16, F32
    if t.dtype not in (torch.bfloat16, torch.float32):
        raise RuntimeError("encoder: bf16 or fp32 tensors expected")
    return BF16 if t.dtype == torch.bfloat16 else F32


def _conv1x1_gemm(x, w, b, relu, residual=None):
    """1x1 convolution (BN folded) over a channels-last tensor as one hipBLASLt GEMM over its
    [n*h*w, c] rows with the bias (+ residual) (+ ReLU) epilogue (tm_conv1x1)."""
    from . import _lib
    from .engine import _p, _stream
    cl = torch.channels_last
    n, c, h, wd = x.shape
    cout = w.shape[0]
    if not x.is_contiguous(memory_format=cl) or w.dtype != x.dtype or (b is not None and b.dtype != x.dtype):
        raise RuntimeError("conv1x1: channels-last input, weight and bias of one dtype expected")
    y = torch.empty((n, h, wd, cout), dtype=x.dtype, device=x.device).permute(0, 3, 1, 2)
    if residual is not None and (residual.shape != y.shape or residual.dtype != y.dtype or
                                 not residual.is_contiguous(memory_format=cl)):
        raise RuntimeError("conv1x1: channels-last residual of the output's shape and dtype expected")
    # stream-ordered scratch from the caching allocator (no library-global workspace)
    ws_bytes = _conv1x1_ws_bytes()
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=x.device)
    args = (_dtype_code(x), _p(x), _p(w.contiguous()), _p(b), _p(residual) if residual is not None else None,
            _p(y), n * h * wd, c, cout, int(relu), _p(ws), ws_bytes, _stream())
    key = (x.device.index, x.dtype, n * h * wd, c, cout, bool(relu), b is not None, residual is not None)
    if key not in _TUNED and _tuning_enabled() and not torch.cuda.is_current_stream_capturing():
        # first call of a shape, outside capture: time hipBLASLt's candidates once (the ABI's one
        # synchronising entry point, tm_conv1x1_tune); y is then written by the real call below
        _lib.call("tm_conv1x1_tune", *args)
        _TUNED.add(key)
    _lib.call("tm_conv1x1", *args)
    return y


_TUNED = set()
_WS = []


def _conv1x1_ws_bytes():
    if not _WS:
        from . import _lib
        _WS.append(_lib.query("tm_conv1x1_workspace_bytes"))
    return _WS[0]


def _tuning_enabled():
    """The timed algorithm search picks hipBLASLt's fastest candidate per process from wall-clock
    timings, so two processes (or ranks) may run different algorithms and their encoder features
    differ by rounding.  Off with TM_CONV1X1_TUNE=0 or under torch.use_deterministic_algorithms(True)
    (then every process runs the heuristic's first choice: run-to-run and rank-to-rank identical)."""
    import os
    if torch.are_deterministic_algorithms_enabled():
        return False
    return os.environ.get("TM_CONV1X1_TUNE", "1") != "0"


def _bias_act_(y, b, relu=True):
    """y = act(y + b[channel]) in place over a channels-last tensor, one HIP pass (tm_bias_act)."""
    from . import _lib
    from .engine import _p, _stream
    if not y.is_contiguous(memory_format=torch.channels_last):
        y = y.contiguous(memory_format=torch.channels_last)
    n, c, h, wd = y.shape
    _lib.call("tm_bias_act", _dtype_code(y), _p(y), _p(b), n * h * wd, c, int(relu), _stream())
    return y


def _stem_pool_(y, b):
    """maxpool3x3/2(relu(y + b)) of the raw channels-last bf16 stem output in one HIP pass
    (tm_bias_relu_maxpool; the same values as tm_bias_act + max_pool2d: + b, ReLU and bf16 rounding
    are monotone, so they commute with the max)."""
    from . import _lib
    from .engine import _p, _stream
    if not y.is_contiguous(memory_format=torch.channels_last):
        y = y.contiguous(memory_format=torch.channels_last)
    n, c, h, wd = y.shape
    out = torch.empty(n, c, (h - 1) // 2 + 1, (wd - 1) // 2 + 1, dtype=y.dtype, device=y.device,
                      memory_format=torch.channels_last)
    _lib.call("tm_bias_relu_maxpool", _p(y), _p(b), _p(out), n, h, wd, c, _stream())
    return out


def _stem_pool_bn_(y, st):
    """maxpool3x3/2(relu(y * scale + shift)) with the stem BatchNorm's batch statistics in one HIP
    pass (tm_bn_relu_maxpool; the same values as tm_bn_apply + max_pool2d)."""
    from . import _lib
    from .engine import _p, _stream
    n, c, h, wd = y.shape
    out = torch.empty(n, c, (h - 1) // 2 + 1, (wd - 1) // 2 + 1, dtype=y.dtype, device=y.device,
                      memory_format=torch.channels_last)
    _lib.call("tm_bn_relu_maxpool", _p(y), _p(st[0]), _p(st[1]), _p(out), n, h, wd, c, _stream())
    return out


def _bn_train_stats(ys, bn, ws):
    """Train-mode BatchNorm statistics of a channels-last activation held as a list of bag pieces
    (tm_bn_train_stats: the statistics span every piece): returns fp32 [2, C] (scale, shift) and
    updates the module's running statistics as nn.BatchNorm2d does (momentum; None = cumulative
    average)."""
    import ctypes as C
    from . import _lib
    from .engine import _p, _stream
    if any(not y.is_contiguous(memory_format=torch.channels_last) for y in ys):
        raise RuntimeError("bn_train_stats: channels-last activations expected")
    c = ys[0].shape[1]
    st = torch.empty(2, c, dtype=torch.float32, device=ys[0].device)
    track = bn.track_running_stats and bn.running_mean is not None
    if track:
        bn.num_batches_tracked.add_(1)
    m = bn.momentum if bn.momentum is not None else (1.0 / float(bn.num_batches_tracked.item()) if track else 0.0)
    g = bn.weight.detach() if bn.weight is not None else torch.ones(c, device=ys[0].device)
    b = bn.bias.detach() if bn.bias is not None else torch.zeros(c, device=ys[0].device)
    ptrs = (C.c_void_p * len(ys))(*[y.data_ptr() for y in ys])
    rows = (C.c_longlong * len(ys))(*[y.numel() // c for y in ys])
    _lib.call("tm_bn_train_stats", _dtype_code(ys[0]), ptrs, rows, len(ys), c, _p(g), _p(b),
              _p(bn.running_mean) if track else None, _p(bn.running_var) if track else None, float(m),
              float(bn.eps), _p(st[0]), _p(st[1]), _p(ws), ws.numel(), _stream())
    return st


def _bn_apply_(y, st, residual=None, rst=None, relu=True):
    """y = act(y * scale + shift (+ residual | + residual * rscale + rshift)) in place
    (tm_bn_apply) over channels-last tensors."""
    from . import _lib
    from .engine import _p, _stream
    if not y.is_contiguous(memory_format=torch.channels_last):
        raise RuntimeError("bn_apply: channels-last activation expected")
    n, c, h, wd = y.shape
    if residual is not None and (residual.shape != y.shape or residual.dtype != y.dtype or
                                 not residual.is_contiguous(memory_format=torch.channels_last)):
        raise RuntimeError("bn_apply: channels-last residual of the output's shape and dtype expected")
    _lib.call("tm_bn_apply", _dtype_code(y), _p(y), _p(st[0]), _p(st[1]), _p(residual),
              _p(rst[0]) if rst is not None else None, _p(rst[1]) if rst is not None else None,
              n * h * wd, c, int(relu), _stream())
    return y


def _stem_conv_pool(x, wp, b):
    """The eval stem (BN folded) in one HIP pass: maxpool3x3/2(relu(conv7x7/2(x) + b)) from bf16
    tiles at any strides to a channels-last bf16 [n, 64, PH, PW] (tm_stem_conv_pool; the
    convolution output never reaches HBM)."""
    from . import _lib
    from .engine import _p, _stream
    n, c, h, wd = x.shape
    if c != 3 or x.dtype != torch.bfloat16 or wp.shape != (64, 224):
        raise RuntimeError("stem_conv_pool: bf16 [n, 3, h, w] tiles and [64, 224] packed weights expected")
    ch, cw = (h - 1) // 2 + 1, (wd - 1) // 2 + 1
    out = torch.empty(n, 64, (ch - 1) // 2 + 1, (cw - 1) // 2 + 1, dtype=x.dtype, device=x.device,
                      memory_format=torch.channels_last)
    sn, sc, sh, sw = x.stride()
    _lib.call("tm_stem_conv_pool", _p(x), _p(wp), _p(b), _p(out), n, h, wd, sn, sc, sh, sw, _stream())
    return out


def _stem_bn_stats(x, wp, bn):
    """Train-mode bn1 statistics of the stem convolution over the whole bag (tm_stem_bn_stats: the
    convolution recomputed, never stored): returns fp32 [2, 64] (scale, shift) and updates the
    module's running statistics as nn.BatchNorm2d does."""
    from . import _lib
    from .engine import _p, _stream
    n, c, h, wd = x.shape
    if c != 3 or x.dtype != torch.bfloat16:
        raise RuntimeError("stem_bn_stats: bf16 [n, 3, h, w] tiles expected")
    st = torch.empty(2, 64, dtype=torch.float32, device=x.device)
    track = bn.track_running_stats and bn.running_mean is not None
    if track:
        bn.num_batches_tracked.add_(1)
    m = bn.momentum if bn.momentum is not None else (1.0 / float(bn.num_batches_tracked.item()) if track else 0.0)
    g = bn.weight.detach() if bn.weight is not None else torch.ones(64, device=x.device)
    b = bn.bias.detach() if bn.bias is not None else torch.zeros(64, device=x.device)
    ws = torch.empty(_lib.query("tm_stem_bn_stats_workspace"), dtype=torch.float64, device=x.device)
    sn, sc, sh, sw = x.stride()
    _lib.call("tm_stem_bn_stats", _p(x), _p(wp), n, h, wd, sn, sc, sh, sw, _p(g), _p(b),
              _p(bn.running_mean) if track else None, _p(bn.running_var) if track else None, float(m),
              float(bn.eps), _p(st[0]), _p(st[1]), _p(ws), ws.numel(), _stream())
    return st


def _stem_conv_pool_bn(x, wp, st):
    """maxpool3x3/2(relu(bn1(conv7x7/2(x)))) with the batch statistics st in one pass
    (tm_stem_conv_pool_bn): channels-last bf16 [n, 64, PH, PW]."""
    from . import _lib
    from .engine import _p, _stream
    n, c, h, wd = x.shape
    ch, cw = (h - 1) // 2 + 1, (wd - 1) // 2 + 1
    out = torch.empty(n, 64, (ch - 1) // 2 + 1, (cw - 1) // 2 + 1, dtype=x.dtype, device=x.device,
                      memory_format=torch.channels_last)
    sn, sc, sh, sw = x.stride()
    _lib.call("tm_stem_conv_pool_bn", _p(x), _p(wp), _p(st[0]), _p(st[1]), _p(out), n, h, wd, sn, sc, sh, sw,
              _stream())
    return out


def _subsample(x, s):
    """x[:, :, ::s, ::s] of a channels-last activation as a channels-last tensor (tm_subsample2d:
    16-B channel pieces; the strided torch copy ran at ~2.7 TB/s)."""
    if s == 1:
        return x
    from . import _lib
    from .engine import _p, _stream
    n, c, h, wd = x.shape
    if not x.is_contiguous(memory_format=torch.channels_last) or (c * x.element_size()) % 16:
        return _cl(x[:, :, ::s, ::s])
    out = torch.empty(n, c, (h - 1) // s + 1, (wd - 1) // s + 1, dtype=x.dtype, device=x.device,
                      memory_format=torch.channels_last)
    _lib.call("tm_subsample2d", _dtype_code(x), _p(x), _p(out), n, h, wd, c, s, _stream())
    return out


def _pack_stem(w):
    """Folded stem weights [64, 3, 7, 7] -> tm_stem_conv_pool's [64][ky][kx 8][c 4] (kx = 7, c = 3 zero)."""
    wp = torch.zeros(64, 7, 8, 4, dtype=w.dtype, device=w.device)
    wp[:, :, :7, :3] = w.permute(0, 2, 3, 1)
    return wp.reshape(64, 224).contiguous()


def _stem_fused_enabled():
    import os
    return os.environ.get("TM_STEM_FUSED", "1") != "0"


def _cl(t):
    return t.contiguous(memory_format=torch.channels_last)


# Every library kernel of the encoder (MIOpen / CK convolutions, PyTorch pooling, hipBLASLt) is
# handed tensors of less than 2 GiB.  Round 5 measured why (scripts/dev/c5_drift.py,
# profiles/r05_c5_drift.json): fed a whole 4096-tile fp32 bag, MIOpen's implicit-GEMM NHWC forward
# kernel for layer2.0's 3x3 / stride-2 convolution (igemm_fwd_gtcx35_nhwc_fp32_..._bt128x128x16)
# returned WRONG outputs for every tile from 2674 on (per-tile relative error up to 0.35; tiles
# 0-2673 bit-identical to the piecewise run, every other op of the network bit-identical) -- a
# 32-bit offset wrapping where 2 x the input's elements (= its bf16 bytes) pass 2^31 although the
# tensor itself has 1.6 G elements.  That is the round-4 one-pass drift (3.35e-3 on the features,
# only on tiles >= 2674), and the same wrap in a bf16 kernel is the likely source of the round-4
# train-mode illegal-address fault.  So the bag is always held in pieces of at most
# max_tiles_per_call() tiles (668 fp32 / 1337 bf16 at 224 x 224), and _lib_guard refuses any
# library tensor of 2 GiB or more before it reaches a library.
LIB_MAX_BYTES = 2 ** 31 - 1


def tile_elems_max(h=224, w=224):
    """The largest activation one h x w tile produces in RetCCL ResNet-50 (elements): the input, the
    stem output (64 x ceil(h/2) x ceil(w/2)) or layer1's output (256 x ceil(h/4) x ceil(w/4))."""
    h2, w2 = (h + 1) // 2, (w + 1) // 2
    h4, w4 = (h2 + 1) // 2, (w2 + 1) // 2
    return max(3 * h * w, 64 * h2 * w2, 256 * h4 * w4)


def max_tiles_per_call(h=224, w=224, elem_bytes=4):
    """Tiles per library call that keep every activation under LIB_MAX_BYTES (224 x 224: 668 tiles
    in fp32, 1337 in bf16)."""
    return max(1, LIB_MAX_BYTES // (tile_elems_max(h, w) * elem_bytes))


def _lib_guard(*ts):
    for t in ts:
        if t is not None and t.numel() * t.element_size() > LIB_MAX_BYTES:
            raise RuntimeError(f"encoder: a library call on {t.numel() * t.element_size()} bytes (shape "
                               f"{tuple(t.shape)}) reaches 2^31; the bag must be held in pieces of "
                               f"<= max_tiles_per_call() tiles")


def _conv_out_numel(x, w, stride, padding):
    n, _, h, wd = x.shape
    k = w.shape[2]
    ho = (h + 2 * padding - k) // stride + 1
    wo = (wd + 2 * padding - k) // stride + 1
    return n * w.shape[0] * ho * wo


def _lib_conv2d(x, w, b=None, stride=1, padding=0):
    """F.conv2d (MIOpen / CK) with input and output sizes checked against LIB_MAX_BYTES first."""
    _lib_guard(x)
    if _conv_out_numel(x, w, stride, padding) * x.element_size() > LIB_MAX_BYTES:
        raise RuntimeError(f"encoder: convolution output of {_conv_out_numel(x, w, stride, padding)} elements "
                           f"reaches 2^31 bytes; hold the bag in pieces of <= max_tiles_per_call() tiles")
    return F.conv2d(x, w, b, stride=stride, padding=padding)


def _lib_max_pool(x):
    _lib_guard(x)
    return F.max_pool2d(x, 3, 2, 1)


def train_pieces(n_tiles, chunk, h=224, w=224, elem_bytes=4, max_pieces=64):
    """Piece size of the train-mode bag: at least ``chunk`` tiles, enough that the statistics call
    combines at most ``max_pieces`` pieces (tm_bn_train_stats), never more than
    max_tiles_per_call(h, w, elem_bytes).  Raises when no piece size satisfies both."""
    cap = max_tiles_per_call(h, w, elem_bytes)
    size = min(max(chunk, -(-n_tiles // max_pieces)), cap)
    if -(-n_tiles // size) > max_pieces:
        raise RuntimeError(f"encoder: a {n_tiles}-tile train-mode bag needs more than {max_pieces} pieces of "
                           f"<= {cap} tiles (tm_bn_train_stats combines at most {max_pieces})")
    return size


class RetCCLResNet50(nn.Module):
    """``ResNet(Bottleneck, [3, 4, 6, 3])`` with ``fc = Identity``: tiles [n, 3, 224, 224] ->
    features [n, 2048] fp32."""

    def __init__(self, momentum_bn=0.1, chunk=512):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, kernel_size=7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64, momentum=momentum_bn)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(kernel_size=3, stride=2, padding=1)
        self.layer1 = self._stage(64, 3, 1, momentum_bn)
        self.layer2 = self._stage(128, 4, 2, momentum_bn)
        self.layer3 = self._stage(256, 6, 2, momentum_bn)
        self.layer4 = self._stage(512, 3, 2, momentum_bn)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Identity()                         # model_interface.py:245
        self.compute_dtype = torch.bfloat16
        self.chunk = chunk
        self.channels_last = True
        self._folded = None
        self._folded_key = None
        self._cast = None               # train mode: conv weights in the compute dtype, channels-last
        self._cast_key = None
        for p in self.parameters():                     # model_interface.py:243-244
            p.requires_grad = False

    def _stage(self, planes, blocks, stride, momentum_bn):
        down = None
        if stride != 1 or self.inplanes != planes * 4:
            down = nn.Sequential(nn.Conv2d(self.inplanes, planes * 4, 1, stride=stride, bias=False),
                                 nn.BatchNorm2d(planes * 4, momentum=momentum_bn))
        layers = [Bottleneck(self.inplanes, planes, stride, down, momentum_bn)]
        self.inplanes = planes * 4
        layers += [Bottleneck(self.inplanes, planes, momentum_bn=momentum_bn) for _ in range(1, blocks)]
        return nn.Sequential(*layers)

    def set_compute_dtype(self, dtype):
        if dtype not in (torch.bfloat16, torch.float32):
            raise ValueError("compute dtype must be torch.bfloat16 or torch.float32")
        self.compute_dtype = dtype
        self._folded = None
        return self

    def load_state_dict(self, state_dict, strict=True, assign=False):
        self._folded = None
        return super().load_state_dict(state_dict, strict=strict, assign=assign)

    def train(self, mode=True):
        self._folded = None
        return super().train(mode)

    def load_retccl_checkpoint(self, path):
        """``load_state_dict(torch.load(path), strict=False)`` as the reference does (:242), with
        the safe loader; the 128-way ``fc`` of the checkpoint is dropped (fc is Identity)."""
        sd = torch.load(path, map_location="cpu", weights_only=True)
        return self.load_state_dict({k: v for k, v in sd.items() if not k.startswith("fc.")}, strict=False)

    # ------------------------------------------------------------------ eval: folded convolutions
    def _fold_key(self):
        """Identity of every parameter and buffer the folded weights derive from (storage and
        in-place version counter): a checkpoint loaded through a parent module, ``.to()``, an
        in-place weight edit or a BatchNorm statistics update all change it, so the next eval
        forward re-folds instead of reading stale conv+BN weights."""
        return tuple((t.data_ptr(), t._version, t.dtype) for t in
                     list(self.parameters()) + list(self.buffers()))

    def _fold_all(self):
        dt, cl = self.compute_dtype, self.channels_last
        f = {"stem": _fold(self.conv1, self.bn1, dt, cl), "blocks": []}
        if dt == torch.bfloat16:
            f["stem_packed"] = _pack_stem(f["stem"][0])
        for stage in (self.layer1, self.layer2, self.layer3, self.layer4):
            for blk in stage:
                d = None
                if blk.downsample is not None:
                    d = _fold(blk.downsample[0], blk.downsample[1], dt, cl) + (blk.downsample[0].stride,)
                f["blocks"].append((_fold(blk.conv1, blk.bn1, dt, cl), _fold(blk.conv2, blk.bn2, dt, cl) + (blk.stride,),
                                    _fold(blk.conv3, blk.bn3, dt, cl), d))
        self._folded = f

    def _forward_folded(self, x):
        """Eval mode, BN folded.  On the GPU with channels-last activations: every 1x1 convolution
        one hipBLASLt GEMM with its epilogue (conv1: bias + ReLU; downsample: bias; conv3: bias +
        residual + ReLU -- the block output is written once), the 3x3 / stem convolutions through
        MIOpen without bias, then bias + ReLU in one in-place pass."""
        f = self._folded
        w, b = f["stem"]
        if self.channels_last and x.is_cuda:
            if "stem_packed" in f and x.dtype == torch.bfloat16 and _stem_fused_enabled():
                x = _stem_conv_pool(x, f["stem_packed"], b)
            else:
                y = _lib_conv2d(_cl(x), w, None, stride=2, padding=3)
                x = _stem_pool_(y, b) if y.dtype == torch.bfloat16 else _lib_max_pool(_bias_act_(y, b))
            for (w1, b1), (w2, b2, s2), (w3, b3), d in f["blocks"]:
                y = _conv1x1_gemm(x, w1, b1, True)
                y = _bias_act_(_lib_conv2d(y, w2, None, stride=s2, padding=1), b2)
                if d is None:
                    idt = x
                else:
                    idt = _conv1x1_gemm(_subsample(x, d[2][0]), d[0], d[1], False)
                x = _conv1x1_gemm(y, w3, b3, True, residual=idt)
            return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
        x = _lib_max_pool(F.relu(_lib_conv2d(x, w, b, stride=2, padding=3)))
        for (w1, b1), (w2, b2, s2), (w3, b3), d in f["blocks"]:
            y = F.relu(_lib_conv2d(x, w1, b1))
            y = F.relu(_lib_conv2d(y, w2, b2, stride=s2, padding=1))
            y = _lib_conv2d(y, w3, b3)
            idt = x if d is None else _lib_conv2d(x, d[0], d[1], stride=d[2][0])
            x = F.relu(y + idt)
        return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)

    def _forward_train_fused(self, x):
        """Train mode (batch-statistics BatchNorm, frozen parameters, no autograd) on the GPU.
        The bag is held as pieces of ``train_pieces(N, chunk)`` tiles (every convolution / pooling
        on one piece, < 2^31 elements) while each BatchNorm's statistics span all pieces
        (tm_bn_train_stats).  Convolutions without bias (1x1: hipBLASLt GEMM; 3x3 / stem: MIOpen),
        each BatchNorm one statistics pass + one apply pass fused with its ReLU, and bn3 + (BN'd
        downsample) identity + ReLU one pass (tm_bn_apply)."""
        key = self._fold_key()
        if self._cast is None or self._cast_key != key:
            self._cast = {n: _cl(p.detach().to(self.compute_dtype)) for n, p in self.named_parameters()
                          if p.dim() == 4}
            self._cast_key = key
        w = self._cast
        ws = torch.empty(self._bn_ws_floats(), dtype=torch.float32, device=x.device)
        piece = train_pieces(x.shape[0], self.chunk, x.shape[2], x.shape[3], x.element_size())
        if x.dtype == torch.bfloat16 and _stem_fused_enabled():
            # the stem in two hand-written passes over the tiles (statistics, then conv + BN + ReLU +
            # pool): the 112 x 112 x 64 conv output is never stored
            if "stem_packed" not in w:
                w["stem_packed"] = _pack_stem(w["conv1.weight"])
            st = _stem_bn_stats(x, w["stem_packed"], self.bn1)
            xs = [_stem_conv_pool_bn(x[i:i + piece], w["stem_packed"], st) for i in range(0, x.shape[0], piece)]
        else:
            xs = [_cl(_lib_conv2d(_cl(x[i:i + piece]), w["conv1.weight"], None, stride=2, padding=3))
                  for i in range(0, x.shape[0], piece)]
            st = _bn_train_stats(xs, self.bn1, ws)
            if x.dtype == torch.bfloat16:
                xs = [_stem_pool_bn_(p, st) for p in xs]
            else:
                xs = [_lib_max_pool(_bn_apply_(p, st)) for p in xs]
        for si, stage in enumerate((self.layer1, self.layer2, self.layer3, self.layer4), start=1):
            for bi, blk in enumerate(stage):
                pre = f"layer{si}.{bi}."
                ys = [_conv1x1_gemm(p, w[pre + "conv1.weight"], None, False) for p in xs]
                st = _bn_train_stats(ys, blk.bn1, ws)
                ys = [_cl(_lib_conv2d(_bn_apply_(y, st), w[pre + "conv2.weight"], None, stride=blk.stride, padding=1))
                      for y in ys]
                st = _bn_train_stats(ys, blk.bn2, ws)
                ys = [_conv1x1_gemm(_bn_apply_(y, st), w[pre + "conv3.weight"], None, False) for y in ys]
                st3 = _bn_train_stats(ys, blk.bn3, ws)
                if blk.downsample is None:
                    for y, p in zip(ys, xs):
                        _bn_apply_(y, st3, residual=p)
                else:
                    s = blk.downsample[0].stride[0]
                    ds = [_conv1x1_gemm(_subsample(p, s), w[pre + "downsample.0.weight"], None, False) for p in xs]
                    sd = _bn_train_stats(ds, blk.downsample[1], ws)
                    for y, d in zip(ys, ds):
                        _bn_apply_(y, st3, residual=d, rst=sd)
                    del ds
                xs = ys
        return torch.cat([torch.flatten(F.adaptive_avg_pool2d(p, 1), 1) for p in xs])

    @staticmethod
    def _bn_ws_floats():
        from . import _lib
        return _lib.query("tm_bn_train_workspace", 2048)

    def _forward_modules(self, x):
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))

    def forward(self, x):
        if not x.is_cuda:
            raise RuntimeError("RetCCL encoder (MI355X path) needs a GPU tensor")
        dt = self.compute_dtype
        out = torch.empty(x.shape[0], 2048, dtype=torch.float32, device=x.device)
        if not self.training:
            key = self._fold_key()
            if self._folded is None or self._folded_key != key:
                self._fold_all()
                self._folded_key = key
        if self.training and self.channels_last and \
                not self.conv1.weight.is_contiguous(memory_format=torch.channels_last):
            self.to(memory_format=torch.channels_last)
        grad = torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters())
        # train-mode BatchNorm normalises with the statistics of the whole [B*bag] batch the
        # reference feeds model_ft in one call (model_interface.py:303-309): the fused train path
        # holds the bag in pieces whose statistics are combined; eval chunks are per-tile exact.
        # No library call sees a tensor of LIB_MAX_BYTES or more on any path (the module path under
        # autocast keeps fp32 BatchNorm outputs: sized as fp32).
        fused_train = self.training and not grad and self.channels_last
        esz = 2 if dt == torch.bfloat16 and (fused_train or not self.training) else 4
        cap = max_tiles_per_call(x.shape[2], x.shape[3], esz)
        chunk = x.shape[0] if self.training else max(1, min(self.chunk, cap))
        if self.training and not fused_train and x.shape[0] > cap:
            # nn.BatchNorm2d needs the whole batch in one module call; above the cap that call
            # would hand the library > 2^31-element tensors
            raise RuntimeError(f"encoder: train mode with autograd (or without channels-last) takes at most {cap} "
                               f"tiles per call (the whole-batch BatchNorm would hand the library >= 2^31 bytes); got "
                               f"{x.shape[0]}")
        autocast = self.training and not fused_train and dt == torch.bfloat16
        with torch.set_grad_enabled(grad), torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
            for s in range(0, x.shape[0], chunk):
                xc = x[s:s + chunk].to(torch.float32 if autocast else dt)
                if not ((not self.training or fused_train) and self.channels_last and dt == torch.bfloat16
                        and _stem_fused_enabled()):
                    # (the fused stem reads the tiles at any strides: no channels-last copy)
                    xc = xc.contiguous(memory_format=torch.channels_last if self.channels_last
                                       else torch.contiguous_format)
                if not self.training:
                    y = self._forward_folded(xc)
                elif fused_train:
                    y = self._forward_train_fused(xc)
                else:
                    y = self._forward_modules(xc)
                out[s:s + chunk] = y.float()
        return out


def retccl_resnet50(**kw):
    """``ResNet.resnet50(num_classes=128, mlp=False, two_branch=False, normlinear=True)`` with
    ``fc = Identity`` and frozen parameters (model_interface.py:238-245)."""
    return RetCCLResNet50(**kw)


class ImageBagModel(nn.Module):
    """``ModelInterface.forward``'s image path (model_interface.py:300-316): tiles
    ``[B, bag, 3, H, W]`` -> frozen encoder -> ``[B, bag, 2048]`` on the device -> the MIL model
    (TransMIL(n_classes, 2048) runs its RCC-2048 _fc1 branch on the fused engine)."""

    def __init__(self, model_ft: nn.Module, model: nn.Module):
        super().__init__()
        self.model_ft = model_ft
        self.model = model
        self.n_classes = getattr(model, "n_classes", None)

    def forward(self, x):
        B, bag = x.shape[0], x.shape[1]
        feats = self.model_ft(x.reshape(B * bag, *x.shape[2:]))
        return self.model(feats.view(B, bag, -1))
