"""CPU oracle (test infrastructure only) for the C5 tile encoder: RetCCL ResNet-50 with
``fc = Identity`` as ``ModelInterface`` builds it (code/models/model_interface.py:238-245:
``ResNet.resnet50(num_classes=128, mlp=False, two_branch=False, normlinear=True)``), restated as a
plain functional forward over a state_dict: eval-mode BatchNorm (running statistics) or, with
``train=True``, train-mode BatchNorm (statistics of the whole batch, running statistics updated
with ``momentum`` as nn.BatchNorm2d does -- the reference's frozen encoder under ``model.train()``).

Follows code/models/ResNet.py:
  * stem: conv1 7x7/2 pad 3 -> bn1 -> ReLU -> maxpool 3/2 pad 1 (ResNet.forward :249-252);
  * layer1..4 = [3, 4, 6, 3] Bottlenecks (_make_layer :214-245): conv1 1x1 -> bn1 -> ReLU ->
    conv2 3x3/stride pad 1 -> bn2 -> ReLU -> conv3 1x1 -> bn3; identity = downsample(x) (1x1/stride
    conv + BN) where the block changes shape; out = ReLU(out + identity) (Bottleneck.forward
    :95-117);
  * global average pool, flatten, fc = Identity (:258-271 with mlp = two_branch = False).

Pinned by tests/golden/retccl_r50_tiles4.npz (features of the reference's own ResNet.py on 4
tiles, fp32 + fp64; tests/test_encoder.py).  Only ``tests/`` import this module.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

BLOCKS = (3, 4, 6, 3)
BN_EPS = 1e-5


def _bn(x, sd, pre):
    given = sd.get("__stats_in__")
    if given is not None and pre in given:
        # train-mode BN whose batch statistics were taken over a larger batch than x (a subset of a
        # bag's tiles normalised with the whole bag's mean / biased variance)
        mean, var = given[pre]
        return F.batch_norm(x, mean.to(x), var.to(x), sd[pre + ".weight"], sd[pre + ".bias"], training=False,
                            eps=BN_EPS)
    return F.batch_norm(x, sd[pre + ".running_mean"], sd[pre + ".running_var"], sd[pre + ".weight"],
                        sd[pre + ".bias"], training=sd["__train__"], momentum=sd["__momentum__"], eps=BN_EPS)


def _bottleneck(x, sd, pre, stride):
    out = F.relu(_bn(F.conv2d(x, sd[pre + ".conv1.weight"]), sd, pre + ".bn1"))
    out = F.relu(_bn(F.conv2d(out, sd[pre + ".conv2.weight"], stride=stride, padding=1), sd, pre + ".bn2"))
    out = _bn(F.conv2d(out, sd[pre + ".conv3.weight"]), sd, pre + ".bn3")
    if pre + ".downsample.0.weight" in sd:
        idt = _bn(F.conv2d(x, sd[pre + ".downsample.0.weight"], stride=stride), sd, pre + ".downsample.1")
    else:
        idt = x
    return F.relu(out + idt)


def features(tiles: torch.Tensor, state_dict: dict, dtype=torch.float64, train=False, momentum=0.1,
             stats_out: dict | None = None, stats_in: dict | None = None) -> torch.Tensor:
    """tiles [n, 3, 224, 224] -> features [n, 2048] (``dtype`` arithmetic on the CPU).  With
    ``train``: batch-statistics BatchNorm over all n tiles; the updated running statistics go into
    ``stats_out`` (name -> tensor) when given.  ``stats_in`` (BN module name, e.g. "layer1.0.bn2" ->
    (mean, biased variance)): those BatchNorms normalise with the given batch statistics instead of
    the n tiles' own (a subset of a bag whose statistics span the whole bag)."""
    sd = {k: v.detach().to("cpu", dtype).clone() for k, v in state_dict.items()
          if not k.endswith("num_batches_tracked")}
    sd["__train__"], sd["__momentum__"] = bool(train), momentum
    sd["__stats_in__"] = None if stats_in is None else {
        k: (m.detach().to("cpu", dtype), v.detach().to("cpu", dtype)) for k, (m, v) in stats_in.items()}
    x = tiles.detach().to("cpu", dtype)
    x = F.relu(_bn(F.conv2d(x, sd["conv1.weight"], stride=2, padding=3), sd, "bn1"))
    x = F.max_pool2d(x, 3, 2, 1)
    for li, nb in enumerate(BLOCKS, start=1):
        for bi in range(nb):
            stride = 2 if (li > 1 and bi == 0) else 1
            x = _bottleneck(x, sd, f"layer{li}.{bi}", stride)
    if stats_out is not None:
        stats_out.update({k: v for k, v in sd.items() if isinstance(k, str) and k.endswith(("running_mean", "running_var"))})
    return torch.flatten(F.adaptive_avg_pool2d(x, 1), 1)
