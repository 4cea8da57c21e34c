"""One rank of the two-rank gradient-averaging test (tests/test_ddp_gpu.py).

Launched twice by the test with RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT in the
environment; both ranks share the one leased GPU, so the process group is gloo (RCCL refuses
two ranks on one device; gloo all-reduces CUDA tensors through host staging).  Each rank runs
the fused HIP TransMIL step (bf16 mode, train mode) on its own bags (argv[4] patches, default
700; 8192 = BASELINE config C4's per-rank workload) through
``TransMILTask.optimization_step`` with ``GradAllReduce(model=..., overlap=True)``: the part-0
all_reduce is issued by the fused backward's mid-backward ``ready(0)`` hook, and with
``accumulate_grad_batches = K`` only every K-th micro-batch reduces (Lightning's DDP no-sync,
code/train.py:178-201).  The final parameters go to ``argv[1]``.

Not collected by pytest (no ``test_`` prefix); imports nothing from ``oracle/``.
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

N_PATCHES = 700


def build_model():
    from transmil_deepgraft_amd.models import TransMIL
    torch.manual_seed(0)
    return TransMIL(2, 512, 512).cuda().train().set_compute_dtype(torch.bfloat16)


def bag(rank, micro, n=N_PATCHES):
    g = torch.Generator(device="cuda").manual_seed(1000 * rank + micro)
    x = torch.rand(1, n, 512, device="cuda", generator=g)
    return x, torch.tensor([(rank + micro) % 2], device="cuda"), None   # (bags, labels, names)


C5_TILES = 8


def build_c5_model():
    """The C5 image path (ImageBagModel: frozen RetCCL ResNet-50, eval-mode BN, bf16 channels-last
    -> TransMIL(2, 2048) on its RCC-2048 _fc1 branch, bf16, train mode); model_interface.py:237-247,
    300-316."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from golden_util import deterministic_encoder_params_
    from transmil_deepgraft_amd.encoder import ImageBagModel, retccl_resnet50
    from transmil_deepgraft_amd.models import TransMIL
    enc = retccl_resnet50()
    deterministic_encoder_params_(enc, 2021)
    enc = enc.set_compute_dtype(torch.bfloat16).eval().cuda()
    torch.manual_seed(0)
    mil = TransMIL(2, 2048).cuda().train().set_compute_dtype(torch.bfloat16)
    return ImageBagModel(enc, mil)


def c5_bag(rank, micro, n=C5_TILES):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from golden_util import encoder_tiles
    x = torch.from_numpy(encoder_tiles(n, seed=500 + 100 * rank + micro)).cuda().view(1, n, 3, 224, 224)
    return x, torch.tensor([(rank + micro) % 2], device="cuda"), None


def main(out_path, k, steps, n=N_PATCHES, mode="feat"):
    import torch.distributed as dist
    from transmil_deepgraft_amd.interface import GradAllReduce, TransMILTask
    torch.cuda.set_device(0)
    dist.init_process_group("gloo")
    rank = dist.get_rank()
    if mode == "c5":
        model = build_c5_model()
        # the frozen encoder has no trainable parameters: the bucket holds the MIL model's
        ar = GradAllReduce(model.parameters(), model=model.model, overlap=True)
        assert len(ar.bucket.ranges) == 3           # world > 1: layer1 cut from the _fc1 part
        data = lambda micro: c5_bag(rank, micro, n)     # noqa: E731
    else:
        model = build_model()
        ar = GradAllReduce(model.parameters(), model=model, overlap=True)
        data = lambda micro: bag(rank, micro, n)        # noqa: E731
    issued = []      # parts whose all_reduce the backward's ready() hook issued (mid-backward)

    def spy(i, inner=ar._on_ready):
        before = set(ar._works)
        inner(i)
        if i in ar._works and i not in before:
            issued.append(i)
    ar.bucket.hooks = [spy]
    task = TransMILTask(model, accumulate_grad_batches=k)
    opt = task.configure_optimizers()[0][0]
    for micro in range(steps * k):
        task.optimization_step(data(micro), opt, allreduce=ar)
    torch.cuda.synchronize()
    trainable = [p for p in model.parameters() if p.requires_grad]
    owned = all(ar.bucket.owns(p) for p in trainable) or all(p.grad is None for p in trainable)
    torch.save({"params": {n: p.detach().cpu() for n, p in model.named_parameters() if p.requires_grad},
                "issued": issued, "owned": owned, "rank": rank, "parts": len(ar.bucket.ranges),
                "exposed_bytes": ar.exposed_bytes()}, out_path)
    ar.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]) if len(sys.argv) > 4 else N_PATCHES,
         sys.argv[5] if len(sys.argv) > 5 else "feat")
