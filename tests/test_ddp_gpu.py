"""The DDP gradient path on the GPU: the fused backward writing into a GradBucket, gradient
accumulation, and the RCCL all_reduce inside a captured hipGraph (world size 1, forced).

Reference: Lightning DDP with ``accumulate_grad_batches=10`` (code/train.py:178-201); the
gradients of the fused path are checked against the same model's gradients without a bucket
(same kernels, so bit-identical), the graph step against eager steps."""
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _model(seed=0, n_classes=2, feat=256):
    from transmil_deepgraft_amd.models import TransMIL
    torch.manual_seed(seed)
    return TransMIL(n_classes, feat, 512).cuda().eval()


def _bag(i, n=700, feat=256):
    g = torch.Generator(device="cuda").manual_seed(50 + i)
    return torch.rand(1, n, feat, device="cuda", generator=g), torch.tensor([i % 2], device="cuda")


def _loss(model, i):
    from transmil_deepgraft_amd.interface import TransMILTask
    x, y = _bag(i)
    return TransMILTask(model).training_step((x, y, None))


def test_fused_backward_writes_into_bucket():
    """p.grad are views of the bucket (no copy), equal to the un-bucketed gradients bit for bit,
    in the two parts the overlap schedule assumes; a second micro-batch accumulates."""
    from transmil_deepgraft_amd.interface import GradAllReduce
    a, b = _model(), _model()
    ar = GradAllReduce(a.parameters(), model=a)
    fired = []
    ar.bucket.hooks.append(fired.append)
    _loss(a, 0).backward()
    _loss(b, 0).backward()
    torch.cuda.synchronize()
    assert fired == [0, 1]
    assert [len(p) for p in ar.bucket.parts_params] == [len(p) for p in a.grad_bucket_parts()]
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        assert ar.bucket.owns(pa), n
        torch.testing.assert_close(pa.grad, pb.grad, rtol=0, atol=0, msg=n)
    first = {n: p.grad.clone() for n, p in b.named_parameters()}
    _loss(a, 1).backward()          # accumulation: added into the bucket views
    _loss(b, 1).backward()          # autograd accumulation
    torch.cuda.synchronize()
    assert fired == [0, 1, 0, 1]
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        assert ar.bucket.owns(pa), n
        torch.testing.assert_close(pa.grad, pb.grad, rtol=1e-6, atol=1e-9, msg=n)
        assert not torch.equal(pa.grad, first[n]) or first[n].abs().max() == 0, n


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rccl_graph_body(overlap, teardown="close"):
    """(Run in a child process by test_rccl_allreduce_inside_captured_graph.)  init_process_group("nccl") at world size 1 with the collective forced: the whole step
    (forward, CE, fused backward whose part-0 hook issues the RCCL all_reduce mid-backward when
    ``overlap``, the wait + 1/world scale, fused RAdam+Lookahead) captured as ONE hipGraph and
    replayed, against the same steps run eagerly without any collective."""
    import torch.distributed as dist
    from transmil_deepgraft_amd.interface import GradAllReduce, TransMILTask
    import gc
    for attempt in range(5):   # a port free at probe time can be taken before the store binds it
        try:
            dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1,
                                    device_id=torch.device("cuda", torch.cuda.current_device()))
            break
        except dist.DistNetworkError:
            if attempt == 4:
                raise
    graph = ar = None
    try:
        a, b = _model(3), _model(3)
        ta, tb = TransMILTask(a), TransMILTask(b)
        oa, ob = ta.configure_optimizers()[0][0], tb.configure_optimizers()[0][0]
        ar = GradAllReduce(a.parameters(), model=a, overlap=overlap, force=True)
        issued = []
        ar.bucket.hooks.insert(0, lambda i: issued.append(i))
        sx, sy = _bag(0)
        sx, sy = sx.clone(), sy.clone()

        def body():
            ta.training_step((sx, sy, None)).backward()
            ar()
            oa.step()

        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(2):          # warm-up steps (as bench.py); b takes the same two steps
                body()
                oa.zero_grad(set_to_none=True)
        torch.cuda.current_stream().wait_stream(side)
        for _ in range(2):
            tb.training_step((sx, sy, None)).backward()
            ob.step()
            ob.zero_grad(set_to_none=True)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            body()
        for i in range(3):
            x, y = _bag(i + 1)
            sx.copy_(x)
            sy.copy_(y)
            graph.replay()
            tb.training_step((sx, sy, None)).backward()
            ob.step()
            ob.zero_grad(set_to_none=True)
        torch.cuda.synchronize()
        assert issued[:2] == [0, 1]
        for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
            torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-6, msg=n)
    finally:
        # teardown order: the captured graph holds the communicator's kernels
        # (and RCCL's registration of the buffers it captured), the model's bucket holds the
        # all-reduce's hook: drop the graph, close the all-reduce, drain, THEN destroy the group
        torch.cuda.synchronize()
        if teardown == "close":
            if graph is not None:
                graph.reset()
            if ar is not None:
                ar.close()
        graph = ar = None       # teardown == "old": the round-5 order (scripts/dev/rccl_teardown.py)
        gc.collect()
        torch.cuda.synchronize()
        dist.destroy_process_group()


def test_rccl_allreduce_inside_captured_graph():
    """_rccl_graph_body for overlap off, then on, in ONE child process: two NCCL process groups
    initialised and destroyed back to back, each after a hipGraph captured over its all-reduce,
    with the teardown order GradAllReduce.close() documents.  (The child process keeps a failure
    from taking the pytest process with it; it is not needed for the two groups to coexist.)"""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    code = (f"import sys; sys.path.insert(0, {here!r}); sys.path.insert(0, {os.path.dirname(here)!r}); "
            f"import test_ddp_gpu as T; T._rccl_graph_body(False); print('RCCL_GRAPH_OK 0', flush=True); "
            f"T._rccl_graph_body(True); print('RCCL_GRAPH_OK 1', flush=True)")
    r = subprocess.run([sys.executable, "-c", code], cwd=os.path.dirname(here), capture_output=True, timeout=300)
    out = (r.stdout + r.stderr).decode(errors="replace")
    assert r.returncode == 0 and "RCCL_GRAPH_OK 1" in out, f"rc={r.returncode}\n{out[-4000:]}"


@pytest.mark.parametrize("k,npatch", [(1, 700), (3, 700), (1, 8192)])
def test_two_ranks_average_through_the_hip_engine(k, npatch, tmp_path):
    """Two processes on the one leased GPU (gloo: RCCL refuses two ranks on one device), each
    running the fused HIP TransMIL step (bf16 mode, train mode) on its own bags with
    ``GradAllReduce(model=..., overlap=True)`` and ``accumulate_grad_batches = k``
    (tests/ddp_two_rank_worker.py; reference: Lightning DDP, code/train.py:178-201, K = 10 at
    :199).  After 2 optimizer steps both ranks hold the same parameters, equal (rtol 1e-5) to one
    process that accumulates both ranks' bags with loss / (2k) -- the gradient average DDP
    computes -- through the same kernels and optimizer, with the dropout stream replayed.  The
    part-0 all_reduce is issued by the fused backward's ready() hook.  n = 8192 is BASELINE config
    C4's per-rank workload (C2: 2-class, N=8192x512, bf16, train mode, one slide per rank)."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    import ddp_two_rank_worker as W
    from transmil_deepgraft_amd.interface import TransMILTask
    steps, world = 2, 2
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(here, "ddp_two_rank_worker.py"),
                                       str(tmp_path / f"rank{r}.pt"), str(k), str(steps), str(npatch)],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    logs = []
    try:
        for p in procs:
            logs.append(p.communicate(timeout=100)[0].decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} failed:\n{logs[r][-3000:]}"
    res = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    for r in range(world):
        # world 2: three bucket parts, each issued by the backward's ready() hook (part 1 before the
        # _fc1 backward, part 2 at its end)
        assert res[r]["parts"] == 3
        assert res[r]["issued"] == [0, 1, 2] * steps, res[r]["issued"]
    for n in res[0]["params"]:
        torch.testing.assert_close(res[0]["params"][n], res[1]["params"][n], rtol=0, atol=0, msg=n)

    # one process, both ranks' bags, the DDP mean taken by the loss scale
    model = W.build_model()
    c0 = model._dropout_counter.clone()
    task = TransMILTask(model)
    opt = task.configure_optimizers()[0][0]
    start = {n: p.detach().clone() for n, p in model.named_parameters()}
    for s in range(steps):
        for micro in range(s * k, (s + 1) * k):
            for r in range(world):
                model._dropout_counter.copy_(c0 + micro)     # each rank's stream at this micro-batch
                task.backward(task.training_step(W.bag(r, micro, npatch)) / (world * k))
        opt.step()
        opt.zero_grad(set_to_none=True)
    torch.cuda.synchronize()
    moved = 0.0
    for n, p in model.named_parameters():
        got = res[0]["params"][n]
        torch.testing.assert_close(got, p.detach().cpu(), rtol=1e-5, atol=1e-7, msg=n)
        moved = max(moved, (p.detach() - start[n]).abs().max().item())
    assert moved > 1e-5      # the steps changed the parameters (the comparison is not vacuous)


def test_two_ranks_average_the_c5_image_path(tmp_path, monkeypatch):
    """BASELINE config C5's image path under DDP: two processes on the one GPU (gloo), each
    running ImageBagModel (frozen RetCCL ResNet-50, bf16, eval-mode BN -> TransMIL(2, 2048) RCC-2048
    branch, bf16, train mode) on its own 8-tile bags through TransMILTask.optimization_step with
    GradAllReduce over the MIL parameters (three bucket parts, each issued mid-backward).  After 2
    optimizer steps both ranks hold the same parameters, equal (rtol 1e-5) to one process that
    runs both ranks' bags with loss / 2 through the same kernels (reference: Lightning DDP,
    code/train.py:178-201; ModelInterface.forward's image branch, model_interface.py:300-316)."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    import ddp_two_rank_worker as W
    from transmil_deepgraft_amd.interface import TransMILTask
    steps, world, k = 2, 2, 1
    # the encoder's 1x1 convolutions on hipBLASLt's heuristic choice in every process: a per-process
    # timed algorithm search (tm_conv1x1_tune) could round the features differently per process
    monkeypatch.setenv("TM_CONV1X1_TUNE", "0")
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.join(here, "ddp_two_rank_worker.py"),
                                       str(tmp_path / f"rank{r}.pt"), str(k), str(steps), str(W.C5_TILES), "c5"],
                                      env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    logs = []
    try:
        for p in procs:
            logs.append(p.communicate(timeout=150)[0].decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} failed:\n{logs[r][-3000:]}"
    res = [torch.load(tmp_path / f"rank{r}.pt", weights_only=True) for r in range(world)]
    for r in range(world):
        assert res[r]["parts"] == 3 and res[r]["issued"] == [0, 1, 2] * steps, res[r]["issued"]
        # only the class token + _fc1 part (+ the has-gradient flags, 64-B alignment) is reduced after
        # the whole backward; layer1's part went out before the _fc1 backward
        tail = 4 * sum(v.numel() for n, v in res[r]["params"].items() if n.startswith(("model._fc1.", "model.cls_token")))
        assert tail <= res[r]["exposed_bytes"] < tail + 4096, (res[r]["exposed_bytes"], tail)
    for n in res[0]["params"]:
        torch.testing.assert_close(res[0]["params"][n], res[1]["params"][n], rtol=0, atol=0, msg=n)

    model = W.build_c5_model()
    mil = model.model
    c0 = mil._dropout_counter.clone()
    task = TransMILTask(model)
    opt = task.configure_optimizers()[0][0]
    start = {n: p.detach().clone() for n, p in model.named_parameters() if p.requires_grad}
    for s in range(steps):
        for r in range(world):
            mil._dropout_counter.copy_(c0 + s)          # each rank's dropout stream at this step
            task.backward(task.training_step(W.c5_bag(r, s)) / world)
        opt.step()
        opt.zero_grad(set_to_none=True)
    torch.cuda.synchronize()
    moved = 0.0
    for n, p in model.named_parameters():
        if not p.requires_grad:
            continue
        got, want = res[0]["params"][n], p.detach().cpu()
        # (the loss / world scale enters before the bf16 products here, after them on the ranks:
        # a few weights of |w| ~ 1e-3 differ by ~1e-7)
        torch.testing.assert_close(got, want, rtol=1e-5, atol=1e-6,
                                   msg=lambda m, n=n, got=got, want=want: f"{n}: max |diff| "
                                   f"{(got - want).abs().max().item():.3e}\n{m}")
        moved = max(moved, (p.detach() - start[n]).abs().max().item())
    assert moved > 1e-5
