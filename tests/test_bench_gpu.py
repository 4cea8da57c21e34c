"""bench.py's timed step (make_step: captured hipGraphs per bag and accumulation phase) against
TransMILTask.optimization_step run eagerly on the same micro-batch sequence: the parameters after
the warm-up + timed micro-batches must be bitwise identical, with accumulate_grad_batches K = 1
(the driver's bench line) and K = 3 (C4's all-reduce every K micro-batches; code/train.py:199)."""
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


@pytest.mark.gpu
@pytest.mark.parametrize("K", [1, 3])
def test_bench_graph_step_equals_eager_optimization_step(K):
    import bench
    from transmil_deepgraft_amd.interface import GradAllReduce, TransMILTask
    from transmil_deepgraft_amd.models import TransMIL

    def build():
        torch.manual_seed(7)
        m = TransMIL(2, 512, 512).cuda().train().set_compute_dtype(torch.float32)
        task = TransMILTask(m, accumulate_grad_batches=K)
        return m, task, task.configure_optimizers()[0][0], GradAllReduce(m.parameters(), model=m)

    g = torch.Generator(device="cuda").manual_seed(3)
    bags = [torch.rand(1, 300, 512, device="cuda", generator=g) for _ in range(2)]
    labels = [torch.tensor([j % 2], device="cuda") for j in range(2)]
    timed = 2 * K

    ma, ta, oa, ara = build()
    st = bench.make_step(ta, oa, ara, bags, labels, K, warmup=1)
    assert st.graph is not None
    for i in range(timed):
        st.step(i)
    torch.cuda.synchronize()

    mb, tb, ob, arb = build()
    assert st.warm_micro == (2 * K, 2 * K)
    # make_step's eager warm-up, its one replay of every captured graph, then the timed ones
    for i in list(range(2 * K)) + list(range(2 * K)) + list(range(timed)):
        tb.optimization_step((bags[i % 2], labels[i % 2], None), ob, allreduce=arb)
    torch.cuda.synchronize()

    pa, pb = dict(ma.named_parameters()), dict(mb.named_parameters())
    moved = any(not torch.equal(pa[n], p0) for n, p0 in [(n, p.detach().clone()) for n, p in build()[0].named_parameters()])
    assert moved
    bad = [n for n in pa if not torch.equal(pa[n], pb[n])]
    assert not bad, bad


@pytest.mark.gpu
def test_two_rank_bench_control_flow_completes():
    """bench.py at N = 2 (torch.distributed.run, two ranks sharing this GPU through the gloo
    rehearsal backend, eager): the timed loop, the post-timed probes (HBM sites, pseudo-inverse
    roofline) and the teardown run their gradient all-reduces on EVERY rank, so the run ends and
    rank 0 prints one JSON line with n_gpus = 2 (a rank-0-only probe step left rank 0 waiting in
    its all-reduce)."""
    import json
    import subprocess
    import socket
    with socket.socket() as sk:        # a free port, not a fixed one (the box is shared)
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    env = dict(os.environ, TM_BENCH_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", "--eager",
           "--n-patches", "1024", "--steps", "3", "--warmup", "1", "--no-cpu-baseline"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["value"] > 0 and d["config"]["parallelism"] == "dp2"
    assert d["hbm_roofline"], "the HBM probe ran on every rank and rank 0 reported it"
