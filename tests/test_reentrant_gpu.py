"""The C ABI is reentrant across streams and threads (SURVEY.md §8(b), C-ABI row): two fused
engines, each on its own HIP stream and driven from its own host thread with the parameter-gradient
reductions deferred (every backward owns a tm_reduce_queue), give bit-identical logits and
gradients to the same calls run one after the other on the default stream."""
import threading

import numpy as np
import pytest
import torch


def _setup(seed, N, n_classes):
    from transmil_deepgraft_amd.models import TransMIL
    torch.manual_seed(seed)
    m = TransMIL(n_classes, 512).cuda()
    params = {n: p.detach().clone() for n, p in m.named_parameters()}
    x = torch.from_numpy(np.random.default_rng(seed).random((1, N, 512), dtype=np.float32)).cuda()
    return params, x


def _run(engine, params, x, stream, reps=1):
    """forward (train-mode dropout, fixed seeds) + backward on ``stream``; returns host copies."""
    with torch.cuda.stream(stream):
        for _ in range(reps):
            logits, ctx = engine.forward(x, params, drop_p=0.7, seeds=(11, 12))
            dl = torch.ones_like(logits)
            g = engine.backward(dl, ctx, params)
    stream.synchronize()
    return logits.cpu(), {k: v.cpu() for k, v in g.items()}


@pytest.mark.gpu
@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_two_engines_two_streams_two_threads_bit_identical(dtype):
    from transmil_deepgraft_amd.engine import TransMILEngine
    cases = [_setup(1, 3000, 2), _setup(2, 1900, 3)]
    engines = [TransMILEngine(dtype), TransMILEngine(dtype)]
    serial = [_run(engines[i], *cases[i], torch.cuda.current_stream()) for i in range(2)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for _ in range(2):
        results, errors = [None, None], []
        gate = threading.Barrier(2)

        def worker(i):
            try:
                gate.wait()
                results[i] = _run(engines[i], *cases[i], streams[i], reps=3)
            except Exception as e:          # surfaced below
                errors.append(e)

        ts = [threading.Thread(target=worker, args=(i,)) for i in range(2)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=100)
        assert not errors, errors
        for i in range(2):
            lo, g = results[i]
            assert torch.equal(lo, serial[i][0]), i
            assert g.keys() == serial[i][1].keys()
            for k in g:
                assert torch.equal(g[k], serial[i][1][k]), (i, k)
