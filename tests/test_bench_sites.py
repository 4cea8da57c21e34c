"""bench.py's GEMM roofline sites against the GEMMs the fused engine actually launches (CPU: every
``_lib`` entry point replaced by a recorder, so the engine's host orchestration runs on CPU tensors
and no kernel executes).  Reference: code/models/TransMIL.py:26-34 (to_qkv / to_out), :128-133
(_fc1); the bench line's ``gemm_roofline`` credits each call site with 2 M N K flops and its
algorithmic bytes, so a site whose shape drifted from the launch would misstate its fraction.

Also the order of the bucket hooks against the launches: with a three-part bucket (world > 1)
part 1 (layer1) is announced after layer1's last parameter-gradient flush and before the _fc1
backward's first launch, part 2 at the end."""
import ctypes as C
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


class _Recorder:
    def __init__(self):
        self.site = []
        self.log = []          # ("gemm", site, M, N, K) / ("call", name) / ("ready", i)

    def call(self, name, *args):
        if name == "tm_gemm":
            g = args[3]._obj
            self.log.append(("gemm", self.site[-1] if self.site else None, g.M, g.N, g.K))
        else:
            self.log.append(("call", name))

    def query(self, name, *args):
        return 1 << 24      # sizes (bytes or floats): big enough for any view the engine takes

    def probe(self, name):
        rec = self

        class _Ctx:
            def __enter__(self):
                rec.site.append(name)

            def __exit__(self, *exc):
                rec.site.pop()
                return False
        return _Ctx()


class _FakeQueue:
    def __init__(self):
        self.handle = C.c_void_p(0)
        self.n = 0

    def pending(self):
        return 1

    def flush(self):
        _REC.log.append(("call", "tm_reduce_flush"))

    def close(self):
        pass


_REC = None


def _run_engine(monkeypatch, N, parts):
    global _REC
    from transmil_deepgraft_amd import engine
    from transmil_deepgraft_amd.models import TransMIL
    _REC = rec = _Recorder()
    monkeypatch.setattr(engine._lib, "call", rec.call)
    monkeypatch.setattr(engine._lib, "query", rec.query)
    monkeypatch.setattr(engine._lib, "lib", lambda: None)
    monkeypatch.setattr(engine, "ReduceQueue", _FakeQueue)
    monkeypatch.setattr(engine, "_stream", lambda: C.c_void_p(0))
    monkeypatch.setattr(engine, "probe", rec.probe)
    torch.manual_seed(0)
    model = TransMIL(2, 512, 512).train()
    names, params = model._engine_params(model._fc1_layout())
    prm = dict(zip(names, [p.detach() for p in params]))
    eng = engine.TransMILEngine(torch.bfloat16, fc1=engine.FC1_PLAIN, head="_fc")
    x = torch.zeros(1, N, 512)
    seed_dev = torch.zeros(1, dtype=torch.int64)
    ce = (torch.zeros(1, dtype=torch.int64), torch.zeros(2, 2, dtype=torch.int32))
    logits, ctx = eng.forward(x, prm, 0.7, seed_dev=seed_dev, counter=torch.zeros(1, dtype=torch.int64), ce=ce)
    out = {n: torch.empty_like(p) for n, p in prm.items()}
    eng.backward(None, ctx, prm, out=out, ready=lambda i: rec.log.append(("ready", i)), gloss=torch.ones(()),
                 parts=parts)
    return rec.log


@pytest.mark.parametrize("N", [8192, 1000])
def test_gemm_sites_match_the_engine_launches(monkeypatch, N):
    import bench
    import math
    log = _run_engine(monkeypatch, N, parts=2)
    G = math.ceil(math.sqrt(N))
    n = (G * G + 1 + 255) // 256 * 256
    launched = {}
    for e in log:
        if e[0] == "gemm" and e[1] in bench.GEMM_SITES:
            launched.setdefault(e[1], []).append(e[2:])
    assert set(launched) == set(bench.GEMM_SITES), set(launched) ^ set(bench.GEMM_SITES)
    for site, (layers, shape, _) in bench.GEMM_SITES.items():
        want = [shape(n, N, layer)[:3] for layer in layers]
        assert launched[site] == want, (site, launched[site], want)
    # layer 2 (the class-row layer) runs the k / v part of to_qkv's backward at K = 2D
    assert launched["dxn_gemm"][0] == (n, 512, 1024)
    assert launched["wgrad_qkv"][0] == (1024, 512, n)


def test_three_part_bucket_announces_layer1_before_the_fc1_backward(monkeypatch):
    log = _run_engine(monkeypatch, 1000, parts=3)
    marks = [(i, e) for i, e in enumerate(log) if e[0] == "ready"]
    assert [e[1] for _, e in marks] == [0, 1, 2]
    i1, i2 = marks[1][0], marks[2][0]
    assert log[i1 - 1] == ("call", "tm_reduce_flush")          # layer1's gradients final
    after = log[i1 + 1:i2]
    assert after[0] == ("call", "tm_fc1_gelu_bwd")             # the _fc1 backward follows part 1
    assert any(e[0] == "gemm" and e[1] == "wgrad_fc1" for e in after)
    assert after[-1] == ("call", "tm_reduce_flush")
    # two parts: no flush between layer1's backward and the _fc1 backward
    log2 = _run_engine(monkeypatch, 1000, parts=2)
    assert [e[1] for e in log2 if e[0] == "ready"] == [0, 1]
    assert log2.count(("call", "tm_reduce_flush")) == log.count(("call", "tm_reduce_flush")) - 1


def test_grad_bucket_parts_split_layer1():
    from transmil_deepgraft_amd.models import TransMIL
    m = TransMIL(2, 512, 512)
    names = {id(p): n for n, p in m.named_parameters()}
    two, three = m.grad_bucket_parts(), m.grad_bucket_parts(split_layer1=True)
    assert three[0] == two[0]
    assert all(names[id(p)].startswith("layer1.") for p in three[1])
    assert {names[id(p)] for p in three[2]} == {"cls_token", "_fc1.0.weight", "_fc1.0.bias"}
    assert {id(p) for p in three[1] + three[2]} == {id(p) for p in two[1]}
