"""Rate of interface.GraphedOptimizationStep (the user-facing graphed training step) against the
eager TransMILTask.optimization_step at the bench shape (1 bag N=8192x512, bf16, train mode):
the graphed step copies each batch into its static inputs and replays one graph."""
import json
import os
import sys
import time

sys.path.insert(0, os.getcwd())
import torch
from transmil_deepgraft_amd.interface import GradAllReduce, GraphedOptimizationStep, TransMILTask
from transmil_deepgraft_amd.models import TransMIL


def run(graphed, steps=200, warm=20):
    torch.manual_seed(1234)
    m = TransMIL(2, 512, 512).cuda().train().set_compute_dtype(torch.bfloat16)
    task = TransMILTask(m)
    opt = task.configure_optimizers()[0][0]
    ar = GradAllReduce(m.parameters(), model=m)
    g = torch.Generator(device="cuda").manual_seed(2021)
    bags = [torch.rand(1, 8192, 512, device="cuda", generator=g) for _ in range(4)]
    labels = [torch.randint(0, 2, (1,), device="cuda", generator=g) for _ in range(4)]
    fn = GraphedOptimizationStep(task, opt, ar) if graphed else \
        (lambda b: task.optimization_step(b, opt, allreduce=ar))
    for i in range(warm):
        fn((bags[i % 4], labels[i % 4], None))
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(steps):
        fn((bags[i % 4], labels[i % 4], None))
    torch.cuda.synchronize()
    return steps / (time.perf_counter() - t)


out = {"eager_optimization_step": round(run(False), 1), "GraphedOptimizationStep": round(run(True), 1),
       "unit": "slides/sec", "workload": "1 bag N=8192x512, bf16, train step, 1 GPU"}
print(json.dumps(out))
