"""cProfile of the eager TransMILTask.optimization_step at the bench shape: where the host time of
an eager step goes (the GPU work is ~1.2 ms; an eager step takes ~1.9 ms)."""
import cProfile
import os
import pstats
import sys

sys.path.insert(0, os.getcwd())
import torch
from transmil_deepgraft_amd.interface import GradAllReduce, TransMILTask
from transmil_deepgraft_amd.models import TransMIL

torch.autograd.set_multithreading_enabled(False)   # the backward on this thread: cProfile sees it
torch.manual_seed(1234)
m = TransMIL(2, 512, 512).cuda().train().set_compute_dtype(torch.bfloat16)
task = TransMILTask(m)
opt = task.configure_optimizers()[0][0]
ar = GradAllReduce(m.parameters(), model=m)
bag = torch.rand(1, 8192, 512, device="cuda")
label = torch.tensor([1], device="cuda")
for _ in range(10):
    task.optimization_step((bag, label, None), opt, allreduce=ar)
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(50):
    task.optimization_step((bag, label, None), opt, allreduce=ar)
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(40)
