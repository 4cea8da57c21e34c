"""Diagnostic for the round-5 abort (commit 92b6c08): two NCCL (RCCL) process groups initialised and
destroyed back to back in ONE process, each after a hipGraph captured over GradAllReduce's
all-reduce (tests/test_ddp_gpu.py::_rccl_graph_body).

    python scripts/dev/rccl_teardown.py old|close

``old``: the round-5 teardown (graph / all-reduce references dropped, the model still holding the
bucket and its hook, destroy_process_group); ``close``: graph.reset() + GradAllReduce.close() first.
Prints which object is still alive at destroy time (gc referrers of the GradAllReduce and of the
captured graph) and each phase as it completes, so an abort names the phase it happened in."""
import gc
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import test_ddp_gpu as T  # noqa: E402
from transmil_deepgraft_amd import interface  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "old"
alive = []
_orig_init = interface.GradAllReduce.__init__


def _spy_init(self, *a, **k):
    _orig_init(self, *a, **k)
    import weakref
    alive.append(weakref.ref(self))


interface.GradAllReduce.__init__ = _spy_init
_orig_destroy = dist.destroy_process_group


def _spy_destroy(*a, **k):
    gc.collect()
    live = [r() for r in alive if r() is not None]
    print(f"# destroy_process_group: {len(live)} GradAllReduce alive", flush=True)
    for ar in live:
        holders = [type(h).__name__ for h in gc.get_referrers(ar) if h is not alive]
        print(f"#   referrers: {holders}; works pending: {len(ar._works)}", flush=True)
    _orig_destroy(*a, **k)
    print("# destroy_process_group returned", flush=True)


dist.destroy_process_group = _spy_destroy
for i, overlap in enumerate((False, True)):
    print(f"# group {i}: overlap={overlap} teardown={mode}", flush=True)
    T._rccl_graph_body(overlap, teardown=mode)
    print(f"# group {i} done", flush=True)
torch.cuda.synchronize()
print("RCCL_TEARDOWN_OK", mode, flush=True)
