"""A/B of a pinv_split diagnostic variant inside the whole bench step (diagnostic build):
    python scripts/dev/ab_split_variant.py V [bench args...]
runs bench.py's main with tm_debug_set_split_variant(V) set first."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
os.environ.setdefault("TRANSMIL_HIP_LIB", os.path.join(ROOT, "transmil_deepgraft_amd", "libtransmil_hip_diag.so"))
import torch  # noqa: E402,F401  (HIP runtime initialised by torch first)
from transmil_deepgraft_amd import _lib  # noqa: E402

_lib.lib().tm_debug_set_split_variant(int(sys.argv[1]))
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
