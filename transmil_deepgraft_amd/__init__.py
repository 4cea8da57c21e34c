"""MI355X-native TransMIL hot path (forward + backward) for Ycblue/TransMIL-DeepGraft.

Drop-in surfaces:
  * ``transmil_deepgraft_amd.models.TransMIL`` -- ``code/models/TransMIL.py``
  * ``transmil_deepgraft_amd.nystrom_attention.NystromAttention`` -- the
    third-party ``nystrom_attention`` package class
  * ``transmil_deepgraft_amd.interface`` -- the Lightning step pieces
    (loss, optimizer, DDP gradient all-reduce)
Compute: hand-written HIP kernels for gfx950 in ``libtransmil_hip.so``
(C ABI: ``include/transmil_hip.h``).
"""
__version__ = "0.1.0"
