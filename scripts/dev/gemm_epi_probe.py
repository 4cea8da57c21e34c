"""Ring GEMM epilogue probe: full epilogue vs image reads only vs bare stores (variant 8 stamps)."""
import sys, os, ctypes
sys.path.insert(0, os.getcwd())
import numpy as np
import torch
from transmil_deepgraft_amd import engine as E
from transmil_deepgraft_amd._lib import BF16, F32, GemmArgs, EPI_PLAIN
from transmil_deepgraft_amd import _lib

L = _lib.lib()
dev = "cuda"
M, N, K = 8192, 512, 512
for cd in (BF16, F32):
    A = (torch.randn(M, K, device=dev) * 0.1).to(torch.bfloat16)
    Bm = (torch.randn(N, K, device=dev) * 0.1).to(torch.bfloat16)
    Cm = torch.empty(M, N, device=dev, dtype=torch.float32 if cd == F32 else torch.bfloat16)
    for mode, ds in (("full", 1.0), ("reads-only", -1.0), ("bare-stores", -2.0)):
        g = GemmArgs()
        g.M, g.N, g.K = M, N, K
        g.lda, g.ldb, g.ldc = K, K, N
        g.a_trans, g.b_kn = 0, 0
        g.ab_dtype, g.c_dtype = BF16, cd
        g.splits, g.k_per_split = 1, K
        g.mode = EPI_PLAIN
        g.alpha = 1.0
        g.drop_scale = ds
        L.tm_debug_set_variant(2, 8)
        for _ in range(4):
            _lib.call("tm_gemm", ctypes.c_void_p(A.data_ptr()), ctypes.c_void_p(Bm.data_ptr()),
                      ctypes.c_void_p(Cm.data_ptr()), ctypes.byref(g), E._stream())
        torch.cuda.synchronize()
        L.tm_debug_set_variant(2, 0)
        nb = (M // 128) * (N // 128)
        buf = (ctypes.c_ulonglong * (nb * 8))()
        assert L.tm_debug_gemm_stamps(buf, nb * 8) == 0
        st = np.frombuffer(buf, dtype=np.uint64).reshape(nb, 8).astype(np.int64)
        d = np.diff(st[:, 1:7], axis=1)
        end = (st[:, 7] - st[:, 0].min()) / 100.0
        print(f"{'bf16' if cd == BF16 else 'f32 '} {mode:11s}: end p50 {np.median(end):5.2f} us | first {np.median(d[:,0]):5.0f} "
              f"k-loop {np.median(d[:,1]):5.0f} stage {np.median(d[:,2]):5.0f} epi {np.median(d[:,3]):5.0f} drain {np.median(d[:,4]):5.0f} cyc", flush=True)
