"""ctypes binding of ``libtransmil_hip.so`` (the C ABI in ``include/transmil_hip.h``).

The product path has no CPU or eager-PyTorch fallback: if the library is
missing or cannot be loaded, :func:`lib` raises.  Every call checks the
returned status and raises ``RuntimeError`` with ``tm_last_error()``.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("TRANSMIL_HIP_LIB", os.path.join(_HERE, "libtransmil_hip.so"))

F32, BF16 = 0, 1
EPI_PLAIN, EPI_QKV, EPI_SPLITK = 0, 1, 2

P = C.c_void_p
I = C.c_int
L = C.c_longlong
Fl = C.c_float
U64 = C.c_uint64


class GemmArgs(C.Structure):
    _fields_ = [("M", I), ("N", I), ("K", I), ("lda", I), ("ldb", I), ("ldc", I),
                ("a_trans", I), ("b_kn", I), ("ab_dtype", I), ("c_dtype", I),
                ("splits", I), ("k_per_split", I), ("mode", I), ("alpha", Fl),
                ("bias", P), ("gelu", I), ("pre", P), ("ld_pre", I),
                ("drop_p", Fl), ("drop_scale", Fl), ("seed", U64), ("resid", P),
                ("accumulate", I), ("grp_in", I), ("skip", I), ("grp_out", I),
                ("out_off", I), ("dup_n", I), ("dup_off", I), ("nbags", I), ("nh", I),
                ("dh", I), ("seq", I), ("qscale", Fl), ("seed_ptr", P), ("colsum", P), ("pre_bf16", I), ("slab_bf16", I)]


class BmmJob(C.Structure):
    _fields_ = [("A", P), ("B", P), ("ta", I), ("tb", I), ("lda", I), ("ldb", I), ("sa", L), ("sb", L),
                ("A2", P), ("B2", P), ("ta2", I), ("tb2", I), ("lda2", I), ("ldb2", I), ("sa2", L), ("sb2", L),
                ("E1", P), ("e1", Fl), ("E2", P), ("e2", Fl), ("alpha", Fl), ("diag", Fl),
                ("C", P), ("ldc", I), ("sc", L), ("M", I), ("N", I), ("K", I),
                ("C2", P), ("c2_alpha", Fl), ("c2_diag", Fl), ("c2_e1", Fl),
                ("Ct", P), ("ct_plane", L), ("ct_mode", I), ("ct_reserved", I), ("Rd", P), ("Rw", P)]


OPTIM_MAX_TENSORS = 40


class OptimTensor(C.Structure):
    _fields_ = [("param", P), ("grad", P), ("numel", L), ("lr", Fl), ("weight_decay", Fl)]


class OptimTable(C.Structure):
    _fields_ = [("count", I), ("reserved", I), ("offset", L * (OPTIM_MAX_TENSORS + 1)),
                ("t", OptimTensor * OPTIM_MAX_TENSORS), ("hyper", P)]


CAST_MAX = 8


class CastTable(C.Structure):
    _fields_ = [("count", I), ("reserved", I), ("src", P * CAST_MAX), ("dst", P * CAST_MAX),
                ("offset", L * (CAST_MAX + 1))]


# name -> (restype, argtypes)
_SIGS = {
    "tm_last_error": (C.c_char_p, []),
    "tm_build_info": (C.c_char_p, []),
    "tm_gemm": (I, [P, P, P, C.POINTER(GemmArgs), P]),
    "tm_splitk_reduce": (I, [P, P, I, L, Fl, I, P, P]),
    "tm_splitk_reduce_bf16": (I, [P, P, I, L, Fl, I, P, P]),
    "tm_colsum_workspace": (L, [I, I, I]),
    "tm_colsum": (I, [P, I, I, I, I, I, P, P, I, P, P]),
    "tm_layernorm_fwd": (I, [P, P, P, Fl, I, I, I, I, I, I, P, P, P, P]),
    "tm_layernorm_bwd_workspace": (L, [I, I, I]),
    "tm_layernorm_bwd": (I, [P, I, P, P, P, P, I, I, I, I, I, I, I, P, P, P, P, P, P]),
    "tm_layernorm_bwd_seg": (I, [P, I, P, P, P, P, I, I, I, I, I, I, I, P, I, I, I, P, P, P, P, P, P]),
    "tm_head_fwd": (I, [P, I, I, I, P, P, Fl, P, P, I, P, P, P, P]),
    "tm_head_bwd": (I, [P, I, I, I, I, P, P, P, P, P, P, P, P, P, P, P]),
    "tm_head_ce_fwd": (I, [P, I, I, I, P, P, Fl, P, P, I, P, P, P, P, P, P, P, P, P]),
    "tm_head_ce_bwd": (I, [P, P, P, P, I, I, I, I, P, P, P, P, P, P, P, P, P, P, P, P]),
    "tm_nys_landmarks": (I, [I, P, P, I, I, P, P, P, P, P]),
    "tm_nys_sim2_softmax": (I, [P, P, I, P, P]),
    "tm_softmax_bwd_rows256": (I, [P, P, P, I, P]),
    "tm_nys_a3_workspace": (L, [I, I]),
    "tm_nys_a3_partials": (L, [I, I]),
    "tm_nys_a3_fwd": (I, [I, P, P, P, I, I, P, P, P, P]),
    "tm_nys_a3_fwd_sim2": (I, [P, P, P, P, I, I, P, P, P, P]),
    "tm_nys_a1_fwd": (I, [I, P, P, P, P, P, I, I, I, P, P, P]),
    "tm_nys_rowdot_cast": (I, [I, P, P, I, P, P, P]),
    "tm_cast_f32": (I, [I, P, P, L, P]),
    "tm_nys_conv_bwd_workspace": (L, [I, I, I]),
    "tm_nys_conv_bwd": (I, [I, P, P, P, P, I, I, I, P, P, P, P, P, P]),
    "tm_nys_a1_bwd_workspace": (L, [I, I, I]),
    "tm_nys_a1_bwd": (I, [I, P, P, P, P, P, P, I, I, I, I, P, P, P, P, I, P, P]),
    "tm_nys_a1_bwd_dqkv": (I, [P, P, P, P, P, P, I, I, I, P, Fl, P, P, P, P, P]),
    "tm_nys_a3_bwd_workspace": (L, [I, I]),
    "tm_nys_a3_bwd": (I, [I, P, P, P, P, P, P, I, I, I, P, P, P, P, I, P, P]),
    "tm_nys_assemble_dqkv": (I, [I, P, P, P, P, P, I, I, I, Fl, P, P]),
    "tm_nys_a3_bwd_fused": (I, [P, P, P, P, P, P, I, I, I, P, I, I, P, P, P, P, P, P]),
    "tm_nys_assemble_q": (I, [I, P, I, P, P, I, I, I, Fl, P, P]),
    "tm_nys_a3_bwd_slabs": (I, [I, I]),
    "tm_nys_assemble_q_slab": (I, [I, P, I, P, P, I, I, I, I, Fl, P, P]),
    "tm_nys_assemble_q_slab_inplace": (I, [P, P, I, I, I, I, Fl, P, P]),
    "tm_nys_attn_row": (I, [I, P, P, P, P, P, P, I, I, I, P, P]),
    "tm_bmm": (I, [C.POINTER(BmmJob), I, I, I, P]),
    "tm_pinv_saved_floats": (L, [I, I]),
    "tm_pinv_fwd": (I, [P, I, I, I, P, P]),
    "tm_pinv_bwd_workspace_floats": (L, [I]),
    "tm_pinv_bwd": (I, [P, I, I, I, P, P, P, P, P]),
    "tm_nys_sim2_softmax_split": (I, [P, P, I, P, P, P]),
    "tm_pinv_split_saved_floats": (L, [I, I]),
    "tm_pinv_fwd_split": (I, [P, P, I, I, P, P]),
    "tm_pinv_fwd_split_a3": (I, [P, P, I, I, P, P, I, P, P, P]),
    "tm_pinv_bwd_split_workspace_floats": (L, [I]),
    "tm_pinv_bwd_split": (I, [P, P, I, I, P, P, I, P, P]),
    "tm_split_f32": (I, [P, P, L, P]),
    "tm_ppeg_fold": (I, [P, P, P, P, P, P, I, P, P, P]),
    "tm_ppeg_fwd": (I, [P, I, I, I, P, P, P, P]),
    "tm_ppeg_bwd_workspace": (L, [I, I, I]),
    "tm_ppeg_bwd": (I, [P, P, I, I, I, P, P, P, P, P, P, P, P, P, I, P, I, I, Fl, U64, P, P, P]),
    "tm_gather_rows": (I, [I, P, I, P, P, P, P, I, P, P]),
    "tm_attmil_fwd_workspace": (L, [I, I]),
    "tm_attmil_fwd": (I, [P, P, P, P, P, P, I, I, I, I, P, P, P, P, P, P]),
    "tm_attmil_bwd_workspace": (L, [I, I, I]),
    "tm_attmil_bwd": (I, [P, P, P, P, P, P, P, I, I, I, I, P, P, P, P, P, P, P, P, P]),
    "tm_put_cls": (I, [P, I, I, I, P, P]),
    "tm_step_prepare": (I, [I, C.POINTER(CastTable), P, P, P, P, P, P, I, P, P, P, P, P, P, I, I, P]),
    "tm_reduce_queue_create": (P, []),
    "tm_reduce_queue_destroy": (None, [P]),
    "tm_reduce_queue_pending": (I, [P]),
    "tm_reduce_flush": (I, [P, P]),
    "tm_ce_fwd": (I, [P, P, I, I, P, P, P, P, P]),
    "tm_ce_bwd": (I, [P, P, I, I, P, P, P]),
    "tm_dropout_bwd_pad": (I, [I, P, I, I, I, I, I, Fl, U64, P, P, P]),
    "tm_add_relu": (I, [I, P, P, P, L, P]),
    "tm_bias_act": (I, [I, P, P, L, I, I, P]),
    "tm_bias_relu_maxpool": (I, [P, P, P, I, I, I, I, P]),
    "tm_bn_relu_maxpool": (I, [P, P, P, P, I, I, I, I, P]),
    "tm_stem_conv_pool": (I, [P, P, P, P, I, I, I, L, L, L, L, P]),
    "tm_subsample2d": (I, [I, P, P, I, I, I, I, I, P]),
    "tm_stem_bn_stats_workspace": (L, []),
    "tm_stem_bn_stats": (I, [P, P, I, I, I, L, L, L, L, P, P, P, P, Fl, Fl, P, P, P, L, P]),
    "tm_stem_conv_pool_bn": (I, [P, P, P, P, P, I, I, I, L, L, L, L, P]),
    "tm_conv1x1_workspace_bytes": (L, []),
    "tm_conv1x1": (I, [I, P, P, P, P, P, L, I, I, I, P, L, P]),
    "tm_conv1x1_tune": (I, [I, P, P, P, P, P, L, I, I, I, P, L, P]),
    "tm_bn_train_workspace": (L, [I]),
    "tm_bn_train_stats": (I, [I, P, P, I, I, P, P, P, P, Fl, Fl, P, P, P, L, P]),
    "tm_bn_apply": (I, [I, P, P, P, P, P, P, L, I, I, P]),
    "tm_cls_a1_row_fwd": (I, [I, P, P, P, P, P, I, I, I, I, P, P, P]),
    "tm_cls_out_fwd": (I, [I, P, P, P, P, I, I, I, I, I, Fl, U64, P, P, P]),
    "tm_cls_out_bwd": (I, [I, P, P, P, I, I, I, I, I, Fl, U64, P, P, P, P, P]),
    "tm_cls_head_out_bwd": (I, [I, P, P, P, I, P, P, P, P, P, P, P, P, P, P, P, P, I, I, I, I, Fl, U64, P, P, P, P, P]),
    "tm_cls_a1_row_bwd": (I, [I, P, P, P, P, P, P, P, I, I, I, I, P, P, P, P, P, P]),
    "tm_cls_q_rows": (I, [P, P, I, P, P, I, I, I, I, P, P, P]),
    "tm_pad_rows": (I, [I, P, I, I, I, I, I, P, P]),
    "tm_fc1_gelu_bwd": (I, [I, P, P, I, I, I, I, I, P, P, P]),
    "tm_gelu_bwd": (I, [I, P, P, L, P, P]),
    "tm_cast_f32_many": (I, [I, C.POINTER(CastTable), P]),
    "tm_radam_counters_len": (L, [L]),
    "tm_radam_lookahead_step": (I, [C.POINTER(OptimTable), P, P, P, P, Fl, Fl, Fl, I, Fl, P]),
}

EXPORTED = tuple(_SIGS)

# Entry points of the diagnostic build only (`make -C transmil_deepgraft_amd/csrc diag` ->
# libtransmil_hip_diag.so, selected with TRANSMIL_HIP_LIB; scripts/microbench.py): kernel-variant
# switches and timing stamps.  Not part of the ABI; the product library does not export them.
DIAG_SIGS = {
    "tm_debug_set_variant": (None, [I, I]),
    "tm_debug_xcc_map": (I, [P, I, I, P]),
    "tm_debug_set_split_variant": (None, [I]),
    "tm_debug_set_split_stamps": (None, [P]),
    "tm_debug_a1_stamps": (I, [P, I]),
    "tm_debug_gemm_stamps": (I, [P, I]),
}

_lib = None


def lib():
    """Load the HIP library (once).  Raises if it is missing: there is no fallback."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"transmil_deepgraft_amd: HIP library not found at {LIB_PATH}; build it with "
                "`make -C transmil_deepgraft_amd/csrc -j8` (or __graft_entry__.build())")
        handle = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        for name, (res, args) in DIAG_SIGS.items():
            if hasattr(handle, name):
                fn = getattr(handle, name)
                fn.restype = res
                fn.argtypes = args
        _lib = handle
    return _lib


def last_error() -> str:
    return lib().tm_last_error().decode()


_FNS = {}


def call(name: str, *args) -> None:
    fn = _FNS.get(name)
    if fn is None:
        fn = _FNS[name] = getattr(lib(), name)
    rc = fn(*args)
    if rc != 0:
        raise RuntimeError(f"{name} failed (rc={rc}): {last_error()}")


def query(name: str, *args) -> int:
    return int(getattr(lib(), name)(*args))
