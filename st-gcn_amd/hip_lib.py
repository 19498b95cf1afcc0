"""ctypes binding of libstgcn_hip.so (the C-ABI in include/stgcn_hip.h).

The library is built in-tree (``st-gcn_amd/lib/libstgcn_hip.so``, see
``build.py``). There is no fallback: if the library or a HIP device is
missing, ``lib()`` raises.

torch is imported first on purpose: torch ships its own HIP runtime
(``libamdhip64.so``, SONAME ``libamdhip64.so.7``); loading it before the
library makes the library bind to that same runtime, so the hipStream_t handed
over from ``torch.cuda.current_stream()`` is valid inside the library.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

LIB_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib")
LIB_PATH = os.path.join(LIB_DIR, "libstgcn_hip.so")
if os.environ.get("STGCN_LIB_VARIANT"):  # A/B kernel experiments (scripts/), in-tree only
    # an explicitly built A/B variant (build.py variant=...); loading it says so
    LIB_PATH = os.path.join(LIB_DIR, f"libstgcn_hip_{os.environ['STGCN_LIB_VARIANT']}.so")
    import sys
    print(f"stgcn: loading the A/B variant library {LIB_PATH}", file=sys.stderr)
ABI_VERSION = 11
F_RESIDUAL = 1  # stgcn_desc_t.flags
F_BF16 = 2      # channel GEMMs on bf16 MFMA (fp32 accumulate, fp32 tensors)
F_F32X3 = 4     # fp32 temporal GEMMs via exact 3-way bf16 operand splits (fp32 accuracy)
F_F16X2 = 8     # ABI 6, with F_F32X3: the folded GEMMs as 2-way fp16 splits (scaled)
F_NO_G = 16     # ABI 7, with F_F16X2: the folded block without G (memory-lean)
# stgcn_block_plan bits (ABI 6)
PLAN_FOLD, PLAN_SP_FWD_FUSED, PLAN_SP_BWD_FUSED, PLAN_ACT_BF16 = 1, 2, 4, 8
PLAN_WSP_SPLIT, PLAN_TCONV_SPLIT, PLAN_TWGRAD_SPLIT, PLAN_F16X2 = 16, 32, 64, 128
PLAN_FOLD_NO_G = 256
PLAN_X_FROM_U = 512  # ABI 8: the input as ReLU(BN2(U)) of the previous block
# ABI 7: a y_stats / x_stats block: 5 * C doubles, then STATS_AMAX_WORDS uint32 (max |y|)
STATS_AMAX_WORDS = 2048


def y_stats_doubles(C):
    """float64 elements of a y_stats block of C channels (STGCN_Y_STATS_BYTES / 8)"""
    return 5 * C + STATS_AMAX_WORDS // 2

_c_int = ctypes.c_int32
_c_float = ctypes.c_float
_vp = ctypes.c_void_p


class Desc(ctypes.Structure):
    _fields_ = [("N", _c_int), ("C_in", _c_int), ("C_out", _c_int), ("T", _c_int),
                ("T_out", _c_int), ("V", _c_int), ("K", _c_int), ("gamma", _c_int),
                ("stride", _c_int), ("pad", _c_int), ("eps", _c_float),
                ("momentum", _c_float), ("training", _c_int), ("need_dx", _c_int),
                ("flags", _c_int)]


class FwdArgs(ctypes.Structure):
    _fields_ = [(n, _vp) for n in (
        "x", "A", "W", "bW", "Wt", "bWt", "g1", "b1", "g2", "b2",
        "rm1", "rv1", "rm2", "rv2", "y", "Z", "U", "stats",
        "Wr", "br", "Za",        # ABI 2: residual block
        "G",                     # ABI 2: optional kept joint contraction
        "x_stats", "y_stats")    # ABI 2: optional stack chaining
    ] + [("dropout_p", _c_float), ("seed", ctypes.c_uint64)  # ABI 2: fused dropout
         ] + [("prep", _vp)                                   # ABI 7: stgcn_fold_prep
              ] + [(n, _vp) for n in ("prev_U", "prev_stats", "prev_g2", "prev_b2")]  # ABI 8


class BwdArgs(ctypes.Structure):
    _fields_ = [(n, _vp) for n in (
        "dy", "x", "Z", "U", "stats", "A", "W", "bW", "Wt", "g1", "b1", "g2", "b2",
        "dx", "dA", "dW", "dbW", "dWt", "dbWt", "dg1", "db1", "dg2", "db2",
        "Wr", "Za", "y", "dWr", "dbr",         # ABI 2: residual block
        "G",                                   # ABI 2: optional kept joint contraction
        "dy_sums", "prev_g2", "prev_b2", "prev_sums")  # ABI 2: optional stack chaining
    ] + [("dropout_p", _c_float), ("seed", ctypes.c_uint64)  # ABI 2: fused dropout
         ] + [("prev_U", _vp), ("prev_stats", _vp)  # ABI 4: chain conditioning fallback
              ] + [("x_stats", _vp), ("dx_coef", _vp), ("dx_deferred", _vp),  # ABI 5:
                   ("dy_coef", _vp)                                          # deferred dx
                   ] + [("prep", _vp)] + [("dy_nc", _vp)]                    # ABI 7, 10


class FoldWeights(ctypes.Structure):  # ABI 7: stgcn_fold_prep
    _fields_ = [(n, _vp) for n in ("A", "W", "bW", "Wt", "bWt")]


class SpatialDesc(ctypes.Structure):  # ABI 4: SpatialConv on its own
    _fields_ = [("N", _c_int), ("C_in", _c_int), ("C_out", _c_int), ("T", _c_int),
                ("V", _c_int), ("K", _c_int), ("flags", _c_int)]


class HeadDesc(ctypes.Structure):  # ABI 3
    _fields_ = [("N", _c_int), ("C", _c_int), ("L", _c_int), ("classes", _c_int)]


class AdamTensor(ctypes.Structure):  # ABI 3
    _fields_ = [("param", _vp), ("grad", _vp), ("exp_avg", _vp), ("exp_avg_sq", _vp),
                ("numel", ctypes.c_int64)]


# Every symbol include/stgcn_hip.h declares (checked by tests/test_capi.py).
EXPORTED = ("stgcn_abi_version", "stgcn_last_error", "stgcn_check_desc",
            "stgcn_fwd_workspace_bytes", "stgcn_bwd_workspace_bytes",
            "stgcn_block_fwd", "stgcn_block_bwd", "stgcn_time_kernel_bytes",
            "stgcn_time_kernel", "stgcn_head_fwd", "stgcn_head_bwd", "stgcn_adam_table_bytes",
            "stgcn_adam_build_table", "stgcn_adam_step", "stgcn_spatial_workspace_bytes",
            "stgcn_spatial_fwd", "stgcn_spatial_bwd", "stgcn_keep_g_bytes",
            "stgcn_block_plan", "stgcn_fold_prep_bytes", "stgcn_fold_prep", "stgcn_head_fwd_u",
            "stgcn_head_bwd_nc", "stgcn_adam_step_dev")

_LIB = None


def load_library(path=LIB_PATH):
    """dlopen the library and declare prototypes (no GPU needed)."""
    if not os.path.exists(path):
        raise RuntimeError(
            f"libstgcn_hip.so not found at {path}; build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'`")
    lib = ctypes.CDLL(path)
    lib.stgcn_abi_version.restype = ctypes.c_int
    lib.stgcn_last_error.restype = ctypes.c_char_p
    lib.stgcn_check_desc.argtypes = [ctypes.POINTER(Desc)]
    lib.stgcn_check_desc.restype = ctypes.c_int
    for f in (lib.stgcn_fwd_workspace_bytes, lib.stgcn_bwd_workspace_bytes,
              lib.stgcn_keep_g_bytes):
        f.argtypes = [ctypes.POINTER(Desc)]
        f.restype = ctypes.c_size_t
    lib.stgcn_block_fwd.argtypes = [ctypes.POINTER(Desc), ctypes.POINTER(FwdArgs), _vp,
                                    ctypes.c_size_t, _vp]
    lib.stgcn_block_fwd.restype = ctypes.c_int
    lib.stgcn_block_bwd.argtypes = [ctypes.POINTER(Desc), ctypes.POINTER(BwdArgs), _vp,
                                    ctypes.c_size_t, _vp]
    lib.stgcn_block_bwd.restype = ctypes.c_int
    lib.stgcn_time_kernel_bytes.argtypes = [ctypes.POINTER(Desc), ctypes.c_int]
    lib.stgcn_time_kernel_bytes.restype = ctypes.c_size_t
    lib.stgcn_time_kernel.argtypes = [ctypes.POINTER(Desc), ctypes.c_int, _vp, ctypes.c_size_t,
                                      ctypes.c_int, _vp, ctypes.POINTER(ctypes.c_float),
                                      ctypes.POINTER(ctypes.c_double)]
    lib.stgcn_time_kernel.restype = ctypes.c_int
    lib.stgcn_head_fwd.argtypes = [ctypes.POINTER(HeadDesc)] + [_vp] * 8 + [_vp]
    lib.stgcn_head_fwd.restype = ctypes.c_int
    lib.stgcn_head_fwd_u.argtypes = [ctypes.POINTER(HeadDesc)] + [_vp] * 11 + [_vp]
    lib.stgcn_head_fwd_u.restype = ctypes.c_int
    lib.stgcn_head_bwd.argtypes = [ctypes.POINTER(HeadDesc)] + [_vp] * 10 + [_vp]
    lib.stgcn_head_bwd.restype = ctypes.c_int
    lib.stgcn_head_bwd_nc.argtypes = [ctypes.POINTER(HeadDesc)] + [_vp] * 10 + [_vp]
    lib.stgcn_head_bwd_nc.restype = ctypes.c_int
    lib.stgcn_adam_table_bytes.argtypes = [ctypes.c_int]
    lib.stgcn_adam_table_bytes.restype = ctypes.c_size_t
    lib.stgcn_adam_build_table.argtypes = [ctypes.POINTER(AdamTensor), ctypes.c_int, _vp,
                                           ctypes.c_size_t, ctypes.POINTER(ctypes.c_int64)]
    lib.stgcn_adam_build_table.restype = ctypes.c_int
    lib.stgcn_adam_step.argtypes = [_vp, ctypes.c_int, ctypes.c_int64] + \
        [ctypes.c_double] * 5 + [ctypes.c_int64, _vp]
    lib.stgcn_adam_step.restype = ctypes.c_int
    lib.stgcn_adam_step_dev.argtypes = [_vp, ctypes.c_int, ctypes.c_int64] + \
        [ctypes.c_double] * 5 + [_vp, _vp]
    lib.stgcn_adam_step_dev.restype = ctypes.c_int
    lib.stgcn_spatial_workspace_bytes.argtypes = [ctypes.POINTER(SpatialDesc), ctypes.c_int]
    lib.stgcn_spatial_workspace_bytes.restype = ctypes.c_size_t
    lib.stgcn_spatial_fwd.argtypes = [ctypes.POINTER(SpatialDesc)] + [_vp] * 6 + \
        [ctypes.c_size_t, _vp]
    lib.stgcn_spatial_fwd.restype = ctypes.c_int
    lib.stgcn_spatial_bwd.argtypes = [ctypes.POINTER(SpatialDesc)] + [_vp] * 10 + \
        [ctypes.c_size_t, _vp]
    lib.stgcn_spatial_bwd.restype = ctypes.c_int
    lib.stgcn_block_plan.argtypes = [ctypes.POINTER(Desc), ctypes.POINTER(ctypes.c_uint32)]
    lib.stgcn_block_plan.restype = ctypes.c_int
    lib.stgcn_fold_prep_bytes.argtypes = [ctypes.POINTER(Desc)]
    lib.stgcn_fold_prep_bytes.restype = ctypes.c_size_t
    lib.stgcn_fold_prep.argtypes = [ctypes.c_int, ctypes.POINTER(Desc),
                                    ctypes.POINTER(FoldWeights), ctypes.POINTER(_vp), _vp]
    lib.stgcn_fold_prep.restype = ctypes.c_int
    if lib.stgcn_abi_version() != ABI_VERSION:
        raise RuntimeError("libstgcn_hip.so ABI version mismatch; rebuild it")
    return lib


def lib():
    """The loaded library, for GPU use. Raises when it cannot run."""
    global _LIB
    if _LIB is None:
        if not torch.cuda.is_available():
            raise RuntimeError("stgcn HIP path requires a ROCm GPU (torch.cuda.is_available() "
                               "is False); there is no CPU fallback")
        _LIB = load_library()
    return _LIB


E_INVALID, E_UNSUPPORTED, E_HIP = -1, -2, -3  # (stgcn_hip.h stgcn_status)


def check(rc):
    if rc != 0:
        msg = lib().stgcn_last_error().decode(errors="replace")
        raise RuntimeError(f"libstgcn_hip error {rc}: {msg}")


def block_plan(desc):
    """stgcn_block_plan: the PLAN_* bitmask the library selects for a descriptor
    (needs no GPU)."""
    plan = ctypes.c_uint32(0)
    rc = load_library().stgcn_block_plan(ctypes.byref(desc), ctypes.byref(plan))
    if rc != 0:
        raise RuntimeError(f"stgcn_block_plan failed ({rc})")
    return plan.value


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_handle(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
