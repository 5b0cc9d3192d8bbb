"""ctypes binding of libpcadv.so (the C ABI declared in include/pcadv.h).

torch is imported first on purpose: the wheel ships its own libamdhip64.so.7,
and loading it before libpcadv.so makes the dynamic loader reuse that HIP
runtime (same soname), so torch's streams and allocations are valid handles
for the library.

There is no fallback: if the shared library is missing every op raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the dlopen below)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PCADV_LIB", os.path.join(_HERE, "lib", "libpcadv.so"))
# the layout of include/pcadv.h these signatures and AdvArgs bind (pcadv_abi_version())
ABI_VERSION = 10

PCADV_OK = 0
ACT_NONE, ACT_RELU, ACT_LRELU = 0, 1, 2

# state_dict-order flat layouts (must equal the enums in include/pcadv.h)
G_LAYOUT = {
    "feat.conv1.weight": 0, "feat.conv1.bias": 192,
    "feat.conv2.weight": 256, "feat.conv2.bias": 4352,
    "feat.conv3.weight": 4416, "feat.conv3.bias": 12608,
    "feat.conv4.weight": 12736, "feat.conv4.bias": 143808,
    "fc1.weight": 144832, "fc1.bias": 669120,
    "fc2.weight": 669632, "fc2.bias": 800704,
    "fc3.weight": 800960, "fc3.bias": 811200,
}
G_NUMEL = 811240
D_LAYOUT = {
    "conv1.weight": 0, "conv1.bias": 20480,
    "conv2.weight": 20992, "conv2.bias": 152064,
    "conv3.weight": 152320, "conv3.bias": 217856,
    "conv4.weight": 218112, "conv4.bias": 234496,
    "conv5.weight": 234560, "conv5.bias": 238656,
    "fc.weight": 238720, "fc.bias": 238784,
}
D_NUMEL = 238785

_vp = ctypes.c_void_p
_i = ctypes.c_int
_f = ctypes.c_float
_sz = ctypes.c_size_t
_i64 = ctypes.c_int64
_u64 = ctypes.c_uint64


class WgradDesc(ctypes.Structure):
    """Mirror of pcadv_wgrad_desc (include/pcadv.h)."""

    _fields_ = [("dz", _vp), ("ldz", _i64), ("x", _vp), ("ldx", _i64), ("rows", _i), ("O", _i),
                ("Kin", _i), ("dw", _vp), ("ldo", _i64), ("db", _vp), ("gsum", _vp),
                ("rows_per_group", _i), ("accumulate", _i), ("workspace", _vp),
                ("workspace_bytes", _sz)]


class GemmDesc(ctypes.Structure):
    """Mirror of pcadv_gemm_desc (include/pcadv.h)."""

    _fields_ = [("a", _vp), ("lda", _i64), ("ta", _i), ("b", _vp), ("ldb", _i64), ("tb", _i),
                ("c", _vp), ("ldc", _i64), ("M", _i), ("N", _i), ("K", _i), ("bias", _vp),
                ("bias_rows", _vp), ("rows_per_group", _i), ("relu", _i), ("accumulate", _i),
                ("cmask", _vp), ("ldm", _i64), ("precise", _i), ("c_hi", _vp), ("c_lo", _vp),
                ("ldcp", _i64)]


class AdvArgs(ctypes.Structure):
    """Mirror of pcadv_adv_args (include/pcadv.h)."""

    _fields_ = [
        ("B", _i), ("N", _i),
        ("pts_gt", _vp), ("labels", _vp), ("pts_nogt", _vp),
        ("drop_mask_gt", _vp), ("drop_mask_nogt", _vp),
        ("soft_gt", _vp), ("soft_nogt", _vp),
        ("g_param", _vp), ("g_grad", _vp), ("g_m", _vp), ("g_v", _vp),
        ("d_param", _vp), ("d_grad", _vp), ("d_m", _vp), ("d_v", _vp),
        ("step_count", _vp),
        ("lr_g", _f), ("lr_d", _f), ("beta1", _f), ("beta2", _f), ("eps", _f),
        ("lambda_cls", _f), ("lambda_adv", _f), ("drop_p", _f),
        ("rng_seed", _u64),
        ("apply_adam", _i),
        ("losses", _vp), ("logits", _vp),
        ("workspace", _vp), ("workspace_bytes", _sz),
        ("semi", _i), ("lambda_semi", _f), ("semi_th", _f),
        ("part", _i),
        ("precision", _i),
        ("rng_rank", _i), ("rng_world", _i),
        ("epi_counters", _vp), ("epi_ncounters", _i), ("epi_ring", _vp), ("epi_slots", _i),
        ("epi_nl", _i), ("epi_ring_count", _vp),
        ("gather", _vp), ("ngather", _i),
        ("feat_gmax", _vp), ("feat_dgmax", _vp),
    ]


class PwWgradJob(ctypes.Structure):
    """Mirror of pcadv_pw_wgrad_job (include/pcadv.h)."""

    _fields_ = [("slabs", _vp), ("M", _i), ("O", _i), ("K", _i), ("dw", _vp), ("db", _vp)]


class PwLayer(ctypes.Structure):
    """Mirror of pcadv_pw_layer (include/pcadv.h)."""

    _fields_ = [("w", _vp), ("b", _vp), ("y", _vp), ("O", _i), ("act", _i), ("w_kmajor", _i),
                ("rows_per_w", _i)]


class GatherJob(ctypes.Structure):
    """Mirror of pcadv_gather_job (include/pcadv.h)."""

    _fields_ = [
        ("src", _vp), ("n_src", _i64), ("npts", _i), ("src_npts", _i),
        ("order", _vp), ("cursor", _vp), ("B", _i),
        ("src_lab", _vp), ("lab_width", _i), ("src_seg", _vp),
        ("sigma", ctypes.c_double), ("clip", ctypes.c_double), ("seed", _u64), ("step", _vp),
        ("out", _vp), ("out_lab", _vp), ("out_seg", _vp), ("rng_row0", _i64),
    ]


# name -> (restype, argtypes); every symbol of include/pcadv.h
SIGNATURES = {
    "pcadv_last_error": (ctypes.c_char_p, []),
    "pcadv_abi_version": (_i, []),
    "pcadv_feat_fwd_workspace_bytes": (_sz, [_i, _i]),
    "pcadv_feat_fwd": (_i, [_vp, _i, _i] + [_vp] * 8 + [_vp] * 3 + [_vp, _sz, _vp]),
    "pcadv_feat_fwd_bf16": (_i, [_vp, _i, _i] + [_vp] * 8 + [_vp] * 3 + [_vp, _sz, _vp]),
    "pcadv_conv4_max": (_i, [_vp, _i, _i, _vp, _vp, _vp, _vp, _i, _vp]),
    "pcadv_feat_bwd_workspace_bytes": (_sz, [_i, _i]),
    "pcadv_feat_bwd": (_i, [_vp, _vp, _vp, _i, _i] + [_vp] * 7 + [_vp] * 8 + [_vp, _sz, _vp]),
    "pcadv_conv_max_fwd": (_i, [_vp, _i, _i, _i, _vp, _vp, _i, _i, _vp, _vp, _vp]),
    "pcadv_linear_fwd": (_i, [_vp, _vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp, _u64, _f, _i, _vp]),
    "pcadv_linear_bwd": (_i, [_vp, _vp, _i, _vp, _vp, _u64, _f, _vp, _vp, _vp, _vp, _vp,
                              _i, _i, _i, _i, _vp]),
    "pcadv_adam": (_i, [_vp, _vp, _vp, _vp, _i64, _vp, _f, _f, _f, _f, _vp]),
    "pcadv_concat2": (_i, [_vp, _i64, _vp, _i64, _vp, _vp, _vp]),
    "pcadv_adam2": (_i, [_vp, _vp, _vp, _vp, _i64, _f, _vp, _vp, _vp, _vp, _i64, _f, _vp, _f, _f,
                         _f, _vp]),
    "pcadv_pw_fwd": (_i, [_vp, _i, _i, _vp, _vp, _i, _i, _i, _i, _vp, _vp]),
    "pcadv_pw_chain": (_i, [_vp, _i, _i, ctypes.POINTER(PwLayer), _i, _vp]),
    "pcadv_pw_bwd_data": (_i, [_vp, _vp, _i, _i, _i, _vp, _i, _i, _i, _vp, _i, _vp]),
    "pcadv_pw_bwd_weight_workspace_bytes": (_sz, [_i, _i, _i]),
    "pcadv_pw_bwd_weight": (_i, [_vp, _vp, _i, _vp, _i, _i, _i, _i, _i, _vp, _vp, _vp, _sz,
                                 _vp]),
    "pcadv_pw_wgrad_finish": (_i, [ctypes.POINTER(PwWgradJob), _i, _vp]),
    "pcadv_conv_max_bwd": (_i, [_vp, _vp, _vp, _vp, _i, _i, _i, _vp, _i, _vp, _vp, _vp, _i, _vp]),
    "pcadv_tnet_reg_fwd": (_i, [_vp, _i, _i, _vp, _vp, _vp]),
    "pcadv_tnet_reg_bwd": (_i, [_vp, _i, _i, _vp, _vp, _vp]),
    "pcadv_tnet_reg_step": (_i, [_vp, _i, _i, _vp, _vp, _vp, _vp, _vp, _vp]),
    "pcadv_gemm": (_i, [_vp, _i64, _i, _vp, _i64, _i, _vp, _i64, _i, _i, _i, _vp, _vp, _i, _i, _i,
                        _vp, _i64, _i, _vp, _vp, _i64, _vp]),
    "pcadv_gemm_bf2": (_i, [_vp, _vp, _i64, _vp, _vp, _i64, _vp, _i64, _vp, _vp, _i64, _i, _i, _i,
                            _vp, _vp, _i, _i, _i, _vp, _i64, _vp]),
    "pcadv_split_bf2": (_i, [_vp, _i64, _i, _i, _vp, _vp, _i64, _vp]),
    "pcadv_split_bf3": (_i, [_vp, _i64, _i, _i, _vp, _vp, _vp, _i64, _vp]),
    "pcadv_gemm_b3": (_i, [_vp, _i64, _vp, _vp, _vp, _i64, _vp, _i64, _i, _i, _i, _vp, _vp, _i, _i,
                           _i, _vp]),
    "pcadv_conv_max_bf2": (_i, [_vp, _i64, _vp, _vp, _i64, _i, _i, _i, _vp, _vp, _vp, _vp, _i, _i,
                                _vp, _vp, _vp, _sz, _vp]),
    "pcadv_gemm_wgrad_workspace_bytes": (_sz, [_i, _i, _i, _i]),
    "pcadv_gemm_wgrad": (_i, [_vp, _i64, _vp, _i64, _i, _i, _i, _vp, _i64, _vp, _vp, _i, _i, _vp,
                              _sz, _vp]),
    "pcadv_gemm_wgrad_slabs": (_i, [ctypes.POINTER(WgradDesc), ctypes.POINTER(GemmDesc), _vp]),
    "pcadv_wgrad_finish": (_i, [ctypes.POINTER(WgradDesc), _i, _vp]),
    "pcadv_wgrad_small": (_i, [_vp, _i64, _i, _i, _vp, _i64, _i, _vp, _vp, _i64, _i, _vp, _i64, _i,
                               _vp]),
    "pcadv_colsum_workspace_bytes": (_sz, [_i, _i]),
    "pcadv_colsum": (_i, [_vp, _vp, _i64, _i64, _i, _i, _vp, _i, _vp, _sz, _vp]),
    "pcadv_group_colsum": (_i, [_vp, _vp, _i64, _i64, _i, _i, _i, _vp, _vp]),
    "pcadv_conv_max_x3_workspace_bytes": (_sz, [_i, _i, _i]),
    "pcadv_conv_max_x3": (_i, [_vp, _i64, _i, _i, _i, _vp, _vp, _i, _i, _vp, _vp, _vp, _sz, _vp]),
    "pcadv_conv_max_x3_bwd": (_i, [_vp, _vp, _vp, _vp, _i64, _i, _i, _i, _i, _vp, _vp, _vp, _vp,
                                   _i64, _i, _vp]),
    "pcadv_h5_info": (_i, [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(_i),
                           ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(_i)]),
    "pcadv_h5_read": (_i, [ctypes.c_char_p, ctypes.c_char_p, _i, _i64, _vp, _sz]),
    "pcadv_gather_clouds": (_i, [_vp, _i64, _i, _i, _vp, _i, _vp, _i, _vp, ctypes.c_double,
                                 ctypes.c_double, _vp, _u64, _vp,
                                 _vp, _vp, _vp, _i64, _vp]),
    "pcadv_gather_clouds_at": (_i, [_vp, _i64, _i, _i, _vp, _vp, _i, _vp, _i, _vp, ctypes.c_double,
                                    ctypes.c_double, _u64, _vp, _vp, _vp, _vp, _i64, _vp]),
    "pcadv_gather_clouds_multi": (_i, [ctypes.POINTER(GatherJob), _i, _vp]),
    "pcadv_iter_epilogue": (_i, [_vp, _i, _vp, _i, _vp, _i, _vp, _vp]),
    "pcadv_row_ce_workspace_bytes": (_sz, [_i]),
    "pcadv_row_ce": (_i, [_vp, _i64, _vp, _i, _i, _f, _vp, _vp, _vp, _sz, _vp]),
    "pcadv_adv_step_workspace_bytes": (_sz, [_i, _i]),
    "pcadv_adv_step": (_i, [ctypes.POINTER(AdvArgs), _vp]),
    "pcadv_adv_step_adam": (_i, [ctypes.POINTER(AdvArgs), _vp]),
    "pcadv_cls_step": (_i, [ctypes.POINTER(AdvArgs), _vp]),
}

_lib = None


class PcadvError(RuntimeError):
    pass


def load():
    """dlopen libpcadv.so once; raise if it is missing (no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise PcadvError(
                f"libpcadv.so not found at {LIB_PATH}: build it with `make` (hipcc, gfx950). "
                "There is no CPU fallback for the pcadv ops.")
        lib = ctypes.CDLL(LIB_PATH)
        lib.pcadv_abi_version.restype = ctypes.c_int
        lib.pcadv_abi_version.argtypes = []
        abi = lib.pcadv_abi_version()
        if abi != ABI_VERSION:
            # a stale build (or an older PCADV_LIB) would bind silently with shifted
            # arguments: e.g. ABI 7's rng_row0 would land in an ABI 5 gather's stream
            raise PcadvError(
                f"{LIB_PATH} implements pcadv ABI {abi}, this package binds ABI {ABI_VERSION}: "
                "rebuild it with `make`")
        for name, (res, args) in SIGNATURES.items():
            if os.environ.get("PCADV_LIB") and not hasattr(lib, name):
                continue  # an older library picked for an A/B timing run
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def check(rc: int, what: str):
    if rc != PCADV_OK:
        msg = load().pcadv_last_error().decode(errors="replace")
        raise PcadvError(f"{what} failed (rc={rc}): {msg}")


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_ptr():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def use_stream_graph_dispatch() -> bool:
    """Opt in to replaying HIP graphs through the stream dispatch path.

    Sets DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 (a ROCm runtime debug switch: graph
    kernel nodes are dispatched like stream launches instead of from
    pre-recorded AQL packets; measured on MI355X: adv step -2.5 %, cls -3.5 %,
    seg unchanged).  The HIP runtime reads it once when it
    initialises, so it changes graph dispatch for EVERY library in the
    process, and only if called before the first GPU call.  Importing the
    package never sets it; bench.py calls this at its start.  An explicit
    setting in the environment is left alone.  Returns True when the runtime
    will see the value 0."""
    if "DEBUG_CLR_GRAPH_PACKET_CAPTURE" not in os.environ:
        if torch.cuda.is_initialized():
            return False
        os.environ["DEBUG_CLR_GRAPH_PACKET_CAPTURE"] = "0"
    return os.environ["DEBUG_CLR_GRAPH_PACKET_CAPTURE"] == "0"
