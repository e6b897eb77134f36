"""ctypes binding of libsdp.so (the C ABI declared in include/sdp.h).

The library must be loaded after ``import torch``: torch's bundled HIP runtime and the one
libsdp.so links share the SONAME ``libamdhip64.so.7``, so the dynamic linker reuses torch's
instance and device pointers / hipStream_t handles from torch are valid in libsdp.
There is no CPU fallback: if the library is missing, every entry point raises.
"""
from __future__ import annotations

import ctypes as C
import os

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SDP_LIB", os.path.join(_HERE, "_lib", "libsdp.so"))

P = C.c_void_p
I = C.c_int
F = C.c_float
D = C.c_double
U64 = C.c_uint64
SZ = C.c_size_t


class NetDesc(C.Structure):
    _fields_ = [("ngf", I), ("channels", I), ("H", I), ("W", I), ("num_classes", I), ("precision", I)]


class MergeParams(C.Structure):
    _fields_ = [("variant", I), ("setting", I), ("sigma", F), ("allowance", F), ("cc", F)]


class LangevinParams(C.Structure):
    _fields_ = [("ref", P), ("mask", P), ("noise", P), ("seed", U64), ("offset", U64), ("step_size", F),
                ("noise_scale", F), ("grad_ref", F), ("nan_to_num", I), ("lik_out", P), ("absmax_bits", P),
                ("grad_out", P)]


PREC = {"fp32": 0, "fp32x3": 1, "bf16": 2}
MERGE_POSES, MERGE_ORIGINS = 0, 1

_SIGS = {
    "sdp_version": (I, []),
    "sdp_last_error": (C.c_char_p, []),
    "sdp_net_create": (I, [C.POINTER(NetDesc), C.POINTER(P)]),
    "sdp_net_set_param": (I, [P, C.c_char_p, P, C.POINTER(C.c_int64), I]),
    "sdp_net_finalize": (I, [P]),
    "sdp_net_workspace_size": (I, [P, I, C.POINTER(SZ)]),
    "sdp_net_forward": (I, [P, P, P, P, I, P, SZ, P]),
    "sdp_net_forward_langevin": (I, [P, P, P, I, C.POINTER(LangevinParams), P, SZ, P]),
    "sdp_net_set_split": (I, [P, I]),
    "sdp_net_set_tape": (I, [P, I]),
    "sdp_net_destroy": (I, [P]),
    "sdp_net_profile_enable": (I, [P, I]),
    "sdp_net_profile_read": (I, [P, C.c_char_p, SZ, C.POINTER(I)]),
    "sdp_net_param_arena_floats": (I, [P, C.POINTER(SZ)]),
    "sdp_net_param_count": (I, [P, C.POINTER(I)]),
    "sdp_net_param_info": (I, [P, I, C.c_char_p, SZ, C.POINTER(SZ), C.POINTER(SZ)]),
    "sdp_net_bind_params": (I, [P, P, P]),
    "sdp_net_repack": (I, [P, P]),
    "sdp_net_train_workspace_size": (I, [P, I, C.POINTER(SZ)]),
    "sdp_net_forward_train": (I, [P, P, P, P, I, P, SZ, P]),
    "sdp_net_backward": (I, [P, P, I, P, SZ, P, P]),
    "sdp_net_backward_buckets": (I, [P, P, I, P, SZ, P, I, C.POINTER(SZ), C.POINTER(P), P]),
    "sdp_dsm_loss": (I, [P, P, P, P, I, I, F, P, P, P, P, P]),
    "sdp_adam_ema_step": (I, [P, P, P, P, P, SZ, D, D, D, D, I, D, P]),
    "sdp_optim_ema_step": (I, [I, P, P, P, P, P, P, SZ, D, D, D, D, D, I, D, P]),
    "sdp_range_project_workspace_size": (I, [I, I, C.POINTER(SZ)]),
    "sdp_range_project": (I, [P, I, I, I, P, I, I, P, P, P, P, P, P, SZ, P]),
    "sdp_view_transform": (I, [P, C.c_int64, P, P, P, P]),
    "sdp_view_gather": (I, [P, I, I, I, P, P, P, P]),
    "sdp_view_finalize": (I, [P, P, P, P, P, P, I, I, I, I, I, I, P, P, P, P, P]),
    "sdp_grid_subsample": (I, [P, C.c_int64, P, I, P, I, F, I, P, P, P, C.POINTER(C.c_int64)]),
    "sdp_langevin_step": (I, [P, P, P, P, P, U64, U64, F, F, F, I, I, I, I, P, P, P]),
    "sdp_axpy_step": (I, [P, P, F, P, P, P, F, I, P]),
    "sdp_merge_workspace_size": (I, [I, I, I, I, C.POINTER(SZ)]),
    "sdp_merge_workspace_bytes": (I, [I, I, I, I, I, C.POINTER(SZ)]),
    "sdp_consistency_merge": (I, [P, I, I, I, I, I, I, P, P, P, P, P, P, C.POINTER(MergeParams), P, P, P, SZ, P]),
    "sdp_consistency_merge_ev": (I, [P, I, I, I, I, I, I, P, P, P, P, P, P, C.POINTER(MergeParams), P, P, P, SZ, P, P]),
}

_lib = None


def lib():
    """Load libsdp.so once, building it first if it is missing or stale (sdp/_build.py). A build
    failure raises with the compiler's output; there is no fallback path."""
    global _lib
    if _lib is None:
        from . import _build
        _build.ensure_built()
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"libsdp.so not found at {LIB_PATH}: build it with `python __graft_entry__.py build` "
                               "(or `make -C simultaneous-diffusion-for-pointclouds_amd/csrc`)")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        raise RuntimeError(f"libsdp {what}: {lib().sdp_last_error().decode()}")


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()


def stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def exported_symbols():
    return list(_SIGS)
