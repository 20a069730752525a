"""ctypes binding of libntt.so (include/ntt.h).

The library is the product: there is no CPU fallback.  ``load()`` raises if the in-tree
``ntt_amd/libntt.so`` is missing (build it with ``python -m ntt_amd.build`` or
``__graft_entry__.build()``).
"""
from __future__ import annotations

import ctypes as C
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("NTT_LIB_PATH") or os.path.join(HERE, "libntt.so")

NTT_OK = 0
NTT_ERR_ARG, NTT_ERR_HIP, NTT_ERR_RCCL, NTT_ERR_FIELD, NTT_ERR_NODEV, NTT_ERR_DEVICE = -1, -2, -3, -4, -5, -6
NTT_FIELD_P469762049 = 0
NTT_FIELD_BN254_FR = 1
NTT_FIELD_BLS12_381_FR = 2
NTT_PLAN_TWIDDLE_ONLY = 1
NTT_PLAN_MONTGOMERY_IO = 2
NTT_PLAN_STOCKHAM = 4
NTT_PLAN_GZKP = 8
NTT_PLAN_IN_PLACE = 16
NTT_PLAN_SINGLE_LAUNCH = 32
NTT_PLAN_NAIVE = 64
NTT_PLAN_NO_SWAP = 128
NTT_PLAN_BELLPERSON = 256
NTT_PLAN_IMPROVED_V1 = 512
NTT_PLAN_IMPROVED_V2 = 1024
NTT_PLAN_IMPROVED_V3 = 2048
NTT_PLAN_IMPROVED_V4 = 4096

# Every symbol declared in include/ntt.h with its ctypes prototype: (restype, argtypes).
_vp = C.c_void_p
PROTOTYPES = {
    "ntt_plan_create": (C.c_int, [C.POINTER(_vp), C.c_int, C.c_uint, C.c_uint, C.c_int]),
    "ntt_plan_create_custom": (C.c_int, [C.POINTER(_vp), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_uint,
                                         C.c_uint, C.c_int]),
    "ntt_forward": (C.c_int, [_vp, _vp, _vp]),
    "ntt_inverse": (C.c_int, [_vp, _vp, _vp]),
    "ntt_forward_batch": (C.c_int, [_vp, _vp, C.c_uint, _vp]),
    "ntt_inverse_batch": (C.c_int, [_vp, _vp, C.c_uint, _vp]),
    "ntt_pointwise_mul": (C.c_int, [_vp, _vp, _vp, _vp, _vp]),
    "ntt_forward_coset": (C.c_int, [_vp, _vp, C.POINTER(C.c_uint64), _vp]),
    "ntt_inverse_coset": (C.c_int, [_vp, _vp, C.POINTER(C.c_uint64), _vp]),
    "ntt_polymul": (C.c_int, [_vp, _vp, _vp, _vp, _vp]),
    "ntt_fill": (C.c_int, [_vp, _vp, C.c_int, C.c_uint64, _vp]),
    "ntt_plan_info": (C.c_int, [_vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint), C.POINTER(C.c_uint),
                                C.POINTER(C.c_uint)]),
    "ntt_plan_destroy": (C.c_int, [_vp]),
    "ntt_plan_set_profiling": (C.c_int, [_vp, C.c_int]),
    "ntt_plan_last_launch_ms": (C.c_int, [_vp, C.POINTER(C.c_float), C.c_uint, C.POINTER(C.c_uint)]),
    "ntt_plan_last_launch_labels": (C.c_int, [_vp, C.c_char_p, C.c_uint]),
    "ntt_plan_profile_group": (C.c_int, [_vp]),
    "ntt_strerror": (C.c_char_p, [C.c_int]),
    "SSIP": (None, [_vp, C.c_longlong, C.c_uint]),
    "NTT_GZKP_256": (C.c_int, [_vp, C.c_uint32, _vp, C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                               C.c_uint32, C.c_uint32]),
    "NTT_GZKP_64": (C.c_int, [_vp, _vp, C.c_longlong, C.c_longlong, C.c_int, C.c_int, C.c_longlong]),
    "ntt_last_error": (C.c_int, []),
    "ntt_plan_create_ex": (C.c_int, [C.POINTER(_vp), C.c_int, C.c_uint, C.c_uint, C.c_int, C.c_uint]),
    "ntt_plan_create_custom_ex": (C.c_int, [C.POINTER(_vp), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.c_uint,
                                            C.c_uint, C.c_int, C.c_uint]),
    "ntt_fill_map": (C.c_int, [_vp, _vp, C.c_uint64, C.c_int, C.c_uint64, C.c_uint64, C.c_uint, C.c_uint, _vp]),
    "ntt_twiddle_pack": (C.c_int, [_vp, _vp, _vp, C.c_uint, C.c_uint, C.c_uint, C.c_uint64, C.c_int, _vp]),
    "ntt_transpose": (C.c_int, [_vp, _vp, _vp, C.c_uint, C.c_uint, _vp]),
    "ntt_mplan_create": (C.c_int, [C.POINTER(_vp), C.c_int, C.c_uint, C.c_uint, C.c_int, C.POINTER(C.c_int)]),
    "ntt_forward_multi": (C.c_int, [_vp, C.POINTER(_vp), C.POINTER(_vp)]),
    "ntt_inverse_multi": (C.c_int, [_vp, C.POINTER(_vp), C.POINTER(_vp)]),
    "ntt_mplan_fill": (C.c_int, [_vp, C.POINTER(_vp), C.c_int, C.c_uint64, C.POINTER(_vp)]),
    "ntt_mplan_info": (C.c_int, [_vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint), C.POINTER(C.c_uint)]),
    "ntt_mplan_set_pieces": (C.c_int, [_vp, C.c_uint]),
    "ntt_mplan_set_pieces2": (C.c_int, [_vp, C.c_uint, C.c_uint]),
    "ntt_mplan_destroy": (C.c_int, [_vp]),
    "ntt_count_noncanonical": (C.c_int, [_vp, _vp, C.c_uint64, C.POINTER(C.c_uint64), _vp]),
    "ntt_plan_device_status": (C.c_int, [_vp, C.POINTER(C.c_uint)]),
    "ntt_plan_set_watchdog": (C.c_int, [_vp, C.c_uint]),
    "ntt_shim_cache_clear": (None, []),
    "ntt_inverse_pointwise_batch": (C.c_int, [_vp, _vp, _vp, _vp, C.c_uint, _vp]),
    "ntt_twiddle_pack_ex": (C.c_int, [_vp, _vp, _vp, C.c_uint, C.c_uint, C.c_uint, C.c_uint64, C.c_int, C.c_uint64,
                                      _vp]),
    "ntt_transpose_ex": (C.c_int, [_vp, _vp, _vp, C.c_uint, C.c_uint, C.c_uint, C.c_uint64, _vp]),
    "ntt_polymul_multi": (C.c_int, [_vp, C.POINTER(_vp), C.POINTER(_vp), C.POINTER(_vp), C.POINTER(_vp)]),
    "ntt_rplan_create": (C.c_int, [C.POINTER(_vp), C.c_int, C.c_uint, C.c_uint, C.c_int, C.c_int, C.c_int]),
    "ntt_rplan_info": (C.c_int, [_vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), C.POINTER(C.c_uint),
                                 C.POINTER(C.c_uint), C.POINTER(C.c_uint)]),
    "ntt_rplan_forward_rows": (C.c_int, [_vp, _vp, _vp, C.c_uint, C.c_uint, _vp]),
    "ntt_rplan_forward_cols": (C.c_int, [_vp, _vp, _vp, C.c_uint, C.c_uint, _vp]),
    "ntt_rplan_inverse_cols": (C.c_int, [_vp, _vp, _vp, _vp, _vp]),
    "ntt_rplan_inverse_rows": (C.c_int, [_vp, _vp, _vp, _vp]),
    "ntt_rplan_forward_rows_range": (C.c_int, [_vp, _vp, _vp, C.c_uint, C.c_uint, C.c_uint64, C.c_uint64, _vp]),
    "ntt_rplan_inverse_rows_range": (C.c_int, [_vp, _vp, _vp, C.c_uint64, C.c_uint64, _vp]),
    "ntt_rplan_forward_rows_piece": (C.c_int, [_vp, _vp, _vp, C.c_uint, C.c_uint, C.c_uint, C.c_uint, C.c_uint, _vp]),
    "ntt_rplan_forward_cols_piece": (C.c_int, [_vp, _vp, _vp, C.c_uint, C.c_uint, C.c_uint, C.c_uint, C.c_uint, _vp]),
    "ntt_rplan_inverse_cols_piece": (C.c_int, [_vp, _vp, _vp, _vp, C.c_uint, C.c_uint, C.c_uint, _vp]),
    "ntt_rplan_inverse_rows_piece": (C.c_int, [_vp, _vp, _vp, C.c_uint, C.c_uint, C.c_uint, _vp]),
    "ntt_rplan_fill": (C.c_int, [_vp, _vp, C.c_int, C.c_uint64, _vp]),
    "ntt_rplan_set_profiling": (C.c_int, [_vp, C.c_int]),
    "ntt_rplan_last_launch_ms": (C.c_int, [_vp, C.c_int, C.POINTER(C.c_float), C.c_uint, C.POINTER(C.c_uint)]),
    "ntt_rplan_last_launch_labels": (C.c_int, [_vp, C.c_int, C.c_char_p, C.c_uint]),
    "ntt_rplan_profile_group": (C.c_int, [_vp]),
    "ntt_rplan_destroy": (C.c_int, [_vp]),
}

_lock = threading.Lock()
_lib = None


class NTTError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        msg = _strerror(status)
        super().__init__(f"{what}: {msg} (status {status})" if what else f"{msg} (status {status})")
        self.status = status


def _strerror(status: int) -> str:
    try:
        return load().ntt_strerror(status).decode()
    except Exception:  # pragma: no cover - library unavailable
        return "error"


def load(path: str = LIB_PATH) -> C.CDLL:
    """Load libntt.so (in-tree) and attach prototypes.  Raises if it is missing."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise FileNotFoundError(
                f"{path} not found: build the HIP extension first (python -m ntt_amd.build); "
                "the NTT has no CPU fallback")
        lib = C.CDLL(path, mode=C.RTLD_GLOBAL)
        for name, (res, args) in PROTOTYPES.items():
            fn = getattr(lib, name, None)
            if fn is None:
                continue
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def check(status: int, what: str = "") -> None:
    if status != NTT_OK:
        raise NTTError(status, what)
