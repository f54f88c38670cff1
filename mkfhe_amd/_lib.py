"""ctypes binding of the C ABI in include/mkfhe_amd.h (libmkfhe_amd.so).

The shared library is built in-tree (mkfhe_amd/lib/) by mkfhe_amd.build or
__graft_entry__.build().  There is no fallback: if the library is missing the
import of the accumulator fails loudly.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# MKFHE_LIB: load another build of the engine (A/B timing of kernel variants)
LIB_PATH = os.environ.get("MKFHE_LIB") or os.path.join(_HERE, "lib", "libmkfhe_amd.so")

MKACC_OK = 0
MKACC_E_ARG = -1
MKACC_E_UNSUPPORTED = -2
MKACC_E_NOKEYS = -3
MKACC_E_DEVICE = -4
MKACC_E_RANGE = -5

METHOD_MKNTRU = 0
METHOD_MKNTRU_B = 1
METHOD_MKNTRU_LWE = 2

_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)


class MkaccParams(ctypes.Structure):
    """struct mkacc_params (include/mkfhe_amd.h)."""

    _fields_ = [
        ("method", ctypes.c_uint32),
        ("k", ctypes.c_uint32),
        ("n", ctypes.c_uint32),
        ("N", ctypes.c_uint32),
        ("Q", ctypes.c_uint64),
        ("q", ctypes.c_uint64),
        ("baseG", ctypes.c_uint32),
        ("digitsG", ctypes.c_uint32),
        ("root", ctypes.c_uint64),
    ]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class MkaccKsParams(ctypes.Structure):
    """struct mkacc_ks_params (include/mkfhe_amd.h)."""

    _fields_ = [("qKS", ctypes.c_uint64), ("baseKS", ctypes.c_uint32), ("n_out", ctypes.c_uint32)]


# every symbol include/mkfhe_amd.h declares, with (restype, argtypes)
SIGNATURES = {
    "mkacc_paramset": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_uint32, ctypes.POINTER(MkaccParams)]),
    "mkacc_create": (ctypes.c_int, [ctypes.POINTER(MkaccParams), ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "mkacc_destroy": (None, [ctypes.c_void_p]),
    "mkacc_get_params": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MkaccParams)]),
    "mkacc_evk_words": (ctypes.c_size_t, [ctypes.c_void_p]),
    "mkacc_pkey_words": (ctypes.c_size_t, [ctypes.c_void_p]),
    "mkacc_upload_keys": (ctypes.c_int, [ctypes.c_void_p, _u32p, _u32p]),
    "mkacc_upload_keys_u64": (ctypes.c_int, [ctypes.c_void_p, _u64p, _u64p]),
    "mkacc_upload_keys_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]),
    "mkacc_eval_batch": (ctypes.c_int, [ctypes.c_void_p, _u32p, _u32p, _u32p, ctypes.c_size_t]),
    "mkacc_eval_batch_u64": (ctypes.c_int, [ctypes.c_void_p, _u32p, _u64p, _u64p, ctypes.c_size_t]),
    "mkacc_is_wide": (ctypes.c_int, [ctypes.c_void_p]),
    "mkacc_ntt_forward_u64": (ctypes.c_int, [ctypes.c_void_p, _u64p, _u64p, ctypes.c_size_t]),
    "mkacc_ntt_inverse_u64": (ctypes.c_int, [ctypes.c_void_p, _u64p, _u64p, ctypes.c_size_t]),
    "mkacc_sdd_u64": (ctypes.c_int, [ctypes.c_void_p, _u64p, _u64p, ctypes.c_size_t]),
    "mkacc_eval_batch_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                               ctypes.c_void_p, ctypes.c_size_t]),
    "mkacc_sync": (ctypes.c_int, [ctypes.c_void_p]),
    "mkacc_stream": (ctypes.c_void_p, [ctypes.c_void_p]),
    "mkacc_ks_digits": (ctypes.c_uint32, [ctypes.POINTER(MkaccKsParams)]),
    "mkacc_upload_ksk_mntru": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MkaccKsParams), _u32p]),
    "mkacc_upload_ksk_mklwe": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MkaccKsParams), _u32p, _u32p]),
    "mkacc_eval_nand_mntru": (ctypes.c_int, [ctypes.c_void_p, _u32p, _u32p, _u32p, _u32p, ctypes.c_size_t]),
    "mkacc_eval_nand_mklwe": (ctypes.c_int, [ctypes.c_void_p, _u32p, _u32p, _u32p, _u32p, _u32p, _u32p,
                                             ctypes.c_size_t]),
    "mkacc_eval_nand_device": (ctypes.c_int, [ctypes.c_void_p] + [ctypes.c_void_p] * 7 + [ctypes.c_size_t]),
    "mkacc_gate_tail": (ctypes.c_int, [ctypes.c_void_p, _u32p, _u32p, _u32p, ctypes.c_size_t]),
    "mkacc_ntt_forward": (ctypes.c_int, [ctypes.c_void_p, _u32p, _u32p, ctypes.c_size_t]),
    "mkacc_ntt_inverse": (ctypes.c_int, [ctypes.c_void_p, _u32p, _u32p, ctypes.c_size_t]),
    "mkacc_sdd": (ctypes.c_int, [ctypes.c_void_p, _u32p, _u32p, ctypes.c_size_t]),
    "mkacc_last_error": (ctypes.c_char_p, []),
    "mkacc_abi_version": (ctypes.c_int, []),
}

_lib = None


def load():
    """Load libmkfhe_amd.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} not found: build the HIP engine first (python -m mkfhe_amd.build)")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def last_error() -> str:
    return load().mkacc_last_error().decode()


class MkaccError(RuntimeError):
    """Raised on a nonzero MKACC status (reference: OPENFHE_THROW config_error / math_error)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"[{code}] {msg}")
        self.code = code


def check(rc: int):
    if rc != MKACC_OK:
        raise MkaccError(rc, last_error())
