"""ctypes binding of the C ABI in include/mkfhe_amd.h (libmkfhe_amd.so).

The shared library is built in-tree (mkfhe_amd/lib/) by mkfhe_amd.build or
__graft_entry__.build().  There is no fallback: if the library is missing the
import of the accumulator fails loudly.
"""
from __future__ import annotations

import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
DEFAULT_LIB_PATH = os.path.join(_HERE, "lib", "libmkfhe_amd.so")
# MKFHE_LIB: load another build of the engine (A/B timing of kernel variants)
LIB_PATH = os.environ.get("MKFHE_LIB") or DEFAULT_LIB_PATH

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
    "mkacc_step_kernel_name": (ctypes.c_char_p, [ctypes.c_void_p, ctypes.c_size_t]),
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
    "mkacc_upload_ksk_mntru_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MkaccKsParams), ctypes.c_void_p]),
    "mkacc_upload_ksk_mklwe_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MkaccKsParams), ctypes.c_void_p,
                                                     ctypes.c_void_p]),
    "mkacc_eval_nand_mntru": (ctypes.c_int, [ctypes.c_void_p, _u32p, _u32p, _u32p, _u32p, ctypes.c_size_t]),
    "mkacc_eval_nand_mklwe": (ctypes.c_int, [ctypes.c_void_p, _u32p, _u32p, _u32p, _u32p, _u32p, _u32p,
                                             ctypes.c_size_t]),
    "mkacc_eval_nand_device": (ctypes.c_int, [ctypes.c_void_p] + [ctypes.c_void_p] * 7 + [ctypes.c_size_t]),
    "mkacc_gate_tail": (ctypes.c_int, [ctypes.c_void_p, _u32p, _u32p, _u32p, ctypes.c_size_t]),
    "mkacc_ntt_forward": (ctypes.c_int, [ctypes.c_void_p, _u32p, _u32p, ctypes.c_size_t]),
    "mkacc_ntt_inverse": (ctypes.c_int, [ctypes.c_void_p, _u32p, _u32p, ctypes.c_size_t]),
    "mkacc_sdd": (ctypes.c_int, [ctypes.c_void_p, _u32p, _u32p, ctypes.c_size_t]),
    "mkacc_group_create": (ctypes.c_int, [ctypes.POINTER(MkaccParams), ctypes.POINTER(ctypes.c_int), ctypes.c_uint32,
                                          ctypes.POINTER(ctypes.c_void_p)]),
    "mkacc_group_destroy": (None, [ctypes.c_void_p]),
    "mkacc_group_size": (ctypes.c_uint32, [ctypes.c_void_p]),
    "mkacc_group_member": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.c_uint32]),
    "mkacc_shard_range": (None, [ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, ctypes.POINTER(ctypes.c_size_t),
                                 ctypes.POINTER(ctypes.c_size_t)]),
    "mkacc_group_upload_keys": (ctypes.c_int, [ctypes.c_void_p, _u32p, _u32p]),
    "mkacc_group_upload_keys_u64": (ctypes.c_int, [ctypes.c_void_p, _u64p, _u64p]),
    "mkacc_group_upload_ksk_mntru": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MkaccKsParams), _u32p]),
    "mkacc_group_upload_ksk_mklwe": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(MkaccKsParams), _u32p, _u32p]),
    "mkacc_group_eval_batch": (ctypes.c_int, [ctypes.c_void_p, _u32p, _u32p, _u32p, ctypes.c_size_t]),
    "mkacc_group_eval_batch_u64": (ctypes.c_int, [ctypes.c_void_p, _u32p, _u64p, _u64p, ctypes.c_size_t]),
    "mkacc_group_eval_nand_mntru": (ctypes.c_int, [ctypes.c_void_p, _u32p, _u32p, _u32p, _u32p, ctypes.c_size_t]),
    "mkacc_group_eval_nand_mklwe": (ctypes.c_int, [ctypes.c_void_p, _u32p, _u32p, _u32p, _u32p, _u32p, _u32p,
                                                   ctypes.c_size_t]),
    "mkacc_last_error": (ctypes.c_char_p, []),
    "mkacc_abi_version": (ctypes.c_int, []),
    "mkacc_build_info": (ctypes.c_char_p, []),
}

_lib = None


class LibraryMismatch(RuntimeError):
    """The library on disk was not built from this tree (ABI, header or sources differ)."""


def header_abi_version(header: str) -> int:
    """The #define ..._ABI_VERSION of a C header in include/."""
    import re
    with open(header) as f:
        m = re.search(r"#define\s+\w+_ABI_VERSION\s+(\d+)", f.read())
    if not m:
        raise LibraryMismatch(f"{header}: no ABI version")
    return int(m.group(1))


def parse_build_info(text: str) -> dict:
    """'abi=2;header=..;source=..;flags=..' -> dict"""
    return dict(kv.split("=", 1) for kv in text.split(";") if "=" in kv)


def verify_build(path: str, info_text: str, abi: int, header: str, ids: dict, require_source: bool) -> dict:
    """Refuse a library whose ABI version, header id or (require_source) source id
    differs from this tree (mkfhe_amd/build.py computes the ids)."""
    info = parse_build_info(info_text)
    want_abi = header_abi_version(header)
    if abi != want_abi or info.get("abi") != str(want_abi):
        raise LibraryMismatch(f"refusing {path}: ABI version {abi} (build info {info.get('abi')}), "
                              f"{os.path.basename(header)} declares {want_abi}")
    if info.get("header") != ids["header"]:
        raise LibraryMismatch(f"refusing {path}: built against header id {info.get('header')}, "
                              f"this tree's is {ids['header']} (rebuild: python -m mkfhe_amd.build)")
    if require_source and info.get("source") != ids["source"]:
        raise LibraryMismatch(f"refusing {path}: built from source id {info.get('source')}, "
                              f"this tree's is {ids['source']} (stale build: python -m mkfhe_amd.build)")
    return info


def open_checked(path: str, require_source: bool | None = None):
    """CDLL of an engine library after its build identity has been checked.
    The default in-tree library must match the sources too; an MKFHE_LIB variant
    (an A/B build with extra -D switches) must match the ABI and the header."""
    from . import build as _build
    if not os.path.exists(path):
        raise RuntimeError(f"{path} not found: build the HIP engine first (python -m mkfhe_amd.build)")
    # One HIP runtime per process.  torch ships its own libamdhip64 (soname
    # libamdhip64.so.7, but NEEDED as "libamdhip64.so"): loaded first, it also
    # satisfies this library's libamdhip64.so.7 dependency; loaded after
    # /opt/rocm's copy, it becomes a second runtime that sees no GPU ("No HIP
    # GPUs are available") and whose tensors this library could not use.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(path)
    for name in ("mkacc_abi_version", "mkacc_build_info"):
        if not hasattr(L, name):
            raise LibraryMismatch(f"refusing {path}: no {name} (a library older than ABI 2)")
    L.mkacc_abi_version.restype = ctypes.c_int
    L.mkacc_abi_version.argtypes = []
    L.mkacc_build_info.restype = ctypes.c_char_p
    L.mkacc_build_info.argtypes = []
    if require_source is None:
        require_source = os.path.realpath(path) == os.path.realpath(DEFAULT_LIB_PATH)
    L.build_info = verify_build(path, L.mkacc_build_info().decode(), L.mkacc_abi_version(),
                                _build.ENGINE_HEADER, _build.engine_ids(), require_source)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    return L


def load():
    """Load libmkfhe_amd.so (raises if it has not been built, or was built from another tree)."""
    global _lib
    if _lib is None:
        _lib = open_checked(LIB_PATH)
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
