"""ctypes binding of the CPU oracle (oracle/mkfhe_oracle.c).

TEST INFRASTRUCTURE ONLY.  Imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py -- never by the mkfhe_amd package.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_DEFAULT_LIB = os.path.join(_HERE, "build", "libmkfhe_oracle.so")
# MKFHE_ORACLE_LIB: another build of the same source (the sanitizer build,
# `make -C oracle asan`, tests/test_sanitize.py); used as is, never rebuilt here
_LIB_PATH = os.environ.get("MKFHE_ORACLE_LIB") or _DEFAULT_LIB

XZW = 0
XZW_B = 1

_u64p = ctypes.POINTER(ctypes.c_uint64)
_u32p = ctypes.POINTER(ctypes.c_uint32)


class OrcParams(ctypes.Structure):
    _fields_ = [
        ("method", ctypes.c_uint32),
        ("k", ctypes.c_uint32),
        ("n", ctypes.c_uint32),
        ("N", ctypes.c_uint32),
        ("Q", ctypes.c_uint64),
        ("q", ctypes.c_uint64),
        ("baseG", ctypes.c_uint32),
        ("digitsG", ctypes.c_uint32),
        ("psi", ctypes.c_uint64),
    ]


def build() -> str:
    """Compile the oracle if needed (plain gcc via oracle/Makefile)."""
    src = os.path.join(_HERE, "mkfhe_oracle.c")

    def stale():
        if _LIB_PATH != _DEFAULT_LIB:
            return False
        return (not os.path.exists(_LIB_PATH)) or os.path.getmtime(_LIB_PATH) < os.path.getmtime(src)

    if stale():
        # the N ranks of a multi-GPU bench may all get here at once: one builds
        import fcntl
        os.makedirs(os.path.dirname(_LIB_PATH), exist_ok=True)
        with open(_LIB_PATH + ".lock", "w") as lk:
            fcntl.flock(lk, fcntl.LOCK_EX)
            if stale():
                subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(_LIB_PATH)
        L.orc_first_prime.restype = ctypes.c_uint64
        L.orc_first_prime.argtypes = [ctypes.c_uint32, ctypes.c_uint64]
        L.orc_next_prime.restype = ctypes.c_uint64
        L.orc_next_prime.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.orc_vec_mod.argtypes = [ctypes.c_int, _u64p, _u64p, _u64p, ctypes.c_size_t, ctypes.c_uint64]
        L.orc_previous_prime.restype = ctypes.c_uint64
        L.orc_previous_prime.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.orc_root_of_unity.restype = ctypes.c_uint64
        L.orc_root_of_unity.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.orc_is_prime.restype = ctypes.c_int
        L.orc_is_prime.argtypes = [ctypes.c_uint64]
        L.orc_modinv.restype = ctypes.c_uint64
        L.orc_modinv.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
        L.orc_digits_g.restype = ctypes.c_uint32
        L.orc_digits_g.argtypes = [ctypes.c_uint64, ctypes.c_uint32]
        L.orc_ntt_forward.argtypes = [_u64p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64]
        L.orc_ntt_inverse.argtypes = [_u64p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64]
        L.orc_transpose_eval.argtypes = [_u64p, _u64p, ctypes.c_uint32]
        L.orc_automorphism_coeff.argtypes = [_u64p, _u64p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32]
        L.orc_sdd.argtypes = [_u64p, _u64p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32]
        L.orc_ctx_create.restype = ctypes.c_void_p
        L.orc_ctx_create.argtypes = [ctypes.POINTER(OrcParams)]
        L.orc_ctx_destroy.argtypes = [ctypes.c_void_p]
        L.orc_evk_words.restype = ctypes.c_size_t
        L.orc_evk_words.argtypes = [ctypes.POINTER(OrcParams)]
        L.orc_evalacc.restype = ctypes.c_int
        L.orc_evalacc.argtypes = [ctypes.c_void_p, _u64p, _u64p, _u64p, _u64p]
        L.orc_evalacc_batch.restype = ctypes.c_int
        L.orc_evalacc_batch.argtypes = [ctypes.c_void_p, _u64p, _u64p, _u64p, _u64p, ctypes.c_size_t, ctypes.c_int]
        L.orc_fill_uniform.argtypes = [_u64p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64]
        L.orc_round_qQ.restype = ctypes.c_uint64
        L.orc_round_qQ.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
        L.orc_ks_digits.restype = ctypes.c_uint32
        L.orc_ks_digits.argtypes = [ctypes.c_uint64, ctypes.c_uint32]
        L.orc_mntru_head.argtypes = [_u64p, _u64p, _u64p, _u64p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]
        L.orc_extract.argtypes = [ctypes.c_void_p, _u64p, _u64p]
        L.orc_keyswitch2.argtypes = [_u64p, _u64p, _u64p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                     ctypes.c_uint64, ctypes.c_uint32]
        L.orc_mntru_tail.argtypes = [ctypes.c_void_p, _u64p, _u64p, ctypes.c_uint64, ctypes.c_uint32,
                                     ctypes.c_uint32, _u64p]
        L.orc_mntru_tail_ksk1.argtypes = [ctypes.c_void_p, _u64p, _u32p, ctypes.c_uint64, ctypes.c_uint32,
                                          ctypes.c_uint32, _u64p]
        L.orc_mklwe_head.argtypes = [ctypes.c_void_p, _u64p, ctypes.c_uint64, _u64p, ctypes.c_uint64,
                                     ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, _u64p, _u64p]
        L.orc_mklwe_keyswitch.argtypes = [_u64p, _u64p, _u64p, ctypes.c_uint64, _u64p, _u64p, ctypes.c_uint32,
                                          ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32]
        L.orc_mklwe_tail.argtypes = [ctypes.c_void_p, _u64p, _u64p, _u64p, ctypes.c_uint64, ctypes.c_uint32,
                                     ctypes.c_uint32, _u64p, _u64p]
        L.orc_fill_uniform_u32.argtypes = [_u32p, ctypes.c_size_t, ctypes.c_uint64, ctypes.c_uint64]
        L.orc_mntru_testvector.argtypes = [ctypes.c_void_p, ctypes.c_uint64, _u64p]
        _lib = L
    return _lib


def _p64(a: np.ndarray):
    assert a.dtype == np.uint64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_u64p)


def first_prime(nbits: int, m: int) -> int:
    return int(lib().orc_first_prime(nbits, m))


def previous_prime(q: int, m: int) -> int:
    return int(lib().orc_previous_prime(q, m))


def next_prime(q: int, m: int) -> int:
    return int(lib().orc_next_prime(q, m))


def vec_mod(op: str, a, b, Q: int) -> np.ndarray:
    """NativeVectorT ModAdd / ModSub / ModMul (op 'add' | 'sub' | 'mul')."""
    x = np.ascontiguousarray(np.asarray(a, dtype=np.uint64))
    y = np.ascontiguousarray(np.asarray(b, dtype=np.uint64))
    out = np.empty_like(x)
    lib().orc_vec_mod({"add": 0, "sub": 1, "mul": 2}[op], _p64(x), _p64(y), _p64(out), x.size, Q)
    return out


def root_of_unity(m: int, Q: int) -> int:
    return int(lib().orc_root_of_unity(m, Q))


def is_prime(n: int) -> bool:
    return bool(lib().orc_is_prime(n))


def digits_g(Q: int, baseG: int) -> int:
    return int(lib().orc_digits_g(Q, baseG))


def ntt_forward(a, Q: int, psi: int) -> np.ndarray:
    x = np.ascontiguousarray(np.asarray(a, dtype=np.uint64)).copy()
    lib().orc_ntt_forward(_p64(x), x.size, Q, psi)
    return x


def ntt_inverse(a, Q: int, psi: int) -> np.ndarray:
    x = np.ascontiguousarray(np.asarray(a, dtype=np.uint64)).copy()
    lib().orc_ntt_inverse(_p64(x), x.size, Q, psi)
    return x


def transpose_eval(a) -> np.ndarray:
    x = np.ascontiguousarray(np.asarray(a, dtype=np.uint64))
    out = np.zeros_like(x)
    lib().orc_transpose_eval(_p64(x), _p64(out), x.size)
    return out


def automorphism_coeff(a, Q: int, k: int) -> np.ndarray:
    x = np.ascontiguousarray(np.asarray(a, dtype=np.uint64))
    out = np.zeros_like(x)
    lib().orc_automorphism_coeff(_p64(x), _p64(out), x.size, Q, k)
    return out


def sdd(a, Q: int, baseG: int, dg: int) -> np.ndarray:
    x = np.ascontiguousarray(np.asarray(a, dtype=np.uint64))
    out = np.zeros((dg, x.size), dtype=np.uint64)
    lib().orc_sdd(_p64(x), _p64(out), x.size, Q, baseG, dg)
    return out


def fill_uniform(n: int, bound: int, seed: int, dtype=np.uint64) -> np.ndarray:
    if dtype == np.uint32:
        out = np.empty(n, dtype=np.uint32)
        lib().orc_fill_uniform_u32(out.ctypes.data_as(_u32p), n, bound, seed)
    else:
        out = np.empty(n, dtype=np.uint64)
        lib().orc_fill_uniform(_p64(out), n, bound, seed)
    return out


class Oracle:
    """EvalAcc restatement for one parameter set (see mkfhe_oracle.h)."""

    def __init__(self, method: int, k: int, n: int, N: int, Q: int, q: int, baseG: int,
                 digitsG: int = 0, psi: int = 0):
        self.params = OrcParams(method, k, n, N, Q, q, baseG, digitsG, psi)
        self._ctx = lib().orc_ctx_create(ctypes.byref(self.params))
        if not self._ctx:
            raise ValueError("bad oracle parameters")
        self.method, self.k, self.n, self.N, self.Q, self.q, self.baseG = method, k, n, N, Q, q, baseG
        self.digitsG = digitsG or digits_g(Q, baseG)
        self.dg = self.digitsG - 1
        self.nk = 2 if method == XZW else 1
        self.psi = psi or root_of_unity(2 * N, Q)

    def __del__(self):
        if getattr(self, "_ctx", None):
            lib().orc_ctx_destroy(self._ctx)
            self._ctx = None

    @property
    def evk_shape(self):
        return (self.k, self.nk, self.n + 1, self.dg, 2, self.N)

    @property
    def pkey_shape(self):
        return (self.k, self.dg, self.N)

    def evalacc(self, evk: np.ndarray, pkey: np.ndarray, ct: np.ndarray, acc: np.ndarray) -> np.ndarray:
        evk = np.ascontiguousarray(evk, dtype=np.uint64)
        pkey = np.ascontiguousarray(pkey, dtype=np.uint64)
        ct = np.ascontiguousarray(ct, dtype=np.uint64)
        out = np.ascontiguousarray(acc, dtype=np.uint64).copy()
        assert evk.size == int(np.prod(self.evk_shape)) and pkey.size == int(np.prod(self.pkey_shape))
        if ct.ndim == 2:
            rc = lib().orc_evalacc(self._ctx, _p64(evk), _p64(pkey), _p64(ct), _p64(out))
        else:
            B = ct.shape[0]
            rc = lib().orc_evalacc_batch(self._ctx, _p64(evk), _p64(pkey), _p64(ct), _p64(out), B,
                                         int(os.environ.get("MKFHE_ORACLE_THREADS", os.cpu_count() or 1)))
        if rc != 0:
            raise ValueError(f"oracle evalacc failed rc={rc}")
        return out

    def evalacc_batch(self, evk, pkey, ct, acc, threads: int) -> np.ndarray:
        out = np.ascontiguousarray(acc, dtype=np.uint64).copy()
        rc = lib().orc_evalacc_batch(self._ctx, _p64(np.ascontiguousarray(evk, dtype=np.uint64)),
                                     _p64(np.ascontiguousarray(pkey, dtype=np.uint64)),
                                     _p64(np.ascontiguousarray(ct, dtype=np.uint64)), _p64(out),
                                     ct.shape[0], threads)
        if rc != 0:
            raise ValueError(f"oracle evalacc failed rc={rc}")
        return out

    def mntru_testvector(self, p: int = 4) -> np.ndarray:
        acc = np.zeros((self.k, self.N), dtype=np.uint64)
        lib().orc_mntru_testvector(self._ctx, p, _p64(acc))
        return acc


# ---- gate head / tail (binfhe-base-scheme.cpp:380-515) ----------------------------

def round_qQ(v: int, q: int, Q: int) -> int:
    return lib().orc_round_qQ(v, q, Q)


def ks_digits(qKS: int, baseKS: int) -> int:
    return lib().orc_ks_digits(qKS, baseKS)


def _u64(a):
    return np.ascontiguousarray(a, dtype=np.uint64)


def mntru_head(ct_nand, ct1, ct2, q: int) -> np.ndarray:
    """ctNAND - (ct1 + ct2) mod q for one gate ([k][n] each)."""
    cn, c1, c2 = _u64(ct_nand), _u64(ct1), _u64(ct2)
    out = np.empty_like(c1)
    k, n = c1.shape
    lib().orc_mntru_head(_p64(cn), _p64(c1), _p64(c2), _p64(out), k, n, q)
    return out


def keyswitch2(ksk2, ct, k: int, N: int, n: int, qKS: int, baseKS: int) -> np.ndarray:
    out = np.empty((k, n), dtype=np.uint64)
    lib().orc_keyswitch2(_p64(_u64(ksk2)), _p64(_u64(ct)), _p64(out), k, N, n, qKS, baseKS)
    return out


def _oracle_methods():
    def extract(self, acc):
        out = np.empty((self.k, self.N), dtype=np.uint64)
        lib().orc_extract(self._ctx, _p64(_u64(acc)), _p64(out))
        return out

    def mntru_tail(self, acc, ksk2, qKS: int, baseKS: int, n_out: int):
        out = np.empty((self.k, n_out), dtype=np.uint64)
        lib().orc_mntru_tail(self._ctx, _p64(_u64(acc)), _p64(_u64(ksk2)), qKS, baseKS, n_out, _p64(out))
        return out

    def mntru_tail_ksk1(self, acc, ksk1, qKS: int, baseKS: int, n_out: int):
        """Tail with the key as KSK2[u][1] ([k][N*dks][n] u32, mkfhe_keys.h layout)."""
        out = np.empty((self.k, n_out), dtype=np.uint64)
        k1 = np.ascontiguousarray(ksk1, dtype=np.uint32)
        lib().orc_mntru_tail_ksk1(self._ctx, _p64(_u64(acc)), k1.ctypes.data_as(_u32p), qKS, baseKS, n_out,
                                  _p64(out))
        return out

    def mklwe_head(self, a1, b1, a2, b2, q: int, p: int = 4):
        a1, a2 = _u64(a1), _u64(a2)
        c = np.empty_like(a1)
        acc = np.empty((self.k, self.N), dtype=np.uint64)
        lib().orc_mklwe_head(self._ctx, _p64(a1), int(b1), _p64(a2), int(b2), q, a1.shape[1], p, _p64(c),
                             _p64(acc))
        return c, acc

    def mklwe_tail(self, acc, A, Bk, qKS: int, baseKS: int, n_out: int):
        oa = np.empty((self.k, n_out), dtype=np.uint64)
        ob = np.zeros(1, dtype=np.uint64)
        lib().orc_mklwe_tail(self._ctx, _p64(_u64(acc)), _p64(_u64(A)), _p64(_u64(Bk)), qKS, baseKS, n_out,
                             _p64(oa), _p64(ob))
        return oa, int(ob[0])

    for f in (extract, mntru_tail, mntru_tail_ksk1, mklwe_head, mklwe_tail):
        setattr(Oracle, f.__name__, f)


_oracle_methods()
