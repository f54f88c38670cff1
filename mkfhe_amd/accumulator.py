"""Host-side mirror of the reference accumulator plugin interface.

Reference seam: ``class UniEncAccumulator`` (src/binfhe/include/mk-acc.h:55-80)
with the concrete ``UniEncAccumulatorXZW`` (mk-acc-xzw.cpp:89-130, MKNTRU) and
``UniEncAccumulatorXZW_B`` (mk-acc-xzw_B.cpp:103-132, MKNTRU_B / MKNTRU_LWE),
selected by ``BinFHEScheme(BINFHE_METHOD)`` (binfhe-base-scheme.h:137-151).

Every call goes through the HIP engine's C ABI (include/mkfhe_amd.h); there is
no CPU fallback.  Arrays use the reference's layouts:

* ``ek``   ``[k][nk][n+1][dg][2][N]`` EVAL residues, nk = 2 (XZW) or 1 (XZW_B)
* ``Pkey`` ``[k][dg][N]`` EVAL
* ``acc``  ``[k][N]`` EVAL, updated in place by ``EvalAcc``
* ``ct``   ``[k][n]`` raw ciphertext words (XZW: mod q, XZW_B: mod 2N)
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import MkaccError, MkaccParams, check

MKNTRU = _lib.METHOD_MKNTRU
MKNTRU_B = _lib.METHOD_MKNTRU_B
MKNTRU_LWE = _lib.METHOD_MKNTRU_LWE

_u32p = ctypes.POINTER(ctypes.c_uint32)
_u64p = ctypes.POINTER(ctypes.c_uint64)

PARAMSETS = [
    "STD128_MKNTRU", "STD128_MKNTRU_2", "STD128_MKNTRU_3", "STD128_MKNTRU_4",
    "STD128_MKNTRU_LWE", "STD128_MKNTRU_LWE_2", "STD128_MKNTRU_LWE_3", "STD128_MKNTRU_LWE_4",
    "STD100_MKNTRU", "STD100_MKNTRU_2", "STD100_MKNTRU_3", "STD100_MKNTRU_4",
    "STD100_MKNTRU_LWE", "STD100_MKNTRU_LWE_2", "STD100_MKNTRU_LWE_3", "STD100_MKNTRU_LWE_4",
]


def paramset(name: str, method: int | None = None) -> MkaccParams:
    """UniEnc parameters of a named BINFHE_PARAMSET (binfhecontext.cpp:129-144).

    ``method`` defaults to MKNTRU_LWE for ``*_LWE*`` sets and MKNTRU otherwise,
    matching the example programs (boolean-mkntru.cpp:14, boolean-mklwe.cpp:13).
    """
    if method is None:
        method = MKNTRU_LWE if "_LWE" in name else MKNTRU
    p = MkaccParams()
    check(_lib.load().mkacc_paramset(name.encode(), method, ctypes.byref(p)))
    return p


def make_params(method: int, k: int, n: int, N: int, Q: int, q: int, baseG: int,
                digitsG: int = 0, root: int = 0) -> MkaccParams:
    return MkaccParams(method, k, n, N, Q, q, baseG, digitsG, root)


def _u32(a: np.ndarray):
    return a.ctypes.data_as(_u32p)


def _fingerprint(*arrays) -> int:
    """Cheap content check of key arrays: shape, dtype and ~4096 strided words each."""
    h = 0
    for a in arrays:
        a = np.asarray(a)
        flat = a.reshape(-1)
        step = max(1, flat.size // 4096)
        h = hash((h, a.shape, a.dtype.str, flat[::step].tobytes()))
    return h


class MKAccumulatorEngine:
    """One device context (mkacc_ctx) with its uploaded keys."""

    def __init__(self, params: MkaccParams, device: int = 0):
        L = _lib.load()
        h = ctypes.c_void_p()
        check(L.mkacc_create(ctypes.byref(params), device, ctypes.byref(h)))
        self._h = h
        eff = MkaccParams()
        check(L.mkacc_get_params(h, ctypes.byref(eff)))
        self.params = eff
        self.method, self.k, self.n, self.N = eff.method, eff.k, eff.n, eff.N
        self.Q, self.q, self.baseG, self.digitsG = eff.Q, eff.q, eff.baseG, eff.digitsG
        self.dg = eff.digitsG - 1
        self.nk = 2 if eff.method == MKNTRU else 1
        self.device = device
        self._keys_ref = None   # (evk, pkey, fingerprint) of the arrays on the device
        self.ks = None

    def close(self):
        if getattr(self, "_h", None):
            _lib.load().mkacc_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    @property
    def handle(self):
        return self._h

    @property
    def evk_shape(self):
        return (self.k, self.nk, self.n + 1, self.dg, 2, self.N)

    @property
    def pkey_shape(self):
        return (self.k, self.dg, self.N)

    # -- keys -----------------------------------------------------------------
    def upload_keys(self, evk: np.ndarray, pkey: np.ndarray):
        L = _lib.load()
        if evk.size != int(np.prod(self.evk_shape)) or pkey.size != int(np.prod(self.pkey_shape)):
            raise MkaccError(_lib.MKACC_E_ARG, "key arrays have the wrong size")
        if evk.dtype == np.uint64 or pkey.dtype == np.uint64:
            e = np.ascontiguousarray(evk, dtype=np.uint64)
            p = np.ascontiguousarray(pkey, dtype=np.uint64)
            check(L.mkacc_upload_keys_u64(self._h, e.ctypes.data_as(_u64p), p.ctypes.data_as(_u64p)))
        else:
            e = np.ascontiguousarray(evk, dtype=np.uint32)
            p = np.ascontiguousarray(pkey, dtype=np.uint32)
            check(L.mkacc_upload_keys(self._h, _u32(e), _u32(p)))
        self._keys_ref = (evk, pkey, _fingerprint(evk, pkey))

    def holds_keys(self, evk, pkey) -> bool:
        """True if exactly these arrays (same objects, same sampled content) are on the device."""
        r = self._keys_ref
        return r is not None and r[0] is evk and r[1] is pkey and r[2] == _fingerprint(evk, pkey)

    def upload_keys_device(self, d_evk, d_pkey):
        """Keys from device memory (torch tensors or ints on this context's device) in
        the reference layout; the layout conversion runs on the GPU (no host copy)."""
        def ptr(t):
            return ctypes.c_void_p(t if isinstance(t, int) else t.data_ptr())
        wb = 8 if self.Q >= (1 << 32) else 4
        if not isinstance(d_evk, int):
            wb = d_evk.element_size()
            if d_evk.numel() != int(np.prod(self.evk_shape)) or d_pkey.numel() != int(np.prod(self.pkey_shape)):
                raise MkaccError(_lib.MKACC_E_ARG, "key arrays have the wrong size")
        check(_lib.load().mkacc_upload_keys_device(self._h, ptr(d_evk), ptr(d_pkey), wb))
        self._keys_ref = None

    # -- evaluation -------------------------------------------------------------
    @property
    def wide(self) -> bool:
        """True if the context runs the 64-bit word path (Q >= 2^27)."""
        return bool(_lib.load().mkacc_is_wide(self._h))

    @property
    def wide_fp(self) -> bool:
        """True if the 64-bit word path runs its FP64 kernels (Q < 2^50, mkacc_fp64.hpp / mkacc_widereg2.hpp)."""
        return _lib.load().mkacc_is_wide(self._h) == 2

    def step_kernel_name(self, B: int) -> str:
        """The batch step kernel this context launches for B gates."""
        return _lib.load().mkacc_step_kernel_name(self._h, int(B)).decode()

    def eval_batch(self, ct: np.ndarray, acc: np.ndarray) -> np.ndarray:
        """EvalAcc on B gates: ct [B][k][n], acc [B][k][N] EVAL -> new acc.
        uint64 accumulators (or Q >= 2^32) go through mkacc_eval_batch_u64."""
        ct32 = np.ascontiguousarray(ct, dtype=np.uint32)
        use64 = acc.dtype == np.uint64 or self.Q >= (1 << 32)
        accw = np.ascontiguousarray(acc, dtype=np.uint64 if use64 else np.uint32)
        if ct32.ndim != 3 or ct32.shape[1:] != (self.k, self.n):
            raise MkaccError(_lib.MKACC_E_ARG, f"ct must be [B][{self.k}][{self.n}]")
        B = ct32.shape[0]
        if accw.shape != (B, self.k, self.N):
            raise MkaccError(_lib.MKACC_E_ARG, f"acc must be [B][{self.k}][{self.N}]")
        out = np.empty_like(accw)
        if use64:
            check(_lib.load().mkacc_eval_batch_u64(self._h, _u32(ct32), accw.ctypes.data_as(_u64p),
                                                   out.ctypes.data_as(_u64p), B))
        else:
            check(_lib.load().mkacc_eval_batch(self._h, _u32(ct32), _u32(accw), _u32(out), B))
        return out

    def eval_batch_device(self, d_ct, d_acc_in, d_acc_out, B: int):
        """Device-pointer batch (torch tensors or raw ints); asynchronous on the context stream."""
        def ptr(t):
            return ctypes.c_void_p(t if isinstance(t, int) else t.data_ptr())
        check(_lib.load().mkacc_eval_batch_device(self._h, ptr(d_ct), ptr(d_acc_in), ptr(d_acc_out), B))

    def sync(self):
        check(_lib.load().mkacc_sync(self._h))

    def stream_handle(self) -> int:
        return _lib.load().mkacc_stream(self._h) or 0

    # -- gate level (head + EvalAcc + tail) ----------------------------------------
    def upload_ksk_mntru(self, ksk: np.ndarray, qKS: int, baseKS: int, n_out: int):
        """KeySwitch2 key: ksk [k][N*dks][n_out] = KSK2[u][1] (mntru-pke.cpp:744-755)."""
        ks = _lib.MkaccKsParams(qKS, baseKS, n_out)
        a = np.ascontiguousarray(ksk, dtype=np.uint32)
        check(_lib.load().mkacc_upload_ksk_mntru(self._h, ctypes.byref(ks), _u32(a)))
        self.ks = ks

    def upload_ksk_mklwe(self, A: np.ndarray, B: np.ndarray, qKS: int, baseKS: int, n_out: int):
        """MK-LWE KeySwitch key: A [k][N][Bks][dks][n_out], B [k][N][Bks][dks] (mklwe-pke.cpp:176-258)."""
        ks = _lib.MkaccKsParams(qKS, baseKS, n_out)
        a = np.ascontiguousarray(A, dtype=np.uint32)
        b = np.ascontiguousarray(B, dtype=np.uint32)
        check(_lib.load().mkacc_upload_ksk_mklwe(self._h, ctypes.byref(ks), _u32(a), _u32(b)))
        self.ks = ks

    def upload_ksk_device(self, qKS: int, baseKS: int, n_out: int, d_ksk=None, d_A=None, d_B=None):
        """Key-switching keys from device memory (torch tensors or ints on this
        context's device, u32 words in the host layouts); converted on the GPU."""
        def ptr(t):
            return ctypes.c_void_p(t if isinstance(t, int) else t.data_ptr())
        ks = _lib.MkaccKsParams(qKS, baseKS, n_out)
        if self.method == MKNTRU:
            check(_lib.load().mkacc_upload_ksk_mntru_device(self._h, ctypes.byref(ks), ptr(d_ksk)))
        else:
            check(_lib.load().mkacc_upload_ksk_mklwe_device(self._h, ctypes.byref(ks), ptr(d_A), ptr(d_B)))
        self.ks = ks

    def _need_ksk(self):
        if self.ks is None:
            raise MkaccError(_lib.MKACC_E_NOKEYS, "Key-switching keys have not been uploaded")

    def eval_nand_mntru(self, ct_nand: np.ndarray, ct1: np.ndarray, ct2: np.ndarray) -> np.ndarray:
        """B MK-NTRU NAND gates (EvalBinGate, binfhe-base-scheme.cpp:467-515) -> [B][k][n_out]."""
        self._need_ksk()
        c1 = np.ascontiguousarray(ct1, dtype=np.uint32)
        c2 = np.ascontiguousarray(ct2, dtype=np.uint32)
        cn = np.ascontiguousarray(ct_nand, dtype=np.uint32)
        B = c1.shape[0]
        out = np.empty((B, self.k, self.ks.n_out), dtype=np.uint32)
        check(_lib.load().mkacc_eval_nand_mntru(self._h, _u32(cn), _u32(c1), _u32(c2), _u32(out), B))
        return out

    def eval_nand_mklwe(self, a1, b1, a2, b2):
        """B MK-LWE NAND gates (binfhe-base-scheme.cpp:380-463) -> (a [B][k][n_out], b [B])."""
        self._need_ksk()
        a1 = np.ascontiguousarray(a1, dtype=np.uint32)
        a2 = np.ascontiguousarray(a2, dtype=np.uint32)
        b1 = np.ascontiguousarray(b1, dtype=np.uint32)
        b2 = np.ascontiguousarray(b2, dtype=np.uint32)
        B = a1.shape[0]
        oa = np.empty((B, self.k, self.ks.n_out), dtype=np.uint32)
        ob = np.empty(B, dtype=np.uint32)
        check(_lib.load().mkacc_eval_nand_mklwe(self._h, _u32(a1), _u32(b1), _u32(a2), _u32(b2), _u32(oa),
                                                _u32(ob), B))
        return oa, ob

    def eval_nand_device(self, d_nand, d_a1, d_b1, d_a2, d_b2, d_out_a, d_out_b, B: int):
        """Device-pointer gates (torch tensors or ints; None for unused); asynchronous."""
        def ptr(t):
            if t is None:
                return ctypes.c_void_p(0)
            return ctypes.c_void_p(t if isinstance(t, int) else t.data_ptr())
        check(_lib.load().mkacc_eval_nand_device(self._h, ptr(d_nand), ptr(d_a1), ptr(d_b1), ptr(d_a2), ptr(d_b2),
                                                 ptr(d_out_a), ptr(d_out_b), B))

    def gate_tail(self, acc: np.ndarray):
        """Extraction + ModSwitch + key switch of B accumulators [B][k][N] (EVAL)."""
        self._need_ksk()
        a = np.ascontiguousarray(acc, dtype=np.uint32)
        B = a.shape[0]
        oa = np.empty((B, self.k, self.ks.n_out), dtype=np.uint32)
        ob = np.empty(B, dtype=np.uint32)
        check(_lib.load().mkacc_gate_tail(self._h, _u32(a), _u32(oa), _u32(ob), B))
        return oa if self.method == MKNTRU else (oa, ob)

    # -- primitives -------------------------------------------------------------
    def _prim(self, name: str, a: np.ndarray, out_mul: int):
        L = _lib.load()
        if a.dtype == np.uint64 or self.wide:   # 64-bit word entry points
            x = np.ascontiguousarray(a, dtype=np.uint64).reshape(-1, self.N)
            out = np.empty((x.shape[0] * out_mul, self.N), dtype=np.uint64)
            check(getattr(L, name + "_u64")(self._h, x.ctypes.data_as(_u64p), out.ctypes.data_as(_u64p), x.shape[0]))
            return out
        x = np.ascontiguousarray(a, dtype=np.uint32).reshape(-1, self.N)
        out = np.empty((x.shape[0] * out_mul, self.N), dtype=np.uint32)
        check(getattr(L, name)(self._h, _u32(x), _u32(out), x.shape[0]))
        return out

    def ntt_forward(self, a: np.ndarray) -> np.ndarray:
        """NativePoly::SetFormat(EVALUATION) on rows of a."""
        return self._prim("mkacc_ntt_forward", a, 1)

    def ntt_inverse(self, a: np.ndarray) -> np.ndarray:
        """NativePoly::SetFormat(COEFFICIENT) on rows of a."""
        return self._prim("mkacc_ntt_inverse", a, 1)

    def sdd(self, a: np.ndarray) -> np.ndarray:
        """SignedDigitDecompose (mk-acc.cpp:54-80): rows -> [rows][dg][N]."""
        out = self._prim("mkacc_sdd", a, self.dg)
        return out.reshape(-1, self.dg, self.N)


def shard_range_c(B: int, parts: int, i: int) -> tuple[int, int]:
    """mkacc_shard_range: the group's split of B gates (same as shard.shard_range)."""
    b, e = ctypes.c_size_t(), ctypes.c_size_t()
    _lib.load().mkacc_shard_range(B, parts, i, ctypes.byref(b), ctypes.byref(e))
    return b.value, e.value


class MKAccumulatorGroup:
    """A multi-device group (mkacc_group): one context per entry of `devices` (a
    device may repeat), keys converted once and copied device to device, batches
    split into contiguous shards that run concurrently.  Same batch interface as
    MKAccumulatorEngine; outputs are bit-identical to one context's."""

    def __init__(self, params: MkaccParams, devices):
        L = _lib.load()
        devs = (ctypes.c_int * len(devices))(*devices)
        h = ctypes.c_void_p()
        check(L.mkacc_group_create(ctypes.byref(params), devs, len(devices), ctypes.byref(h)))
        self._h = h
        self.devices = list(devices)
        eff = MkaccParams()
        check(L.mkacc_get_params(L.mkacc_group_member(h, 0), ctypes.byref(eff)))
        self.params = eff
        self.method, self.k, self.n, self.N = eff.method, eff.k, eff.n, eff.N
        self.Q, self.q, self.baseG, self.digitsG = eff.Q, eff.q, eff.baseG, eff.digitsG
        self.dg = eff.digitsG - 1
        self.nk = 2 if eff.method == MKNTRU else 1
        self.ks = None

    def close(self):
        if getattr(self, "_h", None):
            _lib.load().mkacc_group_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()

    @property
    def size(self) -> int:
        return int(_lib.load().mkacc_group_size(self._h))

    def upload_keys(self, evk: np.ndarray, pkey: np.ndarray):
        L = _lib.load()
        if evk.dtype == np.uint64 or pkey.dtype == np.uint64:
            e = np.ascontiguousarray(evk, dtype=np.uint64)
            p = np.ascontiguousarray(pkey, dtype=np.uint64)
            check(L.mkacc_group_upload_keys_u64(self._h, e.ctypes.data_as(_u64p), p.ctypes.data_as(_u64p)))
        else:
            e = np.ascontiguousarray(evk, dtype=np.uint32)
            p = np.ascontiguousarray(pkey, dtype=np.uint32)
            check(L.mkacc_group_upload_keys(self._h, _u32(e), _u32(p)))

    def eval_batch(self, ct: np.ndarray, acc: np.ndarray) -> np.ndarray:
        ct32 = np.ascontiguousarray(ct, dtype=np.uint32)
        use64 = acc.dtype == np.uint64 or self.Q >= (1 << 32)
        accw = np.ascontiguousarray(acc, dtype=np.uint64 if use64 else np.uint32)
        B = ct32.shape[0]
        if ct32.shape != (B, self.k, self.n) or accw.shape != (B, self.k, self.N):
            raise MkaccError(_lib.MKACC_E_ARG, "ct must be [B][k][n] and acc [B][k][N]")
        out = np.empty_like(accw)
        if use64:
            check(_lib.load().mkacc_group_eval_batch_u64(self._h, _u32(ct32), accw.ctypes.data_as(_u64p),
                                                         out.ctypes.data_as(_u64p), B))
        else:
            check(_lib.load().mkacc_group_eval_batch(self._h, _u32(ct32), _u32(accw), _u32(out), B))
        return out

    def upload_ksk_mntru(self, ksk: np.ndarray, qKS: int, baseKS: int, n_out: int):
        ks = _lib.MkaccKsParams(qKS, baseKS, n_out)
        check(_lib.load().mkacc_group_upload_ksk_mntru(self._h, ctypes.byref(ks),
                                                       _u32(np.ascontiguousarray(ksk, dtype=np.uint32))))
        self.ks = ks

    def upload_ksk_mklwe(self, A: np.ndarray, B: np.ndarray, qKS: int, baseKS: int, n_out: int):
        ks = _lib.MkaccKsParams(qKS, baseKS, n_out)
        check(_lib.load().mkacc_group_upload_ksk_mklwe(self._h, ctypes.byref(ks),
                                                       _u32(np.ascontiguousarray(A, dtype=np.uint32)),
                                                       _u32(np.ascontiguousarray(B, dtype=np.uint32))))
        self.ks = ks

    def eval_nand_mntru(self, ct_nand, ct1, ct2) -> np.ndarray:
        if self.ks is None:
            raise MkaccError(_lib.MKACC_E_NOKEYS, "Key-switching keys have not been uploaded")
        c1 = np.ascontiguousarray(ct1, dtype=np.uint32)
        c2 = np.ascontiguousarray(ct2, dtype=np.uint32)
        cn = np.ascontiguousarray(ct_nand, dtype=np.uint32)
        B = c1.shape[0]
        out = np.empty((B, self.k, self.ks.n_out), dtype=np.uint32)
        check(_lib.load().mkacc_group_eval_nand_mntru(self._h, _u32(cn), _u32(c1), _u32(c2), _u32(out), B))
        return out

    def eval_nand_mklwe(self, a1, b1, a2, b2):
        if self.ks is None:
            raise MkaccError(_lib.MKACC_E_NOKEYS, "Key-switching keys have not been uploaded")
        a1, a2 = np.ascontiguousarray(a1, dtype=np.uint32), np.ascontiguousarray(a2, dtype=np.uint32)
        b1, b2 = np.ascontiguousarray(b1, dtype=np.uint32), np.ascontiguousarray(b2, dtype=np.uint32)
        B = a1.shape[0]
        oa = np.empty((B, self.k, self.ks.n_out), dtype=np.uint32)
        ob = np.empty(B, dtype=np.uint32)
        check(_lib.load().mkacc_group_eval_nand_mklwe(self._h, _u32(a1), _u32(b1), _u32(a2), _u32(b2), _u32(oa),
                                                      _u32(ob), B))
        return oa, ob


class UniEncAccumulator:
    """Mirror of the reference's abstract accumulator (mk-acc.h:55-80)."""

    method: int = -1

    def __init__(self, params: MkaccParams, device: int = 0):
        if params.method not in self._methods:
            raise MkaccError(_lib.MKACC_E_ARG, "method is invalid for this accumulator")
        self.engine = MKAccumulatorEngine(params, device)

    def _ensure_keys(self, ek, Pkey):
        # the engine keeps references to the uploaded arrays, so an identity hit
        # cannot be a recycled id(); the sampled fingerprint catches in-place edits
        if not self.engine.holds_keys(ek, Pkey):
            self.engine.upload_keys(np.asarray(ek), np.asarray(Pkey))
            self.engine._keys_ref = (ek, Pkey, _fingerprint(ek, Pkey))

    def EvalAcc(self, ek, Pkey, skf, acc: np.ndarray, ct) -> None:
        """EvalAcc(params, ek, Pkey, skf, acc, ct): acc [k][N] EVAL updated in place.

        ``skf`` is accepted for signature parity and ignored, as in the reference
        (it is only read by commented-out debug code, mk-acc-xzw.cpp:115-120).
        """
        if ek is None:
            raise MkaccError(_lib.MKACC_E_NOKEYS, "Bootstrapping keys have not been generated. "
                                                  "Please call MKBTKeyGen before calling bootstrapping.")
        self._ensure_keys(ek, Pkey)
        out = self.engine.eval_batch(np.asarray(ct)[None], np.asarray(acc)[None])
        acc[...] = out[0]

    def EvalAccBatch(self, ek, Pkey, acc: np.ndarray, ct: np.ndarray) -> np.ndarray:
        """Batch extension: B independent gates, acc [B][k][N], ct [B][k][n]."""
        self._ensure_keys(ek, Pkey)
        return self.engine.eval_batch(ct, acc)


class UniEncAccumulatorXZW(UniEncAccumulator):
    """MKNTRU accumulator, ternary secret (mk-acc-xzw.cpp)."""

    _methods = (MKNTRU,)


class UniEncAccumulatorXZW_B(UniEncAccumulator):
    """MKNTRU_B / MKNTRU_LWE accumulator, binary secret (mk-acc-xzw_B.cpp)."""

    _methods = (MKNTRU_B, MKNTRU_LWE)


def accumulator_for(params: MkaccParams, device: int = 0) -> UniEncAccumulator:
    """BinFHEScheme(BINFHE_METHOD) accumulator choice (binfhe-base-scheme.h:137-151)."""
    if params.method == MKNTRU:
        return UniEncAccumulatorXZW(params, device)
    if params.method in (MKNTRU_B, MKNTRU_LWE):
        return UniEncAccumulatorXZW_B(params, device)
    raise MkaccError(_lib.MKACC_E_ARG, "method is invalid")
