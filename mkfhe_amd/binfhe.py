"""Python mirror of the reference's multi-key BinFHEContext
(src/binfhe/include/binfhecontext.h:98-338, binfhecontext.cpp:235-577) for the
boolean-mkntru / boolean-mklwe examples:

    cc = BinFHEContext()
    cc.GenerateBinFHEContext("STD128_MKNTRU", MKNTRU)
    sk = cc.MNTRU_KeyGen()
    cc.MKBTKeyGen(sk)
    cc.ctGateGen(sk, NAND)
    ct1, ct2 = cc.Encrypt(sk, 1), cc.Encrypt(sk, 0)
    ct = cc.EvalBinGate(NAND, ct1, ct2)          # HIP engine (one MI355X)
    assert cc.Decrypt(sk, ct) == 1

Key generation, encryption and decryption run on the host
(libmkfhe_keys.so); EvalBinGate runs on the GPU through the C ABI
(libmkfhe_amd.so), created on first use.  Ciphertexts are numpy arrays:
MK-NTRU ``[k][n]`` (or ``[B][k][n]`` for a batch), MK-LWE ``(a [k][n], b)``
(or ``(a [B][k][n], b [B])``).
"""
from __future__ import annotations

import numpy as np

from . import keys as K
from .accumulator import MKNTRU, MKNTRU_B, MKNTRU_LWE, MKAccumulatorEngine, MKAccumulatorGroup

NAND = 3  # BINGATE value (binfhe-constants.h)


class ConfigError(ValueError):
    """OPENFHE_THROW(config_error, ...)."""


class BinFHEContext:
    def __init__(self):
        self.kp = None
        self.method = None
        self.device = 0
        self._eng = None
        self._seed = 0
        self._calls = 0
        self.BTKey = None
        self.ctNAND = None

    # ---- context ------------------------------------------------------------------
    def GenerateBinFHEContext(self, paramset: str, method: int = MKNTRU, device=0):
        """device: one HIP device, or a list of devices -- batches of gates then shard
        across them (mkacc_group; keys converted once and copied device to device)."""
        if method not in (MKNTRU, MKNTRU_B, MKNTRU_LWE):
            raise ConfigError("method is invalid")
        self.kp = K.paramset(paramset, method)
        self.method = method
        self.device = device
        self._eng = None
        self.BTKey = None
        self.ctNAND = None

    def SetSeed(self, seed: int):
        """Extension: deterministic sampling (0 = random, the reference's behaviour)."""
        self._seed = seed
        self._calls = 0

    def _next(self) -> int:
        if not self._seed:
            return 0
        self._calls += 1
        return (self._seed + self._calls * 0x9E3779B97F4A7C15) & ((1 << 64) - 1) or 1

    def engine(self):
        if self._eng is None:
            if isinstance(self.device, (list, tuple)):
                self._eng = MKAccumulatorGroup(self.kp.acc, list(self.device))
            else:
                self._eng = MKAccumulatorEngine(self.kp.acc, self.device)
        return self._eng

    @property
    def params(self):
        return self.kp

    # ---- keys ---------------------------------------------------------------------
    def MNTRU_KeyGen(self) -> K.MNTRUPrivateKey:
        return K.mntru_keygen(self.kp, self._next())

    def MKLWE_KeyGen(self) -> K.MKLWEPrivateKey:
        if self.kp.lwe_keydist != K.DIST_BINARY:
            raise ConfigError("Support BINARY PrivateKey Only")
        return K.mklwe_keygen(self.kp, self._next())

    def MKBTKeyGen(self, sk, rdefect: str = "keep"):
        """MKKeyGen (binfhe-base-scheme.cpp:198-338) + upload to the engine.

        rdefect (extension): "keep" (the reference's keys; GetRDefects() counts keys
        whose DggR sample r is nonzero), "reject" (keys.KeyDefectError) or
        "resample" -- the reference's KeyGenXZW defect, include/mkfhe_keys.h."""
        is_lwe = isinstance(sk, K.MKLWEPrivateKey)
        if is_lwe != (self.method == MKNTRU_LWE):
            raise ConfigError("secret key type does not match the context method")
        seed = self._next()
        self.rdefects = 0
        try:
            bk = K.bt_keygen(self.kp, sk, seed=seed, crs_seed=(seed ^ 0xC25) if seed else None, rdefect=rdefect)
        except K.KeyDefectError as e:
            self.rdefects = e.rdefects   # GetRDefects() reports the rejected draw's count
            raise
        self.rdefects = bk.rdefects
        self._upload(bk)

    def GetRDefects(self) -> int:
        """Bootstrapping keys of the last MKBTKeyGen that drew DggR r != 0 (gates may decrypt wrong)."""
        return getattr(self, "rdefects", 0)

    def _upload(self, bk: K.UniEncBTKey):
        eng = self.engine()
        eng.upload_keys(bk.evk, bk.pkey)
        ks = self.kp.ks
        if self.method == MKNTRU_LWE:
            eng.upload_ksk_mklwe(bk.ksk_A, bk.ksk_B, ks.qKS, ks.baseKS, ks.n_out)
        else:
            eng.upload_ksk_mntru(bk.ksk, ks.qKS, ks.baseKS, ks.n_out)
        self.BTKey = bk

    # ---- key files (mkfhe_keys.h wire format) ---------------------------------------------
    def SaveBTKey(self, path: str):
        if self.BTKey is None:
            raise ConfigError("no bootstrapping key generated")
        K.save_btkey(path, self.kp, self.BTKey)

    def LoadBTKey(self, path: str):
        p, bk = K.load_btkey(path)
        a, b = p.acc, self.kp.acc
        if (a.method, a.k, a.n, a.Q, a.baseG, p.ks.qKS) != (b.method, b.k, b.n, b.Q, b.baseG, self.kp.ks.qKS):
            raise ConfigError(f"{path} was generated for a different context")
        self._upload(bk)

    def ctGateGen(self, sk: K.MNTRUPrivateKey, gate: int = NAND):
        if gate != NAND:
            raise ConfigError("Support NAND gate Only")
        self.ctNAND = K.mntru_ctgate(self.kp, sk, self._next())

    # ---- encryption ------------------------------------------------------------------
    def Encrypt(self, sk, m, p: int = 4):
        """One plaintext -> one ciphertext; an array of plaintexts -> a batch."""
        batch = np.ndim(m) > 0
        if isinstance(sk, K.MKLWEPrivateKey):
            a, b = K.mklwe_encrypt(self.kp, sk, m, p, self._next())
            return (a, b) if batch else (a[0], b[0])
        ct = K.mntru_encrypt(self.kp, sk, m, p, self._next())
        return ct if batch else ct[0]

    def Decrypt(self, sk, ct, p: int = 4, mod: int = 0):
        if isinstance(sk, K.MKLWEPrivateKey):
            a, b = ct
            r = K.mklwe_decrypt(self.kp, sk, a, b, p, K.DECRYPT, mod)
            return r if np.ndim(b) > 0 else int(r[0])
        r = K.mntru_decrypt(self.kp, sk, ct, p, K.DECRYPT, mod)
        return r if np.ndim(ct) == 3 else int(r[0])

    # ---- gates ---------------------------------------------------------------------------
    def EvalBinGate(self, gate: int, ct1, ct2):
        """NAND of one pair or of a batch (same shapes), on the GPU.  Outputs are mod qKS."""
        if gate != NAND:
            raise NotImplementedError("only NAND is supported (ctGateGen, binfhe-base-scheme.cpp:341-342)")
        if ct1 is ct2:
            raise ConfigError("Input ciphertexts should be independant")
        if self.method == MKNTRU_B:
            # the reference hands mod-q MNTRU words to XZW_B as monomial exponents
            # (binfhecontext.cpp:174, binfhe-base-scheme.cpp:1127, mk-acc-xzw_B.cpp:120,290):
            # an out-of-range GetMonomial, i.e. undefined behaviour -- rejected here
            raise ConfigError("MKNTRU_B NAND gates are undefined in the reference; use MKNTRU or MKNTRU_LWE")
        if self.BTKey is None:
            raise ConfigError("Bootstrapping keys have not been generated. Please call MKBTKeyGen before calling "
                              "bootstrapping.")
        eng = self.engine()
        if self.method == MKNTRU_LWE:
            (a1, b1), (a2, b2) = ct1, ct2
            single = np.ndim(b1) == 0
            k, n = self.kp.acc.k, self.kp.acc.n
            oa, ob = eng.eval_nand_mklwe(np.reshape(a1, (-1, k, n)), np.atleast_1d(b1),
                                         np.reshape(a2, (-1, k, n)), np.atleast_1d(b2))
            return (oa[0], ob[0]) if single else (oa, ob)
        if self.ctNAND is None:
            raise ConfigError("ctNAND has not been generated (ctGateGen)")
        single = np.ndim(ct1) == 2
        k, n = self.kp.acc.k, self.kp.acc.n
        out = eng.eval_nand_mntru(self.ctNAND, np.reshape(ct1, (-1, k, n)), np.reshape(ct2, (-1, k, n)))
        return out[0] if single else out

    def DecryptGate(self, sk, ct, p: int = 4):
        """Decrypt a gate output (modulus qKS)."""
        return self.Decrypt(sk, ct, p, mod=self.kp.ks.qKS)
