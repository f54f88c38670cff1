#!/usr/bin/env python3
"""Fresh-key (seed 0) NAND truth tables on the GPU, as the reference examples run
them: per trial new MNTRU keys, bootstrapping keys and ctNAND, then the four
input pairs as single-gate EvalBinGate calls and as one batch.  Every output is
decrypted; any wrong gate is recomputed by the CPU oracle (test infrastructure)
from the same keys and inputs, which tells a device defect (GPU != oracle) from
a key/noise failure (GPU == oracle, wrong plaintext).

usage: tools/fresh_key_trials.py TRIALS [PARAMSET]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

N = 2048


def main():
    trials = int(sys.argv[1])
    ps = sys.argv[2] if len(sys.argv) > 2 else "STD128_MKNTRU"
    import pyoracle as oracle
    from mkfhe_amd import keys as K
    from mkfhe_amd.binfhe import NAND, BinFHEContext
    m1, m2 = np.array([0, 0, 1, 1]), np.array([0, 1, 0, 1])
    want = 1 - (m1 & m2)
    bad_sets = 0
    for t in range(trials):
        K.entropy_set(None)          # a fresh seed-0 master per trial, printed on failure
        master = K.entropy_get()[0]
        cc = BinFHEContext()
        cc.GenerateBinFHEContext(ps, 0)
        sk = cc.MNTRU_KeyGen()
        cc.MKBTKeyGen(sk)
        cc.ctGateGen(sk, NAND)
        c1, c2 = cc.Encrypt(sk, m1), cc.Encrypt(sk, m2)
        single = np.stack([cc.EvalBinGate(NAND, c1[i], c2[i]) for i in range(4)])
        batch = cc.EvalBinGate(NAND, c1, c2)
        d1, d2 = cc.DecryptGate(sk, single), cc.DecryptGate(sk, batch)
        ok = np.array_equal(d1, want) and np.array_equal(d2, want)
        line = f"trial {t}: single {list(map(int, d1))} batch {list(map(int, d2))} same={np.array_equal(single, batch)}"
        if not ok:
            bad_sets += 1
            line += f" | MKFHE_ENTROPY={master}"
            p, bk = cc.params, cc.BTKey
            k, n = p.acc.k, p.acc.n
            orc = oracle.Oracle(oracle.XZW, k, n, N, p.acc.Q, p.acc.q, p.acc.baseG)
            heads = np.stack([oracle.mntru_head(cc.ctNAND, c1[i], c2[i], p.acc.q) for i in range(4)])
            acc0 = np.broadcast_to(orc.mntru_testvector(4), (4, k, N)).copy()
            acc = orc.evalacc_batch(bk.evk, bk.pkey, heads, acc0, 4)
            exp = np.stack([orc.mntru_tail_ksk1(acc[i], bk.ksk, p.ks.qKS, p.ks.baseKS, n) for i in range(4)])
            line += (f" | oracle dec {list(map(int, cc.DecryptGate(sk, exp.astype(np.uint32))))}"
                     f" gpu==oracle single {np.array_equal(single.astype(np.uint64), exp)}"
                     f" batch {np.array_equal(batch.astype(np.uint64), exp)}")
        print(line, flush=True)
    print(f"{bad_sets} of {trials} key sets with a wrong gate", flush=True)


if __name__ == "__main__":
    main()
