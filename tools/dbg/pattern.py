import sys, os, ctypes, numpy as np
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests")); sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
import pyoracle, mkfhe_amd as mk
from conftest import make_case, Q_MK
B = 512
for (k, n, logB) in [(1, 1, 7), (2, 1, 7)]:
    orc, evk, pkey, ct, acc = make_case(pyoracle, pyoracle.XZW, k, n, 45181, 1 << logB, B, seed=5)
    eng = mk.MKAccumulatorEngine(mk.make_params(mk.MKNTRU, k, n, 2048, Q_MK, 45181, 1 << logB))
    eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    exp = orc.evalacc_batch(evk, pkey, ct, acc, 16).astype(np.uint32)
    for run in range(4):
        r = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
        bad = [g for g in range(B) if (r[g] != exp[g]).any()]
        desc = []
        for g in bad[:6]:
            d = (r[g] != exp[g])
            desc.append((g, [int(d[u].sum()) for u in range(k)]))
        print(f"k={k} run {run}: {len(bad)} bad; (gate, bad coeffs per party): {desc}")
