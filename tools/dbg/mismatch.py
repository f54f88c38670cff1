import sys, os, numpy as np
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests")); sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
import pyoracle, mkfhe_amd as mk
from conftest import make_case, Q_MK
pyoracle.build()
for (k, n, B, meth) in [(2, 1, 5, 0), (2, 1, 8, 0), (2, 1, 9, 0), (2, 1, 16, 0), (2, 1, 6, 1), (3, 1, 12, 0)]:
    om = pyoracle.XZW if meth == 0 else pyoracle.XZW_B
    q = 45181 if meth == 0 else 32749
    orc, evk, pkey, ct, acc = make_case(pyoracle, om, k, n, q, 1 << 9, B, seed=k * 100 + n)
    exp = orc.evalacc_batch(evk, pkey, ct, acc, 8).astype(np.uint32)
    eng = mk.MKAccumulatorEngine(mk.make_params(mk.MKNTRU if meth == 0 else mk.MKNTRU_LWE, k, n, 2048, Q_MK, q, 1 << 9))
    eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    got = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
    bad = (got != exp)
    print(k, n, B, meth, "bad gates:", [g for g in range(B) if bad[g].any()])
# determinism: same inputs twice
orc, evk, pkey, ct, acc = make_case(pyoracle, pyoracle.XZW, 2, 1, 45181, 1 << 9, 64, seed=5)
eng = mk.MKAccumulatorEngine(mk.make_params(mk.MKNTRU, 2, 1, 2048, Q_MK, 45181, 1 << 9))
eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
r = [eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32)) for _ in range(4)]
exp = orc.evalacc_batch(evk, pkey, ct, acc, 8).astype(np.uint32)
for i in range(4):
    print("run", i, "bad gates vs oracle:", [g for g in range(64) if (r[i][g] != exp[g]).any()])
