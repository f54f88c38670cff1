import sys, os, numpy as np
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests")); sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
import pyoracle, mkfhe_amd as mk
from conftest import make_case, Q_MK
pyoracle.build()
B = 128
for (k, n, meth, logB) in [(1, 1, 0, 9), (2, 1, 0, 9), (1, 2, 0, 9), (1, 2, 1, 9), (1, 2, 0, 7)]:
    om = pyoracle.XZW if meth == 0 else pyoracle.XZW_B
    q = 45181 if meth == 0 else 32749
    orc, evk, pkey, ct, acc = make_case(pyoracle, om, k, n, q, 1 << logB, B, seed=5)
    eng = mk.MKAccumulatorEngine(mk.make_params(mk.MKNTRU if meth == 0 else mk.MKNTRU_LWE, k, n, 2048, Q_MK, q, 1 << logB))
    eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    exp = orc.evalacc_batch(evk, pkey, ct, acc, 8).astype(np.uint32)
    bads = []
    for _ in range(3):
        r = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
        bads.append([g for g in range(B) if (r[g] != exp[g]).any()])
    print(f"k={k} n={n} meth={meth} logB={logB}: bad gates per run {bads}")
