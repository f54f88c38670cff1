import sys, os, ctypes, numpy as np
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests")); sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
import pyoracle, mkfhe_amd as mk
from mkfhe_amd import _lib
from conftest import make_case, Q_MK
L = _lib.load()
B = 128
orc, evk, pkey, ct, acc = make_case(pyoracle, pyoracle.XZW, 2, 2, 45181, 1 << 7, B, seed=5)
eng = mk.MKAccumulatorEngine(mk.make_params(mk.MKNTRU, 2, 2, 2048, Q_MK, 45181, 1 << 7))
eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
exp = orc.evalacc_batch(evk, pkey, ct, acc, 16).astype(np.uint32)
buf = (ctypes.c_uint * 64)()
L.mkacc_debug_counters(buf)
for run in range(8):
    r = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
    L.mkacc_debug_counters(buf)
    bad = [g for g in range(B) if (r[g] != exp[g]).any()]
    print("run", run, "bad gates", bad, "image mismatches start/end per wave:", list(buf[0:8]), list(buf[8:16]))
