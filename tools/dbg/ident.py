"""B identical gates through a short EvalAcc (k=2, n=N_STEPS): every output must
equal gate 0's; for the gates that differ, print where (party, EVAL slot ->
lane/register of the C4 layout) and by how much."""
import os, sys, collections
import numpy as np
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests")); sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
import pyoracle, mkfhe_amd as mk
from conftest import make_case, Q_MK
B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
n = int(sys.argv[2]) if len(sys.argv) > 2 else 2
R = int(sys.argv[3]) if len(sys.argv) > 3 else 4
orc, evk, pkey, ct, acc = make_case(pyoracle, pyoracle.XZW, 2, n, 45181, 1 << 7, 1, seed=5)
ct = np.broadcast_to(ct, (B,) + ct.shape[1:]).copy(); acc = np.broadcast_to(acc, (B,) + acc.shape[1:]).copy()
exp = orc.evalacc_batch(evk, pkey, ct[:1], acc[:1], 1).astype(np.uint32)[0]
eng = mk.MKAccumulatorEngine(mk.make_params(mk.MKNTRU, 2, n, 2048, Q_MK, 45181, 1 << 7))
eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
tot = collections.Counter()
for rep in range(R):
    out = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
    bad = [b for b in range(B) if (out[b] != exp).any()]
    print(f"rep {rep}: {len(bad)} bad gates: {bad[:20]}", flush=True)
    for b in bad[:6]:
        d = out[b] != exp
        for u in range(2):
            js = np.nonzero(d[u])[0]
            if len(js) == 0: continue
            lanes = sorted(set(int(j) >> 5 for j in js)); regs = sorted(set(int(j) & 31 for j in js))
            print(f"   gate {b} (wg {b // 4} wave {b % 4}) party {u}: {len(js)} slots differ; lanes {lanes[:12]}{'...' if len(lanes) > 12 else ''} regs {regs[:12]}")
    for b in bad: tot[(b // 4 < 256, b % 4)] += 1
print("bad by (first 256 WGs, wave):", dict(tot))
