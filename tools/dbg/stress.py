"""Run-to-run determinism stress of the step kernel: B gates, R runs; reports
gates that differ from the oracle (first 256 gates) and from the run majority."""
import sys, os, collections, numpy as np
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests")); sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
import pyoracle, mkfhe_amd as mk
from conftest import make_case, Q_MK
pyoracle.build()
B, R = int(sys.argv[1]) if len(sys.argv) > 1 else 2048, int(sys.argv[2]) if len(sys.argv) > 2 else 6
tot = collections.Counter()
for (k, n, meth, logB) in [(2, 2, 0, 7), (1, 1, 0, 9)]:
    om = pyoracle.XZW if meth == 0 else pyoracle.XZW_B
    q = 45181 if meth == 0 else 32749
    orc, evk, pkey, ct, acc = make_case(pyoracle, om, k, n, q, 1 << logB, B, seed=5)
    eng = mk.MKAccumulatorEngine(mk.make_params(mk.MKNTRU if meth == 0 else mk.MKNTRU_LWE, k, n, 2048, Q_MK, q, 1 << logB))
    eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    exp = orc.evalacc_batch(evk, pkey, ct[:256], acc[:256], 16).astype(np.uint32)
    runs = [eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32)) for _ in range(R)]
    ref = runs[0].copy()
    # majority per gate
    for g in range(B):
        vals = collections.Counter(r[g].tobytes() for r in runs)
        ref[g] = np.frombuffer(vals.most_common(1)[0][0], dtype=np.uint32).reshape(ref[g].shape)
    assert (ref[:256] == exp).all(), "majority differs from oracle"
    for i, r in enumerate(runs):
        bad = [g for g in range(B) if (r[g] != ref[g]).any()]
        for g in bad: tot[g % 8] += 1
        print(f"k={k} n={n} logB={logB} run {i}: {len(bad)} bad gates; wave slots {sorted(set(g % 8 for g in bad))}")
print("bad count by wave slot:", dict(tot))
