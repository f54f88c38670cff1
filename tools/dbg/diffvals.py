"""ph4-style diagnosis: for gates whose 2-WG/CU output differs from the 1-WG/CU
output, locate the wrong words (party, lane, register of the C4 layout) and
search where the wrong values come from (other lanes/registers/gates of the
correct output)."""
import os, sys, collections
import numpy as np
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests")); sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
import pyoracle, mkfhe_amd as mk
from conftest import make_case, Q_MK
B, n = 4096, 2
orc, evk, pkey, ct, acc = make_case(pyoracle, pyoracle.XZW, 2, n, 45181, 1 << 7, B, seed=7)
eng = mk.MKAccumulatorEngine(mk.make_params(mk.MKNTRU, 2, n, 2048, Q_MK, 45181, 1 << 7))
eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
os.environ["MKACC_DBG_LDS"] = "10240"
ref = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
os.environ["MKACC_DBG_LDS"] = "0"
out = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
# the engine returns reference EVAL order; EVAL slot j = (lane << 5) | reg
index = collections.defaultdict(list)
for g in range(B):
    for u in range(2):
        for j, v in enumerate(ref[g, u]):
            index[int(v)].append((g, u, j))
bad = [g for g in range(B) if (out[g] != ref[g]).any()]
print("bad gates", len(bad))
pat = collections.Counter()
for g in bad[:12]:
    for u in range(2):
        js = np.nonzero(out[g, u] != ref[g, u])[0]
        if len(js) == 0:
            continue
        lanes = sorted(set(int(j) >> 5 for j in js)); regs = sorted(set(int(j) & 31 for j in js))
        print(f"gate {g} (wg {g // 4} w{g % 4}) party {u}: {len(js)} words; lanes {lanes[:16]} regs {regs[:16]}")
        for j in js[:4]:
            v = int(out[g, u, j])
            src = index.get(v, [])[:3]
            print(f"    slot (lane {j >> 5}, reg {j & 31}): got {v} want {int(ref[g, u, j])}; value found in the correct output at {src}")
            for s in index.get(v, [])[:1]:
                pat[(s[0] - g, s[1] - u, (s[2] >> 5) - (j >> 5), (s[2] & 31) - (j & 31))] += 1
print("source offsets (dgate, dparty, dlane, dreg):", pat.most_common(10))
