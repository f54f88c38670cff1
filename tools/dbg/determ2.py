"""Co-residency determinism: the same batch with two workgroups per CU and with
one (extra dynamic LDS, MKACC_DBG_LDS) must give identical outputs; reports the
gates that differ.  No oracle needed, so stubbed diagnostic kernels work too."""
import os, sys
import numpy as np
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests")); sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
import pyoracle, mkfhe_amd as mk
from conftest import make_case, Q_MK
B, n = int(sys.argv[1]) if len(sys.argv) > 1 else 4096, int(sys.argv[2]) if len(sys.argv) > 2 else 2
orc, evk, pkey, ct, acc = make_case(pyoracle, pyoracle.XZW, 2, n, 45181, 1 << 7, B, seed=7)
eng = mk.MKAccumulatorEngine(mk.make_params(mk.MKNTRU, 2, n, 2048, Q_MK, 45181, 1 << 7))
eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
os.environ["MKACC_DBG_LDS"] = "10240"
ref = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
os.environ["MKACC_DBG_LDS"] = "0"
tag = os.path.basename(os.environ.get("MKFHE_LIB", "default"))
for rep in range(3):
    out = eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32))
    bad = [b for b in range(B) if (out[b] != ref[b]).any()]
    print(f"{tag} rep {rep}: {len(bad)} gates differ from the 1-WG/CU run; <1024: {sum(b < 1024 for b in bad)}; {bad[:10]}", flush=True)
