"""B = 4096 full-n STD128_MKNTRU EvalAcc against the committed oracle fixture:
counts wrong gates (first / second half of the batch) and run-to-run changes."""
import hashlib, json, os, sys
import numpy as np
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests", "golden"))
import make_golden, mkfhe_amd as mk
g = json.load(open("tests/golden/evalacc_b4096.json"))
orc, evk, pkey, ct, acc = make_golden.big_batch_inputs()
eng = mk.MKAccumulatorEngine(mk.make_params(mk.MKNTRU, 2, 765, 2048, 134176769, 45181, 1 << 7))
eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
runs = [eng.eval_batch(ct.astype(np.uint32), acc.astype(np.uint32)) for _ in range(2)]
for i, r in enumerate(runs):
    bad = [b for b in range(4096) if hashlib.sha256(np.ascontiguousarray(r[b], dtype="<u8").tobytes()).hexdigest()[:16] != g["gate_sha256_16"][b]]
    lo = sum(1 for b in bad if b < 1024); hi = len(bad) - lo
    print(f"{os.path.basename(os.environ.get('MKFHE_LIB', 'default'))} run {i}: {len(bad)} bad (<1024: {lo}, >=1024: {hi}) first {bad[:8]}", flush=True)
print("run-to-run differing gates:", int(sum(1 for b in range(4096) if (runs[0][b] != runs[1][b]).any())))
