"""The NTT primitive kernels (same LDS image and per-wave scratch as the step
kernel, low VGPR use) on many polynomials: every one against the oracle."""
import os, sys
import numpy as np
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "oracle"))
import pyoracle, mkfhe_amd as mk
Q = 134176769
cnt = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
eng = mk.MKAccumulatorEngine(mk.make_params(mk.MKNTRU, 2, 4, 2048, Q, 45181, 1 << 7))
psi = pyoracle.root_of_unity(4096, Q)
a = pyoracle.fill_uniform(cnt * 2048, Q, 99).reshape(cnt, 2048)
ref = np.stack([pyoracle.ntt_forward(a[i], Q, psi) for i in range(0, cnt, 64)])   # every 64th
for rep in range(3):
    fw = eng.ntt_forward(a.astype(np.uint32))
    bad = [i for i in range(0, cnt, 64) if not np.array_equal(fw[i], ref[i // 64].astype(np.uint32))]
    inv = eng.ntt_inverse(fw)
    badi = [i for i in range(cnt) if not np.array_equal(inv[i], a[i].astype(np.uint32))]
    print(f"rep {rep}: forward bad (sampled) {len(bad)} {bad[:8]}; round-trip bad {len(badi)} {badi[:8]}", flush=True)
