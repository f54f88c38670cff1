#!/usr/bin/env python3
"""Repeated small-batch EvalAcc (the mk_lat_kernel path: one workgroup per gate,
one wave per party) against the CPU oracle (test infrastructure), counting runs
whose output differs.  The engine library is the one MKFHE_LIB names (A/B of a
fix against the build that showed the intermittent wrong accumulators).

usage: tools/lat_stress.py ITERATIONS"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    iters = int(sys.argv[1])
    import pyoracle
    import mkfhe_amd as mk
    from conftest import Q_MK, make_case
    k, n, q, baseG, B = 2, 16, 45181, 1 << 7, 3   # STD128_MKNTRU shape: dg = 3
    orc, evk, pkey, ct, acc = make_case(pyoracle, pyoracle.XZW, k, n, q, baseG, B, seed=7)
    exp = orc.evalacc_batch(evk, pkey, ct, acc, 8).astype(np.uint32)
    eng = mk.MKAccumulatorEngine(mk.make_params(mk.MKNTRU, k, n, 2048, Q_MK, q, baseG))
    eng.upload_keys(evk.astype(np.uint32), pkey.astype(np.uint32))
    ct32, acc32 = ct.astype(np.uint32), acc.astype(np.uint32)
    bad = 0
    for it in range(iters):
        got = eng.eval_batch(ct32, acc32)
        if not np.array_equal(got, exp):
            bad += 1
            wrong = [int(np.any(got[b] != exp[b])) for b in range(B)]
            print(f"iteration {it}: wrong gates {wrong}", flush=True)
        if it % 50 == 49:
            print(f"{it + 1} iterations, {bad} wrong", flush=True)
    print(f"{os.path.basename(os.environ.get('MKFHE_LIB', 'libmkfhe_amd.so'))}: {bad} of {iters} runs "
          f"({iters * k * n} step launches) differ from the oracle", flush=True)


if __name__ == "__main__":
    main()
