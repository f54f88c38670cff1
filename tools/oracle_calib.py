#!/usr/bin/env python3
"""Single-thread EvalAcc time of the CPU oracle (test infrastructure) against
the reference's own EvalAcc probe (SURVEY.md s6, 1 core of this container type),
for bench.py's cpu_baseline calibration.

Each paramset: real keys from the keys library (seed 1), one NAND input's head
(XZW) or the MK-LWE head (XZW_B) with the test-vector accumulator, evalacc on 1
thread, best of --reps.  Writes JSON {paramset: {oracle_s, reference_s, ratio}}.

usage: tools/oracle_calib.py [--reps 3] [--out profiles/oracle_calibration.json]
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

N = 2048


def time_one(K, oracle, ps: str, reps: int) -> float:
    lwe = "_LWE" in ps
    p = K.paramset(ps, 2 if lwe else 0)
    k, n = p.acc.k, p.acc.n
    orc = oracle.Oracle(oracle.XZW_B if lwe else oracle.XZW, k, n, N, p.acc.Q, 2 * N if lwe else p.acc.q, p.acc.baseG)
    K.entropy_set("11" * 32)
    sk = K.mklwe_keygen(p, 0) if lwe else K.mntru_keygen(p, 0)
    bk = K.bt_keygen(p, sk, seed=0)
    rng = np.random.default_rng(1)
    if lwe:
        ct = rng.integers(0, 2 * N, (1, k, n)).astype(np.uint64)
        acc = rng.integers(0, p.acc.Q, (1, k, N)).astype(np.uint64)
    else:
        ct = rng.integers(0, p.acc.q, (1, k, n)).astype(np.uint64)
        acc = orc.mntru_testvector(4)[None]
    best = float("inf")
    for _ in range(reps):
        t0 = time.perf_counter()
        orc.evalacc_batch(bk.evk, bk.pkey, ct, acc, 1)
        best = min(best, time.perf_counter() - t0)
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--paramsets", default="STD100_MKNTRU,STD128_MKNTRU,STD100_MKNTRU_LWE_2,STD100_MKNTRU_3,STD128_MKNTRU_3")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import pyoracle as oracle
    import bench
    from mkfhe_amd import keys as K
    model = next((l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")),
                 platform.processor() or platform.machine())
    flags = next((l for l in open("/proc/cpuinfo") if l.startswith("flags")), "")
    out = {"host": platform.machine(), "threads": 1,
           "oracle_cpu": model + (" (AVX-512)" if "avx512f" in flags else ""),
           "reference_cpu": "8-vCPU AMD EPYC (SURVEY.md s6: the survey's probe session)",
           "same_machine": False,
           "note": ("the reference cannot be rebuilt here under the rules for an oracle/_ref build (its headers "
                    "need CMake-generated config_core.h and its library its own build system; DESIGN.md s3), so "
                    "the ratio divides times from two different CPUs and is an estimate")}
    for ps in a.paramsets.split(","):
        t = time_one(K, oracle, ps, a.reps)
        ref = bench.REF_CPU_S_PER_EVALACC.get(ps)
        out[ps] = {"oracle_s": round(t, 4), "reference_s": ref, "oracle_over_reference": round(t / ref, 3) if ref else None}
        print(ps, out[ps], flush=True)
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
