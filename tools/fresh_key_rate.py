#!/usr/bin/env python3
"""Fresh-key (seed-0) decryption-failure rate of the MK NAND gate, measured on
the CPU through the oracle (test infrastructure) -- no GPU involved, so a
failure here is a key/noise property of the scheme, not a device defect.

Each trial replays the reference example's call sequence exactly as the C++
mirror's examples/boolean-mk{ntru,lwe}.cpp make it (boolean-mkntru.cpp:9-48,
boolean-mklwe.cpp:9-42): a fresh entropy master, then
    MNTRU_KeyGen | MKLWE_KeyGen, MKBTKeyGen, [ctGateGen], and for the input
    pairs (0,0) (0,1) (1,0) (1,1): Encrypt(m0), Encrypt(m1),
every seed-0 call keyed by the journal (mkfhe_keys.h), and evaluates the four
NAND gates with the oracle (head, EvalAcc, extraction, ModSwitch, key switch)
and the mirror's Decrypt.  The master key of every trial is printed, so any
set can be replayed: --replay HEX recomputes one example run (e.g. the
"replay: MKFHE_ENTROPY=..." line an example prints when a gate is wrong).

usage: tools/fresh_key_rate.py [--paramset PS] [--sets N] [--out FILE]
       tools/fresh_key_rate.py --replay HEX [--paramset PS]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

N = 2048
PAIRS = [(0, 0), (0, 1), (1, 0), (1, 1)]


def r_defects(oracle, p, bk):
    """Bootstrapping keys whose DggR sample r is nonzero, as [(u, s, i)].

    KeyGenXZW / KDMKeyGenXZW (mk-acc-xzw.cpp:141-167, mk-acc-xzw_B.cpp:135-220)
    put r into f as the polynomial g_t * r but into d only as the scalar
    r^[t] * CRS_t (skrPoly[i], an EVALUATION slot), so the r-terms of a key
    cancel in HbProd only when r = 0.  With sigma_r = 0.15 a coefficient of r
    is nonzero with probability ~4.4e-10, i.e. ~9e-7 per key; such a key adds
    a full-size error to every step that uses it.  Found here from f_0 * s_u =
    e1 + baseG * r: a coefficient of magnitude >= baseG/2 means r != 0."""
    N, Q = p.acc.N, p.acc.Q
    psi = oracle.root_of_unity(2 * N, Q)
    ev = bk.evk
    out = []
    for u in range(ev.shape[0]):
        s_eval = bk.skN_eval[u].astype(np.uint64)
        for s_ in range(ev.shape[1]):
            for i in range(ev.shape[2]):
                f0 = ev[u, s_, i, 0, 1].astype(np.uint64)
                if not f0.any():
                    continue
                x = oracle.ntt_inverse(f0 * s_eval % Q, Q, psi).astype(np.int64)
                x = np.where(x > Q // 2, x - Q, x)
                if int(np.abs(x).max()) >= p.acc.baseG // 2:
                    out.append((u, s_, i))
    return out


def example_run(K, oracle, p, orcs, lwe: bool, threads: int, rdefect: str = "keep"):
    """The example's seed-0 calls in its order; returns the decrypted gates and the key set."""
    sk = K.mklwe_keygen(p, 0) if lwe else K.mntru_keygen(p, 0)
    bk = K.bt_keygen(p, sk, seed=0, rdefect=rdefect)
    ct_nand = None if lwe else K.mntru_ctgate(p, sk, 0)
    cts = []
    for m0, m1 in PAIRS:
        if lwe:
            cts.append((K.mklwe_encrypt(p, sk, m0, 4, 0), K.mklwe_encrypt(p, sk, m1, 4, 0)))
        else:
            cts.append((K.mntru_encrypt(p, sk, m0, 4, 0)[0], K.mntru_encrypt(p, sk, m1, 4, 0)[0]))
    k, n = p.acc.k, p.acc.n
    orc = orcs
    if lwe:
        heads = [orc.mklwe_head(a1[0], b1[0], a2[0], b2[0], p.acc.q) for (a1, b1), (a2, b2) in cts]
        cs = np.stack([h[0] for h in heads])
        acc0 = np.stack([h[1] for h in heads])
    else:
        cs = np.stack([oracle.mntru_head(ct_nand, c1, c2, p.acc.q) for c1, c2 in cts])
        acc0 = np.broadcast_to(orc.mntru_testvector(4), (4, k, N)).copy()
    acc = orc.evalacc_batch(bk.evk, bk.pkey, cs, acc0, threads)
    dec = []
    for i in range(4):
        if lwe:
            oa, ob = orc.mklwe_tail(acc[i], bk.ksk_A.astype(np.uint64), bk.ksk_B.astype(np.uint64), p.ks.qKS,
                                    p.ks.baseKS, n)
            dec.append(int(K.mklwe_decrypt(p, sk, oa.astype(np.uint32)[None], np.array([ob], np.uint32), 4,
                                           K.DECRYPT, p.ks.qKS)[0]))
        else:
            out = orc.mntru_tail_ksk1(acc[i], bk.ksk, p.ks.qKS, p.ks.baseKS, n)
            dec.append(int(K.mntru_decrypt(p, sk, out.astype(np.uint32)[None], 4, K.DECRYPT, p.ks.qKS)[0]))
    return dec, bk


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--paramset", default="STD128_MKNTRU")
    ap.add_argument("--sets", type=int, default=200)
    ap.add_argument("--replay", default=None, help="64 hex digits: recompute one example run")
    ap.add_argument("--threads", type=int, default=min(8, os.cpu_count() or 1))
    ap.add_argument("--out", default=None, help="JSON-lines record, one line per key set")
    ap.add_argument("--scan", default=None, help="JSON-lines record of an earlier run: regenerate each set's "
                    "bootstrapping keys (no gates) and tabulate r-defects against the recorded wrong gates")
    a = ap.parse_args()
    import pyoracle as oracle
    from mkfhe_amd import keys as K
    lwe = "_LWE" in a.paramset
    p = K.paramset(a.paramset, 2 if lwe else 0)
    orc = oracle.Oracle(oracle.XZW_B if lwe else oracle.XZW, p.acc.k, p.acc.n, N, p.acc.Q,
                        2 * N if lwe else p.acc.q, p.acc.baseG)
    want = [1 - (m0 & m1) for m0, m1 in PAIRS]
    if a.replay:
        K.entropy_set(a.replay)
        dec, bk = example_run(K, oracle, p, orc, lwe, a.threads)
        print(f"{a.paramset} MKFHE_ENTROPY={a.replay}: NAND of {PAIRS} -> {dec} (expected {want}): "
              f"{'all correct' if dec == want else 'WRONG'}; keys with r != 0 (u, s, i): {r_defects(oracle, p, bk)}",
              flush=True)
        return 0 if dec == want else 1
    if a.scan:
        tab = {}
        recs = [json.loads(line) for line in open(a.scan)]
        t0 = time.time()
        for j, rec in enumerate(recs):
            K.entropy_set(rec["entropy"])
            sk = K.mklwe_keygen(p, 0) if lwe else K.mntru_keygen(p, 0)
            rdef = r_defects(oracle, p, K.bt_keygen(p, sk, seed=0))
            key = (bool(rdef), rec["wrong"] > 0)
            tab[key] = tab.get(key, 0) + 1
            if rdef or rec["wrong"]:
                print(f"set {rec['set']}: wrong gates {rec['wrong']}, keys with r != 0 (u, s, i) {rdef}", flush=True)
            if j % 100 == 99:
                print(f"[{j + 1} sets, {time.time() - t0:.0f} s]", flush=True)
        print(json.dumps({"paramset": a.paramset, "key_sets": len(recs),
                          "r_defect_and_wrong": tab.get((True, True), 0), "r_defect_all_correct": tab.get((True, False), 0),
                          "no_defect_wrong": tab.get((False, True), 0), "no_defect_all_correct": tab.get((False, False), 0)}),
              flush=True)
        return 0
    fout = open(a.out, "a") if a.out else None
    bad_sets = bad_gates = n_rdef = 0
    t0 = time.time()
    for t in range(a.sets):
        K.entropy_set(None)
        master = K.entropy_get()[0]
        dec, bk = example_run(K, oracle, p, orc, lwe, a.threads)
        rdef = r_defects(oracle, p, bk)
        n_rdef += bool(rdef)
        wrong = sum(int(d != w) for d, w in zip(dec, want))
        bad_sets += wrong > 0
        bad_gates += wrong
        rec = {"paramset": a.paramset, "set": t, "entropy": master, "dec": dec, "wrong": wrong,
               "r_defect_keys": rdef}
        if fout:
            fout.write(json.dumps(rec) + "\n")
            fout.flush()
        if wrong or t % 20 == 19:
            print(f"set {t}: {'WRONG ' + str(dec) + ' MKFHE_ENTROPY=' + master if wrong else 'ok'} "
                  f"{'r!=0 keys ' + str(rdef) if rdef else ''} "
                  f"[{bad_sets} bad sets / {t + 1}, {time.time() - t0:.0f} s]", flush=True)
    print(json.dumps({"paramset": a.paramset, "key_sets": a.sets, "gates": 4 * a.sets, "bad_sets": bad_sets,
                      "bad_gates": bad_gates,
                      "sets_with_r_defect": n_rdef, "seconds": round(time.time() - t0, 1)}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
