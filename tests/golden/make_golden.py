#!/usr/bin/env python3
"""Generate tests/golden/*.json (committed fixtures; run here, never on the GPU box).

  python tests/golden/make_golden.py [--kats-only | --big-batch [mkntru|mklwe] | --gates-only]

reference_kats.json
    Known-answer vectors held by the reference's own unit tests for the
    primitives on this path, copied as data with their file:line (the
    reference has no MK/accumulator test), plus the MK ring
    constants the reference probe printed.
evalacc_full.json
    Full-size EvalAcc fixtures: for each BASELINE configuration shape, seeded
    synthetic keys / ciphertexts (oracle fill_uniform, SplitMix64) and the
    MNTRU test-vector accumulator, run through the CPU oracle; stored as the
    SHA-256 of the little-endian uint64 output plus sample coefficients.
    The GPU tests regenerate the inputs from the seeds and compare digests.
evalacc_b4096.json (--big-batch mkntru), evalacc_b4096_mklwe.json (--big-batch mklwe)
    The benched shapes: STD128_MKNTRU (headline) and STD100_MKNTRU_LWE_2
    (config 3, MK-LWE k = 4), full n, B = 4096 seeded gates in one batch,
    whole-output SHA-256 and per-gate digests.
gates_realkeys.json (--gates-only regenerates just this file)
    NAND gates with real keys (seeded NTL-free key generation,
    mkfhe_amd/keys.py), evaluated by the oracle: digest of the output
    ciphertexts and their decryptions, at every BASELINE configuration's
    parameter set: STD128_MKNTRU (configs 1/2), STD100_MKNTRU_LWE (the
    boolean-mklwe example), STD100_MKNTRU_LWE_2 (config 3, MK-LWE k = 4) and
    STD128_MKNTRU_3 (config 4, MK-NTRU k = 8).  The seeds draw no
    r-defective key (KEEP policy): asserted here.
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import pyoracle  # noqa: E402

N = 2048
Q_MK = 134176769
Q50 = 1125899906826241

REFERENCE_KATS = {
    "first_prime": [
        {"bits": 30, "m": 2048, "q": 1073750017, "src": "src/core/unittest/UnitTestNbTheory.cpp:170-175"},
        {"bits": 49, "m": 4096, "q": 562949953548289, "src": "src/core/unittest/UnitTestNbTheory.cpp:178-185"},
    ],
    "switch_format_forward": {"q": 73, "root": 22, "in": [2, 1, 3, 2], "out": [69, 65, 44, 49],
                              "src": "src/core/unittest/UnitTestPolyElements.cpp:388-399"},
    "switch_format_inverse": {"q": 73, "root": 22, "in": [2, 3, 1, 2], "out": [2, 3, 50, 3],
                              "src": "src/core/unittest/UnitTestPolyElements.cpp:401-411"},
    "transpose": {"q": 73, "root": 22, "in": [31, 21, 15, 34], "out": [31, 39, 58, 52],
                  "src": "src/core/unittest/UnitTestPolyElements.cpp:540-571"},
    "automorphism": {"q": 73, "k": 3, "in": [56, 1, 37, 2], "out": [56, 2, 36, 1],
                     "src": "src/core/unittest/UnitTestPolyElements.cpp:512-521"},
    "crt_mult": {"q": 113, "m": 8, "a": [1, 2, 4, 1], "out": [94, 109, 11, 18],
                 "src": "src/core/unittest/UnitTestTransform.cpp:58-93"},
    "next_prime": {"bits": 22, "m": 2048,
                   "chain": [4208641, 4263937, 4270081, 4274177, 4294657, 4300801, 4304897, 4319233, 4323329, 4360193],
                   "src": "src/core/unittest/UnitTestNbTheory.cpp:380-397 (test_nextQ: FirstPrime(22, 2048), then NextPrime x10)"},
    "vec_mod_1limb": {
        "q": 163841,
        "a": [127753, 77706, 17133, 22582, 112132, 27625, 126773, 8924,
              125972, 2551, 113837, 112045, 100953, 77352, 132013, 57029],
        "b": [66773, 69572, 142134, 141115, 123182, 155822, 128147, 94818,
              135782, 30844, 88634, 99407, 53647, 111689, 28502, 26401],
        "add": [30685, 147278, 159267, 163697, 71473, 19606, 91079, 103742,
                97913, 33395, 38630, 47611, 154600, 25200, 160515, 83430],
        "sub": [60980, 8134, 38840, 45308, 152791, 35644, 162467, 77947,
                154031, 135548, 25203, 12638, 47306, 129504, 103511, 30628],
        "mul": [69404, 64196, 13039, 115321, 28519, 151998, 89117, 80908,
                57386, 39364, 8355, 146135, 61336, 31598, 25961, 87680],
        "src": "src/core/unittest/UnitTestMubintvec.cpp:276-358 (basic_vector_vector_mod_math_1_limb)"},
    "vec_mod_2limb": {
        "q": 4057816419532801,
        "a": [185225172798255, 98879665709163, 3497410031351258, 4012431933509255,
              1543020758028581, 135094568432141, 3976954337141739, 4030348521557120,
              175940803531155, 435236277692967, 3304652649070144, 2032520019613814,
              375749152798379, 3933203511673255, 2293434116159938, 1201413067178193],
        "b": [698898215124963, 39832572186149, 1835473200214782, 1041547470449968,
              1076152419903743, 433588874877196, 2336100673132075, 2990190360138614,
              754647536064726, 702097990733190, 2102063768035483, 119786389165930,
              3976652902630043, 3238750424196678, 2978742255253796, 2124827461185795],
        "add": [884123387923218, 138712237895312, 1275066812033239, 996162984426422,
                2619173177932324, 568683443309337, 2255238590741013, 2962722462162933,
                930588339595881, 1137334268426157, 1348899997572826, 2152306408779744,
                294585635895621, 3114137516337132, 1214359951880933, 3326240528363988],
        "sub": [3544143377206093, 59047093523014, 1661936831136476, 2970884463059287,
                466868338124838, 3759322113087746, 1640853664009664, 1040158161418506,
                3479109686999230, 3790954706492578, 1202588881034661, 1912733630447884,
                456912669701137, 694453087476577, 3372508280438943, 3134402025525199],
        "mul": [585473140075497, 3637571624495703, 1216097920193708, 1363577444007558,
                694070384788800, 2378590980295187, 903406520872185, 559510929662332,
                322863634303789, 1685429502680940, 1715852907773825, 2521152917532260,
                781959737898673, 2334258943108700, 2573793300043944, 1273980645866111],
        "src": "src/core/unittest/UnitTestMubintvec.cpp:402-484 (basic_vector_vector_mod_math_2_limb)"},
    "mk_ring": {"Q": Q_MK, "psi": 100530, "src": "binfhecontext.cpp:157-158 + reference probe, SURVEY.md s0"},
    "cfg5_ring": {"Q": Q50, "psi": 1080667890455, "src": "reference probe at NATIVE_SIZE=64, SURVEY.md s0 item 2"},
}

# name, method, k, n, q, baseG, Q, B  (the BASELINE.json configuration shapes)
EVALACC_CASES = [
    ("STD100_MKNTRU", pyoracle.XZW, 2, 560, 45181, 1 << 9, Q_MK, 2),
    ("STD128_MKNTRU", pyoracle.XZW, 2, 765, 45181, 1 << 7, Q_MK, 2),
    ("STD100_MKNTRU_LWE", pyoracle.XZW_B, 2, 500, 32749, 1 << 9, Q_MK, 2),
    ("STD100_MKNTRU_LWE_2", pyoracle.XZW_B, 4, 500, 32749, 1 << 9, Q_MK, 2),
    ("STD128_MKNTRU_3", pyoracle.XZW, 8, 765, 45181, 1 << 6, Q_MK, 1),
    ("CFG5_Q50_STD100_SHAPE", pyoracle.XZW, 2, 560, 45181, 1 << 10, Q50, 2),
    # the reference's k = 16 rows (binfhecontext.cpp:129-144): STD128_MKNTRU_4 at dg = 5
    # (a 2.0 GB bootstrapping key in u32 words)
    ("STD128_MKNTRU_4", pyoracle.XZW, 16, 765, 45181, 1 << 5, Q_MK, 1),
]


def digest(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a, dtype="<u8").tobytes()).hexdigest()


def evalacc_inputs(method, k, n, q, baseG, Q, B, seed):
    """Seeded inputs, identical to what tests/test_golden.py rebuilds."""
    orc = pyoracle.Oracle(method, k, n, N, Q, q, baseG)
    evk = pyoracle.fill_uniform(int(np.prod(orc.evk_shape)), Q, seed + 1).reshape(orc.evk_shape)
    pkey = pyoracle.fill_uniform(int(np.prod(orc.pkey_shape)), Q, seed + 2).reshape(orc.pkey_shape)
    bound = q if method == pyoracle.XZW else 2 * N
    ct = pyoracle.fill_uniform(B * k * n, bound, seed + 3).reshape(B, k, n)
    acc = np.broadcast_to(orc.mntru_testvector(4), (B, k, N)).copy()
    return orc, evk, pkey, ct, acc


def make_evalacc():
    out = []
    for i, (name, method, k, n, q, baseG, Q, B) in enumerate(EVALACC_CASES):
        seed = 7000 + 100 * i
        orc, evk, pkey, ct, acc = evalacc_inputs(method, k, n, q, baseG, Q, B, seed)
        res = orc.evalacc_batch(evk, pkey, ct, acc, min(8, os.cpu_count() or 1))
        out.append({"name": name, "method": "XZW" if method == pyoracle.XZW else "XZW_B", "k": k, "n": n,
                    "q": q, "baseG": baseG, "Q": Q, "B": B, "seed": seed, "sha256": digest(res),
                    "sample": [int(x) for x in res[0, 0, :8]] + [int(x) for x in res[-1, -1, -8:]]})
        print(name, out[-1]["sha256"][:16], flush=True)
    return out


# paramset, method, seed
GATE_CASES = [("STD128_MKNTRU", 0, 9100), ("STD100_MKNTRU_LWE", 2, 9200),
              ("STD100_MKNTRU_LWE_2", 2, 9300), ("STD128_MKNTRU_3", 0, 9400),
              # k = 16 (binfhecontext.cpp:129-144): MK-NTRU at dg = 2, MK-LWE at dg = 3
              ("STD100_MKNTRU_4", 0, 9500), ("STD128_MKNTRU_LWE_4", 2, 9600)]


def make_gates():
    from mkfhe_amd import keys as K
    out = []
    m1 = np.array([0, 0, 1, 1]); m2 = np.array([0, 1, 0, 1])
    threads = min(8, os.cpu_count() or 1)
    for ps, method, seed in GATE_CASES:
        p = K.paramset(ps, method)
        k, n, _, dg, nk, dks = K.dims(p)
        if method == 0:
            sk = K.mntru_keygen(p, seed)
            bk = K.bt_keygen(p, sk, seed=seed + 1)
            assert bk.rdefects == 0, (ps, "r-defective key drawn: pick another seed")
            ctn = K.mntru_ctgate(p, sk, seed + 2)
            c1, c2 = K.mntru_encrypt(p, sk, m1, seed=seed + 3), K.mntru_encrypt(p, sk, m2, seed=seed + 4)
            orc = pyoracle.Oracle(pyoracle.XZW, k, n, N, p.acc.Q, p.acc.q, p.acc.baseG)
            heads = np.stack([pyoracle.mntru_head(ctn, c1[i], c2[i], p.acc.q) for i in range(4)])
            acc0 = np.broadcast_to(orc.mntru_testvector(4), (4, k, N)).copy()
            acc = orc.evalacc_batch(bk.evk, bk.pkey, heads, acc0, threads)
            res = np.stack([orc.mntru_tail_ksk1(acc[i], bk.ksk, p.ks.qKS, p.ks.baseKS, n) for i in range(4)])
            dec = K.mntru_decrypt(p, sk, res.astype(np.uint32), mod=p.ks.qKS)
            inputs = {"ct_nand": digest(ctn), "ct1": digest(c1), "ct2": digest(c2)}
        else:
            sk = K.mklwe_keygen(p, seed)
            bk = K.bt_keygen(p, sk, seed=seed + 1)
            assert bk.rdefects == 0, (ps, "r-defective key drawn: pick another seed")
            a1, b1 = K.mklwe_encrypt(p, sk, m1, seed=seed + 3)
            a2, b2 = K.mklwe_encrypt(p, sk, m2, seed=seed + 4)
            orc = pyoracle.Oracle(pyoracle.XZW_B, k, n, N, p.acc.Q, 2 * N, p.acc.baseG)
            cs, accs = zip(*[orc.mklwe_head(a1[i], b1[i], a2[i], b2[i], p.acc.q) for i in range(4)])
            acc = orc.evalacc_batch(bk.evk, bk.pkey, np.stack(cs), np.stack(accs), threads)
            A, Bk = bk.ksk_A.astype(np.uint64), bk.ksk_B.astype(np.uint64)
            outs = [orc.mklwe_tail(acc[i], A, Bk, p.ks.qKS, p.ks.baseKS, n) for i in range(4)]
            res = np.concatenate([np.stack([o[0] for o in outs]).reshape(4, -1),
                                  np.array([[o[1]] for o in outs], dtype=np.uint64)], axis=1)
            dec = K.mklwe_decrypt(p, sk, np.stack([o[0] for o in outs]).astype(np.uint32),
                                  np.array([o[1] for o in outs], dtype=np.uint32), mod=p.ks.qKS)
            inputs = {"a1": digest(a1), "b1": digest(b1), "a2": digest(a2), "b2": digest(b2)}
        assert np.array_equal(dec, 1 - (m1 & m2)), (ps, dec)
        out.append({"paramset": ps, "method": method, "seed": seed, "m1": m1.tolist(), "m2": m2.tolist(),
                    "keys": {"evk": digest(bk.evk), "pkey": digest(bk.pkey)}, "inputs": inputs,
                    "sha256": digest(res), "decrypted": dec.tolist()})
        print(ps, out[-1]["sha256"][:16], flush=True)
    return out


# The bench shapes themselves, full n, B = 4096 gates in one batch (every wave
# slot of every workgroup, two rounds of the 2048 slots; the batch kernels cut it
# into two slices on two streams): the headline's STD128_MKNTRU and config 3's
# STD100_MKNTRU_LWE_2 (MK-LWE, k = 4, the XZW_B step kernel).
# key: (name, method, k, n, q, baseG, Q, B, seed, fixture file)
BIG_BATCHES = {
    "mkntru": ("STD128_MKNTRU_B4096", pyoracle.XZW, 2, 765, 45181, 1 << 7, Q_MK, 4096, 8100, "evalacc_b4096.json"),
    "mklwe": ("STD100_MKNTRU_LWE_2_B4096", pyoracle.XZW_B, 4, 500, 32749, 1 << 9, Q_MK, 4096, 8200,
              "evalacc_b4096_mklwe.json"),
}
BIG_BATCH = BIG_BATCHES["mkntru"][:9]


def big_batch_inputs(B=None, which="mkntru"):
    name, method, k, n, q, baseG, Q, B0, seed, _ = BIG_BATCHES[which]
    return evalacc_inputs(method, k, n, q, baseG, Q, B or B0, seed)


def make_big_batch(which="mkntru"):
    """SHA-256 of the whole [4096][k][2048] output plus per-gate digests (so a
    failure names the gates); 20-40 CPU-minutes of oracle time."""
    name, method, k, n, q, baseG, Q, B, seed, _ = BIG_BATCHES[which]
    orc, evk, pkey, ct, acc = big_batch_inputs(which=which)
    res = orc.evalacc_batch(evk, pkey, ct, acc, os.cpu_count() or 1)
    per_gate = [hashlib.sha256(np.ascontiguousarray(res[b], dtype="<u8").tobytes()).hexdigest()[:16]
                for b in range(B)]
    return {"name": name, "method": "XZW" if method == pyoracle.XZW else "XZW_B", "k": k, "n": n, "q": q,
            "baseG": baseG, "Q": Q, "B": B, "seed": seed, "sha256": digest(res), "gate_sha256_16": per_gate}


def main():
    pyoracle.build()
    json.dump(REFERENCE_KATS, open(os.path.join(HERE, "reference_kats.json"), "w"), indent=1)
    if "--kats-only" in sys.argv:
        return
    if "--big-batch" in sys.argv:
        i = sys.argv.index("--big-batch")
        which = sys.argv[i + 1] if i + 1 < len(sys.argv) else "mkntru"
        json.dump(make_big_batch(which), open(os.path.join(HERE, BIG_BATCHES[which][9]), "w"))
        return
    json.dump(make_gates(), open(os.path.join(HERE, "gates_realkeys.json"), "w"), indent=1)
    if "--gates-only" in sys.argv:
        return
    json.dump(make_evalacc(), open(os.path.join(HERE, "evalacc_full.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
