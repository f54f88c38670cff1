#!/usr/bin/env python3
"""Exact-integer model of the quarter-polynomial transforms (mkacc_quad.hpp).

mk_quad_kernel spreads one ring polynomial of N = 2048 residues over the four
waves of a workgroup: wave q, lane l, register r (8 per lane).  Every layout
below maps (q, l, r) to the coefficient / EVAL index j; a transform runs its
radix-2 stages on register bits, and LDS exchanges move bits between registers,
lanes and waves (one exchange per transform crosses waves: one barrier).

This model runs the transforms exactly as the kernel orders them -- stage by
stage, each butterfly reading its twiddle from the index the kernel computes --
and checks them against the oracle (oracle/mkfhe_oracle.c, the reference's
EVAL order).  It also checks the LDS word map: every exchange's writes and reads
are conflict-free per half-wave (32 banks of 4 bytes), and the map is injective.

    python tools/quad_model.py            # all checks, prints a summary
"""
from __future__ import annotations

import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, LOGN = 2048, 11

# ---- layouts: (q, l, r) -> j --------------------------------------------------------
# bits of j held by (register bits, wave bits, lane bits), most significant first
LAYOUTS = {
    # forward: QA -> QB -> QC (wave bits 1, 0) -> QD (wave bits 4, 3)
    "QA": ((10, 9, 8), (1, 0), (7, 6, 5, 4, 3, 2)),
    "QB": ((7, 6, 5), (1, 0), (10, 9, 8, 4, 3, 2)),
    "QC": ((4, 3, 2), (1, 0), (10, 9, 8, 7, 6, 5)),
    "QD": ((2, 1, 0), (4, 3), (10, 9, 8, 7, 6, 5)),
    # inverse: QD -> IB -> IC -> QA (wave bits 1, 0 after the first exchange)
    "IB": ((5, 4, 3), (1, 0), (10, 9, 8, 7, 6, 2)),
    "IC": ((8, 7, 6), (1, 0), (10, 9, 5, 4, 3, 2)),
}


def jmap(name: str, q: int, l: int, r: int) -> int:
    rb, wb, lb = LAYOUTS[name]
    j = 0
    for k, b in enumerate(rb):
        j |= ((r >> (len(rb) - 1 - k)) & 1) << b
    for k, b in enumerate(wb):
        j |= ((q >> (len(wb) - 1 - k)) & 1) << b
    for k, b in enumerate(lb):
        j |= ((l >> (len(lb) - 1 - k)) & 1) << b
    return j


def table(name: str) -> np.ndarray:
    """[4][64][8] -> j"""
    t = np.empty((4, 64, 8), dtype=np.int64)
    for q in range(4):
        for l in range(64):
            for r in range(8):
                t[q, l, r] = jmap(name, q, l, r)
    assert sorted(t.reshape(-1)) == list(range(N)), name
    return t


# ---- LDS word map: an XOR swizzle inside each 32-word row (bijective, no padding) --------
# word(j) = (j & ~31) | ((j & 31) ^ H(j)),  H(j) = XOR of HX[k] over the set bits k >= 5 of j.
# The bank of a word is linear in j over GF(2); a half-wave access is conflict-free iff
# the bank columns of its five low lane bits are independent -- true for every layout.
HX = {5: 1, 6: 2, 7: 8, 8: 17, 9: 7, 10: 0}
LDS_WORDS = N


def word(j: int) -> int:
    h = 0
    for k, v in HX.items():
        if (j >> k) & 1:
            h ^= v
    return (j & ~31) | ((j & 31) ^ h)


def check_lds():
    words = [word(j) for j in range(N)]
    assert len(set(words)) == N, "LDS map not injective"
    worst = 1
    for name in LAYOUTS:
        t = table(name)
        for q in range(4):
            for r in range(8):
                for half in range(2):
                    banks = [word(int(t[q, l, r])) % 32 for l in range(32 * half, 32 * half + 32)]
                    worst = max(worst, max(banks.count(b) for b in set(banks)))
    return worst, max(words) + 1


# ---- transforms -----------------------------------------------------------------------
def brv(x: int, bits: int) -> int:
    return int(f"{x:0{bits}b}"[::-1], 2)


def fwd_model(a, Q, psi):
    """Forward CT with the reference's table tw[i] = psi^brv(i), stages by bit b = 10..0,
    run per layout: stages on bits (10, 9, 8) in QA, (7, 6, 5) in QB, (4, 3, 2) in QC,
    (1, 0) in QD; twiddle index 2^s + (j >> (b + 1)), s = 10 - b."""
    tw = [pow(psi, brv(i, LOGN), Q) for i in range(N)]
    x = {}   # j -> value, but accessed only through (q, l, r) of the current layout
    vals = list(int(v) for v in a)
    for lay, bits in (("QA", (10, 9, 8)), ("QB", (7, 6, 5)), ("QC", (4, 3, 2)), ("QD", (1, 0))):
        t = table(lay)
        rb = LAYOUTS[lay][0]
        for b in bits:
            rbit = 2 - rb.index(b)            # which register bit carries j's bit b
            h = 1 << rbit
            s = 10 - b
            for q in range(4):
                for l in range(64):
                    for r in range(8):
                        if r & h:
                            continue
                        j0, j1 = int(t[q, l, r]), int(t[q, l, r + h])
                        assert j1 == j0 + (1 << b)
                        w = tw[(1 << s) + (j0 >> (b + 1))]
                        U, V = vals[j0], vals[j1] * w % Q
                        vals[j0], vals[j1] = (U + V) % Q, (U - V) % Q
    return vals


def inv_model(A, Q, psi):
    """Inverse without N^-1: DIT butterflies on bits 0..10 with psi^-(t 2^(11-b)),
    t = j mod 2^b, then psi^-i per coefficient; stages (0, 1, 2) in QD, (3, 4, 5) in IB,
    (6, 7, 8) in IC, (9, 10) and the twist in QA."""
    pinv = pow(psi, -1, Q)
    vals = list(int(v) for v in A)
    for lay, bits in (("QD", (0, 1, 2)), ("IB", (3, 4, 5)), ("IC", (6, 7, 8)), ("QA", (9, 10))):
        t = table(lay)
        rb = LAYOUTS[lay][0]
        for b in bits:
            rbit = 2 - rb.index(b)
            h = 1 << rbit
            for q in range(4):
                for l in range(64):
                    for r in range(8):
                        if r & h:
                            continue
                        j0, j1 = int(t[q, l, r]), int(t[q, l, r + h])
                        assert j1 == j0 + (1 << b)
                        tt = j0 & ((1 << b) - 1)
                        w = pow(pinv, tt << (LOGN - b), Q)
                        U, V = vals[j0], vals[j1] * w % Q
                        vals[j0], vals[j1] = (U + V) % Q, (U - V) % Q
    return [vals[i] * pow(pinv, i, Q) % Q for i in range(N)]


def main() -> int:
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle
    pyoracle.build()
    Q = 134176769
    psi = pyoracle.root_of_unity(2 * N, Q)
    rng = np.random.default_rng(5)
    a = rng.integers(0, Q, size=N, dtype=np.uint64)
    F = fwd_model(a, Q, psi)
    ref = pyoracle.ntt_forward(a, Q, psi)
    assert [int(v) for v in ref] == F, "forward model != oracle"
    inv = inv_model(ref, Q, psi)
    ninv = pow(N, -1, Q)
    ref_inv = pyoracle.ntt_inverse(ref, Q, psi)
    assert [v * ninv % Q for v in inv] == [int(v) for v in ref_inv], "inverse model != oracle"
    worst, words = check_lds()
    print(f"quad model: forward and inverse equal the oracle; LDS map injective over {words} words, "
          f"worst bank multiplicity {worst} per half-wave")
    return 0 if worst == 1 else 1


if __name__ == "__main__":
    sys.exit(main())
