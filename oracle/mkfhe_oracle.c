/*
 * mkfhe_oracle.c -- CPU restatement of the MKFHE multi-key accumulator.
 *
 * TEST INFRASTRUCTURE ONLY: this is the parity checker for the HIP engine.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load
 * it.  Nothing under mkfhe_amd/ links or calls it.
 *
 * Every function cites the reference file:line it restates (paths relative to
 * the reference's src/).  Pinning status is documented in mkfhe_oracle.h and
 * DESIGN.md section 3.
 */
#include "mkfhe_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>
#ifdef __AVX512F__
#include <immintrin.h>
#endif
#ifdef _OPENMP
#include <omp.h>
#endif

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------------ */
/* modular helpers                                                          */
/* ------------------------------------------------------------------------ */

uint64_t orc_mulmod(uint64_t a, uint64_t b, uint64_t Q) {
    if (Q <= 0xFFFFFFFFull) return (a * b) % Q; /* a,b < Q < 2^32: product fits */
    return (uint64_t)(((u128)a * b) % Q);
}

uint64_t orc_powmod(uint64_t a, uint64_t e, uint64_t Q) {
    uint64_t r = 1 % Q;
    a %= Q;
    while (e) {
        if (e & 1) r = orc_mulmod(r, a, Q);
        a = orc_mulmod(a, a, Q);
        e >>= 1;
    }
    return r;
}

/* branch-free conditional corrections (random residues defeat the branch predictor) */
static inline uint64_t csub(uint64_t r, uint64_t Q) { return r - (Q & (0 - (uint64_t)(r >= Q))); }
static inline uint64_t addmod(uint64_t a, uint64_t b, uint64_t Q) { return csub(a + b, Q); }
static inline uint64_t submod(uint64_t a, uint64_t b, uint64_t Q) {
    return a - b + (Q & (0 - (uint64_t)(a < b)));
}

/* Exact reductions used by the accumulator loops.  The reference's pointwise
 * product is a plain 64-bit `%` (ubintnat.h:1304-1310) and its NTT uses
 * Shoup-precomputed twiddles (ubintnat.h:1488-1494); every form returns the
 * canonical residue, so the choice only changes the speed of the oracle.
 *   Q < 2^32 : Barrett with mu = floor(2^64 / Q) on the 64-bit product
 *              (q_est in {q-1, q}: one conditional subtraction);
 *   otherwise: 128-bit product and `%`.                                      */
typedef struct modq {
    uint64_t Q, mu;
    int big;
} modq;

static modq make_modq(uint64_t Q) {
    modq m;
    m.Q = Q;
    m.big = Q > 0xFFFFFFFFull;
    m.mu = m.big ? 0 : (uint64_t)((((u128)1) << 64) / Q);
    return m;
}
static inline uint64_t mm(const modq* m, uint64_t a, uint64_t b) {
    if (!m->big) {
        const uint64_t p = a * b;
        const uint64_t qe = (uint64_t)(((u128)p * m->mu) >> 64);
        return csub(p - qe * m->Q, m->Q);
    }
    return (uint64_t)(((u128)a * b) % m->Q);
}
/* Shoup companion floor(w 2^64 / Q) and product a*w mod Q (any a < 2^64, Q < 2^63) */
static inline uint64_t shoup_pre(uint64_t w, uint64_t Q) { return (uint64_t)((((u128)w) << 64) / Q); }
static inline uint64_t shoup_mul(uint64_t a, uint64_t w, uint64_t wp, uint64_t Q) {
    const uint64_t qe = (uint64_t)(((u128)a * wp) >> 64);
    return csub(a * w - qe * Q, Q);
}

uint64_t orc_modinv(uint64_t a, uint64_t Q) {
    /* extended Euclid over signed 128-bit */
    __int128 t = 0, nt = 1, r = (__int128)Q, nr = (__int128)(a % Q);
    while (nr != 0) {
        __int128 qt = r / nr, tmp;
        tmp = t - qt * nt; t = nt; nt = tmp;
        tmp = r - qt * nr; r = nr; nr = tmp;
    }
    if (r != 1) return 0;
    if (t < 0) t += (__int128)Q;
    return (uint64_t)t;
}

/* ------------------------------------------------------------------------ */
/* number theory                                                            */
/* ------------------------------------------------------------------------ */

/* Miller-Rabin with the deterministic base set for 64-bit n.  The reference
 * (nbtheory-impl.h:258-287) uses random witnesses; for primes both accept,
 * so FirstPrime/PreviousPrime return the same values. */
int orc_is_prime(uint64_t n) {
    static const uint64_t bases[] = {2, 3, 5, 7, 11, 13, 17, 19, 23, 29, 31, 37};
    if (n < 2) return 0;
    for (int i = 0; i < 12; ++i) {
        if (n == bases[i]) return 1;
        if (n % bases[i] == 0) return 0;
    }
    uint64_t d = n - 1;
    int s = 0;
    while ((d & 1) == 0) { d >>= 1; ++s; }
    for (int i = 0; i < 12; ++i) {
        uint64_t x = orc_powmod(bases[i], d, n);
        if (x == 1 || x == n - 1) continue;
        int comp = 1;
        for (int r = 1; r < s; ++r) {
            x = (uint64_t)(((u128)x * x) % n);
            if (x == n - 1) { comp = 0; break; }
        }
        if (comp) return 0;
    }
    return 1;
}

/* FirstPrime: nbtheory-impl.h:334-357.  Smallest prime q > 2^nbits with q = 1 mod m. */
uint64_t orc_first_prime(uint32_t nbits, uint64_t m) {
    uint64_t q = 1ull << nbits;
    uint64_t r = q % m;
    uint64_t q2 = q + 1;
    if (r > 0) q2 += (m - r);
    while (!orc_is_prime(q2)) q2 += m;
    return q2;
}

/* NextPrime: nbtheory-impl.h:361-369.  Smallest prime q' > q with q' = q mod m. */
uint64_t orc_next_prime(uint64_t q, uint64_t m) {
    uint64_t c = q + m;
    while (!orc_is_prime(c)) {
        if (c + m < c) return 0; /* the reference throws math_error on overflow */
        c += m;
    }
    return c;
}

/* PreviousPrime: nbtheory-impl.h:369-377. */
uint64_t orc_previous_prime(uint64_t q, uint64_t m) {
    uint64_t c = q - m;
    while (!orc_is_prime(c)) c -= m;
    return c;
}

/* RootOfUnity: nbtheory-impl.h:183-231.  The reference finds a random
 * generator, raises it to (Q-1)/m and then returns the MINIMUM over all
 * primitive m-th roots (odd powers for power-of-two m) -- a value that does
 * not depend on the generator.  We do the same from a deterministic generator. */
uint64_t orc_root_of_unity(uint64_t m, uint64_t Q) {
    if ((Q - 1) % m != 0) return 0;
    /* factor Q-1 by trial division (Q < 2^62; fine for the moduli used here) */
    uint64_t fac[64];
    int nf = 0;
    uint64_t t = Q - 1;
    for (uint64_t p = 2; p * p <= t; p += (p == 2 ? 1 : 2)) {
        if (t % p == 0) {
            fac[nf++] = p;
            while (t % p == 0) t /= p;
        }
    }
    if (t > 1) fac[nf++] = t;
    uint64_t g = 2;
    for (;; ++g) {
        int ok = 1;
        for (int i = 0; i < nf; ++i)
            if (orc_powmod(g, (Q - 1) / fac[i], Q) == 1) { ok = 0; break; }
        if (ok) break;
    }
    uint64_t w = orc_powmod(g, (Q - 1) / m, Q);
    /* cycle over powers coprime to m; m is a power of two here -> odd powers */
    uint64_t w2 = orc_mulmod(w, w, Q), x = w, best = w;
    for (uint64_t e = 1; e < m; e += 2) {
        if (x < best && x != 1) best = x;
        x = orc_mulmod(x, w2, Q);
    }
    return best;
}

/* mk-cryptoparameters.h:141-142: digitsG = ceil(log(Q)/log(baseG)) in double. */
uint32_t orc_digits_g(uint64_t Q, uint32_t baseG) {
    double logQ = log((double)Q);
    return (uint32_t)ceil(logQ / log((double)baseG));
}

/* Element-wise vector arithmetic of NativeVectorT (mubintvecnat.cpp:235-244
 * ModAdd, :279-288 ModSub, :324-340 ModMul) with the same reductions the
 * accumulator loops use (mm / addmod / submod).  op: 0 add, 1 sub, 2 mul. */
void orc_vec_mod(int op, const uint64_t* a, const uint64_t* b, uint64_t* out, size_t n, uint64_t Q) {
    const modq m = make_modq(Q);
    for (size_t i = 0; i < n; ++i)
        out[i] = op == 0 ? addmod(a[i], b[i], Q) : op == 1 ? submod(a[i], b[i], Q) : mm(&m, a[i], b[i]);
}

/* ------------------------------------------------------------------------ */
/* NTT (transformnat-impl.h)                                                */
/* ------------------------------------------------------------------------ */

/* the 32-bit word transforms and digit decomposition (defined with the accumulator below) */
static void ntt_fwd32(uint32_t* restrict a, uint32_t N, uint32_t Q, const uint32_t* restrict w,
                      const uint32_t* restrict wp);
static void ntt_inv32(uint32_t* restrict a, uint32_t N, uint32_t Q, const uint32_t* restrict w,
                      const uint32_t* restrict wp, uint32_t ninv, uint32_t ninvp);
static void sdd32(const uint32_t* restrict in, uint32_t* restrict out, uint32_t N, uint32_t Q, uint32_t gBits,
                  uint32_t dg);

static uint32_t brv(uint32_t x, uint32_t bits) {
    uint32_t r = 0;
    for (uint32_t i = 0; i < bits; ++i) r |= ((x >> i) & 1u) << (bits - 1 - i);
    return r;
}
static uint32_t ilog2u(uint32_t x) { uint32_t r = 0; while ((1u << r) < x) ++r; return r; }

/* Tables exactly as ChineseRemainderTransformFTTNat::PreCompute
 * (transformnat-impl.h:705-760): table[brv(i)] = psi^i, tableI[brv(i)] = psi^-i,
 * each followed by its Shoup companions: floor(w 2^64 / Q) at +N and, for
 * Q < 2^32, floor(w 2^32 / Q) at +2N. */
static void make_tables(uint64_t* tab, uint64_t* tabI, uint32_t N, uint64_t Q, uint64_t psi) {
    uint32_t lg = ilog2u(N);
    uint64_t x = 1, xi = 1, psiI = orc_modinv(psi, Q);
    for (uint32_t i = 0; i < N; ++i) {
        uint32_t r = brv(i, lg);
        tab[r] = x;
        tabI[r] = xi;
        tab[N + r] = shoup_pre(x, Q);
        tabI[N + r] = shoup_pre(xi, Q);
        tab[2 * N + r] = Q <= 0xFFFFFFFFull ? (x << 32) / Q : 0;
        tabI[2 * N + r] = Q <= 0xFFFFFFFFull ? (xi << 32) / Q : 0;
        x = orc_mulmod(x, psi, Q);
        xi = orc_mulmod(xi, psiI, Q);
    }
}

/* ForwardTransformToBitReverseInPlace, transformnat-impl.h:300-354. */
/* Q < 2^32: Shoup with the 32-bit companion floor(w 2^32 / Q) on 32x32->64
 * products, written so that the butterfly loops vectorize (vpmuludq). */
static inline uint64_t shoup32(uint64_t x, uint64_t w, uint64_t wp32, uint64_t Q) {
    const uint64_t qe = ((uint64_t)(uint32_t)x * (uint32_t)wp32) >> 32;
    return csub((uint64_t)(uint32_t)x * (uint32_t)w - (uint64_t)(uint32_t)qe * (uint32_t)Q, Q);
}
static void ntt_fwd_tab32(uint64_t* restrict a, uint32_t N, uint64_t Q, const uint64_t* tab) {
    uint32_t t = N;
    for (uint32_t m = 1; m < N; m <<= 1) {
        t >>= 1;
        for (uint32_t i = 0; i < m; ++i) {
            const uint64_t w = tab[m + i], wp = tab[2 * N + m + i];
            uint64_t* restrict x = a + 2 * i * t;
            uint64_t* restrict y = x + t;
            for (uint32_t j = 0; j < t; ++j) {
                const uint64_t U = x[j], V = shoup32(y[j], w, wp, Q);
                x[j] = csub(U + V, Q);
                y[j] = U - V + (Q & (0 - (uint64_t)(U < V)));
            }
        }
    }
}
static void ntt_inv_tab32(uint64_t* restrict a, uint32_t N, uint64_t Q, const uint64_t* tabI, uint64_t Ninv) {
    const uint64_t NinvP = (Ninv << 32) / Q;
    for (uint32_t i = 0; i < N; i += 2) {
        uint64_t w = tabI[(i + N) >> 1], wp = tabI[2 * N + ((i + N) >> 1)];
        uint64_t lo = a[i], hi = a[i + 1];
        uint64_t d = submod(lo, hi, Q);
        lo = addmod(lo, hi, Q);
        a[i] = shoup32(lo, Ninv, NinvP, Q);
        a[i + 1] = shoup32(shoup32(d, w, wp, Q), Ninv, NinvP, Q);
    }
    for (uint32_t m = N >> 2, t = 2; m >= 1; m >>= 1, t <<= 1) {
        for (uint32_t i = 0; i < m; ++i) {
            const uint64_t w = tabI[i + m], wp = tabI[2 * N + i + m];
            uint64_t* restrict x = a + 2 * i * t;
            uint64_t* restrict y = x + t;
            for (uint32_t j = 0; j < t; ++j) {
                const uint64_t lo = x[j], hi = y[j];
                x[j] = csub(lo + hi, Q);
                y[j] = shoup32(lo - hi + (Q & (0 - (uint64_t)(lo < hi))), w, wp, Q);
            }
        }
    }
}

static void ntt_fwd_tab(uint64_t* a, uint32_t N, uint64_t Q, const uint64_t* tab) {
    if (Q <= 0xFFFFFFFFull) {
        ntt_fwd_tab32(a, N, Q, tab);
        return;
    }
    uint32_t t = N;
    for (uint32_t m = 1; m < N; m <<= 1) {
        t >>= 1;
        for (uint32_t i = 0; i < m; ++i) {
            uint64_t w = tab[m + i], wp = tab[N + m + i];
            uint32_t j1 = 2 * i * t;
            for (uint32_t j = j1; j < j1 + t; ++j) {
                uint64_t U = a[j], V = shoup_mul(a[j + t], w, wp, Q);
                a[j] = addmod(U, V, Q);
                a[j + t] = submod(U, V, Q);
            }
        }
    }
}

/* InverseTransformFromBitReverseInPlace, transformnat-impl.h:492-552
 * (stride-1 stage first with N^-1 fused, then GS stages of growing stride). */
static void ntt_inv_tab(uint64_t* a, uint32_t N, uint64_t Q, const uint64_t* tabI, uint64_t Ninv) {
    if (Q <= 0xFFFFFFFFull) {
        ntt_inv_tab32(a, N, Q, tabI, Ninv);
        return;
    }
    const uint64_t NinvP = shoup_pre(Ninv, Q);
    for (uint32_t i = 0; i < N; i += 2) {
        uint64_t w = tabI[(i + N) >> 1], wp = tabI[N + ((i + N) >> 1)];
        uint64_t lo = a[i], hi = a[i + 1];
        uint64_t d = submod(lo, hi, Q);
        lo = addmod(lo, hi, Q);
        a[i] = shoup_mul(lo, Ninv, NinvP, Q);
        a[i + 1] = shoup_mul(shoup_mul(d, w, wp, Q), Ninv, NinvP, Q);
    }
    for (uint32_t m = N >> 2, t = 2; m >= 1; m >>= 1, t <<= 1) {
        for (uint32_t i = 0; i < m; ++i) {
            uint64_t w = tabI[i + m], wp = tabI[N + i + m];
            uint32_t j1 = 2 * i * t;
            for (uint32_t j = j1; j < j1 + t; ++j) {
                uint64_t lo = a[j], hi = a[j + t];
                a[j] = addmod(lo, hi, Q);
                a[j + t] = shoup_mul(submod(lo, hi, Q), w, wp, Q);
            }
        }
    }
}

/* Q < 2^30: through the 32-bit word transforms the accumulator uses, so the
 * reference's known-answer vectors pin that code (tests/test_oracle_kat.py) */
static void ntt32_entry(uint64_t* a, uint32_t N, uint64_t Q, const uint64_t* tab, uint64_t Ninv, int inverse) {
    uint32_t* w = (uint32_t*)malloc(sizeof(uint32_t) * N * 3);
    uint32_t *wp = w + N, *x = w + 2 * N;
    for (uint32_t i = 0; i < N; ++i) {
        w[i] = (uint32_t)tab[i];
        wp[i] = (uint32_t)tab[2 * N + i];
        x[i] = (uint32_t)a[i];
    }
    if (inverse)
        ntt_inv32(x, N, (uint32_t)Q, w, wp, (uint32_t)Ninv, (uint32_t)((Ninv << 32) / Q));
    else
        ntt_fwd32(x, N, (uint32_t)Q, w, wp);
    for (uint32_t i = 0; i < N; ++i) a[i] = x[i];
    free(w);
}

void orc_ntt_forward(uint64_t* a, uint32_t N, uint64_t Q, uint64_t psi) {
    uint64_t* tab = (uint64_t*)malloc(sizeof(uint64_t) * N * 6);
    make_tables(tab, tab + 3 * N, N, Q, psi);
    if (Q < (1ull << 30))
        ntt32_entry(a, N, Q, tab, 0, 0);
    else
        ntt_fwd_tab(a, N, Q, tab);
    free(tab);
}

void orc_ntt_inverse(uint64_t* a, uint32_t N, uint64_t Q, uint64_t psi) {
    uint64_t* tab = (uint64_t*)malloc(sizeof(uint64_t) * N * 6);
    make_tables(tab, tab + 3 * N, N, Q, psi);
    if (Q < (1ull << 30))
        ntt32_entry(a, N, Q, tab + 3 * N, orc_modinv(N, Q), 1);
    else
        ntt_inv_tab(a, N, Q, tab + 3 * N, orc_modinv(N, Q));
    free(tab);
}

/* PolyImpl::AutomorphismTransform EVALUATION branch (poly-impl.h:348-355) with k = 2N-1. */
void orc_transpose_eval(const uint64_t* in, uint64_t* out, uint32_t N) {
    uint32_t logn = ilog2u(N), mask = N - 1, k = 2 * N - 1;
    uint64_t jk = k;
    for (uint32_t j = 0; j < N; ++j, jk += 2ull * k) {
        uint32_t jrev = brv(j, logn);
        uint32_t idxrev = brv((uint32_t)((jk >> 1) & mask), logn);
        out[jrev] = in[idxrev];
    }
}

/* PolyImpl::AutomorphismTransform COEFFICIENT branch (poly-impl.h:357-361).
 * Note: reproduces the reference's q - 0 = q (non-canonical) for zero entries. */
void orc_automorphism_coeff(const uint64_t* in, uint64_t* out, uint32_t N, uint64_t Q, uint32_t k) {
    uint32_t logn = ilog2u(N), mask = N - 1;
    uint64_t jk = 0;
    for (uint32_t j = 0; j < N; ++j, jk += k)
        out[jk & mask] = ((jk >> logn) & 1) ? Q - in[j] : in[j];
}

/* ------------------------------------------------------------------------ */
/* SignedDigitDecompose (mk-acc.cpp:54-80)                                   */
/* ------------------------------------------------------------------------ */

static inline int64_t sext_low(int64_t d, uint32_t gBits) {
    /* (d << (W - gBits)) >> (W - gBits): sign-extend the low gBits bits */
    uint64_t m = 1ull << gBits;
    uint64_t low = (uint64_t)d & (m - 1);
    return (low >= (m >> 1)) ? (int64_t)low - (int64_t)m : (int64_t)low;
}

void orc_sdd(const uint64_t* in, uint64_t* out, uint32_t N, uint64_t Q, uint32_t baseG, uint32_t dg) {
    uint64_t QHalf = Q >> 1;
    uint32_t gBits = (uint32_t)__builtin_ctz(baseG);
    if (Q < (1ull << 30) && gBits * (dg + 1) <= 30) {
        /* through the 32-bit word decomposition the accumulator uses */
        uint32_t* x = (uint32_t*)calloc((size_t)N * (dg + 1), sizeof(uint32_t));
        for (uint32_t k = 0; k < N; ++k) x[k] = (uint32_t)in[k];
        sdd32(x, x + N, N, (uint32_t)Q, gBits, dg);
        for (size_t k = 0; k < (size_t)N * dg; ++k) out[k] = x[N + k];
        free(x);
        return;
    }
    for (uint32_t k = 0; k < N; ++k) {
        uint64_t t0 = in[k];
        int64_t d0 = t0 < QHalf ? (int64_t)t0 : (int64_t)t0 - (int64_t)Q;
        int64_t r0 = sext_low(d0, gBits);
        d0 = (d0 - r0) >> gBits; /* lowest digit dropped (approximate gadget) */
        for (uint32_t d = 0; d < dg; ++d) {
            r0 = sext_low(d0, gBits);
            d0 = (d0 - r0) >> gBits;
            if (r0 < 0) r0 += (int64_t)Q;
            out[(size_t)d * N + k] = (uint64_t)r0;
        }
    }
}

/* ------------------------------------------------------------------------ */
/* accumulator context                                                       */
/* ------------------------------------------------------------------------ */

/* ------------------------------------------------------------------------ */
/* 32-bit word path (Q < 2^27: every MK parameter set)                       */
/* ------------------------------------------------------------------------ */
/* The reference's README build is NATIVE_SIZE=32: NativeInteger is a 32-bit
 * word (basicint.h:56-59) and its NTT uses Shoup companions floor(w 2^32 / Q)
 * (ubintnat.h:1488-1494).  The accumulator runs on u32 words here too, with
 * lazy (Harvey) butterflies -- values stay below 4Q < 2^32 and are made
 * canonical once per transform -- and lazy 64-bit sums for the pointwise
 * multiply-adds, reduced once per slot.  Every reduction is exact, so the
 * canonical outputs equal the reference's per-operation reductions
 * (ubintnat.h:1304-1310 ModMulFastEq, mubintvecnat.cpp:246-296 ModAdd/ModSub). */
typedef struct m32 {
    uint32_t Q, mu, sh;   /* Barrett: q = ((x >> sh) * mu) >> 32, sh = L - 1, mu = floor(2^(L+31) / Q) */
} m32;

static m32 make_m32(uint32_t Q) {
    m32 m;
    uint32_t L = 32 - (uint32_t)__builtin_clz(Q);
    m.Q = Q;
    m.sh = L - 1;
    m.mu = (uint32_t)((1ull << (L + 31)) / Q);
    return m;
}
/* x < 2^(L+31) (a sum of up to 16 products of residues when L <= 27) -> [0, Q):
 * the quotient estimate is at most 2 below floor(x / Q) */
static inline uint32_t bred(uint64_t x, uint32_t Q, uint32_t mu, uint32_t sh) {
    /* x >> sh < 2^32: a 32 x 32 -> 64-bit product (vpmuludq when vectorized) */
    const uint32_t q = (uint32_t)(((uint64_t)(uint32_t)(x >> sh) * mu) >> 32);
    uint32_t r = (uint32_t)x - q * Q; /* < 3Q */
    r = r >= Q ? r - Q : r;
    return r >= Q ? r - Q : r;
}
/* lazy Shoup product y * w in [0, 2Q) for any 32-bit y (wp = floor(w 2^32 / Q)) */
static inline uint32_t shoup_lazy32(uint32_t y, uint32_t w, uint32_t wp, uint32_t Q) {
    const uint32_t q = (uint32_t)(((uint64_t)y * wp) >> 32);
    return y * w - q * Q;
}
static inline uint32_t min32(uint32_t a, uint32_t b) { return a < b ? a : b; }

#ifdef __AVX512F__
/* 16 lanes of the lazy Shoup product (W, WP broadcast or per lane): the high
 * words of y * wp from the even and odd 64-bit products, low words by vpmulld */
static inline __m512i shoup_lazy_v(__m512i y, __m512i W, __m512i WP, __m512i Qv) {
    const __m512i pe = _mm512_mul_epu32(y, WP);
    const __m512i po = _mm512_mul_epu32(_mm512_srli_epi64(y, 32), _mm512_srli_epi64(WP, 32));
    const __m512i q = _mm512_mask_blend_epi32(0xAAAA, _mm512_srli_epi64(pe, 32), po);
    return _mm512_sub_epi32(_mm512_mullo_epi32(y, W), _mm512_mullo_epi32(q, Qv));
}
/* strides t < 16: 32 consecutive words hold 16/t butterfly groups; gather
 * their x and y halves into two registers (idx_x, idx_y), the twiddle of lane
 * L is entry L / t of the stage's run (idx_w), and idx_o scatters back */
typedef struct short_perm { __m512i ix, iy, iw, io0, io1; } short_perm;
static short_perm make_short_perm(uint32_t t) {
    uint32_t ix[16], iy[16], iw[16], io[32];
    for (uint32_t L = 0; L < 16; ++L) {
        const uint32_t g = L / t, o = L % t;
        ix[L] = g * 2 * t + o;
        iy[L] = g * 2 * t + t + o;
        iw[L] = g;
    }
    for (uint32_t P = 0; P < 32; ++P) {
        const uint32_t g = P / (2 * t), r = P % (2 * t);
        io[P] = r < t ? g * t + r : 16 + g * t + r - t;
    }
    short_perm s;
    s.ix = _mm512_loadu_si512(ix);
    s.iy = _mm512_loadu_si512(iy);
    s.iw = _mm512_loadu_si512(iw);
    s.io0 = _mm512_loadu_si512(io);
    s.io1 = _mm512_loadu_si512(io + 16);
    return s;
}
#endif

/* ForwardTransformToBitReverseInPlace (transformnat-impl.h:300-354) on u32
 * words: the same CT loop and tables, lazy: U in [0, 2Q), V = Shoup in [0, 2Q),
 * outputs in [0, 4Q); canonical at the end.  Input canonical (or < 4Q). */
static void ntt_fwd32(uint32_t* restrict a, uint32_t N, uint32_t Q, const uint32_t* restrict w,
                      const uint32_t* restrict wp) {
    const uint32_t Q2 = 2 * Q;
    uint32_t t = N;
    for (uint32_t m = 1; m < N; m <<= 1) {
        t >>= 1;
#ifdef __AVX512F__
        const __m512i Qv = _mm512_set1_epi32((int)Q), Q2v = _mm512_set1_epi32((int)Q2);
        if (t >= 16) {
            for (uint32_t i = 0; i < m; ++i) {
                const __m512i W = _mm512_set1_epi32((int)w[m + i]), WP = _mm512_set1_epi32((int)wp[m + i]);
                uint32_t* x = a + 2 * i * t;
                uint32_t* y = x + t;
                for (uint32_t j = 0; j < t; j += 16) {
                    __m512i U = _mm512_loadu_si512(x + j);
                    U = _mm512_min_epu32(U, _mm512_sub_epi32(U, Q2v));
                    const __m512i V = shoup_lazy_v(_mm512_loadu_si512(y + j), W, WP, Qv);
                    _mm512_storeu_si512(x + j, _mm512_add_epi32(U, V));
                    _mm512_storeu_si512(y + j, _mm512_add_epi32(_mm512_sub_epi32(U, V), Q2v));
                }
            }
            continue;
        }
        if (N >= 32) {
            const short_perm sp = make_short_perm(t);
            const uint32_t gpb = 16 / t; /* groups per 32 words */
            for (uint32_t b = 0; b < N; b += 32) {
                const __m512i A = _mm512_loadu_si512(a + b), Bv = _mm512_loadu_si512(a + b + 16);
                const uint32_t g0 = m + b / (2 * t);
                (void)gpb;
                const __m512i W = _mm512_permutexvar_epi32(sp.iw, _mm512_loadu_si512(w + g0));
                const __m512i WP = _mm512_permutexvar_epi32(sp.iw, _mm512_loadu_si512(wp + g0));
                __m512i U = _mm512_permutex2var_epi32(A, sp.ix, Bv);
                U = _mm512_min_epu32(U, _mm512_sub_epi32(U, Q2v));
                const __m512i V = shoup_lazy_v(_mm512_permutex2var_epi32(A, sp.iy, Bv), W, WP, Qv);
                const __m512i X = _mm512_add_epi32(U, V), Y = _mm512_add_epi32(_mm512_sub_epi32(U, V), Q2v);
                _mm512_storeu_si512(a + b, _mm512_permutex2var_epi32(X, sp.io0, Y));
                _mm512_storeu_si512(a + b + 16, _mm512_permutex2var_epi32(X, sp.io1, Y));
            }
            continue;
        }
#endif
        for (uint32_t i = 0; i < m; ++i) {
            const uint32_t W = w[m + i], WP = wp[m + i];
            uint32_t* restrict x = a + 2 * i * t;
            uint32_t* restrict y = x + t;
            for (uint32_t j = 0; j < t; ++j) {
                const uint32_t U = min32(x[j], x[j] - Q2);
                const uint32_t V = shoup_lazy32(y[j], W, WP, Q);
                x[j] = U + V;
                y[j] = U - V + Q2;
            }
        }
    }
    for (uint32_t j = 0; j < N; ++j) {
        uint32_t x = min32(a[j], a[j] - Q2);
        a[j] = min32(x, x - Q);
    }
}

/* InverseTransformFromBitReverseInPlace (transformnat-impl.h:492-552) on u32
 * words: the GS stages of growing stride with the reference's inverse table,
 * lazy in [0, 2Q); N^-1 (fused into the stride-1 stage there) applied with
 * the canonical reduction at the end.  Input canonical (or < 2Q). */
static void ntt_inv32(uint32_t* restrict a, uint32_t N, uint32_t Q, const uint32_t* restrict w,
                      const uint32_t* restrict wp, uint32_t ninv, uint32_t ninvp) {
    const uint32_t Q2 = 2 * Q;
    for (uint32_t m = N >> 1, t = 1; m >= 1; m >>= 1, t <<= 1) {
#ifdef __AVX512F__
        const __m512i Qv = _mm512_set1_epi32((int)Q), Q2v = _mm512_set1_epi32((int)Q2);
        if (t >= 16) {
            for (uint32_t i = 0; i < m; ++i) {
                const __m512i W = _mm512_set1_epi32((int)w[m + i]), WP = _mm512_set1_epi32((int)wp[m + i]);
                uint32_t* x = a + 2 * i * t;
                uint32_t* y = x + t;
                for (uint32_t j = 0; j < t; j += 16) {
                    const __m512i U = _mm512_loadu_si512(x + j), V = _mm512_loadu_si512(y + j);
                    const __m512i S = _mm512_add_epi32(U, V);
                    _mm512_storeu_si512(x + j, _mm512_min_epu32(S, _mm512_sub_epi32(S, Q2v)));
                    _mm512_storeu_si512(y + j, shoup_lazy_v(_mm512_add_epi32(_mm512_sub_epi32(U, V), Q2v), W, WP, Qv));
                }
            }
            continue;
        }
        if (N >= 32) {
            const short_perm sp = make_short_perm(t);
            for (uint32_t b = 0; b < N; b += 32) {
                const __m512i A = _mm512_loadu_si512(a + b), Bv = _mm512_loadu_si512(a + b + 16);
                const uint32_t g0 = m + b / (2 * t);
                const __m512i W = _mm512_permutexvar_epi32(sp.iw, _mm512_loadu_si512(w + g0));
                const __m512i WP = _mm512_permutexvar_epi32(sp.iw, _mm512_loadu_si512(wp + g0));
                const __m512i U = _mm512_permutex2var_epi32(A, sp.ix, Bv);
                const __m512i V = _mm512_permutex2var_epi32(A, sp.iy, Bv);
                const __m512i S = _mm512_add_epi32(U, V);
                const __m512i X = _mm512_min_epu32(S, _mm512_sub_epi32(S, Q2v));
                const __m512i Y = shoup_lazy_v(_mm512_add_epi32(_mm512_sub_epi32(U, V), Q2v), W, WP, Qv);
                _mm512_storeu_si512(a + b, _mm512_permutex2var_epi32(X, sp.io0, Y));
                _mm512_storeu_si512(a + b + 16, _mm512_permutex2var_epi32(X, sp.io1, Y));
            }
            continue;
        }
#endif
        for (uint32_t i = 0; i < m; ++i) {
            const uint32_t W = w[m + i], WP = wp[m + i];
            uint32_t* restrict x = a + 2 * i * t;
            uint32_t* restrict y = x + t;
            for (uint32_t j = 0; j < t; ++j) {
                const uint32_t U = x[j], V = y[j];
                x[j] = min32(U + V, U + V - Q2);
                y[j] = shoup_lazy32(U - V + Q2, W, WP, Q);
            }
        }
    }
    for (uint32_t j = 0; j < N; ++j) {
        const uint32_t x = shoup_lazy32(a[j], ninv, ninvp, Q);
        a[j] = min32(x, x - Q);
    }
}

/* SignedDigitDecompose (mk-acc.cpp:54-80) on u32 words, one pass per digit
 * over the running value d (kept in out's last row until it is overwritten) */
static void sdd32(const uint32_t* restrict in, uint32_t* restrict out, uint32_t N, uint32_t Q, uint32_t gBits,
                  uint32_t dg) {
    const int32_t QHalf = (int32_t)(Q >> 1), half = 1 << (gBits - 1), mask = (1 << gBits) - 1;
    int32_t* dv = (int32_t*)(out + (size_t)(dg - 1) * N);
    for (uint32_t k = 0; k < N; ++k) {
        const int32_t t0 = (int32_t)in[k];
        const int32_t d0 = t0 < QHalf ? t0 : t0 - (int32_t)Q;
        const int32_t r0 = ((d0 + half) & mask) - half; /* sign-extended low gBits bits */
        dv[k] = (d0 - r0) >> gBits;                     /* lowest digit dropped */
    }
    for (uint32_t d = 0; d + 1 < dg; ++d) {
        uint32_t* restrict o = out + (size_t)d * N;
        for (uint32_t k = 0; k < N; ++k) {
            const int32_t x = dv[k];
            const int32_t r0 = ((x + half) & mask) - half;
            dv[k] = (x - r0) >> gBits;
            o[k] = (uint32_t)(r0 < 0 ? r0 + (int32_t)Q : r0);
        }
    }
    for (uint32_t k = 0; k < N; ++k) {   /* the last digit replaces the running value */
        const int32_t x = dv[k];
        const int32_t r0 = ((x + half) & mask) - half;
        dv[k] = r0 < 0 ? r0 + (int32_t)Q : r0;
    }
}

struct orc_ctx {
    orc_params p;
    uint32_t dg, nk;
    uint64_t Ninv;
    modq m;
    uint64_t* tab;   /* forward table [N] + Shoup companions [2N] (make_tables) */
    uint64_t* tabI;  /* inverse table [N] + Shoup companions [2N] */
    uint64_t* mono;  /* [2N][N] monomials X^m - 1 in EVAL (mk-cryptoparameters.cpp:51-70); 64-bit path */
    /* 32-bit word path (Q < 2^27) */
    int w32;
    m32 b;
    uint32_t ninv32, ninvp32;
    uint32_t *tw32, *twp32, *twi32, *twip32;   /* reference tables and Shoup companions */
    uint32_t* mono32;                          /* [2N][N] monomials, u32 */
};

orc_ctx* orc_ctx_create(const orc_params* p) {
    if (!p || p->N < 4 || (p->N & (p->N - 1)) || p->k == 0 || p->n == 0) return NULL;
    if (p->baseG < 2 || (p->baseG & (p->baseG - 1))) return NULL;
    orc_ctx* c = (orc_ctx*)calloc(1, sizeof(orc_ctx));
    c->p = *p;
    if (c->p.digitsG == 0) c->p.digitsG = orc_digits_g(p->Q, p->baseG);
    if (c->p.psi == 0) c->p.psi = orc_root_of_unity(2ull * p->N, p->Q);
    c->dg = c->p.digitsG - 1;
    c->nk = (p->method == ORC_XZW) ? 2 : 1;
    uint32_t N = p->N;
    uint64_t Q = p->Q;
    c->Ninv = orc_modinv(N, Q);
    c->m = make_modq(Q);
    c->tab = (uint64_t*)malloc(sizeof(uint64_t) * N * 3);
    c->tabI = (uint64_t*)malloc(sizeof(uint64_t) * N * 3);
    make_tables(c->tab, c->tabI, N, Q, c->p.psi);
    c->w32 = Q < (1ull << 27);
    if (c->w32) {
        c->b = make_m32((uint32_t)Q);
        c->ninv32 = (uint32_t)c->Ninv;
        c->ninvp32 = (uint32_t)((c->Ninv << 32) / Q);
        uint32_t* t = (uint32_t*)malloc(sizeof(uint32_t) * N * 4);
        c->tw32 = t; c->twp32 = t + N; c->twi32 = t + 2 * N; c->twip32 = t + 3 * N;
        for (uint32_t i = 0; i < N; ++i) {
            c->tw32[i] = (uint32_t)c->tab[i];
            c->twp32[i] = (uint32_t)c->tab[2 * N + i];
            c->twi32[i] = (uint32_t)c->tabI[i];
            c->twip32[i] = (uint32_t)c->tabI[2 * N + i];
        }
        /* monomials X^i - 1 and -X^i - 1 (= X^(N+i) - 1), mk-cryptoparameters.cpp:51-70 */
        c->mono32 = (uint32_t*)calloc((size_t)2 * N * N, sizeof(uint32_t));
        for (uint32_t i = 0; i < 2 * N; ++i) {
            uint32_t* a = c->mono32 + (size_t)i * N;
            const uint32_t e = i % N;
            a[0] = (uint32_t)Q - 1;
            a[e] = i < N ? (uint32_t)addmod(a[e], 1, Q) : (uint32_t)submod(a[e], 1, Q);
            ntt_fwd32(a, N, (uint32_t)Q, c->tw32, c->twp32);
        }
        return c;
    }
    c->mono = (uint64_t*)calloc((size_t)2 * N * N, sizeof(uint64_t));
    for (uint32_t i = 0; i < N; ++i) {               /* X^i - 1 */
        uint64_t* a = c->mono + (size_t)i * N;
        a[0] = submod(a[0], 1, Q);
        a[i] = addmod(a[i], 1, Q);
        ntt_fwd_tab(a, N, Q, c->tab);
    }
    for (uint32_t i = 0; i < N; ++i) {               /* -X^i - 1 (= X^(N+i) - 1) */
        uint64_t* a = c->mono + (size_t)(N + i) * N;
        a[0] = submod(a[0], 1, Q);
        a[i] = submod(a[i], 1, Q);
        ntt_fwd_tab(a, N, Q, c->tab);
    }
    return c;
}

void orc_ctx_destroy(orc_ctx* c) {
    if (!c) return;
    free(c->tab); free(c->tabI); free(c->mono); free(c->tw32); free(c->mono32); free(c);
}

size_t orc_evk_words(const orc_params* p) {
    uint32_t dg = (p->digitsG ? p->digitsG : orc_digits_g(p->Q, p->baseG)) - 1;
    uint32_t nk = (p->method == ORC_XZW) ? 2 : 1;
    return (size_t)p->k * nk * (p->n + 1) * dg * 2 * p->N;
}

/* key poly pointer: evk[u][j][i][digit][part] */
static inline const uint64_t* keyp(const orc_ctx* c, const uint64_t* evk, uint32_t u, uint32_t j, uint32_t i,
                                   uint32_t digit, uint32_t part) {
    size_t N = c->p.N;
    size_t idx = ((((size_t)u * c->nk + j) * (c->p.n + 1) + i) * c->dg + digit) * 2 + part;
    return evk + idx * N;
}

/* HbProd: mk-acc-xzw.cpp:231-290 (identical in mk-acc-xzw_B.cpp:221-279).
 *   acc[u] <- sum_i NTT(g^-1(iNTT(acc[u])))_i * d_i            for every u
 *   acc[index] += sum_i NTT(g^-1(iNTT(sum_u sum_i dct_{u,i} * P[u][i])))_i * f_i */
static void hbprod(const orc_ctx* c, const uint64_t* d, const uint64_t* f, uint32_t index,
                   const uint64_t* pkey, uint64_t* acc, uint64_t* scratch) {
    const uint32_t N = c->p.N, k = c->p.k, dg = c->dg;
    const uint64_t Q = c->p.Q;
    uint64_t* ct = scratch;                  /* N */
    uint64_t* dct = ct + N;                  /* dg*N */
    uint64_t* sumV = dct + (size_t)dg * N;   /* N */
    memset(sumV, 0, sizeof(uint64_t) * N);
    for (uint32_t u = 0; u < k; ++u) {
        memcpy(ct, acc + (size_t)u * N, sizeof(uint64_t) * N);
        ntt_inv_tab(ct, N, Q, c->tabI, c->Ninv);
        orc_sdd(ct, dct, N, Q, c->p.baseG, dg);
        for (uint32_t i = 0; i < dg; ++i) ntt_fwd_tab(dct + (size_t)i * N, N, Q, c->tab);
        uint64_t* out = acc + (size_t)u * N;
        const uint64_t* Pu = pkey + (size_t)u * dg * N;
        for (uint32_t s = 0; s < N; ++s) {
            uint64_t uj = 0, v = 0;
            for (uint32_t i = 0; i < dg; ++i) {
                uint64_t g = dct[(size_t)i * N + s];
                uj = addmod(uj, mm(&c->m, g, d[(size_t)i * N + s]), Q);
                v = addmod(v, mm(&c->m, g, Pu[(size_t)i * N + s]), Q);
            }
            sumV[s] = addmod(sumV[s], v, Q);
            out[s] = uj;
        }
    }
    ntt_inv_tab(sumV, N, Q, c->tabI, c->Ninv);
    orc_sdd(sumV, dct, N, Q, c->p.baseG, dg);
    for (uint32_t i = 0; i < dg; ++i) ntt_fwd_tab(dct + (size_t)i * N, N, Q, c->tab);
    uint64_t* out = acc + (size_t)index * N;
    for (uint32_t s = 0; s < N; ++s) {
        uint64_t w = 0;
        for (uint32_t i = 0; i < dg; ++i)
            w = addmod(w, mm(&c->m, dct[(size_t)i * N + s], f[(size_t)i * N + s]), Q);
        out[s] = addmod(out[s], w, Q);
    }
}

/* HbProd (mk-acc-xzw.cpp:231-290) on u32 words: the same loop nest as hbprod();
 * the per-slot sums over the digits are lazy 64-bit (at most 2 dg products of
 * residues below Q < 2^27) and reduced once. */
static void hbprod32(const orc_ctx* c, const uint32_t* restrict d, const uint32_t* restrict f, uint32_t index,
                     const uint32_t* restrict pkey, uint32_t* restrict acc, uint32_t* restrict scratch) {
    const uint32_t N = c->p.N, k = c->p.k, dg = c->dg, Q = (uint32_t)c->p.Q;
    const uint32_t mu = c->b.mu, sh = c->b.sh, gBits = (uint32_t)__builtin_ctz(c->p.baseG);
    uint32_t* ct = scratch;                    /* N */
    uint32_t* dct = ct + N;                    /* dg*N */
    uint32_t* sumV = dct + (size_t)dg * N;     /* N */
    uint64_t* sU = (uint64_t*)(sumV + N);      /* N lazy sums (u64) */
    uint64_t* sVv = sU + N;                    /* N */
    memset(sumV, 0, sizeof(uint32_t) * N);
    for (uint32_t u = 0; u < k; ++u) {
        memcpy(ct, acc + (size_t)u * N, sizeof(uint32_t) * N);
        ntt_inv32(ct, N, Q, c->twi32, c->twip32, c->ninv32, c->ninvp32);
        sdd32(ct, dct, N, Q, gBits, dg);
        for (uint32_t i = 0; i < dg; ++i) ntt_fwd32(dct + (size_t)i * N, N, Q, c->tw32, c->twp32);
        uint32_t* out = acc + (size_t)u * N;
        const uint32_t* Pu = pkey + (size_t)u * dg * N;
        for (uint32_t s = 0; s < N; ++s) {
            sU[s] = 0;
            sVv[s] = 0;
        }
        for (uint32_t i = 0; i < dg; ++i) {
            const uint32_t* restrict g = dct + (size_t)i * N;
            const uint32_t* restrict di = d + (size_t)i * N;
            const uint32_t* restrict pi = Pu + (size_t)i * N;
            for (uint32_t s = 0; s < N; ++s) {
                sU[s] += (uint64_t)g[s] * di[s];
                sVv[s] += (uint64_t)g[s] * pi[s];
            }
        }
        for (uint32_t s = 0; s < N; ++s) {
            const uint32_t sv = sumV[s] + bred(sVv[s], Q, mu, sh);
            sumV[s] = min32(sv, sv - Q);
            out[s] = bred(sU[s], Q, mu, sh);
        }
    }
    ntt_inv32(sumV, N, Q, c->twi32, c->twip32, c->ninv32, c->ninvp32);
    sdd32(sumV, dct, N, Q, gBits, dg);
    for (uint32_t i = 0; i < dg; ++i) ntt_fwd32(dct + (size_t)i * N, N, Q, c->tw32, c->twp32);
    uint32_t* out = acc + (size_t)index * N;
    for (uint32_t s = 0; s < N; ++s) sU[s] = out[s];
    for (uint32_t i = 0; i < dg; ++i) {
        const uint32_t* restrict g = dct + (size_t)i * N;
        const uint32_t* restrict fi = f + (size_t)i * N;
        for (uint32_t s = 0; s < N; ++s) sU[s] += (uint64_t)g[s] * fi[s];
    }
    for (uint32_t s = 0; s < N; ++s) out[s] = bred(sU[s], Q, mu, sh);
}

/* EvalAcc (mk-acc-xzw.cpp:89-130 / mk-acc-xzw_B.cpp:103-132) on u32 words: the
 * loop of evalacc_one() with the same key combinations (xzw.cpp:322-325,
 * 375-378; xzw_B.cpp:311-314, 368-371), reduced once per slot. */
static int evalacc_one32(const orc_ctx* c, const uint64_t* evk, const uint32_t* pkey, const uint64_t* ct,
                         uint64_t* acc64, uint32_t* work) {
    const uint32_t N = c->p.N, k = c->p.k, n = c->p.n, dg = c->dg, Q = (uint32_t)c->p.Q;
    const uint32_t mu = c->b.mu, sh = c->b.sh;
    const uint64_t M = 2ull * N;
    uint32_t* acc = work;                         /* k*N */
    uint32_t* d = acc + (size_t)k * N;            /* dg*N */
    uint32_t* f = d + (size_t)dg * N;             /* dg*N */
    uint32_t* acctemp = f + (size_t)dg * N;       /* k*N */
    uint32_t* scratch = acctemp + (size_t)k * N;  /* (dg+2)*N u32 + 2N u64 */
    for (size_t s = 0; s < (size_t)k * N; ++s) {
        if (acc64[s] >= Q) return 2;
        acc[s] = (uint32_t)acc64[s];
    }
    for (uint32_t u = 0; u < k; ++u) {
        for (uint32_t i = 0; i < n; ++i) {
            uint64_t raw = ct[(size_t)u * n + i];
            uint64_t cval;
            if (c->p.method == ORC_XZW) {
                if (raw >= c->p.q) return 2;
                cval = raw * 2 * N / c->p.q;          /* mk-acc-xzw.cpp:110,125: floor(ct*2N/q) */
            } else {
                if (raw > M) return 2;
                cval = raw;                           /* mk-acc-xzw_B.cpp:119,124 */
            }
            uint32_t ipos = (uint32_t)(cval == M ? 0 : cval);
            uint32_t ineg = (uint32_t)(cval == 0 ? 0 : M - cval); /* ModSubFast(0 - c) mod 2N */
            if (ineg == M) ineg = 0;
            const uint32_t* restrict mono = c->mono32 + (size_t)ipos * N;
            const uint32_t* restrict monoN = c->mono32 + (size_t)ineg * N;
            const int first = (u == 0 && i == 0);
            for (uint32_t dgt = 0; dgt < dg; ++dgt) {
                for (uint32_t part = 0; part < 2; ++part) {
                    uint32_t* restrict out = (part == 0 ? d : f) + (size_t)dgt * N;
                    const uint64_t* restrict e1 = keyp(c, evk, u, 0, i, dgt, part);
                    if (c->p.method == ORC_XZW) {
                        const uint64_t* restrict e2 = keyp(c, evk, u, 1, i, dgt, part);
                        if (first) {
                            /* AddToAccXZW0 xzw.cpp:375-378: evs + ev1*(X^c-1) + ev2*(X^-c-1) */
                            const uint64_t* restrict es = keyp(c, evk, u, 0, n, dgt, part);
                            for (uint32_t s = 0; s < N; ++s)
                                out[s] = bred(es[s] + (uint64_t)(uint32_t)e1[s] * mono[s] + (uint64_t)(uint32_t)e2[s] * monoN[s], Q, mu, sh);
                        } else {
                            /* AddToAccXZW xzw.cpp:322-325: ev1 - ev2*(X^-c-1) - ev2
                             * = ev1 + ev2 * (Q - (X^-c - 1) - 1), a sum below 2 Q^2 */
                            for (uint32_t s = 0; s < N; ++s)
                                out[s] = bred(e1[s] + (uint64_t)(uint32_t)e2[s] * (Q - 1 - monoN[s]), Q, mu, sh);
                        }
                    } else {
                        if (first) {
                            /* AddToAccXZW0 xzw_B.cpp:368-371: evs + ev1*(X^c-1) */
                            const uint64_t* restrict es = keyp(c, evk, u, 0, n, dgt, part);
                            for (uint32_t s = 0; s < N; ++s) out[s] = bred(es[s] + (uint64_t)(uint32_t)e1[s] * mono[s], Q, mu, sh);
                        } else {
                            /* AddToAccXZW xzw_B.cpp:311-314: d = ev1 */
                            for (uint32_t s = 0; s < N; ++s) out[s] = (uint32_t)e1[s];
                        }
                    }
                }
            }
            if (first) {
                hbprod32(c, d, f, u, pkey, acc, scratch); /* acc is REPLACED (xzw.cpp:380) */
            } else {
                /* acctemp = acc * (X^c - 1); HbProd(acctemp); acc += acctemp (xzw.cpp:327-344) */
                for (uint32_t w = 0; w < k; ++w)
                    for (uint32_t s = 0; s < N; ++s)
                        acctemp[(size_t)w * N + s] = bred((uint64_t)acc[(size_t)w * N + s] * mono[s], Q, mu, sh);
                hbprod32(c, d, f, u, pkey, acctemp, scratch);
                for (size_t s = 0; s < (size_t)k * N; ++s) {
                    const uint32_t x = acc[s] + acctemp[s];
                    acc[s] = x >= Q ? x - Q : x;
                }
            }
        }
    }
    for (size_t s = 0; s < (size_t)k * N; ++s) acc64[s] = acc[s];
    return 0;
}

static int evalacc_one(const orc_ctx* c, const uint64_t* evk, const uint64_t* pkey, const uint64_t* ct,
                       uint64_t* acc, uint64_t* work) {
    const uint32_t N = c->p.N, k = c->p.k, n = c->p.n, dg = c->dg;
    const uint64_t Q = c->p.Q, M = 2ull * N;
    uint64_t* d = work;                          /* dg*N */
    uint64_t* f = d + (size_t)dg * N;            /* dg*N */
    uint64_t* acctemp = f + (size_t)dg * N;      /* k*N */
    uint64_t* scratch = acctemp + (size_t)k * N; /* (dg+2)*N */
    for (uint32_t u = 0; u < k; ++u) {
        for (uint32_t i = 0; i < n; ++i) {
            uint64_t raw = ct[(size_t)u * n + i];
            uint64_t cval;
            if (c->p.method == ORC_XZW) {
                if (raw >= c->p.q) return 2;
                cval = raw * 2 * N / c->p.q;          /* mk-acc-xzw.cpp:110,125: floor(ct*2N/q) */
            } else {
                if (raw > M) return 2;
                cval = raw;                           /* mk-acc-xzw_B.cpp:119,124 */
            }
            uint32_t ipos = (uint32_t)(cval == M ? 0 : cval);
            uint32_t ineg = (uint32_t)(cval == 0 ? 0 : M - cval); /* ModSubFast(0 - c) mod 2N */
            if (ineg == M) ineg = 0;
            const uint64_t* mono = c->mono + (size_t)ipos * N;
            const uint64_t* monoN = c->mono + (size_t)ineg * N;
            int first = (u == 0 && i == 0);
            for (uint32_t dgt = 0; dgt < dg; ++dgt) {
                for (uint32_t part = 0; part < 2; ++part) {
                    uint64_t* out = (part == 0 ? d : f) + (size_t)dgt * N;
                    const uint64_t* e1 = keyp(c, evk, u, 0, i, dgt, part);
                    if (c->p.method == ORC_XZW) {
                        const uint64_t* e2 = keyp(c, evk, u, 1, i, dgt, part);
                        if (first) {
                            /* AddToAccXZW0 xzw.cpp:375-378: evs + ev1*(X^c-1) + ev2*(X^-c-1) */
                            const uint64_t* es = keyp(c, evk, u, 0, n, dgt, part);
                            for (uint32_t s = 0; s < N; ++s)
                                out[s] = addmod(addmod(es[s], mm(&c->m, e1[s], mono[s]), Q),
                                                mm(&c->m, e2[s], monoN[s]), Q);
                        } else {
                            /* AddToAccXZW xzw.cpp:322-325: ev1 - ev2*(X^-c-1) - ev2 */
                            for (uint32_t s = 0; s < N; ++s)
                                out[s] = submod(submod(e1[s], mm(&c->m, e2[s], monoN[s]), Q), e2[s], Q);
                        }
                    } else {
                        if (first) {
                            /* AddToAccXZW0 xzw_B.cpp:368-371: evs + ev1*(X^c-1) */
                            const uint64_t* es = keyp(c, evk, u, 0, n, dgt, part);
                            for (uint32_t s = 0; s < N; ++s)
                                out[s] = addmod(es[s], mm(&c->m, e1[s], mono[s]), Q);
                        } else {
                            /* AddToAccXZW xzw_B.cpp:311-314: d = ev1 */
                            memcpy(out, e1, sizeof(uint64_t) * N);
                        }
                    }
                }
            }
            if (first) {
                hbprod(c, d, f, u, pkey, acc, scratch); /* acc is REPLACED (xzw.cpp:380) */
            } else {
                /* acctemp = acc * (X^c - 1); HbProd(acctemp); acc += acctemp (xzw.cpp:327-344) */
                for (uint32_t w = 0; w < k; ++w)
                    for (uint32_t s = 0; s < N; ++s)
                        acctemp[(size_t)w * N + s] = mm(&c->m, acc[(size_t)w * N + s], mono[s]);
                hbprod(c, d, f, u, pkey, acctemp, scratch);
                for (size_t s = 0; s < (size_t)k * N; ++s) acc[s] = addmod(acc[s], acctemp[s], Q);
            }
        }
    }
    return 0;
}

static size_t work_words(const orc_ctx* c) {
    /* 64-bit path in u64 words; the 32-bit path (u32 words) also holds the
     * accumulator and two u64 rows of lazy sums */
    return (size_t)c->p.N * (2 * c->dg + c->p.k + c->dg + 2) + (size_t)c->p.k * c->p.N + 2 * (size_t)c->p.N;
}

/* one gate through the word path of the context; pk32 = pkey narrowed (32-bit path) */
static int evalacc_dispatch(const orc_ctx* c, const uint64_t* evk, const uint64_t* pkey, const uint32_t* pk32,
                            const uint64_t* ct, uint64_t* acc, uint64_t* work) {
    if (c->w32) return evalacc_one32(c, evk, pk32, ct, acc, (uint32_t*)work);
    return evalacc_one(c, evk, pkey, ct, acc, work);
}

/* pkey as u32 words for the 32-bit path (NULL on the 64-bit path, or on a non-canonical word) */
static uint32_t* narrow_pkey(const orc_ctx* c, const uint64_t* pkey, int* bad) {
    *bad = 0;
    if (!c->w32) return NULL;
    const size_t w = (size_t)c->p.k * c->dg * c->p.N;
    uint32_t* p = (uint32_t*)malloc(sizeof(uint32_t) * w);
    for (size_t i = 0; i < w; ++i) {
        if (pkey[i] >= c->p.Q) *bad = 1;
        p[i] = (uint32_t)pkey[i];
    }
    return p;
}

int orc_evalacc(const orc_ctx* c, const uint64_t* evk, const uint64_t* pkey, const uint64_t* ct, uint64_t* acc) {
    if (!c) return 1;
    int bad;
    uint32_t* pk32 = narrow_pkey(c, pkey, &bad);
    uint64_t* work = (uint64_t*)malloc(sizeof(uint64_t) * work_words(c));
    int rc = bad ? 2 : evalacc_dispatch(c, evk, pkey, pk32, ct, acc, work);
    free(work);
    free(pk32);
    return rc;
}

int orc_evalacc_batch(const orc_ctx* c, const uint64_t* evk, const uint64_t* pkey, const uint64_t* ct,
                      uint64_t* acc, size_t B, int threads) {
    if (!c) return 1;
    int rc = 0;
    const size_t ctw = (size_t)c->p.k * c->p.n, accw = (size_t)c->p.k * c->p.N;
    int bad;
    uint32_t* pk32 = narrow_pkey(c, pkey, &bad);
    if (bad) {
        free(pk32);
        return 2;
    }
#ifdef _OPENMP
    if (threads < 1) threads = 1;
#pragma omp parallel num_threads(threads) reduction(| : rc)
    {
        uint64_t* work = (uint64_t*)malloc(sizeof(uint64_t) * work_words(c));
#pragma omp for schedule(dynamic, 1)
        for (long g = 0; g < (long)B; ++g)
            rc |= evalacc_dispatch(c, evk, pkey, pk32, ct + g * ctw, acc + g * accw, work);
        free(work);
    }
#else
    (void)threads;
    uint64_t* work = (uint64_t*)malloc(sizeof(uint64_t) * work_words(c));
    for (size_t g = 0; g < B; ++g) rc |= evalacc_dispatch(c, evk, pkey, pk32, ct + g * ctw, acc + g * accw, work);
    free(work);
#endif
    free(pk32);
    return rc;
}

/* ------------------------------------------------------------------------ */
/* test vectors                                                              */
/* ------------------------------------------------------------------------ */

static inline uint64_t splitmix64(uint64_t* s) {
    uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

/* Uniform in [0, bound) by 128-bit multiply-shift of a SplitMix64 stream
 * (bias < 2^-32 for bound < 2^32, irrelevant for bit-exactness tests). */
void orc_fill_uniform(uint64_t* out, size_t n, uint64_t bound, uint64_t seed) {
    uint64_t s = seed;
    for (size_t i = 0; i < n; ++i) out[i] = (uint64_t)(((u128)splitmix64(&s) * bound) >> 64);
}

void orc_fill_uniform_u32(uint32_t* out, size_t n, uint64_t bound, uint64_t seed) {
    uint64_t s = seed;
    for (size_t i = 0; i < n; ++i) out[i] = (uint32_t)(((u128)splitmix64(&s) * bound) >> 64);
}

/* BootstrapGateCore (MNTRU) test vector, binfhe-base-scheme.cpp:1085-1115:
 * Q2p = Q/(2p)+1; Rx[j] = j < N/2 ? Q - Q2p : Q2p; acc[0] = NTT(Rx); acc[u>0] = 0. */
void orc_mntru_testvector(const orc_ctx* c, uint64_t p, uint64_t* acc) {
    const uint32_t N = c->p.N;
    const uint64_t Q = c->p.Q, Q2p = Q / (2 * p) + 1, Q2pNeg = Q - Q2p;
    memset(acc, 0, sizeof(uint64_t) * (size_t)c->p.k * N);
    for (uint32_t j = 0; j < N; ++j) acc[j] = j < N / 2 ? Q2pNeg : Q2p;
    ntt_fwd_tab(acc, N, Q, c->tab);
}

/* ------------------------------------------------------------------------ */
/* Gate head and tail                                */
/* ------------------------------------------------------------------------ */

/* MNTRUEncryptionScheme::RoundqQ (mntru-pke.cpp:11-16) and the identical
 * MKLWEEncryptionScheme::RoundqQ: floor(0.5 + v * q / Q) in IEEE double,
 * left to right, then Mod(q). */
uint64_t orc_round_qQ(uint64_t v, uint64_t q, uint64_t Q) {
    double x = floor(0.5 + (double)v * (double)q / (double)Q);
    return ((uint64_t)x) % q;
}

/* MNTRU gate head, BinFHEScheme::EvalBinGate (binfhe-base-scheme.cpp:478-490):
 * ct_temp = ctNAND - (ct1 + ct2), element-wise mod q (EvalAddEq / EvalSubEq,
 * mntru-pke.cpp:826-838).  All arrays [k][n]. */
void orc_mntru_head(const uint64_t* ctNAND, const uint64_t* ct1, const uint64_t* ct2, uint64_t* out,
                    uint32_t k, uint32_t n, uint64_t q) {
    for (size_t i = 0; i < (size_t)k * n; ++i) out[i] = submod(ctNAND[i], addmod(ct1[i], ct2[i], q), q);
}

/* Extraction (binfhe-base-scheme.cpp:498-506 / :441-449): per party
 * accVec[u] = accVec[u].Transpose() then SetFormat(COEFFICIENT).
 * acc [k][N] EVAL -> out [k][N] COEFFICIENT. */
void orc_extract(const orc_ctx* c, const uint64_t* acc, uint64_t* out) {
    const uint32_t N = c->p.N;
    for (uint32_t u = 0; u < c->p.k; ++u) {
        orc_transpose_eval(acc + (size_t)u * N, out + (size_t)u * N, N);
        ntt_inv_tab(out + (size_t)u * N, N, c->p.Q, c->tabI, c->Ninv);
    }
}

static uint32_t ks_digits(uint64_t qKS, uint32_t baseKS) {
    /* static_cast<size_t>(std::ceil(log(qKS) / log(baseKS)))  (mntru-pke.cpp:771, mklwe-pke.cpp:266) */
    return (uint32_t)ceil(log((double)qKS) / log((double)baseKS));
}
uint32_t orc_ks_digits(uint64_t qKS, uint32_t baseKS) { return ks_digits(qKS, baseKS); }

/* MNTRUEncryptionScheme::KeySwitch2 (mntru-pke.cpp:763-823).
 *   ksk2 [k][Bks][N*dks][n] mod qKS (KSK2 of KeySwitchGen2, mntru-pke.cpp:744-755)
 *   ct   [k][N] mod qKS (ModSwitch output)
 *   out  [k][n] mod qKS                                                      */
void orc_keyswitch2(const uint64_t* ksk2, const uint64_t* ct, uint64_t* out, uint32_t k, uint32_t N, uint32_t n,
                    uint64_t qKS, uint32_t baseKS) {
    const uint32_t dks = ks_digits(qKS, baseKS);
    const size_t L = (size_t)N * dks;
    uint32_t* hat = (uint32_t*)malloc(L * sizeof(uint32_t));
    for (uint32_t u = 0; u < k; ++u) {
        for (uint32_t i = 0; i < N; ++i) {
            uint64_t t = ct[(size_t)u * N + i];
            for (uint32_t j = 0; j < dks; ++j) {
                hat[(size_t)i * dks + j] = (uint32_t)(t % baseKS);
                t /= baseKS;
            }
        }
        uint64_t* c = out + (size_t)u * n;
        memset(c, 0, n * sizeof(uint64_t));
        for (size_t l = 0; l < L; ++l) {
            const uint32_t index = hat[l];
            if (index == 0) continue;
            const uint64_t* row = ksk2 + (((size_t)u * baseKS + index) * L + l) * n;
            for (uint32_t i = 0; i < n; ++i) c[i] = addmod(c[i], row[i], qKS);
        }
    }
    free(hat);
}

/* Full MNTRU NAND gate after EvalAcc: extraction, ModSwitch(qKS)
 * (mntru-pke.cpp:359-374), KeySwitch2.  acc [k][N] EVAL -> out [k][n]. */
void orc_mntru_tail(const orc_ctx* c, const uint64_t* acc, const uint64_t* ksk2, uint64_t qKS, uint32_t baseKS,
                    uint32_t n_out, uint64_t* out) {
    const uint32_t N = c->p.N, k = c->p.k;
    uint64_t* ext = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)k * N);
    orc_extract(c, acc, ext);
    for (size_t i = 0; i < (size_t)k * N; ++i) ext[i] = orc_round_qQ(ext[i], qKS, c->p.Q);
    orc_keyswitch2(ksk2, ext, out, k, N, n_out, qKS, baseKS);
    free(ext);
}

/* orc_mntru_tail with the key given as KSK2[u][1] only ([k][N*dks][n]): the
 * row KeySwitch2 adds for digit j is KSK2[u][j][l] = j * KSK2[u][1][l] mod qKS,
 * exactly as KeySwitchGen2 stores the table (mntru-pke.cpp:744-755). */
void orc_mntru_tail_ksk1(const orc_ctx* c, const uint64_t* acc, const uint32_t* ksk1, uint64_t qKS,
                         uint32_t baseKS, uint32_t n_out, uint64_t* out) {
    const uint32_t N = c->p.N, k = c->p.k, dks = ks_digits(qKS, baseKS);
    const size_t L = (size_t)N * dks;
    uint64_t* ext = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)k * N);
    orc_extract(c, acc, ext);
    for (size_t i = 0; i < (size_t)k * N; ++i) ext[i] = orc_round_qQ(ext[i], qKS, c->p.Q);
    for (uint32_t u = 0; u < k; ++u) {
        uint64_t* o = out + (size_t)u * n_out;
        memset(o, 0, n_out * sizeof(uint64_t));
        for (uint32_t i = 0; i < N; ++i) {
            uint64_t t = ext[(size_t)u * N + i];
            for (uint32_t j = 0; j < dks; ++j) {
                const uint64_t index = t % baseKS;
                t /= baseKS;
                if (index == 0) continue;
                const uint32_t* row = ksk1 + ((size_t)u * L + (size_t)i * dks + j) * n_out;
                for (uint32_t x = 0; x < n_out; ++x) o[x] = addmod(o[x], index * row[x] % qKS, qKS);
            }
        }
    }
    free(ext);
}

/* MK-LWE gate head (binfhe-base-scheme.cpp:380-406, 1004-1065):
 *   ct_temp = (0, 5q/8) - (ct1 + ct2) mod q; ModSwitch to 2N (mklwe-pke.cpp:160-174);
 *   acc[0] = NTT(X^b * Rx), Rx[j] = j < N/2 ? Q/8+1 : Q - (Q/8+1)  (:1017-1043);
 *   c = GetAneg() = -a mod 2N (mklwe-ciphertext.h:86-96).
 * a1, a2 [k][n] mod q; outputs c [k][n] in [0, 2N], acc [k][N] EVAL. */
void orc_mklwe_head(const orc_ctx* c, const uint64_t* a1, uint64_t b1, const uint64_t* a2, uint64_t b2, uint64_t q,
                    uint32_t n, uint64_t p, uint64_t* cout, uint64_t* acc) {
    const uint32_t N = c->p.N, k = c->p.k;
    const uint64_t M = 2ull * N, Q = c->p.Q;
    const uint64_t b_tmp = submod((5 * q / 8) % q, addmod(b1, b2, q), q);
    const uint64_t bms = orc_round_qQ(b_tmp, M, q);
    for (size_t i = 0; i < (size_t)k * n; ++i) {
        const uint64_t at = submod(0, addmod(a1[i], a2[i], q), q);
        const uint64_t ams = orc_round_qQ(at, M, q);
        cout[i] = ams == 0 ? 0 : M - ams;              /* zero.ModSub(a) mod 2N */
    }
    const uint64_t Q2p = Q / (2 * p) + 1, Q2pNeg = Q - Q2p;
    const uint64_t bhat = bms * M / M;                 /* b*2N/q with q = 2N (:1026) */
    memset(acc, 0, sizeof(uint64_t) * (size_t)k * N);
    for (uint32_t j = 0; j < N; ++j) {
        const uint64_t rx = j < N / 2 ? Q2p : Q2pNeg;
        const uint64_t index = bhat + j;
        if (index >= N && index < 2ull * N) acc[index % N] = Q - rx;
        else acc[index % N] = rx;
    }
    ntt_fwd_tab(acc, N, Q, c->tab);
}

/* MKLWEEncryptionScheme::KeySwitch (mklwe-pke.cpp:260-298).
 *   A [k][N][Bks][dks][n], B [k][N][Bks][dks] mod qKS; a [k][N], b mod qKS.
 *   out_a [k][n], *out_b.                                                    */
void orc_mklwe_keyswitch(const uint64_t* A, const uint64_t* Bk, const uint64_t* a, uint64_t b, uint64_t* out_a,
                         uint64_t* out_b, uint32_t k, uint32_t N, uint32_t n, uint64_t qKS, uint32_t baseKS) {
    const uint32_t dks = ks_digits(qKS, baseKS);
    memset(out_a, 0, sizeof(uint64_t) * (size_t)k * n);
    for (uint32_t u = 0; u < k; ++u)
        for (uint32_t i = 0; i < N; ++i) {
            uint64_t t = a[(size_t)u * N + i];
            for (uint32_t j = 0; j < dks; ++j) {
                const uint64_t a0 = t % baseKS;
                t /= baseKS;
                const size_t e = (((size_t)u * N + i) * baseKS + a0) * dks + j;
                b = submod(b, Bk[e], qKS);
                const uint64_t* row = A + e * n;
                for (uint32_t l = 0; l < n; ++l) out_a[(size_t)u * n + l] = submod(out_a[(size_t)u * n + l], row[l], qKS);
            }
        }
    *out_b = b;
}

/* MK-LWE gate tail: extraction, b = Q/8 + 1 (binfhe-base-scheme.cpp:451),
 * ModSwitch(qKS), KeySwitch.  acc [k][N] EVAL -> out_a [k][n], *out_b. */
void orc_mklwe_tail(const orc_ctx* c, const uint64_t* acc, const uint64_t* A, const uint64_t* Bk, uint64_t qKS,
                    uint32_t baseKS, uint32_t n_out, uint64_t* out_a, uint64_t* out_b) {
    const uint32_t N = c->p.N, k = c->p.k;
    uint64_t* ext = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)k * N);
    orc_extract(c, acc, ext);
    for (size_t i = 0; i < (size_t)k * N; ++i) ext[i] = orc_round_qQ(ext[i], qKS, c->p.Q);
    const uint64_t b = orc_round_qQ((c->p.Q >> 3) + 1, qKS, c->p.Q);
    orc_mklwe_keyswitch(A, Bk, ext, b, out_a, out_b, k, N, n_out, qKS, baseKS);
    free(ext);
}
