/* fp64_modmul_check.c -- host check of the exact FP64 modular product used by
 * the FP64 variant of the 64-bit word path (Q < 2^50), against __int128.
 *
 *   mm(a, b):  h = a*b;  l = fma(a, b, -h);  q = rint(h * Qi);  r = fma(-q, Q, h) + l
 *
 * a, b are exact integers held in doubles (signed, balanced).  h - q Q is an
 * integer below 2^53 in magnitude, so the fma is exact; l is the exact low part
 * of a*b, so r = a*b - q*Q exactly.  The check asserts r == a*b - q*Q (no
 * rounding anywhere) and records max |r| / Q over random operands drawn up to
 * the input bounds |a| <= A*Q, |b| <= B*Q the butterflies rely on, plus the
 * extreme corners.  The same arithmetic runs on the GPU (IEEE binary64 fma /
 * rint are exact-rounded on both).
 *
 *   gcc -O2 -ffp-contract=off -o /tmp/fp64chk tools/fp64_modmul_check.c -lm && /tmp/fp64chk
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef __int128 i128;

static uint64_t s[4] = {0x9E3779B97F4A7C15ull, 0xBF58476D1CE4E5B9ull, 0x94D049BB133111EBull, 0x2545F4914F6CDD1Dull};
static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
static uint64_t rnd(void) {
    const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
    return r;
}
/* uniform integer in [-M, M] */
static double pick(double M) {
    const uint64_t m = (uint64_t)M;
    return (double)(int64_t)(rnd() % (2 * m + 1)) - (double)m;
}

static int check(double Q, double A, double B, long n, double* worst) {
    const double Qi = 1.0 / Q;
    int bad = 0;
    for (long i = 0; i < n + 16; ++i) {
        double a, b;
        if (i < 16) {   /* corners */
            a = ((i & 1) ? -1 : 1) * floor(A * Q);
            b = ((i & 2) ? -1 : 1) * floor(B * Q);
            if (i & 4) a = ((i & 1) ? -1 : 1) * floor(A * Q / 2 + 0.5);
            if (i & 8) b = ((i & 2) ? -1 : 1) * floor(B * Q / 2 + 0.5);
        } else {
            a = pick(A * Q);
            b = pick(B * Q);
        }
        const double h = a * b;
        const double l = fma(a, b, -h);
        const double q = rint(h * Qi);
        const double r = fma(-q, Q, h) + l;
        const i128 exact = (i128)(int64_t)a * (int64_t)b - (i128)(int64_t)q * (int64_t)Q;
        if ((i128)(int64_t)r != exact || fabs(r) >= 9007199254740992.0) {
            if (bad++ < 5) printf("  MISMATCH a=%.0f b=%.0f r=%.0f\n", a, b, r);
        }
        const double m = fabs(r) / Q;
        if (m > *worst) *worst = m;
    }
    return bad;
}

int main(void) {
    /* config 5 stress modulus and the largest prime of the FP64 range below 2^50 */
    const double Qs[] = {1125899906826241.0, 1125899906629633.0, 134176769.0};
    /* (A, B): operand bounds in units of Q -- twiddle/key products with a
     * lazily reduced data word, and data x data */
    const double AB[][2] = {{8, 0.5}, {4, 1}, {2, 2}, {1, 1}, {0.5, 0.5}};
    int bad = 0;
    for (int qi = 0; qi < 3; ++qi)
        for (int k = 0; k < 5; ++k) {
            double worst = 0;
            const int b = check(Qs[qi], AB[k][0], AB[k][1], 2000000, &worst);
            printf("Q=%.0f |a|<=%.1fQ |b|<=%.1fQ: %s, max |r| = %.3f Q\n", Qs[qi], AB[k][0], AB[k][1],
                   b ? "FAIL" : "exact", worst);
            bad += b;
        }
    return bad ? 1 : 0;
}
