/*
 * mkfhe_oracle.h -- CPU restatement of the SKLC-FHE/MKFHE multi-key
 * blind-rotation accumulator (TEST INFRASTRUCTURE ONLY).
 *
 * This library is the parity checker for the HIP engine in mkfhe_amd/.  Only
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it;
 * the product path never links or calls it.
 *
 * Pinning: the number-theory and NTT primitives are checked against the
 * known-answer vectors in the reference's own unit tests (see
 * tests/test_oracle_kat.py).  The accumulator composition (SDD, HbProd,
 * EvalAcc) is a restatement of the reference source cited per function; no
 * reference test covers it and the reference cannot be built in this image
 * (its headers need the cmake-generated config_core.h), so that part is
 * "parity unpinned" beyond the primitives -- see DESIGN.md section 3.
 *
 * All arrays are uint64_t words holding canonical residues; any Q < 2^62 works.
 */
#ifndef MKFHE_ORACLE_H
#define MKFHE_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- number theory (reference src/core/include/math/nbtheory-impl.h) ---- */
int      orc_is_prime(uint64_t n);
uint64_t orc_first_prime(uint32_t nbits, uint64_t m);     /* nbtheory-impl.h:334-357 */
uint64_t orc_previous_prime(uint64_t q, uint64_t m);      /* nbtheory-impl.h:369-377 */
uint64_t orc_next_prime(uint64_t q, uint64_t m);          /* nbtheory-impl.h:361-369 (0 on overflow) */
uint64_t orc_root_of_unity(uint64_t m, uint64_t Q);       /* nbtheory-impl.h:183-231 (minimal root) */
uint64_t orc_modinv(uint64_t a, uint64_t Q);
uint64_t orc_mulmod(uint64_t a, uint64_t b, uint64_t Q);
uint64_t orc_powmod(uint64_t a, uint64_t e, uint64_t Q);

/* ---- NativeVectorT element-wise ModAdd / ModSub / ModMul (mubintvecnat.cpp:235-350);
 *      op 0 add, 1 sub, 2 mul; inputs canonical residues mod Q < 2^62 ---- */
void orc_vec_mod(int op, const uint64_t* a, const uint64_t* b, uint64_t* out, size_t n, uint64_t Q);

/* ---- negacyclic NTT in the reference's EVALUATION order ----
 * forward: transformnat-impl.h:300-354 (CT, bit-reversed output)
 * inverse: transformnat-impl.h:492-552 (GS, N^-1 fused)          */
void orc_ntt_forward(uint64_t* a, uint32_t N, uint64_t Q, uint64_t psi);
void orc_ntt_inverse(uint64_t* a, uint32_t N, uint64_t Q, uint64_t psi);
/* PolyImpl::Transpose (poly-interface.h:443-450): automorphism 2N-1 in EVAL */
void orc_transpose_eval(const uint64_t* in, uint64_t* out, uint32_t N);
/* PolyImpl::AutomorphismTransform in COEFFICIENT form (poly-impl.h:312-365) */
void orc_automorphism_coeff(const uint64_t* in, uint64_t* out, uint32_t N, uint64_t Q, uint32_t k);

/* ---- UniEnc parameters (mk-cryptoparameters.h:124-181) ---- */
uint32_t orc_digits_g(uint64_t Q, uint32_t baseG);        /* ceil(log Q / log B_g), h:142 */

/* ---- approximate signed gadget decomposition (mk-acc.cpp:54-80) ----
 * out: dg = digitsG-1 polys of N residues                          */
void orc_sdd(const uint64_t* in, uint64_t* out, uint32_t N, uint64_t Q, uint32_t baseG, uint32_t dg);

/* ---- accumulator ---- */
enum { ORC_XZW = 0, ORC_XZW_B = 1 };

typedef struct orc_params {
    uint32_t method;   /* ORC_XZW (MKNTRU) or ORC_XZW_B (MKNTRU_B / MKNTRU_LWE) */
    uint32_t k;        /* parties */
    uint32_t n;        /* LWE dimension */
    uint32_t N;        /* ring dimension */
    uint64_t Q;        /* ring modulus */
    uint64_t q;        /* LWE modulus (XZW rescale c = ct*2N/q) */
    uint32_t baseG;    /* gadget base (power of two) */
    uint32_t digitsG;  /* total digits; dg = digitsG-1 are used */
    uint64_t psi;      /* primitive 2N-th root (reference: minimal root) */
} orc_params;

typedef struct orc_ctx orc_ctx;

orc_ctx* orc_ctx_create(const orc_params* p);
void     orc_ctx_destroy(orc_ctx* c);

/* Number of key polys: evk is [k][nk][n+1][dg][2][N] with nk = 2 (XZW) or 1 (XZW_B). */
size_t orc_evk_words(const orc_params* p);

/*
 * UniEncAccumulatorXZW{,_B}::EvalAcc (mk-acc-xzw.cpp:89-130, mk-acc-xzw_B.cpp:103-132).
 *   evk  [k][nk][n+1][dg][2][N]  EVAL form
 *   pkey [k][dg][N]              EVAL form
 *   ct   [k][n]                  raw ciphertext values (XZW: mod q; XZW_B: mod 2N)
 *   acc  [k][N]                  EVAL form, updated in place
 * Returns 0 on success, nonzero on a bad input.
 */
int orc_evalacc(const orc_ctx* c, const uint64_t* evk, const uint64_t* pkey,
                const uint64_t* ct, uint64_t* acc);

/* Same over B independent gates (ct [B][k][n], acc [B][k][N]) on `threads` host threads. */
int orc_evalacc_batch(const orc_ctx* c, const uint64_t* evk, const uint64_t* pkey,
                      const uint64_t* ct, uint64_t* acc, size_t B, int threads);

/* Test-vector helpers. SplitMix64 stream, uniform residues in [0, bound). */
void orc_fill_uniform(uint64_t* out, size_t n, uint64_t bound, uint64_t seed);
void orc_fill_uniform_u32(uint32_t* out, size_t n, uint64_t bound, uint64_t seed);
/* BootstrapGateCore MNTRU test vector (binfhe-base-scheme.cpp:1093-1115): acc[0] = NTT(Rx), acc[u>0] = 0 */
void orc_mntru_testvector(const orc_ctx* c, uint64_t p, uint64_t* acc);


/* ---- gate head / tail (binfhe-base-scheme.cpp:380-515, mntru-pke.cpp, mklwe-pke.cpp) ---- */
uint64_t orc_round_qQ(uint64_t v, uint64_t q, uint64_t Q);          /* RoundqQ, mntru-pke.cpp:11-16 */
uint32_t orc_ks_digits(uint64_t qKS, uint32_t baseKS);                 /* ceil(log qKS / log baseKS) */
void orc_mntru_head(const uint64_t* ctNAND, const uint64_t* ct1, const uint64_t* ct2, uint64_t* out,
                    uint32_t k, uint32_t n, uint64_t q);
void orc_extract(const orc_ctx* c, const uint64_t* acc, uint64_t* out);
void orc_keyswitch2(const uint64_t* ksk2, const uint64_t* ct, uint64_t* out, uint32_t k, uint32_t N, uint32_t n,
                    uint64_t qKS, uint32_t baseKS);
void orc_mntru_tail(const orc_ctx* c, const uint64_t* acc, const uint64_t* ksk2, uint64_t qKS, uint32_t baseKS,
                    uint32_t n_out, uint64_t* out);
/* same, with the key as KSK2[u][1] ([k][N*dks][n], u32); row j = j*KSK2[u][1] */
void orc_mntru_tail_ksk1(const orc_ctx* c, const uint64_t* acc, const uint32_t* ksk1, uint64_t qKS,
                         uint32_t baseKS, uint32_t n_out, uint64_t* out);
void orc_mklwe_head(const orc_ctx* c, const uint64_t* a1, uint64_t b1, const uint64_t* a2, uint64_t b2, uint64_t q,
                    uint32_t n, uint64_t p, uint64_t* cout, uint64_t* acc);
void orc_mklwe_keyswitch(const uint64_t* A, const uint64_t* Bk, const uint64_t* a, uint64_t b, uint64_t* out_a,
                         uint64_t* out_b, uint32_t k, uint32_t N, uint32_t n, uint64_t qKS, uint32_t baseKS);
void orc_mklwe_tail(const orc_ctx* c, const uint64_t* acc, const uint64_t* A, const uint64_t* Bk, uint64_t qKS,
                    uint32_t baseKS, uint32_t n_out, uint64_t* out_a, uint64_t* out_b);

#ifdef __cplusplus
}
#endif
#endif
