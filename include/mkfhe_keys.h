/*
 * mkfhe_keys.h -- C ABI of the host-side key material for the MK gate path:
 * key generation, encryption and decryption for MK-NTRU (MNTRU + XZW) and
 * MK-LWE (MKLWE + XZW_B), without NTL.
 *
 * Library: mkfhe_amd/lib/libmkfhe_keys.so (plain C++, CPU only; no GPU is
 * touched).  Its outputs are exactly the inputs of include/mkfhe_amd.h:
 *   evk/pkey        -> mkacc_upload_keys
 *   ksk (MK-NTRU)   -> mkacc_upload_ksk_mntru
 *   A/B (MK-LWE)    -> mkacc_upload_ksk_mklwe
 *   ciphertexts     -> mkacc_eval_nand_mntru / mkacc_eval_nand_mklwe
 *
 * What each entry point replaces in the reference (src/binfhe/lib/):
 *   mkkg_mntru_keygen   MNTRUEncryptionScheme::KeyGen / KeyGenGaussian +
 *                       Get_invertible_Matrix (mntru-pke.cpp:19-156; NTL's
 *                       mat_ZZ_p inv -> Gauss-Jordan mod q)
 *   mkkg_mklwe_keygen   MKLWEEncryptionScheme::KeyGenBinary (mklwe-pke.cpp:19-34)
 *   mkkg_crs            UniEncCryptoParams CRS (mk-cryptoparameters.h:173-178)
 *   mkkg_ring_secrets   Get_invertible_NativeVector (binfhe-base-scheme.cpp:104-195;
 *                       NTL's InvMod mod X^N+1 -> pointwise inverse in EVAL)
 *   mkkg_pkey           Pkey = e - CRS_i * s_u (binfhe-base-scheme.cpp:255-268, 318-331)
 *   mkkg_acc_keygen     UniEncAccumulatorXZW{,_B}::KeyGenAcc + KeyGenXZW /
 *                       KDMKeyGenXZW (mk-acc-xzw.cpp:38-87, 132-228;
 *                       mk-acc-xzw_B.cpp:38-101, 135-220)
 *   mkkg_ksk_mntru      MNTRUEncryptionScheme::KeySwitchGen2 (mntru-pke.cpp:624-760),
 *                       KSK2[u][1] (the engine derives KSK2[u][j] = j*KSK2[u][1])
 *   mkkg_ksk_mklwe      MKLWEEncryptionScheme::KeySwitchGen (mklwe-pke.cpp:176-258)
 *   mkkg_mntru_encrypt  MNTRUEncryptionScheme::Encrypt (mntru-pke.cpp:158-206)
 *   mkkg_mntru_ctgate   BinFHEScheme::ctGateGen(NAND) (binfhe-base-scheme.cpp:340-376)
 *   mkkg_mntru_decrypt  MNTRUEncryptionScheme::Decrypt / Decrypt2 / DecryptNAND
 *                       (mntru-pke.cpp:208-357)
 *   mkkg_mklwe_encrypt  MKLWEEncryptionScheme::Encrypt (mklwe-pke.cpp:36-64)
 *   mkkg_mklwe_decrypt  MKLWEEncryptionScheme::Decrypt / DecryptNAND (mklwe-pke.cpp:66-158)
 *
 * Sampling follows the reference's distributions (OpenFHE's Peikert-inversion
 * discrete Gaussian, std::normal_distribution truncated to an integer where
 * the reference assigns a double to an NTL ZZ_p, uniform ternary / binary).
 * The reference seeds from the clock, so its keys are not reproducible
 * (binfhe-base-scheme.cpp:111, mntru-pke.cpp:27).  Here every call takes a
 * 64-bit seed:
 *   seed != 0  reproducible test keys: xoshiro256** streams keyed by
 *              SplitMix64(seed) -- NOT a CSPRNG;
 *   seed == 0  fresh keys, the reference's behaviour: ChaCha20 streams under a
 *              256-bit call key derived from the process's entropy journal
 *              (a master key from std::random_device and a counter of seed-0
 *              calls).  After an explicit mkkg_entropy_replay(1) the master
 *              can be exported (mkkg_entropy_get) or taken from MKFHE_ENTROPY,
 *              so a run with a wrong gate can be replayed exactly
 *              (tools/fresh_key_rate.py --replay).
 * Outputs are independent of the thread count.
 *
 * Layouts (row-major, canonical residues):
 *   F, Finv  [k][n][n] mod qKS: F[u][l][j] = row l, column j of party u's
 *            matrix (MNTRUPrivateKeyImpl m_F / m_F_inv); F_col0[u][l] = F[u][l][0]
 *   s (LWE)  [k][n] mod q (MKLWEPrivateKeyImpl)
 *   skN      [k][N] mod Q, COEFF (UniEncBTKey::fvec); skN_eval / skNinv_eval EVAL
 *   crs      [dg][N] EVAL, dg = digitsG - 1
 *   pkey     [k][dg][N] EVAL;  evk [k][nk][n+1][dg][2][N] EVAL (mkfhe_amd.h)
 *   MNTRU ct [count][k][n] mod q;  MKLWE a [count][k][n], b [count] mod q
 *   EVAL is the reference's bit-reversed NTT order (mkfhe_amd.h).
 * Status codes are those of mkfhe_amd.h (MKACC_OK / MKACC_E_*).
 */
#ifndef MKFHE_KEYS_H
#define MKFHE_KEYS_H

#include <stddef.h>
#include <stdint.h>

#include "mkfhe_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

#define MKKG_ABI_VERSION 3

/* SecretKeyDist values used by the MK parameter sets (binfhe-constants.h) */
#define MKKG_DIST_TERNARY  0  /* UNIFORM_TERNARY */
#define MKKG_DIST_GAUSSIAN 1  /* GAUSSIAN        */
#define MKKG_DIST_BINARY   2  /* BINARY          */

/* Decryption variants of MNTRUEncryptionScheme (mntru-pke.cpp:208-357) */
#define MKKG_DECRYPT      0  /* Decrypt:     floor(p * (<c,F_col0> + q/p) / q)        */
#define MKKG_DECRYPT2     1  /* Decrypt2:    floor(p * (<c,F_col0> + q/(2p)) / q)     */
#define MKKG_DECRYPT_NAND 2  /* DecryptNAND: floor(p/2 * (<c,F_col0> + q/(p/2*2)) / q) */

typedef struct mkkg_params {
    mkacc_params acc;     /* accumulator parameters (method, k, n, N, Q, q, baseG, digitsG, root) */
    mkacc_ks_params ks;   /* key switching (qKS, baseKS, n_out = n) */
    double sigma;         /* stdDev column: MNTRU/MKLWE dgg and dggKS (binfhecontext.cpp:85-87) */
    double sigma_unienc;  /* UniEncCryptoParams m_dgg  = 0.25 (mk-cryptoparameters.h:143) */
    double sigma_r;       /* UniEncCryptoParams m_dggR = 0.15 (mk-cryptoparameters.h:144) */
    uint32_t lwe_keydist; /* MKKG_DIST_*: keyDist column (MNTRU_KeyGen / MKLWE_KeyGen) */
    uint32_t ring_keydist;/* MKKG_DIST_*: ring secret s_u (GAUSSIAN for MKNTRU, TERNARY for MKNTRU_LWE) */
} mkkg_params;

/* Fill *out for a named MK parameter set (binfhecontext.cpp:129-144) and a
 * method (MKACC_METHOD_*): GenerateBinFHEContext(set, method). */
int mkkg_paramset(const char* name, uint32_t method, mkkg_params* out);

/* Word counts of the buffers below for *p. */
size_t mkkg_evk_words(const mkkg_params* p);   /* k * nk * (n+1) * dg * 2 * N */
size_t mkkg_pkey_words(const mkkg_params* p);  /* k * dg * N */
size_t mkkg_ksk_mntru_words(const mkkg_params* p);   /* k * N * dks * n */
size_t mkkg_ksk_mklwe_a_words(const mkkg_params* p); /* k * N * baseKS * dks * n */
size_t mkkg_ksk_mklwe_b_words(const mkkg_params* p); /* k * N * baseKS * dks */

/* ---- secret keys -------------------------------------------------------- */
/* MNTRU_KeyGen: k invertible n x n matrices mod qKS and their inverses. */
int mkkg_mntru_keygen(const mkkg_params* p, uint64_t seed, uint32_t* F, uint32_t* Finv);
/* MKLWE_KeyGen: k binary vectors of length n (mod qKS). */
int mkkg_mklwe_keygen(const mkkg_params* p, uint64_t seed, uint32_t* s);

/* ---- bootstrapping key (MKBTKeyGen) --------------------------------------- */
/* Common reference string: dg polys sampled from m_dgg, EVAL. */
int mkkg_crs(const mkkg_params* p, uint64_t seed, uint32_t* crs);
/* k invertible ring secrets s_u: COEFF, EVAL and EVAL inverse. */
int mkkg_ring_secrets(const mkkg_params* p, uint64_t seed, uint32_t* skN, uint32_t* skN_eval,
                      uint32_t* skNinv_eval);
/* Pkey[u][i] = NTT(e) - CRS[i] * s_u (EVAL). */
int mkkg_pkey(const mkkg_params* p, uint64_t seed, const uint32_t* crs, const uint32_t* skN_eval, uint32_t* pkey);
/* KeyGenAcc: uni-encryptions of the LWE secret bits (lwe_sk [k][n] mod q:
 * F_col0 for MK-NTRU, s for MK-LWE) under 1/s_u. */
int mkkg_acc_keygen(const mkkg_params* p, uint64_t seed, const uint32_t* crs, const uint32_t* skNinv_eval,
                    const uint32_t* lwe_sk, uint32_t* evk);
/* Same with a policy for the reference's r-defect: KeyGenXZW / KDMKeyGenXZW
 * (mk-acc-xzw.cpp:141-167, mk-acc-xzw_B.cpp:135-220) put the DggR sample r into
 * f as the polynomial g_t*r but into d only as the scalar r^[t]*CRS_t, so the
 * r-terms cancel in HbProd only when r = 0; a key with r != 0 (about 9e-7 per
 * key, 2.8e-3 per STD128_MKNTRU key set) can break every gate that uses it.
 *   MKKG_RDEFECT_KEEP     the reference's keys bit for bit (mkkg_acc_keygen);
 *   MKKG_RDEFECT_REJECT   same keys, but MKKG_E_RDEFECT if any key has r != 0;
 *   MKKG_RDEFECT_RESAMPLE redraw r from the slot's stream until it is zero
 *                         (deviates from the reference only in affected slots).
 * *defective (may be NULL) = the number of keys that drew r != 0 (under RESAMPLE:
 * the number of slots that were redrawn). */
#define MKKG_RDEFECT_KEEP     0u
#define MKKG_RDEFECT_REJECT   1u
#define MKKG_RDEFECT_RESAMPLE 2u
#define MKKG_E_RDEFECT      -20  /* REJECT: a bootstrapping key drew r != 0 (keys are still written) */
int mkkg_acc_keygen_ex(const mkkg_params* p, uint64_t seed, const uint32_t* crs, const uint32_t* skNinv_eval,
                       const uint32_t* lwe_sk, uint32_t* evk, uint32_t rdefect_policy, uint64_t* defective);
/* KeySwitchGen2 (MK-NTRU): ksk [k][N*dks][n] = KSK2[u][1]. */
int mkkg_ksk_mntru(const mkkg_params* p, uint64_t seed, const uint32_t* skN, const uint32_t* Finv, uint32_t* ksk);
/* KeySwitchGen (MK-LWE): A [k][N][baseKS][dks][n], B [k][N][baseKS][dks]. */
int mkkg_ksk_mklwe(const mkkg_params* p, uint64_t seed, const uint32_t* skN, const uint32_t* s, uint32_t* A,
                   uint32_t* B);

/* ---- encryption / decryption ------------------------------------------------ */
/* count MNTRU encryptions of m[i] (plaintext modulus pt, reference default 4). */
int mkkg_mntru_encrypt(const mkkg_params* p, uint64_t seed, const uint32_t* Finv, const uint32_t* m, uint32_t pt,
                       size_t count, uint32_t* ct);
/* ctGateGen(sk, NAND): the encryption of 5q/8 the NAND head subtracts from. */
int mkkg_mntru_ctgate(const mkkg_params* p, uint64_t seed, const uint32_t* Finv, uint32_t* ct_nand);
/* count MNTRU decryptions (variant MKKG_DECRYPT*; ct modulus `mod`, 0 = q). */
int mkkg_mntru_decrypt(const mkkg_params* p, const uint32_t* F, const uint32_t* ct, uint64_t mod, uint32_t pt,
                       uint32_t variant, size_t count, uint32_t* m);
int mkkg_mklwe_encrypt(const mkkg_params* p, uint64_t seed, const uint32_t* s, const uint32_t* m, uint32_t pt,
                       size_t count, uint32_t* a, uint32_t* b);
/* variant MKKG_DECRYPT (Decrypt, + q/(2p)) or MKKG_DECRYPT_NAND (DecryptNAND). */
int mkkg_mklwe_decrypt(const mkkg_params* p, const uint32_t* s, const uint32_t* a, const uint32_t* b, uint64_t mod,
                       uint32_t pt, uint32_t variant, size_t count, uint32_t* m);

/* ---- key wire format ------------------------------------
 * The reference has no serialization for the MK key types (binfhecontext-ser.h
 * registers the single-key schemes only).  A key file is little-endian:
 *   "MKFHEKEY" | u32 version (1) | u32 kind (MKKG_FILE_*) |
 *   parameter block: 18 x u64 (every mkkg_params field; doubles as IEEE bits) |
 *   u32 section count | per section: char name[16], u64 words, u32 data[words],
 *   u64 FNV-1a of the data bytes
 * so a file names the exact context it belongs to.  Readers reject a bad magic,
 * version, truncated data or checksum with MKACC_E_ARG. */
#define MKKG_FILE_MNTRU_SK   1  /* F, Finv                                                  */
#define MKKG_FILE_MKLWE_SK   2  /* s                                                        */
#define MKKG_FILE_BTKEY      3  /* crs, skN, skN_eval, skNinv, pkey, evk + ksk | ksk_a, ksk_b */
#define MKKG_FILE_CIPHERTEXT 4  /* ct (MNTRU) | a, b (MKLWE)                                 */

typedef struct mkkg_section {
    char name[16];         /* NUL-padded */
    uint64_t words;
    const uint32_t* data;  /* source of mkkg_file_write */
} mkkg_section;

int mkkg_file_write(const char* path, uint32_t kind, const mkkg_params* p, const mkkg_section* sections,
                    uint32_t count);
/* kind, parameters and section count of a file (any output may be NULL). */
int mkkg_file_info(const char* path, uint32_t* kind, mkkg_params* p, uint32_t* count);
/* words of section `name`; 0 if the file has no such section or is unreadable. */
uint64_t mkkg_file_section_words(const char* path, const char* name);
/* read section `name` (exactly `words` words) into out, verifying its checksum. */
int mkkg_file_read_section(const char* path, const char* name, uint32_t* out, uint64_t words);

/* ---- host ring transform (the reference's EVAL order), for tests ------------ */
int mkkg_ntt_forward(const mkkg_params* p, const uint32_t* in, uint32_t* out, size_t count);
int mkkg_ntt_inverse(const mkkg_params* p, const uint32_t* in, uint32_t* out, size_t count);

/* ---- seed-0 entropy journal --------------------------------------------------
 * WHOEVER HOLDS THE MASTER HOLDS EVERY SEED-0 KEY AND CIPHERTEXT OF THE PROCESS.
 * Exporting or importing it is therefore an explicit opt-in; by default the
 * master is drawn from std::random_device, MKFHE_ENTROPY is not read and
 * mkkg_entropy_get fails.
 * master: 8 words = 64 hex digits, word 0 first.
 * mkkg_entropy_replay(1): opt in.  If MKFHE_ENTROPY is set, the journal
 *   restarts at that master (MKACC_E_ARG, and no opt-in, if it is not 64 hex
 *   digits, or if a seed-0 call has already drawn from another master: a
 *   restarted counter would reuse earlier call keys; the same master keeps its
 *   counter); otherwise the current master stays.  mkkg_entropy_replay(0)
 *   opts out again (the master stays, it is just no longer exported).
 * mkkg_entropy_get: the master (drawn now if no seed-0 call has drawn it yet)
 *   and the number of seed-0 calls made since it was set; MKACC_E_ARG unless
 *   the journal was opted in.
 * mkkg_entropy_set: restart the journal at (master, calls) and opt in; master
 *   NULL draws a fresh master from std::random_device. */
int mkkg_entropy_replay(int enable);
int mkkg_entropy_get(uint32_t master[8], uint64_t* calls);
int mkkg_entropy_set(const uint32_t master[8], uint64_t calls);

const char* mkkg_last_error(void);
int mkkg_abi_version(void);
/* "abi=..;header=<id>;source=<id>;flags=": SHA-256 prefixes of mkfhe_keys.h +
 * mkfhe_amd.h and of the library's sources (mkfhe_amd/build.py). */
const char* mkkg_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* MKFHE_KEYS_H */
