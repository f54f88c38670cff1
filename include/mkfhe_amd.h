/*
 * mkfhe_amd.h -- C ABI of the MI355X multi-key blind-rotation accumulator.
 *
 * Drop-in boundary for the reference's plugin seam
 *   class UniEncAccumulator { virtual void EvalAcc(params, ek, Pkey, skf, acc, ct) const; }
 *   (reference src/binfhe/include/mk-acc.h:55-80; concrete classes
 *    UniEncAccumulatorXZW   src/binfhe/lib/mk-acc-xzw.cpp:89-130   (MKNTRU)
 *    UniEncAccumulatorXZW_B src/binfhe/lib/mk-acc-xzw_B.cpp:103-132 (MKNTRU_B, MKNTRU_LWE),
 *    chosen by BinFHEScheme(BINFHE_METHOD) at binfhe-base-scheme.h:137-151).
 *
 * Plain pointers and sizes only.  The caller owns host buffers; a context owns
 * its device buffers and one HIP stream (calls on one context are serialised).
 * Every function returns MKACC_OK (0) or a negative MKACC_E* status; the text
 * of the last error on the calling thread is available from mkacc_last_error().
 * The C++ host layer (include/mkfhe_amd_binfhe.hpp) converts a status into the
 * reference's exception types (OPENFHE_THROW config_error / math_error,
 * reference src/core/include/utils/exception.h:162).
 *
 * Polynomial layouts at this boundary are the reference's:
 *   EVAL  = NativePoly in Format::EVALUATION, i.e. the bit-reversed output of
 *           ForwardTransformToBitReverseInPlace (transformnat-impl.h:300-354)
 *           with the minimal primitive 2N-th root of unity;
 *   COEFF = Format::COEFFICIENT.
 * All words are canonical residues in [0, Q).
 */
#ifndef MKFHE_AMD_H
#define MKFHE_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MKACC_ABI_VERSION 2

/* status codes */
#define MKACC_OK            0
#define MKACC_E_ARG        -1  /* bad argument / shape (reference: config_error) */
#define MKACC_E_UNSUPPORTED -2 /* parameter set outside what the engine supports */
#define MKACC_E_NOKEYS     -3  /* EvalAcc before keys were uploaded (binfhe-base-scheme.cpp:1075-1080) */
#define MKACC_E_DEVICE     -4  /* HIP runtime error */
#define MKACC_E_RANGE      -5  /* an input word is not a canonical residue */

/* BINFHE_METHOD values that reach the accumulator (binfhe-constants.h:129-137) */
#define MKACC_METHOD_MKNTRU     0  /* UniEncAccumulatorXZW   */
#define MKACC_METHOD_MKNTRU_B   1  /* UniEncAccumulatorXZW_B */
#define MKACC_METHOD_MKNTRU_LWE 2  /* UniEncAccumulatorXZW_B */

/* Mirrors the UniEncCryptoParams fields EvalAcc reads
 * (mk-cryptoparameters.h:124-181). */
typedef struct mkacc_params {
    uint32_t method;   /* MKACC_METHOD_* */
    uint32_t k;        /* number of parties (numUser) */
    uint32_t n;        /* LWE / NTRU dimension (latticeParam) */
    uint32_t N;        /* ring dimension; the engine supports N = 2048 */
    uint64_t Q;        /* ring modulus, prime, Q = 1 mod 2N, 2^26 < Q < 2^61: Q < 2^27 runs the 32-bit
                          register-resident kernel, larger Q the 64-bit word path (EvalAcc only) */
    uint64_t q;        /* ciphertext modulus (mod); XZW computes c = floor(ct*2N/q) */
    uint32_t baseG;    /* gadget base B_g, power of two */
    uint32_t digitsG;  /* 0 = derive ceil(log Q / log B_g) as the reference does */
    uint64_t root;     /* 0 = derive the minimal primitive 2N-th root (ilparams.h:90-91) */
} mkacc_params;

typedef struct mkacc_ctx mkacc_ctx;

/* Parameter-set table (binfhecontext.cpp:129-144).  Fills *out for the named
 * set (e.g. "STD128_MKNTRU", "STD100_MKNTRU_LWE_2") with Q derived as
 * PreviousPrime(FirstPrime(27, 4096), 4096).  method selects MKNTRU/…_B/…_LWE. */
int mkacc_paramset(const char* name, uint32_t method, mkacc_params* out);

/* Create a context on HIP device `device`; derives digitsG / root when 0. */
int mkacc_create(const mkacc_params* p, int device, mkacc_ctx** out);
void mkacc_destroy(mkacc_ctx* ctx);

/* Effective parameters (digitsG and root filled in). */
int mkacc_get_params(const mkacc_ctx* ctx, mkacc_params* out);

/* Element counts of the boundary arrays. */
size_t mkacc_evk_words(const mkacc_ctx* ctx);   /* k * nk * (n+1) * (digitsG-1) * 2 * N, nk = 2 (XZW) / 1 (XZW_B) */
size_t mkacc_pkey_words(const mkacc_ctx* ctx);  /* k * (digitsG-1) * N */

/*
 * Upload the accumulator keys (UniEncACCKeyImpl, mk-acckey.h:44-51) and the
 * public "Pkey" polynomials that BinFHEScheme passes to EvalAcc.
 *   evk  [k][nk][n+1][dg][2][N]  EVAL   -- (*ek)[u][j][i] -> GetElements()[digit][0|1]
 *   pkey [k][dg][N]              EVAL
 * Keys are converted once into the device layout.  Re-uploading replaces them.
 */
int mkacc_upload_keys(mkacc_ctx* ctx, const uint32_t* evk, const uint32_t* pkey);
int mkacc_upload_keys_u64(mkacc_ctx* ctx, const uint64_t* evk, const uint64_t* pkey);
/* Same from DEVICE memory on the context's device (word_bytes 4 or 8), e.g. the
 * buffer a multi-GPU run received from the one-time key broadcast: the layout
 * conversion runs on the GPU, keys never return to the host.  Synchronous;
 * MKACC_E_RANGE (and no keys) if a word is not a canonical residue. */
int mkacc_upload_keys_device(mkacc_ctx* ctx, const void* d_evk, const void* d_pkey, uint32_t word_bytes);

/*
 * EvalAcc over a batch of B independent gates (host buffers, synchronous).
 *   ct      [B][k][n]  raw ciphertext words: XZW mod q (MNTRU GetElements()),
 *                      XZW_B mod 2N (MK-LWE GetAneg() after ModSwitch to 2N)
 *   acc_in  [B][k][N]  EVAL, the initial accumulator (BootstrapGateCore test vector)
 *   acc_out [B][k][N]  EVAL, the accumulator after EvalAcc; may alias acc_in
 * Equivalent to calling the reference EvalAcc once per gate.
 */
int mkacc_eval_batch(mkacc_ctx* ctx, const uint32_t* ct, const uint32_t* acc_in, uint32_t* acc_out, size_t B);
/* Same with 64-bit accumulator words (NATIVE_SIZE=64, NativeInteger of 64 bits):
 * required when Q >= 2^32; valid for every context. */
int mkacc_eval_batch_u64(mkacc_ctx* ctx, const uint32_t* ct, const uint64_t* acc_in, uint64_t* acc_out, size_t B);
/* Nonzero if the context runs the 64-bit word path (mkfhe_amd/csrc/mkacc_wide.hpp):
 * then mkacc_eval_batch_device takes uint64_t accumulators and the gate calls are
 * unsupported.  1: integer kernels; 2: the FP64 kernels (mkacc_widefp.hpp, Q < 2^50). */
int mkacc_is_wide(const mkacc_ctx* ctx);
/* Name of the batch step kernel a context launches for B gates (diagnostics:
 * bench.py's roofline record and kernel-trace matching), e.g. "mk_step2_kernel";
 * a static string, "" for a null context. */
const char* mkacc_step_kernel_name(const mkacc_ctx* ctx, size_t B);

/* Same with DEVICE pointers on the context's device; enqueued on the context
 * stream and returns without waiting (use mkacc_sync).  Used by bench.py so
 * the timed region starts with inputs resident in HBM.  Input words are
 * range-checked by the kernels that read them; a violation is reported by the
 * next mkacc_sync (MKACC_E_RANGE), and the outputs of that batch are garbage
 * (never an out-of-bounds access: monomial exponents are masked to [0, 2N)). */
int mkacc_eval_batch_device(mkacc_ctx* ctx, const uint32_t* d_ct, const uint32_t* d_acc_in,
                            uint32_t* d_acc_out, size_t B);
int mkacc_sync(mkacc_ctx* ctx);   /* waits for the stream; reports device-side input-range errors */

/* The context's HIP stream (hipStream_t as void*), for event timing. */
void* mkacc_stream(mkacc_ctx* ctx);

/* ---- gate level: head + EvalAcc + tail -------------------------------------
 * BinFHEScheme::EvalBinGate for MK-NTRU (binfhe-base-scheme.cpp:467-515) and
 * MK-LWE (binfhe-base-scheme.cpp:380-463): gate head, BootstrapGateCore
 * (test vector + EvalAcc, :1004-1130), extraction (Transpose + iNTT,
 * :498-506 / :441-449), ModSwitch to qKS (RoundqQ in double,
 * mntru-pke.cpp:11-16, 359-374) and the key switch (KeySwitch2,
 * mntru-pke.cpp:763-823 / KeySwitch, mklwe-pke.cpp:260-298).
 * Only NAND is supported, as in the reference (ctGateGen, :340-376). */
typedef struct mkacc_ks_params {
    uint64_t qKS;      /* key-switching modulus (modKS; 45181 / 32749 in every MK set) */
    uint32_t baseKS;   /* key-switching digit base (baseKS = 32); at most 256 */
    uint32_t n_out;    /* dimension of the output ciphertext (latticeParam n) */
} mkacc_ks_params;

/* Digits per coefficient: ceil(log qKS / log baseKS) (mntru-pke.cpp:771). */
uint32_t mkacc_ks_digits(const mkacc_ks_params* ks);

/* MK-NTRU KeySwitch2 key.  ksk [k][N*dks][n_out] = KSK2[u][1] of
 * KeySwitchGen2 (mntru-pke.cpp:744-755); the engine relies on
 * KSK2[u][j] = j * KSK2[u][1] mod qKS, which KeySwitchGen2 guarantees. */
int mkacc_upload_ksk_mntru(mkacc_ctx* ctx, const mkacc_ks_params* ks, const uint32_t* ksk);
/* MK-LWE KeySwitch key (mklwe-pke.cpp:176-258): A [k][N][baseKS][dks][n_out],
 * B [k][N][baseKS][dks] (GetElementsA / GetElementsB). */
int mkacc_upload_ksk_mklwe(mkacc_ctx* ctx, const mkacc_ks_params* ks, const uint32_t* A, const uint32_t* B);

/* Same two uploads from DEVICE memory on the context's device (u32 words in the
 * layouts above), e.g. the buffer of the one-time key broadcast of a multi-GPU
 * run: converted on the GPU, no host round trip.  Synchronous; MKACC_E_RANGE
 * (and no key-switching keys) if a word is not a canonical residue mod qKS. */
int mkacc_upload_ksk_mntru_device(mkacc_ctx* ctx, const mkacc_ks_params* ks, const void* d_ksk);
int mkacc_upload_ksk_mklwe_device(mkacc_ctx* ctx, const mkacc_ks_params* ks, const void* d_A, const void* d_B);

/* B NAND gates, MK-NTRU.  ct_nand [k][n] (ctGateGen), ct1/ct2 [B][k][n] mod q
 * -> out [B][k][n_out] mod qKS.  Host buffers, synchronous. */
int mkacc_eval_nand_mntru(mkacc_ctx* ctx, const uint32_t* ct_nand, const uint32_t* ct1, const uint32_t* ct2,
                          uint32_t* out, size_t B);
/* B NAND gates, MK-LWE.  a1/a2 [B][k][n], b1/b2 [B] mod q
 * -> out_a [B][k][n_out], out_b [B] mod qKS.  Host buffers, synchronous. */
int mkacc_eval_nand_mklwe(mkacc_ctx* ctx, const uint32_t* a1, const uint32_t* b1, const uint32_t* a2,
                          const uint32_t* b2, uint32_t* out_a, uint32_t* out_b, size_t B);
/* Device-pointer form of both (ct_nand unused for MK-LWE, b1/b2/out_b unused
 * for MK-NTRU); enqueued on the context stream. */
int mkacc_eval_nand_device(mkacc_ctx* ctx, const uint32_t* d_ct_nand, const uint32_t* d_a1, const uint32_t* d_b1,
                           const uint32_t* d_a2, const uint32_t* d_b2, uint32_t* d_out_a, uint32_t* d_out_b,
                           size_t B);
/* The tail alone on B accumulators acc [B][k][N] (EVAL, reference order):
 * extraction + ModSwitch + key switch -> out_a [B][k][n_out] (+ out_b [B]). */
int mkacc_gate_tail(mkacc_ctx* ctx, const uint32_t* acc, uint32_t* out_a, uint32_t* out_b, size_t B);

/* ---- primitives exposed for parity tests (same layouts as above) ---- */
/* NativePoly::SetFormat(EVALUATION) on `count` polys: COEFF -> EVAL. */
int mkacc_ntt_forward(mkacc_ctx* ctx, const uint32_t* in, uint32_t* out, size_t count);
/* NativePoly::SetFormat(COEFFICIENT) on `count` polys: EVAL -> COEFF. */
int mkacc_ntt_inverse(mkacc_ctx* ctx, const uint32_t* in, uint32_t* out, size_t count);
/* UniEncAccumulator::SignedDigitDecompose(poly) (mk-acc.cpp:54-80) on `count`
 * COEFF polys: out [count][dg][N]. */
int mkacc_sdd(mkacc_ctx* ctx, const uint32_t* in, uint32_t* out, size_t count);
/* 64-bit-word forms of the three primitives (any context). */
int mkacc_ntt_forward_u64(mkacc_ctx* ctx, const uint64_t* in, uint64_t* out, size_t count);
int mkacc_ntt_inverse_u64(mkacc_ctx* ctx, const uint64_t* in, uint64_t* out, size_t count);
int mkacc_sdd_u64(mkacc_ctx* ctx, const uint64_t* in, uint64_t* out, size_t count);

/* ---- multi-device groups ----------------------------------------------------
 * A batch of independent gates shards across the GPUs of one node
 * (BinFHEContext::EvalBinGate over a batch, binfhecontext.cpp:415-426, has no
 * multi-device form in the reference): a group holds one context per entry of
 * devices[] (a device may repeat).  Keys are converted once on member 0 and
 * copied device to device (hipMemcpyPeer, xGMI) to the others; a batch is split
 * into contiguous shards (mkacc_shard_range), each member runs its shard on
 * its own stream from its own host thread, and the calls return when every
 * shard is done.  Outputs are bit-identical to one context's. */
typedef struct mkacc_group mkacc_group;
int mkacc_group_create(const mkacc_params* p, const int* devices, uint32_t count, mkacc_group** out);
void mkacc_group_destroy(mkacc_group* g);
uint32_t mkacc_group_size(const mkacc_group* g);
/* member i (owned by the group), e.g. for mkacc_stream / mkacc_get_params */
mkacc_ctx* mkacc_group_member(mkacc_group* g, uint32_t i);
/* [*begin, *end) of shard i of B gates over `parts` members; sizes differ by at most one */
void mkacc_shard_range(size_t B, uint32_t parts, uint32_t i, size_t* begin, size_t* end);
int mkacc_group_upload_keys(mkacc_group* g, const uint32_t* evk, const uint32_t* pkey);
int mkacc_group_upload_keys_u64(mkacc_group* g, const uint64_t* evk, const uint64_t* pkey);
int mkacc_group_upload_ksk_mntru(mkacc_group* g, const mkacc_ks_params* ks, const uint32_t* ksk);
int mkacc_group_upload_ksk_mklwe(mkacc_group* g, const mkacc_ks_params* ks, const uint32_t* A, const uint32_t* B);
/* host-buffer forms of mkacc_eval_batch / _u64 / mkacc_eval_nand_mntru / _mklwe over the group */
int mkacc_group_eval_batch(mkacc_group* g, const uint32_t* ct, const uint32_t* acc_in, uint32_t* acc_out, size_t B);
int mkacc_group_eval_batch_u64(mkacc_group* g, const uint32_t* ct, const uint64_t* acc_in, uint64_t* acc_out,
                               size_t B);
int mkacc_group_eval_nand_mntru(mkacc_group* g, const uint32_t* ct_nand, const uint32_t* ct1, const uint32_t* ct2,
                                uint32_t* out, size_t B);
int mkacc_group_eval_nand_mklwe(mkacc_group* g, const uint32_t* a1, const uint32_t* b1, const uint32_t* a2,
                                const uint32_t* b2, uint32_t* out_a, uint32_t* out_b, size_t B);

/* Per-thread text of the last error ("" if none). */
const char* mkacc_last_error(void);
int mkacc_abi_version(void);
/* "abi=..;header=<id>;source=<id>;dg=<digit counts built>;flags=<A/B switches>":
 * SHA-256 prefixes of this header and of the engine sources the library was
 * built from (mkfhe_amd/build.py); loaders refuse a mismatch. */
const char* mkacc_build_info(void);

#ifdef __cplusplus
}
#endif
#endif /* MKFHE_AMD_H */
