// mkacc_device.hpp -- gfx950 device building blocks of the multi-key accumulator:
// 27-bit modular arithmetic and the wave-resident negacyclic NTT (N = 2048).
//
// One wavefront owns one ring polynomial: 32 residues per lane held in VGPRs.
// The 11 butterfly stages run in three register passes separated by two LDS
// transposes through an 8 KiB per-wave scratch (no workgroup barriers):
//
//   layout A  x[r] <-> j = (r << 6) | lane                 regs = bits 10..6
//   layout B  x[r] <-> j = ((lane>>1) << 6) | (r<<1) | (lane&1)   regs = bits 5..1
//   layout C  x[r] <-> j = (lane << 5) | r                 regs = bits 4..0
//   layout D  x[r] <-> j = ((lane>>5) << 10) | (r<<5) | (lane&31)   regs = bits 9..5
//
// Forward (coefficient, layout A) -> stages on bits 10..6 (A) -> 5..1 (B) -> 0 (C)
// produces the reference's EVALUATION order (bit-reversed CT output,
// transformnat-impl.h:300-354) in layout C.  The inverse (ntt_inv) runs
// decimation-in-time butterflies on bits 0..4 (C), 5..9 (D), 10 (A) and a
// psi^-i post-twist, the same map as the reference's GS inverse
// (transformnat-impl.h:492-552); its N^-1 factor is folded into the keys and
// the accumulator by the host.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mkacc {

constexpr int kN = 2048;
constexpr int kLogN = 11;
constexpr int kRegs = 32;          // residues per lane

struct Mod {
    uint32_t Q;      // modulus, 2^26 < Q < 2^27
    uint32_t mu;     // floor(2^58 / Q)
    uint32_t r32;    // 2^32 mod Q
    uint32_t qinv;   // -Q^-1 mod 2^32 (Montgomery reduction, R = 2^32)
    uint32_t m1;     // floor(2^32 / Q): Shoup companion of 1
};

// ---- buffer-resource memory access -------------------------------------------
// A wave-uniform 128-bit descriptor in SGPRs + one shared 32-bit lane offset:
// the per-group / per-array variation goes into the scalar soffset, so loops of
// loads from many arrays cost no address VGPRs (guide T8).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ u32x4 bload4(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, 0);
}
__device__ __forceinline__ u32x2 bload2(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    return __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0);
}
// A 16-byte store reads its data VGPRs after it issues: they must not be
// rewritten for 2 wait states (gfx950: VMEM store of more than 8 bytes ->
// VALU write of its data registers).  hipcc (ROCm 7.2) inserts no wait states
// for buffer stores with an SGPR soffset and reuses the data registers on the
// next instruction; under load (two workgroups per CU) the store then wrote
// the NEXT group's values for part of the wave (lanes 12-15 of each row), the
// wrong-result "race" of round 1.  The s_nop sits between scheduling barriers
// so nothing is moved into the gap.  tools/isa_audit.py checks every build.
__device__ __forceinline__ void bstore4(u32x4 v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, soff, 0);
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 1");
    __builtin_amdgcn_sched_barrier(0);
}

// ---- modular arithmetic ---------------------------------------------------
// Canonical residues in [0, Q).  Conditional subtraction by unsigned min:
// if s < Q then s - Q wraps above s.
__device__ __forceinline__ uint32_t add_mod(uint32_t a, uint32_t b, uint32_t Q) {
    uint32_t s = a + b;
    return min(s, s - Q);
}
__device__ __forceinline__ uint32_t sub_mod(uint32_t a, uint32_t b, uint32_t Q) {
    uint32_t d = a - b;
    return min(d, d + Q);
}
// Shoup multiplication by a constant w with companion wp = floor(w * 2^32 / Q).
__device__ __forceinline__ uint32_t mul_shoup(uint32_t x, uint32_t w, uint32_t wp, uint32_t Q) {
    uint32_t q = __umulhi(x, wp);
    uint32_t r = x * w - q * Q;   // in [0, 2Q)
    return min(r, r - Q);
}
// Barrett reduction of x < 2^58 (a sum of up to 16 products of residues).
__device__ __forceinline__ uint32_t reduce58(uint64_t x, const Mod& m) {
    uint32_t xh = (uint32_t)(x >> 26);
    uint32_t q = __umulhi(xh, m.mu);
    uint32_t r = (uint32_t)x - q * m.Q;   // in [0, 3Q)
    r = min(r, r - m.Q);
    return min(r, r - m.Q);
}
// ... to [0, 2Q) (the accumulator between steps is kept in this range)
__device__ __forceinline__ uint32_t reduce58_lazy(uint64_t x, const Mod& m) {
    uint32_t xh = (uint32_t)(x >> 26);
    uint32_t q = __umulhi(xh, m.mu);
    uint32_t r = (uint32_t)x - q * m.Q;   // in [0, 3Q)
    return min(r, r - m.Q);
}
__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {
    return (uint64_t)a * b + c;           // v_mad_u64_u32
}
// v_mad_u64_u32 pinned as ONE instruction.  Where only the low word of a*b + c
// is used the compiler narrows C++ to v_mul_lo_u32 + v_add_u32; the 64-bit
// form does both in one issue slot (tools/ubench_isa.hip: all three cost about
// the same).  SB: b is wave-uniform (SGPR operand).  Carry-out goes to VCC.
// gfx950 needs a wait state between a VALU that writes an SGPR (this carry-out)
// and a VALU that reads any SGPR: with a wave-uniform b in an SGPR, hipcc puts an
// s_nop 0 between back-to-back multiply-adds (the s_nop is not what the wave waits
// on).
template <bool SB>
__device__ __forceinline__ uint64_t mad64_pin(uint32_t a, uint32_t b, uint64_t c) {
    uint64_t r;
    if constexpr (SB)
        asm("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(c) : "vcc");
    else
        asm("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c) : "vcc");
    return r;
}
template <bool SB>
__device__ __forceinline__ uint64_t mul64_pin(uint32_t a, uint32_t b) {
    uint64_t r;
    if constexpr (SB)
        asm("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(r) : "v"(a), "s"(b) : "vcc");
    else
        asm("v_mad_u64_u32 %0, vcc, %1, %2, 0" : "=v"(r) : "v"(a), "v"(b) : "vcc");
    return r;
}

// The pinned multiply-adds write their carry-out to VCC from an asm body, which
// hipcc does not count as a VALU write of VCC: an SALU write/read of VCC (a
// wave-uniform branch) right after them can see the late VALU write (DESIGN.md
// s2, the mk_lat_kernel defect).  Put this between such multiply-adds and the
// next wave-uniform branch; tools/isa_audit.py checks every build.
__device__ __forceinline__ void vcc_fence() {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_nop 7" ::: "vcc");
    __builtin_amdgcn_sched_barrier(0);
}

// Montgomery reduction (R = 2^32) of a lazy 64-bit sum x < Q * 2^32:
// m = x * (-Q^-1) mod 2^32 makes x + m Q divisible by 2^32, and
// (x + m Q) / 2^32 < 2Q is congruent to x * 2^-32 mod Q.  Two instructions
// (v_mul_lo_u32 + v_mad_u64_u32, result = the high word).  The step kernel's
// keys are stored times 2^32 mod Q, so the reduction returns the plain sum.
// Since Q < 2^27, Q * 2^32 > 32 Q^2: sums of up to 32 products of residues
// below Q (or their equivalent, e.g. 8 products of values < 4Q and < Q) qualify.
__device__ __forceinline__ uint32_t redc(uint64_t x, uint32_t Q, uint32_t qinv) {
    const uint32_t m = (uint32_t)x * qinv;
    return (uint32_t)(mad64_pin<true>(m, Q, x) >> 32);
}
// x < Q * 2^32 -> hi * (2^32 mod Q) + lo < Q^2 + 2^32 < 2 Q^2: same residue;
// keeps a long lazy sum inside redc's range
__device__ __forceinline__ uint64_t fold64(uint64_t x, uint32_t r32) {
    return (uint64_t)(uint32_t)(x >> 32) * r32 + (uint32_t)x;
}

// ---- LDS transposes ---------------------------------------------------------
// Row padding of one word per 32 (addr = j + j/32) makes every layout's access
// conflict-free for ds_*_b32 AND additive in (lane, reg), so each transpose uses
// one address VGPR plus immediate offsets (derivation in DESIGN.md s4.1).
constexpr int kLdsWords = kN + kN / 32;   // per-wave transpose scratch (8448 B)

__device__ __forceinline__ uint32_t pad(uint32_t j) { return j + (j >> 5); }
// lane part and register part of pad(j) for each layout
__device__ __forceinline__ uint32_t baseA(uint32_t l) { return l + (l >> 5); }
__device__ __forceinline__ constexpr uint32_t offA(int r) { return 66u * r; }
__device__ __forceinline__ uint32_t baseB(uint32_t l) { return 66u * (l >> 1) + (l & 1u); }
__device__ __forceinline__ constexpr uint32_t offB(int r) { return 2u * r + (r >> 4); }
__device__ __forceinline__ uint32_t baseC(uint32_t l) { return 33u * l; }
__device__ __forceinline__ constexpr uint32_t offC(int r) { return (uint32_t)r; }
// layout D (inverse transform, pass 2): x[r] <-> j = ((lane>>5) << 10) | (r << 5) | (lane & 31),
// regs = bits 9..5; pad(j) = 1056 (lane>>5) + (lane & 31) + 33 r: lanes 0..31 and
// 32..63 each hit 32 consecutive words, the two halves 32 banks apart
__device__ __forceinline__ uint32_t baseD(uint32_t l) { return 1056u * (l >> 5) + (l & 31u); }
__device__ __forceinline__ constexpr uint32_t offD(int r) { return 33u * r; }

__device__ __forceinline__ uint32_t jA(uint32_t l, uint32_t r) { return (r << 6) | l; }
__device__ __forceinline__ uint32_t jB(uint32_t l, uint32_t r) { return ((l >> 1) << 6) | (r << 1) | (l & 1u); }
__device__ __forceinline__ uint32_t jC(uint32_t l, uint32_t r) { return (l << 5) | r; }
__device__ __forceinline__ uint32_t jD(uint32_t l, uint32_t r) { return ((l >> 5) << 10) | (r << 5) | (l & 31u); }

// Keeps the scheduler from hoisting a later stage's twiddle loads (and their
// VGPRs) above the current stage.
__device__ __forceinline__ void sched_fence() { __builtin_amdgcn_sched_barrier(0); }

__device__ __forceinline__ void wave_lds_sync() {
    // A wave's LDS instructions execute in issue order, so a read after the
    // wave's own writes sees them and later writes cannot overtake earlier
    // reads: only the compiler must be kept from reordering (no s_waitcnt).
    asm volatile("" ::: "memory");
}

template <int LAYOUT>
__device__ __forceinline__ uint32_t lbase(uint32_t l) {
    return LAYOUT == 0 ? baseA(l) : (LAYOUT == 1 ? baseB(l) : (LAYOUT == 2 ? baseC(l) : baseD(l)));
}
template <int LAYOUT>
__device__ __forceinline__ constexpr uint32_t loff(int r) {
    return LAYOUT == 0 ? offA(r) : (LAYOUT == 1 ? offB(r) : (LAYOUT == 2 ? offC(r) : offD(r)));
}

template <int SRC, int DST>
__device__ __forceinline__ void transpose(uint32_t (&x)[kRegs], uint32_t* lds, uint32_t l) {
    uint32_t* ws = lds + lbase<SRC>(l);
#pragma unroll
    for (int r = 0; r < kRegs; ++r) ws[loff<SRC>(r)] = x[r];
    wave_lds_sync();
    const uint32_t* rs = lds + lbase<DST>(l);
#pragma unroll
    for (int r = 0; r < kRegs; ++r) x[r] = rs[loff<DST>(r)];
    wave_lds_sync();
}

// ---- forward NTT (Cooley-Tukey, reference table indexing) -------------------
// tw[i] = { psi^brv(i), companion }, i in [0, N): reference rootOfUnityTable.
// Lazy butterflies.  Shoup's product T = b*w - q*Q lies in [0, 2Q) for ANY
// 32-bit b, so the forward transform never reduces b, and it reduces a only
// once, at the last stage: a stage maps values below A to values below A + 2Q
// (a + T, a - T + 2Q), so inputs below 4Q stay below 4Q + 10*2Q = 24Q < 2^32
// (Q < 2^27) through stages 0..9; stage 10 brings a back under 2Q and emits
// [0, 4Q).  Shoup's product is formed negated so both outputs take one
// instruction.  The inverse (GS) keeps values in [0, 2Q).
// Forward twiddle pairs hold { -w mod 2^32, floor(w 2^32 / Q) }: the negated
// Shoup product -T = q*Q - b*w is then two pinned multiply-adds.
// MKACC_BFLY_C (a per-unit flag, mkfhe_amd/build.py): the Shoup product's two
// multiply-adds written in C instead of pinned asm.  hipcc cannot see what an asm
// statement does, so it puts an s_nop 0 before every VALU that reads a register an
// asm statement wrote (one per butterfly: the second multiply-add reads the first's
// result, or the add/sub reads the second's); in C it emits v_mul_lo_u32 +
// v_mad_u64_u32 for the same low word and no wait state.  Faster for the headline
// kernel (-1.7 to -2.1 % per step, profiles/r5/ab_hl_bfly_c.txt) and for
// mk_lat_kernel (-4 %, ab_lat_bfly_c.txt): build.py sets 1 (every product) for the
// step2 and lat units.  mk_step_kernel at dg = 4 needs more registers with it (8 B
// of scratch, +0.6 %); 2 (the forward transforms only) is spill-free there and
// 1.0-1.1 % faster (ab_c4_bfly_c.txt) -- in the MK-NTRU kernels only: the MK-LWE
// (XZW_B) one at dg = 4 would spill 16 B (mkacc_kernels.hpp fwd_c).
#ifndef MKACC_BFLY_C
#define MKACC_BFLY_C 0
#endif
constexpr bool kFwdC = MKACC_BFLY_C == 1 || MKACC_BFLY_C == 2;
constexpr bool kInvC = MKACC_BFLY_C == 1;
static_assert(MKACC_BFLY_C >= 0 && MKACC_BFLY_C <= 2, "MKACC_BFLY_C: 0 (asm), 1 (C), 2 (C in the forward transforms)");
template <bool SW, bool C>
__device__ __forceinline__ uint32_t shoup_neg(uint32_t b, uint2 w, uint32_t Q) {
    const uint32_t q = __umulhi(b, w.y);
    if constexpr (C) return (uint32_t)((uint64_t)q * Q + (uint64_t)(b * w.x));
    return (uint32_t)mad64_pin<true>(q, Q, mul64_pin<SW>(b, w.x));   // -T, T in [0, 2Q)
}
template <bool SW, bool C>
__device__ __forceinline__ void ct_bfly_lazy(uint32_t& a, uint32_t& b, uint2 w, uint32_t Q) {
    const uint32_t X = a;
    const uint32_t Tn = shoup_neg<SW, C>(b, w, Q);
    a = X - Tn;                                                  // X + T
    b = X + Tn + 2u * Q;                                         // X - T + 2Q
}
// last stage: a in [0, 24Q) -> X in [0, 2Q) as Shoup's product by 1
// (companion m1 = floor(2^32 / Q)); outputs in [0, 4Q)
template <bool C>
__device__ __forceinline__ void ct_bfly_last(uint32_t& a, uint32_t& b, uint2 w, uint32_t Q, uint32_t m1) {
    const uint32_t X = a - __umulhi(a, m1) * Q;                  // [0, 2Q)
    const uint32_t Tn = shoup_neg<false, C>(b, w, Q);
    a = X - Tn;                                                  // [0, 4Q)
    b = X + Tn + 2u * Q;                                         // (0, 4Q)
}
// [0, 4Q) -> [0, Q)
__device__ __forceinline__ uint32_t canon4(uint32_t x, uint32_t Q) {
    x = min(x, x - 2u * Q);
    return min(x, x - Q);
}

// Wave-uniform table reads go through the constant address space so they are
// issued as scalar loads into SGPRs instead of occupying VGPRs.
typedef const __attribute__((address_space(4))) uint64_t const_u64;
struct ConstTable {
    const_u64* p;
    __device__ __forceinline__ uint2 operator[](int i) const {
        const uint64_t v = p[i];
        return make_uint2((uint32_t)v, (uint32_t)(v >> 32));
    }
};

// The twiddle tables are loop-invariant inside a kernel; without this the
// compiler hoists every NTT's table loads (and addresses) out of the party /
// digit loops and keeps them live across the whole step, exhausting registers.
__device__ __forceinline__ uint32_t opaque_v(uint32_t v) {
    asm volatile("" : "+v"(v));
    return v;
}
__device__ __forceinline__ const uint2* opaque(const uint2* p) {
    uint64_t v = (uint64_t)p;
    asm volatile("" : "+s"(v));
    return (const uint2*)v;
}

// ---- per-lane twiddles ----------------------------------------------------------
// Pass B (stages 5..9) and pass C (stage 10) need per-lane twiddles.  They are
// stored in an interleaved order so that a wave's read of "twiddle m" is one
// fully coalesced 512-byte dwordx2 load (or, from LDS, one conflict-free
// ds_read_b64) at a lane-dependent base plus an immediate offset:
//   stage s in 5..9 : pair (m, lhi) at  twl_off(s) + 32*m + lhi   (lhi = lane >> 1)
//   stage 10        : pair (m, lane) at kTwlC + 64*m + lane
// Entry (m, lhi) of stage s is reference table index 2^s + lhi*2^(s-5) + m, and
// entry (m, lane) of stage 10 is 1024 + 16*lane + m (transformnat-impl.h:705-760);
// the inverse NTT's bit-B stage uses the layout of stage s = 10 - B.
__host__ __device__ constexpr int twl_off(int s) { return 32 * ((1 << (s - 5)) - 1); }
constexpr int kTwlC = 992;                 // = twl_off(10)
constexpr int kTwlPairs = kTwlC + 1024;    // 2016 pairs per direction


// Per-lane twiddle streams, software-pipelined: the loads of chunk I+1 are
// issued before the butterflies of chunk I (double-buffered 4-pair chunks: the
// same 16 live twiddle VGPRs as one 8-pair chunk), and the first chunk is issued
// before the LDS transpose that precedes the stream, so L1/L2 latency overlaps
// arithmetic instead of stalling the wave.  A stream is a list of chunks
// {stage, first pair m0, pair count}; LD / AP are the direction's load and
// butterfly functors.
// MKACC_TW_FENCE = 0 lets the scheduler move work across chunk boundaries (more
// independent butterflies in flight for a lone wave per SIMD; more live registers).
#ifndef MKACC_TW_FENCE
#define MKACC_TW_FENCE 1
#endif
struct TwChunk { int s, m0, cnt; };
template <class SEQ, int I, int W, class LD, class AP>
__device__ __forceinline__ void tw_pipe(uint2 (&wa)[W], uint2 (&wb)[W], const LD& ld, const AP& ap) {
    constexpr TwChunk c = SEQ::at(I);
    if constexpr (I + 1 < SEQ::N) {
        constexpr TwChunk n = SEQ::at(I + 1);
        ld.template go<n.s, n.m0, n.cnt>((I + 1) % 2 ? wb : wa);
    }
    ap.template go<c.s, c.m0, c.cnt>(I % 2 ? wb : wa);
    if constexpr (MKACC_TW_FENCE) sched_fence();
    if constexpr (I + 1 < SEQ::N) tw_pipe<SEQ, I + 1>(wa, wb, ld, ap);
}
// forward pass A (stages 0..4, layout A): wave-uniform twiddles, scalar loads
// double-buffered in 8-pair chunks (the 16 pairs of stage 4 never all live)
struct FwdASeq {
    static constexpr int N = 6;
    static constexpr TwChunk at(int i) {
        constexpr TwChunk c[N] = {{0, 0, 1}, {1, 0, 2}, {2, 0, 4}, {3, 0, 8}, {4, 0, 8}, {4, 8, 8}};
        return c[i];
    }
};
struct FwdALoad {
    const ConstTable& twc;
    template <int S, int M0, int CNT>
    __device__ __forceinline__ void go(uint2 (&w)[8]) const {
#pragma unroll
        for (int j = 0; j < CNT; ++j) w[j] = twc[(1 << S) + M0 + j];
    }
};
template <bool C>
struct FwdAApply {
    uint32_t (&x)[kRegs];
    uint32_t Q;
    template <int S, int M0, int CNT>
    __device__ __forceinline__ void go(const uint2 (&w)[8]) const {
        constexpr int H = 16 >> S;
#pragma unroll
        for (int r = 0; r < kRegs; ++r) {
            if (r & H) continue;
            const int m = r >> (5 - S);
            if (m < M0 || m >= M0 + CNT) continue;
            ct_bfly_lazy<true, C>(x[r], x[r + H], w[m - M0], Q);
        }
    }
};
// forward passes B (stages 5..9, layout B) and C (stage 10, layout C)
struct FwdSeq {
    static constexpr int N = 13;
    static constexpr TwChunk at(int i) {
        constexpr TwChunk c[N] = {{5, 0, 1},  {6, 0, 2},  {7, 0, 4},  {8, 0, 4},  {8, 4, 4},
                                  {9, 0, 4},  {9, 4, 4},  {9, 8, 4},  {9, 12, 4}, {10, 0, 4},
                                  {10, 4, 4}, {10, 8, 4}, {10, 12, 4}};
        return c[i];
    }
};
struct FwdLoad {
    const uint2* twl;    // stages 5..9: + twl_off(s) + 32 m + (lane >> 1)
    const uint2* tw10;   // stage 10: + 64 m + lane
    __device__ __forceinline__ FwdLoad(const uint2* t, const uint2* t10, uint32_t lo)
        : twl(t + (lo >> 1)), tw10(t10 + lo) {}
    template <int S, int M0, int CNT>
    __device__ __forceinline__ void go(uint2 (&w)[4]) const {
#pragma unroll
        for (int j = 0; j < CNT; ++j) w[j] = S < 10 ? twl[twl_off(S < 10 ? S : 5) + 32 * (M0 + j)] : tw10[64 * (M0 + j)];
    }
};
template <bool C>
struct FwdApply {
    uint32_t (&x)[kRegs];
    uint32_t* lds;
    uint32_t l, Q, m1;
    template <int S, int M0, int CNT>
    __device__ __forceinline__ void go(const uint2 (&w)[4]) const {
        if constexpr (S < 10) {
            constexpr int H = 1 << (9 - S), SH = 10 - S;
#pragma unroll
            for (int r = 0; r < kRegs; ++r) {
                if (r & H) continue;
                const int m = r >> SH;
                if (m < M0 || m >= M0 + CNT) continue;
                ct_bfly_lazy<false, C>(x[r], x[r + H], w[m - M0], Q);
            }
        } else {
            if constexpr (M0 == 0) transpose<1, 2>(x, lds, l);
#pragma unroll
            for (int j = 0; j < CNT; ++j) ct_bfly_last<C>(x[2 * (M0 + j)], x[2 * (M0 + j) + 1], w[j], Q, m1);
        }
    }
};

// Forward negacyclic NTT of one polynomial per wave, reference EVAL order.
//   tw_g : reference forward table (pairs) in global memory, pass A reads it
//          with scalar loads (wave-uniform indices 1..31)
//   twl  : this direction's per-lane LDS table (layout above)
// Input residues in [0, 4Q); output EVAL values in [0, 4Q) (not canonical).
//   tw10 : stage-10 twiddles (pairs (m, lane) at tw10 + 64*m + lane); twl + kTwlC
//          or a copy of that block in LDS
template <bool C = kFwdC>
__device__ __forceinline__ void ntt_fwd(uint32_t (&x)[kRegs], uint32_t* lds, const uint2* tw_g, const uint2* twl,
                                        const uint2* tw10, uint32_t l, uint32_t Q, uint32_t m1) {
    // pass A: stages 0..4 (bits 10..6); twiddle index uniform across the wave
    const ConstTable twc{(const_u64*)opaque(tw_g)};
    {
        const FwdALoad ld{twc};
        const FwdAApply<C> ap{x, Q};
        uint2 sa[8], sb[8];
        ld.template go<0, 0, 1>(sa);
        tw_pipe<FwdASeq, 0>(sa, sb, ld, ap);
    }
    const uint32_t lo = opaque_v(l);
    // passes B (stages 5..9, bits 5..1) and C (stage 10, bit 0), one twiddle stream
    {
        const FwdLoad ld(twl, tw10, lo);
        const FwdApply<C> ap{x, lds, l, Q, m1};
        uint2 wa[4], wb[4];
        ld.template go<5, 0, 1>(wa);
        transpose<0, 1>(x, lds, l);
        tw_pipe<FwdSeq, 0>(wa, wb, ld, ap);
    }
}

// ---- inverse NTT WITHOUT the N^-1 factor: DIT butterflies + post-twist --------
// The reference's inverse (Gentleman-Sande, transformnat-impl.h:492-552) maps the
// EVAL vector A (slot j = evaluation at psi^(2 brv(j) + 1)) to
//   a_i = N^-1 psi^-i sum_k A[brv(k)] w^-ik,   w = psi^2.
// A is the natural-order evaluation vector stored bit-reversed, so radix-2
// decimation-in-time butterflies on bits 0, 1, ..., 10 (bit b: pairs (j, j + 2^b),
// twiddle psi^-(t 2^(11-b)), t = j mod 2^b) produce the cyclic sum in natural
// order, and one Shoup product by psi^-i per coefficient finishes the transform
// (N^-1 is folded into keys and accumulator).  Every butterfly is
// the forward transform's lazy 5-instruction CT butterfly (values grow by < 2Q
// per stage; the final Shoup product accepts any 32-bit word and returns a
// canonical residue), and butterflies with twiddle 1 (t = 0, resolved per
// register in pass 1) drop the product while the bounds allow -- against 8
// instructions for a lazy GS butterfly.
//   pass 1 (layout C, regs = bits 4..0): bits 0..4, wave-uniform twiddles (scalar)
//   pass 2 (layout D, regs = bits 9..5): bits 5..9, per-lane twiddles (lane & 31)
//   pass 3 (layout A, regs = bits 10..6): bit 10 and the twist, per-lane
// Tables (mkacc_engine.hip builds them):
//   tis  [2^b + t], b < 5, t < 2^b  : {-w, w'} of psi^-(t 2^(11-b))   (global, scalar reads)
//   twl  [twl_off(b) + 32 m + (l & 31)], b = 5..9 : t = (l & 31) | (m << 5)
//        [kTwlC + 64 m + l]                        : bit 10, t = (m << 6) | l
//        [kTwlPairs + 64 r + l]                    : {psi^-i, companion}, i = (r << 6) | l
constexpr int kInvImgPairs = kTwlPairs + kN;

// Pass-1 schedule: value bounds in units of Q per register; a twiddle-1
// butterfly skips the product when its doubled bound still leaves room for the
// remaining stages (+2 each); everything entering pass 2 stays below 20 Q, so
// the six per-lane stages end below 32 Q <= 2^32 (Q < 2^27).
struct InvPlan {
    bool skip[5][kRegs];
    int bound[5][kRegs];   // bound of each register entering stage b
    int maxb;
    constexpr explicit InvPlan(int b0) : skip{}, bound{}, maxb(0) {
        int bd[kRegs] = {};
        for (int r = 0; r < kRegs; ++r) bd[r] = b0;
        for (int b = 0; b < 5; ++b) {
            const int h = 1 << b;
            for (int r = 0; r < kRegs; ++r) bound[b][r] = bd[r];
            for (int r = 0; r < kRegs; ++r) {
                if (r & h) continue;
                const int s = bd[r] + bd[r + h];
                if ((r & (h - 1)) == 0 && s + 2 * (4 - b) <= 20) {
                    skip[b][r] = true;
                    bd[r] = bd[r + h] = s;
                } else {
                    bd[r] = bd[r + h] = bd[r] + 2;
                }
            }
        }
        for (int r = 0; r < kRegs; ++r) maxb = bd[r] > maxb ? bd[r] : maxb;
    }
};
constexpr InvPlan kInvPlan(2);   // inputs in [0, 2Q)
static_assert(kInvPlan.maxb <= 20, "inverse NTT bounds");


// inverse pass 1 (bits 0..4, layout C): scalar twiddle chunks; t = 0 entries
// entries (twiddle 1) are loaded even where the butterflies skip the product
struct Inv1Seq {
    static constexpr int N = 6;
    static constexpr TwChunk at(int i) {
        constexpr TwChunk c[N] = {{0, 0, 0}, {1, 0, 2}, {2, 0, 4}, {3, 0, 8}, {4, 0, 8}, {4, 8, 8}};
        return c[i];
    }
};
struct Inv1Load {
    const ConstTable& twc;
    template <int S, int M0, int CNT>
    __device__ __forceinline__ void go(uint2 (&w)[8]) const {
#pragma unroll
        for (int j = 0; j < CNT; ++j) w[j] = twc[(1 << S) + M0 + j];
    }
};
template <bool C>
struct Inv1Apply {
    uint32_t (&x)[kRegs];
    uint32_t Q;
    template <int S, int M0, int CNT>
    __device__ __forceinline__ void go(const uint2 (&w)[8]) const {
        constexpr int H = 1 << S;
#pragma unroll
        for (int r = 0; r < kRegs; ++r) {
            if (r & H) continue;
            const int t = r & (H - 1);
            if (S > 0 && (t < M0 || t >= M0 + CNT)) continue;
            if (S == 0 && M0 != 0) continue;
            if (kInvPlan.skip[S][r]) {
                const uint32_t X = x[r], Y = x[r + H];
                x[r] = X + Y;
                x[r + H] = X - Y + (uint32_t)kInvPlan.bound[S][r + H] * Q;
            } else {
                ct_bfly_lazy<true, C>(x[r], x[r + H], w[t - M0], Q);
            }
        }
    }
};
// inverse pass 2 (stages 5..9, layout D), bit 10 (layout A) and the twist
struct InvSeq {
    static constexpr int N = 21;
    static constexpr TwChunk at(int i) {
        constexpr TwChunk c[N] = {{5, 0, 1},   {6, 0, 2},   {7, 0, 4},   {8, 0, 4},   {8, 4, 4},   {9, 0, 4},
                                  {9, 4, 4},   {9, 8, 4},   {9, 12, 4},  {10, 0, 4},  {10, 4, 4},  {10, 8, 4},
                                  {10, 12, 4}, {11, 0, 4},  {11, 4, 4},  {11, 8, 4},  {11, 12, 4}, {11, 16, 4},
                                  {11, 20, 4}, {11, 24, 4}, {11, 28, 4}};
        return c[i];
    }
};
struct InvLoad {
    const uint2* t31;   // stages 5..9: + twl_off(s) + 32 m + (lane & 31)
    const uint2* t64;   // bit 10: + kTwlC + 64 m + lane; twist: + kTwlPairs + 64 r + lane
    __device__ __forceinline__ InvLoad(const uint2* twl, uint32_t lo) : t31(twl + (lo & 31u)), t64(twl + lo) {}
    template <int S, int M0, int CNT>
    __device__ __forceinline__ void go(uint2 (&w)[4]) const {
#pragma unroll
        for (int j = 0; j < CNT; ++j)
            w[j] = S < 10 ? t31[twl_off(S < 10 ? S : 5) + 32 * (M0 + j)]
                          : t64[(S == 10 ? kTwlC : kTwlPairs) + 64 * (M0 + j)];
    }
};
template <bool C>
struct InvApply {
    uint32_t (&x)[kRegs];
    uint32_t* lds;
    uint32_t l, Q;
    template <int S, int M0, int CNT>
    __device__ __forceinline__ void go(const uint2 (&w)[4]) const {
        if constexpr (S < 10) {
            constexpr int H = 1 << (S - 5);
#pragma unroll
            for (int r = 0; r < kRegs; ++r) {
                if (r & H) continue;
                const int m = r & (H - 1);
                if (m < M0 || m >= M0 + CNT) continue;
                ct_bfly_lazy<false, C>(x[r], x[r + H], w[m - M0], Q);
            }
        } else if constexpr (S == 10) {
            if constexpr (M0 == 0) transpose<3, 0>(x, lds, l);
#pragma unroll
            for (int j = 0; j < CNT; ++j) ct_bfly_lazy<false, C>(x[M0 + j], x[M0 + j + 16], w[j], Q);
        } else {
#pragma unroll
            for (int j = 0; j < CNT; ++j) x[M0 + j] = mul_shoup(x[M0 + j], w[j].x, w[j].y, Q);
        }
    }
};

// Input residues in [0, 2Q), layout C; output canonical coefficients, layout A.
template <bool C = kInvC>
__device__ __forceinline__ void ntt_inv(uint32_t (&x)[kRegs], uint32_t* lds, const uint2* tis, const uint2* twl,
                                        uint32_t l, uint32_t Q) {
    // pass 1: bits 0..4 on registers, twiddle index (r mod 2^b) wave-uniform
    const ConstTable twc{(const_u64*)opaque(tis)};
    {
        const Inv1Load ld{twc};
        const Inv1Apply<C> ap{x, Q};
        uint2 sa[8], sb[8];
        tw_pipe<Inv1Seq, 0>(sa, sb, ld, ap);
    }
    const uint32_t lo = opaque_v(l);
    {
        const InvLoad ld(twl, lo);
        const InvApply<C> ap{x, lds, l, Q};
        uint2 wa[4], wb[4];
        ld.template go<5, 0, 1>(wa);
        transpose<2, 3>(x, lds, l);
        tw_pipe<InvSeq, 0>(wa, wb, ld, ap);
    }
}

// ---- device EVAL layout in HBM ("C4") --------------------------------------
// Element (lane l, reg r) of layout C lives at ((r>>2) << 8) | (l << 2) | (r&3):
// one dwordx4 per lane per 4 registers, 1 KiB contiguous per wave instruction.
__device__ __forceinline__ void load_c4(uint32_t (&x)[kRegs], const uint32_t* __restrict__ p, uint32_t l) {
    const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
    for (int g = 0; g < 8; ++g) {
        uint4 v = q[g * 64 + l];
        x[4 * g + 0] = v.x; x[4 * g + 1] = v.y; x[4 * g + 2] = v.z; x[4 * g + 3] = v.w;
    }
}
__device__ __forceinline__ void store_c4(const uint32_t (&x)[kRegs], uint32_t* __restrict__ p, uint32_t l) {
    uint4* q = reinterpret_cast<uint4*>(p);
#pragma unroll
    for (int g = 0; g < 8; ++g) q[g * 64 + l] = make_uint4(x[4 * g], x[4 * g + 1], x[4 * g + 2], x[4 * g + 3]);
}
__host__ __device__ __forceinline__ uint32_t c4_index(uint32_t j) {
    // logical EVAL slot j = (l << 5) | r  ->  physical C4 index
    uint32_t l = j >> 5, r = j & 31u;
    return ((r >> 2) << 8) | (l << 2) | (r & 3u);
}

// ---- signed digit decomposition (mk-acc.cpp:54-80) -----------------------------
// The reference centres t (d = t < Q/2 ? t : t - Q), then repeatedly takes the
// balanced low digit r = sext_b(d), d = (d - r) >> b; digit 0 is dropped and
// digits 1..dg are emitted as r < 0 ? r + Q : r.
//
// Equivalent closed form used on the GPU: with C = sum_{i<G} 2^(b-1) 2^(b*i)
// (G = digitsG) and D = d + C (0 <= D < 2^32 when b*G <= 32), every balanced
// digit is r_i = bfe(D, b*i, b) - 2^(b-1).  By induction on i: D >> (b*i) equals
// the reference's running d_i plus sum_{j=i}^{G-1} 2^(b-1) 2^(b(j-i)), whose
// residue mod 2^b is d_i + 2^(b-1) = r_i + 2^(b-1) (in [0, 2^b)).
// The NTT consumes r_i + Q (in [Q - 2^(b-1), Q + 2^(b-1)) subset [0, 2Q)), the
// same residue class as the reference digit; the canonical form is r_i + Q mod Q.
struct SddConsts {
    uint32_t qhalf;    // Q >> 1
    uint32_t cpos;     // C          (added when t <  Q/2)
    uint32_t cneg;     // C - Q      (added when t >= Q/2), mod 2^32
    uint32_t gbits;    // b
    uint32_t qm;       // Q - 2^(b-1)
};
__device__ __forceinline__ uint32_t sdd_offset(uint32_t t, const SddConsts& s) {
    return t + (t < s.qhalf ? s.cpos : s.cneg);
}
// digit i (1..dg) of offset word D as an NTT input in [0, 2Q)
__device__ __forceinline__ uint32_t sdd_digit(uint32_t D, uint32_t i, const SddConsts& s) {
    return __builtin_amdgcn_ubfe(D, i * s.gbits, s.gbits) + s.qm;
}

// Digits 2..DG of every element, kept between the digit NTTs as the field
// F = bits [2b, 2b + (DG-1) b) of the offset word D.
//   DG <= 3: (DG-1) b <= 16 (b = 9..13 at DG = 2, b = 7..8 at DG = 3): two
//            elements per register (16 VGPRs).
//   DG >= 4: (DG-1) b <= 20 (b = 6 at DG = 4, b = 5 at DG = 5): the low 16 bits
//            two per register, the high 4 bits eight per register (20 VGPRs).
template <int DG, int R = kRegs>
struct PackedDigits {
    static constexpr bool kWide = DG > 3;
    uint32_t lo[R / 2];
    uint32_t hi[kWide ? R / 8 : 1];

    // element r with offset word D: returns digit 1 (NTT input), stores the rest
    __device__ __forceinline__ uint32_t put(int r, uint32_t D, const SddConsts& s) {
        const uint32_t f = __builtin_amdgcn_ubfe(D, 2u * s.gbits, kWide ? 20u : 16u);
        if ((r & 1) == 0) lo[r >> 1] = kWide ? (f & 0xFFFFu) : f;
        else lo[r >> 1] |= f << 16;
        if (kWide) {
            const uint32_t h = f >> 16;
            if ((r & 7) == 0) hi[r >> 3] = h;
            else hi[r >> 3] |= h << (4 * (r & 7));
            if ((r & 7) == 7) asm volatile("" : "+v"(hi[r >> 3]));
        }
        // pin the packed word: otherwise the compiler sinks the packing to
        // the later unpack and keeps every D live across the NTTs
        if (r & 1) asm volatile("" : "+v"(lo[r >> 1]));
        return sdd_digit(D, 1, s);
    }
    // digit i (2..DG) of element r as an NTT input
    __device__ __forceinline__ uint32_t get(int r, int i, const SddConsts& s) const {
        if (!kWide)
            return __builtin_amdgcn_ubfe(lo[r >> 1], (r & 1) * 16u + (uint32_t)(i - 2) * s.gbits, s.gbits) + s.qm;
        const uint32_t f = __builtin_amdgcn_ubfe(lo[r >> 1], (r & 1) * 16u, 16u) |
                           (__builtin_amdgcn_ubfe(hi[r >> 3], 4u * (r & 7), 4u) << 16);
        return __builtin_amdgcn_ubfe(f, (uint32_t)(i - 2) * s.gbits, s.gbits) + s.qm;
    }
};

}  // namespace mkacc

