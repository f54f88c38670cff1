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
//
// Forward (coefficient, layout A) -> stages on bits 10..6 (A) -> 5..1 (B) -> 0 (C)
// produces the reference's EVALUATION order (bit-reversed CT output,
// transformnat-impl.h:300-354) in layout C.  The inverse runs the GS stages in
// the opposite order (transformnat-impl.h:492-552) and returns layout A; its
// N^-1 factor is folded into the keys by the host.
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
__device__ __forceinline__ void bstore4(u32x4 v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
    __builtin_amdgcn_raw_buffer_store_b128(v, r, voff, soff, 0);
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
__device__ __forceinline__ uint64_t mad64(uint32_t a, uint32_t b, uint64_t c) {
    return (uint64_t)a * b + c;           // v_mad_u64_u32
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

__device__ __forceinline__ uint32_t jA(uint32_t l, uint32_t r) { return (r << 6) | l; }
__device__ __forceinline__ uint32_t jB(uint32_t l, uint32_t r) { return ((l >> 1) << 6) | (r << 1) | (l & 1u); }
__device__ __forceinline__ uint32_t jC(uint32_t l, uint32_t r) { return (l << 5) | r; }

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
    return LAYOUT == 0 ? baseA(l) : (LAYOUT == 1 ? baseB(l) : baseC(l));
}
template <int LAYOUT>
__device__ __forceinline__ constexpr uint32_t loff(int r) {
    return LAYOUT == 0 ? offA(r) : (LAYOUT == 1 ? offB(r) : offC(r));
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
// Lazy (Harvey) butterflies: the forward NTT keeps values in [0, 4Q), the
// inverse in [0, 2Q) (4Q < 2^29, so nothing overflows 32 bits).  Shoup's
// product q*Q - x*w is formed negated so both outputs take one instruction.
__device__ __forceinline__ void ct_bfly(uint32_t& a, uint32_t& b, uint2 w, uint32_t Q) {
    const uint32_t X = min(a, a - 2u * Q);                      // [0, 2Q)
    const uint32_t q = __umulhi(b, w.y);
    const uint32_t Tn = q * Q - b * w.x;                         // -(b*w mod~ Q), T in [0, 2Q)
    a = X - Tn;                                                  // X + T      in [0, 4Q)
    b = X + Tn + 2u * Q;                                         // X - T + 2Q in (0, 4Q)
}
__device__ __forceinline__ void gs_bfly(uint32_t& a, uint32_t& b, uint2 w, uint32_t Q) {
    const uint32_t lo = a, hi = b;                               // [0, 2Q)
    const uint32_t s = lo + hi;
    a = min(s, s - 2u * Q);                                      // [0, 2Q)
    const uint32_t d = lo - hi + 2u * Q;                         // (0, 4Q)
    const uint32_t q = __umulhi(d, w.y);
    b = d * w.x - q * Q;                                         // [0, 2Q)
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

// NP consecutive (w, w') pairs of a per-lane twiddle run starting at p:
// dwordx4 loads off one 64-bit base with immediate offsets.
template <int NP>
__device__ __forceinline__ void load_pairs(uint2 (&w)[NP], const uint2* p) {
    if (NP == 1) {
        w[0] = p[0];
    } else {
        const uint4* q = reinterpret_cast<const uint4*>(p);
#pragma unroll
        for (int j = 0; j < NP / 2; ++j) {
            const uint4 t = q[j];
            w[2 * j] = make_uint2(t.x, t.y);
            w[2 * j + 1] = make_uint2(t.z, t.w);
        }
    }
}

// forward pass-B stage s (5..9) on bit 10-s: twiddle 2^s + (lhi << (s-5)) + (r >> (10-s))
template <int S>
__device__ __forceinline__ void fwd_stage_b(uint32_t (&x)[kRegs], const uint2* tw, uint32_t lhi, uint32_t Q) {
    // twiddle runs longer than 8 pairs are processed in chunks of 8 to cap the
    // live twiddle registers at 16
    constexpr int NP = 1 << (S - 5), H = 1 << (9 - S), CH = NP > 8 ? 8 : NP, SH = 10 - S;
#pragma unroll
    for (int c0 = 0; c0 < NP; c0 += CH) {
        uint2 w[CH];
        load_pairs<CH>(w, tw + (1u << S) + (lhi << (S - 5)) + c0);
#pragma unroll
        for (int r = 0; r < kRegs; ++r) {
            if (r & H) continue;
            const int m = r >> SH;
            if (m < c0 || m >= c0 + CH) continue;
            ct_bfly(x[r], x[r + H], w[m - c0], Q);
        }
        sched_fence();
    }
}
// inverse pass-B stage on bit B (1..5): twiddle 2^(10-B) + (lhi << (5-B)) + (r >> B)
template <int B>
__device__ __forceinline__ void inv_stage_b(uint32_t (&x)[kRegs], const uint2* twi, uint32_t lhi, uint32_t Q) {
    constexpr int NP = 1 << (5 - B), H = 1 << (B - 1), CH = NP > 8 ? 8 : NP;
#pragma unroll
    for (int c0 = 0; c0 < NP; c0 += CH) {
        uint2 w[CH];
        load_pairs<CH>(w, twi + (1u << (10 - B)) + (lhi << (5 - B)) + c0);
#pragma unroll
        for (int r = 0; r < kRegs; ++r) {
            if (r & H) continue;
            const int m = r >> B;
            if (m < c0 || m >= c0 + CH) continue;
            gs_bfly(x[r], x[r + H], w[m - c0], Q);
        }
        sched_fence();
    }
}

// Input residues in [0, 4Q); output EVAL values in [0, 4Q) (not canonical).
__device__ __forceinline__ void ntt_fwd(uint32_t (&x)[kRegs], uint32_t* lds, const uint2* tw_in,
                                        uint32_t l, uint32_t Q) {
    const uint2* tw = opaque(tw_in);
    // pass A: stages 0..4 (bits 10..6); twiddle index uniform across the wave
    const ConstTable twc{(const_u64*)tw};
#pragma unroll
    for (int s = 0; s < 5; ++s) {
        const int h = 16 >> s;
#pragma unroll
        for (int r = 0; r < kRegs; ++r) {
            if (r & h) continue;
            const uint2 w = twc[(1 << s) + (r >> (5 - s))];
            ct_bfly(x[r], x[r + h], w, Q);
        }
        sched_fence();
    }
    transpose<0, 1>(x, lds, l);
    // pass B: stages 5..9 (bits 5..1)
    const uint32_t lo = opaque_v(l);
    const uint32_t lhi = lo >> 1;
    fwd_stage_b<5>(x, tw, lhi, Q);
    fwd_stage_b<6>(x, tw, lhi, Q);
    fwd_stage_b<7>(x, tw, lhi, Q);
    fwd_stage_b<8>(x, tw, lhi, Q);
    fwd_stage_b<9>(x, tw, lhi, Q);
    transpose<1, 2>(x, lds, l);
    // pass C: stage 10 (bit 0): index 1024 + (l << 4) + r/2, in two halves
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
        uint2 w[8];
        load_pairs<8>(w, tw + 1024u + (lo << 4) + 8u * hf);
#pragma unroll
        for (int m = 0; m < 8; ++m) ct_bfly(x[16 * hf + 2 * m], x[16 * hf + 2 * m + 1], w[m], Q);
        sched_fence();
    }
}

// ---- inverse NTT WITHOUT the N^-1 factor (Gentleman-Sande) -------------------
// twi[i] = { psi^-brv(i), companion }: reference rootOfUnityInverseTable.
// Input residues in [0, 2Q); output canonical coefficients in [0, Q).
__device__ __forceinline__ void ntt_inv_noscale(uint32_t (&x)[kRegs], uint32_t* lds, const uint2* twi_in,
                                                uint32_t l, uint32_t Q) {
    const uint2* twi = opaque(twi_in);
    const uint32_t lo = opaque_v(l);
    // pass C: bit 0
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
        uint2 w[8];
        load_pairs<8>(w, twi + 1024u + (lo << 4) + 8u * hf);
#pragma unroll
        for (int m = 0; m < 8; ++m) gs_bfly(x[16 * hf + 2 * m], x[16 * hf + 2 * m + 1], w[m], Q);
        sched_fence();
    }
    transpose<2, 1>(x, lds, l);
    // pass B: bits 1..5
    const uint32_t lhi = lo >> 1;
    inv_stage_b<1>(x, twi, lhi, Q);
    inv_stage_b<2>(x, twi, lhi, Q);
    inv_stage_b<3>(x, twi, lhi, Q);
    inv_stage_b<4>(x, twi, lhi, Q);
    inv_stage_b<5>(x, twi, lhi, Q);
    transpose<1, 0>(x, lds, l);
    // pass A: bits 6..10 ; uniform twiddles
    const ConstTable twc{(const_u64*)twi};
#pragma unroll
    for (int b = 6; b <= 10; ++b) {
        const int h = 1 << (b - 6);
#pragma unroll
        for (int r = 0; r < kRegs; ++r) {
            if (r & h) continue;
            const uint2 w = twc[(1 << (10 - b)) + (r >> (b - 5))];
            gs_bfly(x[r], x[r + h], w, Q);
        }
        sched_fence();
    }
#pragma unroll
    for (int r = 0; r < kRegs; ++r) x[r] = min(x[r], x[r] - Q);
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

// ---- signed digit decomposition helpers (mk-acc.cpp:54-80) ------------------
// sext of the low gbits bits: (d << (W-gBits)) >> (W-gBits)
__device__ __forceinline__ int32_t sext_low(int32_t d, uint32_t gbits) {
    return __builtin_amdgcn_sbfe(d, 0, gbits);
}
// centred value with the lowest digit already dropped
__device__ __forceinline__ int32_t sdd_start(uint32_t t, uint32_t Q, uint32_t qhalf, uint32_t gbits) {
    int32_t d = t < qhalf ? (int32_t)t : (int32_t)t - (int32_t)Q;
    int32_t r = sext_low(d, gbits);
    return (d - r) >> gbits;
}
// next digit as a residue; advances the running value
__device__ __forceinline__ uint32_t sdd_next(int32_t& d, uint32_t Q, uint32_t gbits) {
    int32_t r = sext_low(d, gbits);
    d = (d - r) >> gbits;
    return r < 0 ? (uint32_t)(r + (int32_t)Q) : (uint32_t)r;
}

// Digits 1..DG-1 of every element packed as signed bitfields: two elements per
// register when DG <= 3 (16-bit slots), one otherwise.  Digit 0 goes straight
// into the NTT, so only the rest is kept -- 16 VGPRs instead of a 32-VGPR
// running remainder for the common parameter sets.
template <int DG>
struct PackedDigits {
    static constexpr int kPer = DG <= 3 ? 2 : 1;           // elements per register
    static constexpr int kSlot = 32 / kPer;                // bits per element
    static constexpr int kField = kSlot / (DG - 1 > 0 ? DG - 1 : 1);
    static constexpr int kWords = kRegs / kPer;
    uint32_t w[kWords];

    // decompose coefficient t: returns digit 0 (as residue), stores 1..DG-1
    __device__ __forceinline__ uint32_t put(int r, uint32_t t, uint32_t Q, uint32_t qhalf, uint32_t gbits) {
        int32_t d = sdd_start(t, Q, qhalf, gbits);
        const uint32_t g0 = sdd_next(d, Q, gbits);
        uint32_t acc = 0;
#pragma unroll
        for (int i = 1; i < DG; ++i) {
            const int32_t rr = sext_low(d, gbits);
            d = (d - rr) >> gbits;
            acc |= ((uint32_t)rr & ((1u << kField) - 1u)) << ((i - 1) * kField);
        }
        if (kPer == 1 || (r % kPer) == 0) w[r / kPer] = acc;
        else w[r / kPer] |= acc << kSlot;
        // pin the packed word here: otherwise the compiler sinks the packing to
        // the later unpack and keeps every unpacked digit live across the NTTs
        if ((r % kPer) == kPer - 1) asm volatile("" : "+v"(w[r / kPer]));
        return g0;
    }
    // digit i (1..DG-1) of element r as a residue
    __device__ __forceinline__ uint32_t get(int r, int i, uint32_t Q) const {
        const int32_t rr = __builtin_amdgcn_sbfe((int32_t)w[r / kPer], (r % kPer) * kSlot + (i - 1) * kField, kField);
        return rr < 0 ? (uint32_t)(rr + (int32_t)Q) : (uint32_t)rr;
    }
};

}  // namespace mkacc

