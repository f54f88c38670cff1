// mkacc_layout2.hpp -- register / lane / LDS layouts of the TWO-waves-per-gate
// transforms (widereg2::step_kernel, FP64; round 4's 27-bit two-wave kernel and
// its EVAL layout LC4 were retired in round 5 -- git history, 7a372b6).
// Included inside mkacc_kernels.hpp's anonymous namespace.
//
// A polynomial of N = 2048 positions p (11 bits) is split over the two waves of a
// 128-thread workgroup, 16 elements per lane.  Position p sits at (wave w, lane l,
// register r) in one of four layouts (l written l5..l0):
//   LA  r = p10..p7, w = p6,  l = p5..p0                  coefficients
//   LB  r = p6..p3,  w = p10, l = (p9, p8, p7, p2, p1, p0)
//   LC  r = p3..p0,  w = p10, l = (p8, p4, p7, p9, p6, p5) EVAL slots ("C16")
//   LD  r = p7..p4,  w = p10, l = (p9, p8, p3, p2, p1, p0)
// Forward: LA stages 0-3 (wave-uniform twiddles) -> LB stages 4-6 -> LC stages
// 7-10; inverse: LC bits 0-3 (wave-uniform) -> LD bits 4-7 -> LA bits 8-10.
// The LDS element of position p is sum_k W_k p_k with
// W = 1, 2, 4, 8, 16, 33, 66, 136, 272, 548, 1088 -- injective, additive in every
// bit (a per-lane base plus a compile-time register offset, so one address VGPR and
// immediate offsets), and in every layout the 32 lanes of each half-wave hit 32
// distinct values mod 32 and the 16 lanes of each quarter 16 distinct
// values mod 16: conflict-free ds_read/ds_write_b32, ds_read_b64 and the 16-lane
// groups of ds_write_b64 / ds_read2_b64 (MI355X_MICROARCH.md s LDS; the first LC
// map, l = (p8, p9, p7, p6, p5, p4), put p4 -- weight 16 -- in a 16-lane group:
// 2.0 conflict cycles per LDS instruction, profiles/r4/pmc_c5_widereg2.txt).  tools/widereg2_model.py checks the maps
// exhaustively and runs both transforms on them in exact integers against the oracle.
#pragma once

namespace lay2 {

constexpr int kR = 16;                 // elements per lane and polynomial
constexpr int kBufE = 2175;            // LDS elements of one transpose buffer (max index 2174)
enum { LA = 0, LB = 1, LC = 2, LD = 3 };
constexpr int kW[11] = {1, 2, 4, 8, 16, 33, 66, 136, 272, 548, 1088};

// register offset of register r in layout L (compile time)
template <int L>
__host__ __device__ constexpr int roff(int r) {
    const int b0 = r & 1, b1 = (r >> 1) & 1, b2 = (r >> 2) & 1, b3 = (r >> 3) & 1;
    return L == LA   ? b0 * kW[7] + b1 * kW[8] + b2 * kW[9] + b3 * kW[10]
           : L == LB ? b0 * kW[3] + b1 * kW[4] + b2 * kW[5] + b3 * kW[6]
           : L == LD ? b0 * kW[4] + b1 * kW[5] + b2 * kW[6] + b3 * kW[7]
                     : r;   // LC: registers are p3..p0
}
// lane / wave base of layout L
template <int L>
__host__ __device__ __forceinline__ uint32_t lbase(uint32_t l, uint32_t w) {
    const uint32_t l0 = l & 1u, l1 = (l >> 1) & 1u, l2 = (l >> 2) & 1u, l3 = (l >> 3) & 1u, l4 = (l >> 4) & 1u,
                   l5 = (l >> 5) & 1u;
    if (L == LA) return (l & 31u) + l5 * kW[5] + w * kW[6];
    if (L == LB) return (l & 7u) + l3 * kW[7] + l4 * kW[8] + l5 * kW[9] + w * kW[10];
    if (L == LC) return l0 * kW[5] + l1 * kW[6] + l2 * kW[9] + l3 * kW[7] + l4 * kW[4] + l5 * kW[8] + w * kW[10];
    return (l & 15u) + l4 * kW[8] + l5 * kW[9] + w * kW[10];
}
// positions of (w, l, r)
__host__ __device__ __forceinline__ uint32_t pos_a(uint32_t w, uint32_t l, uint32_t r) { return (r << 7) | (w << 6) | l; }
__host__ __device__ __forceinline__ uint32_t pos_b(uint32_t w, uint32_t l, uint32_t r) {
    return (r << 3) | (l & 7u) | (((l >> 3) & 1u) << 7) | (((l >> 4) & 1u) << 8) | (((l >> 5) & 1u) << 9) | (w << 10);
}
__host__ __device__ __forceinline__ uint32_t pos_c(uint32_t w, uint32_t l, uint32_t r) {
    return r | (((l >> 4) & 1u) << 4) | ((l & 1u) << 5) | (((l >> 1) & 1u) << 6) | (((l >> 3) & 1u) << 7) |
           (((l >> 5) & 1u) << 8) | (((l >> 2) & 1u) << 9) | (w << 10);
}
__host__ __device__ __forceinline__ uint32_t pos_d(uint32_t w, uint32_t l, uint32_t r) {
    return (r << 4) | (l & 15u) | (((l >> 4) & 1u) << 8) | (((l >> 5) & 1u) << 9) | (w << 10);
}

// ---- per-lane twiddle tables (HBM, built by the host) ---------------------------------
// Entry k of sub-table T for (w, l) lives in pair row kTG0[T] + k / 2 at element k % 2:
// a row is 128 lanes x 16 bytes, so a wave loads two entries per lane with one 1 KiB
// dwordx4.  Entries are 8 bytes: a balanced double (FP64 kernel) or a {w, w'} Shoup
// pair (27-bit kernel).
//   TFB  forward LB stages 4..6:  k = (2^(s-4) - 1) + (r >> (8 - s))       (7 entries)
//   TFC  forward LC stages 7..10: k = (2^(s-7) - 1) + (r >> (11 - s))      (15)
//   TID  inverse LD bits 4..7:    k = (H - 1) + (r & (H - 1)), H = 2^(b-4) (15)
//   TIA  inverse LA bits 8..10:   k = (H - 2) + (r & (H - 1)), H = 2^(b-7) (14)
//   TTW  twist psi^-p (times N^-1 for the FP64 kernel): k = r             (16)
enum { TFB = 0, TFC = 1, TID = 2, TIA = 3, TTW = 4 };
constexpr int kTG0[5] = {0, 4, 12, 20, 27};
constexpr int kTPairs = 35;
constexpr int kTabE = kTPairs * 128 * 2;   // 8-byte entries
__host__ __device__ constexpr size_t tab_index(int T, uint32_t w, uint32_t l, int k) {
    return ((size_t)(kTG0[T] + k / 2) * 128 + w * 64 + l) * 2 + (size_t)(k & 1);
}

template <int NP>
struct TwPairs {
    u32x4 v[NP];
    __device__ __forceinline__ u32x2 raw(int k) const {
        const u32x4& q = v[k >> 1];
        return (k & 1) ? u32x2{q.z, q.w} : u32x2{q.x, q.y};
    }
};
template <int T, int NP>
__device__ __forceinline__ void tload(TwPairs<NP>& t, __amdgpu_buffer_rsrc_t rt, uint32_t vo) {
#pragma unroll
    for (int g = 0; g < NP; ++g) t.v[g] = bload4(rt, vo, (uint32_t)(kTG0[T] + g) * 2048u);
}

struct Lane {
    uint32_t l, w;      // lane, wave of the gate (0 / 1)
    uint32_t vt;        // byte offset of this lane in a twiddle pair row: (w * 64 + l) * 16
};

// ---- cross-wave transpose --------------------------------------------------------------
// Both waves write their elements, wait for their own LDS writes and meet at the
// 2-wave workgroup's barrier, then read.  A transform alternates two buffers, so the
// next write into a buffer comes after the partner passed the barrier that followed
// its last read of it (one barrier per transpose).
__device__ __forceinline__ void pair_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
template <int SRC, int DST, typename T>
__device__ __forceinline__ void transpose(T (&x)[kR], T* buf, uint32_t l, uint32_t w) {
    T* ws = buf + lbase<SRC>(l, w);
#pragma unroll
    for (int r = 0; r < kR; ++r) ws[roff<SRC>(r)] = x[r];
    pair_sync();
    const T* rs = buf + lbase<DST>(l, w);
#pragma unroll
    for (int r = 0; r < kR; ++r) x[r] = rs[roff<DST>(r)];
    asm volatile("" ::: "memory");
}

// Transposes between layouts with the same wave bit (LB, LC and LD all have w = p10)
// stay inside the wave's own half of the buffer (p10 carries W_10 = 1088, every other
// bit sums to at most 1086): no barrier, and no s_waitcnt either -- a wave's LDS
// accesses execute in order.  Buffer rule (ping-pong with one barrier per cross-wave
// transpose, Bufs below): a cross-wave transpose moves to the other buffer, a local
// one uses the buffer of the latest cross-wave transpose.  Then every write into a
// region the partner reads is separated from that read by a barrier both waves pass:
// LA -> LB (partner reads only its own half) may be followed by a local transpose in
// the same buffer; LD -> LA (partner reads both halves) is always followed by the
// next transform's LA -> LB, which moves to the other buffer.
template <int SRC, int DST, typename T>
__device__ __forceinline__ void transpose_local(T (&x)[kR], T* buf, uint32_t l, uint32_t w) {
    static_assert(SRC != LA && DST != LA, "wave-local transposes keep w = p10");
    T* ws = buf + lbase<SRC>(l, w);
#pragma unroll
    for (int r = 0; r < kR; ++r) ws[roff<SRC>(r)] = x[r];
    asm volatile("" ::: "memory");
    const T* rs = buf + lbase<DST>(l, w);
#pragma unroll
    for (int r = 0; r < kR; ++r) x[r] = rs[roff<DST>(r)];
    asm volatile("" ::: "memory");
}
template <typename T>
struct Bufs {
    T* base;
    uint32_t cb;   // buffer of the latest cross-wave transpose (wave-uniform)
    __device__ __forceinline__ T* cross() {
        cb ^= 1u;
        return base + cb * kBufE;
    }
    __device__ __forceinline__ T* cur() const { return base + cb * kBufE; }
};

}  // namespace lay2
