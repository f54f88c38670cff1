// mkkeys.cpp -- host key material for the MK gate path (include/mkfhe_keys.h):
// key generation, encryption and decryption for MK-NTRU and MK-LWE without
// NTL.  CPU only; init-time work, never on the bootstrapping path.
//
// The two NTL calls of the reference are replaced by exact equivalents:
//  * InvMod(inv, s, X^N+1) over Z_Q (binfhe-base-scheme.cpp:152-157): Q is a
//    prime = 1 mod 2N, so X^N+1 splits and s is a unit iff none of its NTT
//    values is zero; the inverse is the pointwise inverse in EVAL form (the
//    inverse is unique, so this is the polynomial NTL returns).
//  * inv(mat_ZZ_p) (mntru-pke.cpp:60-62): Gauss-Jordan elimination mod q
//    (q prime), with 64-bit lazy accumulation of the row updates.
// Everything else restates the reference line by line (citations per function).
#include "mkfhe_keys.h"

#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <exception>
#include <mutex>
#include <random>
#include <stdexcept>
#include <string>
#include <sys/types.h>
#include <thread>
#include <vector>

#include "mkacc_host_math.hpp"

namespace {

using namespace mkacc;

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

// ---------------------------------------------------------------------------
// randomness.  seed != 0 (tests, reproducible runs): xoshiro256** streams keyed by
// SplitMix64(seed, stream ids) -- fast, not cryptographic.  seed == 0 (the
// reference's behaviour: fresh keys every call): ChaCha20 with a 256-bit call
// key, one stream per (a, b, c) id in the nonce, so no secret is a function of
// a short seed.  The call keys come from the process's entropy journal: a
// 256-bit master key (std::random_device when first needed) and a counter of
// seed-0 calls; call key = ChaCha20 block of the master at nonce = counter.
// Whoever holds the master holds every seed-0 key of the process, so exporting
// it is an explicit opt-in: mkkg_entropy_replay(1) (which is also the only
// place MKFHE_ENTROPY is read; a malformed value is an error) or
// mkkg_entropy_set.  With it, a run whose gates decrypt wrong can be replayed
// exactly -- the reference's clock-seeded keys (binfhe-base-scheme.cpp:111,
// mntru-pke.cpp:27) cannot be.
// ---------------------------------------------------------------------------
inline uint64_t splitmix(uint64_t& x) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct Seed {
    uint64_t s = 0;        // explicit seed (xoshiro)
    bool secure = false;   // ChaCha20 with key[]
    uint32_t key[8] = {};
};

struct ChaCha20;
void chacha_block(const uint32_t key[8], uint32_t n0, uint32_t n1, uint32_t out[16]);

struct Entropy {
    std::mutex mu;
    bool init = false;
    bool replay = false;   // master exportable (mkkg_entropy_replay / mkkg_entropy_set)
    uint32_t master[8] = {};
    uint64_t calls = 0;
};
Entropy& entropy() {
    static Entropy e;
    return e;
}
bool parse_hex256(const char* h, uint32_t out[8]) {
    if (!h || std::strlen(h) != 64) return false;
    for (int i = 0; i < 8; ++i) {
        uint32_t w = 0;
        for (int j = 0; j < 8; ++j) {
            const char ch = h[8 * i + j];
            const int v = ch >= '0' && ch <= '9' ? ch - '0' : ch >= 'a' && ch <= 'f' ? ch - 'a' + 10
                        : ch >= 'A' && ch <= 'F' ? ch - 'A' + 10 : -1;
            if (v < 0) return false;
            w = (w << 4) | (uint32_t)v;
        }
        out[i] = w;
    }
    return true;
}
// caller holds e.mu
void entropy_init_locked(Entropy& e) {
    if (e.init) return;
    std::random_device rd;
    for (auto& w : e.master) w = rd();
    e.calls = 0;
    e.init = true;
}

Seed resolve_seed(uint64_t seed) {
    Seed r;
    if (seed) {
        r.s = seed;
        return r;
    }
    Entropy& e = entropy();
    uint64_t call;
    uint32_t master[8];
    {
        std::lock_guard<std::mutex> lk(e.mu);
        entropy_init_locked(e);
        call = e.calls++;
        std::memcpy(master, e.master, sizeof master);
    }
    uint32_t blk[16];
    chacha_block(master, (uint32_t)call, (uint32_t)(call >> 32) | 0x80000000u, blk);
    std::memcpy(r.key, blk, sizeof r.key);
    r.secure = true;
    return r;
}

// ChaCha20 block function (RFC 8439 s2.3, 20 rounds; 64-bit block counter and
// 64-bit nonce as in the original construction)
struct ChaCha20 {
    uint32_t st[16];
    uint32_t buf[16];
    int pos = 16;
    ChaCha20(const uint32_t key[8], uint32_t n0, uint32_t n1) {
        st[0] = 0x61707865u; st[1] = 0x3320646eu; st[2] = 0x79622d32u; st[3] = 0x6b206574u;
        for (int i = 0; i < 8; ++i) st[4 + i] = key[i];
        st[12] = st[13] = 0;   // block counter
        st[14] = n0;
        st[15] = n1;
    }
    static uint32_t rotl(uint32_t v, int k) { return (v << k) | (v >> (32 - k)); }
    static void qr(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
        a += b; d ^= a; d = rotl(d, 16);
        c += d; b ^= c; b = rotl(b, 12);
        a += b; d ^= a; d = rotl(d, 8);
        c += d; b ^= c; b = rotl(b, 7);
    }
    void refill() {
        uint32_t x[16];
        for (int i = 0; i < 16; ++i) x[i] = st[i];
        for (int r = 0; r < 10; ++r) {
            qr(x[0], x[4], x[8], x[12]); qr(x[1], x[5], x[9], x[13]);
            qr(x[2], x[6], x[10], x[14]); qr(x[3], x[7], x[11], x[15]);
            qr(x[0], x[5], x[10], x[15]); qr(x[1], x[6], x[11], x[12]);
            qr(x[2], x[7], x[8], x[13]); qr(x[3], x[4], x[9], x[14]);
        }
        for (int i = 0; i < 16; ++i) buf[i] = x[i] + st[i];
        if (++st[12] == 0) ++st[13];
        pos = 0;
    }
    uint64_t next() {
        if (pos > 14) refill();
        const uint64_t v = (uint64_t)buf[pos] | ((uint64_t)buf[pos + 1] << 32);
        pos += 2;
        return v;
    }
};
void chacha_block(const uint32_t key[8], uint32_t n0, uint32_t n1, uint32_t out[16]) {
    ChaCha20 c(key, n0, n1);
    c.refill();
    std::memcpy(out, c.buf, 16 * sizeof(uint32_t));
}

struct Rng {
    uint64_t s[4];
    bool secure;
    ChaCha20 cc;
    // stream ids: a < 2^8 (call kind), b < 2^24, c < 2^32
    Rng(const Seed& sd, uint64_t a, uint64_t b = 0, uint64_t c = 0)
        : secure(sd.secure), cc(sd.key, (uint32_t)(a | (b << 8)), (uint32_t)c) {
        if (secure) {
            if (a >= 256 || b >= (1u << 24) || c >> 32) throw std::runtime_error("random stream id out of range");
            return;
        }
        uint64_t x = sd.s;
        x ^= splitmix(x) + a * 0xD1B54A32D192ED03ull;
        x ^= splitmix(x) + b * 0xABC98388FB8FAC03ull;
        x ^= splitmix(x) + c * 0x8CB92BA72F3D8DD7ull;
        for (auto& w : s) w = splitmix(x);
    }
    static uint64_t rotl(uint64_t v, int k) { return (v << k) | (v >> (64 - k)); }
    uint64_t next() {
        if (secure) return cc.next();
        const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
        s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3];
        s[2] ^= t; s[3] = rotl(s[3], 45);
        return r;
    }
    double u01() { return (double)(next() >> 11) * 0x1.0p-53; }  // [0, 1)
    // std::normal_distribution(0, sd) (Box-Muller; the reference's engine is
    // clock-seeded, so only the distribution is reproduced)
    double normal(double sd) {
        double u1;
        do u1 = u01(); while (u1 <= 0.0);
        return sd * std::sqrt(-2.0 * std::log(u1)) * std::cos(2.0 * M_PI * u01());
    }
    // uniform_int_distribution<int>(-1, 1)
    int ternary() {
        for (;;) {
            const uint32_t v = (uint32_t)(next() >> 62);
            if (v < 3) return (int)v - 1;
        }
    }
    int binary() { return (int)(next() >> 63); }
};

// OpenFHE DiscreteGaussianGeneratorImpl, Peikert inversion sampling
// (reference src/core/include/math/discretegaussiangenerator-impl.h:82-156):
// cumulative table of exp(-x^2 / 2 sigma^2), x = 1 .. ceil(sigma * sqrt(-2 ln 5e-32)).
struct Dgg {
    double a = 1.0;
    std::vector<double> vals;
    explicit Dgg(double sd) {
        const double M = std::sqrt(-2.0 * std::log(5e-32));
        const int fin = (int)std::ceil(sd * M);
        const double var = 2.0 * sd * sd;
        double cusum = 0.0;
        for (int x = 1; x <= fin; ++x) {
            cusum += std::exp(-((double)(x * x) / var));
            vals.push_back(cusum);
        }
        a = 1.0 / (2.0 * cusum + 1.0);
        for (auto& v : vals) v *= a;
    }
    int32_t sample(Rng& r) const {
        const double seed = r.u01() - 0.5;
        const double tmp = std::fabs(seed) - a / 2;
        if (tmp <= 0) return 0;
        size_t idx = (size_t)(std::lower_bound(vals.begin(), vals.end(), tmp) - vals.begin()) + 1;
        if (idx > vals.size()) idx = vals.size();  // reference throws (probability < 5e-32)
        return (int32_t)idx * (seed > 0 ? 1 : -1);
    }
};

// encryptions per call: the item index is the 24-bit stream id b of Rng
constexpr size_t kMaxPerCall = (size_t)1 << 24;

inline uint32_t to_mod(int64_t v, uint64_t m) {
    int64_t r = v % (int64_t)m;
    return (uint32_t)(r < 0 ? r + (int64_t)m : r);
}
inline int64_t centered(uint32_t v, uint64_t m) { return v > m / 2 ? (int64_t)v - (int64_t)m : (int64_t)v; }
// NativeVector::SwitchModulus (centred lift, used where the reference switches q -> mod)
inline uint32_t switch_mod(uint32_t v, uint64_t from, uint64_t to) {
    return from == to ? v : to_mod(centered(v, from), to);
}

// ---------------------------------------------------------------------------
// threads
// ---------------------------------------------------------------------------
unsigned n_threads() {
    unsigned h = std::thread::hardware_concurrency();
    if (const char* e = std::getenv("OMP_NUM_THREADS")) {
        const int v = std::atoi(e);
        if (v > 0) h = std::min<unsigned>(h ? h : v, (unsigned)v);
    }
    return std::max(1u, std::min(h ? h : 1u, 16u));
}

template <class F>
void parallel_for(size_t n, F&& f) {
    const unsigned T = (unsigned)std::min<size_t>(n_threads(), n);
    if (T <= 1) {
        for (size_t i = 0; i < n; ++i) f(i);
        return;
    }
    std::atomic<size_t> next{0};
    std::vector<std::thread> th;
    std::exception_ptr err;
    std::mutex emu;
    for (unsigned t = 0; t < T; ++t)
        th.emplace_back([&] {
            try {
                for (size_t i; (i = next.fetch_add(1)) < n;) f(i);
            } catch (...) {   // an exception must not leave a worker thread (std::terminate)
                std::lock_guard<std::mutex> lk(emu);
                if (!err) err = std::current_exception();
                next = n;
            }
        });
    for (auto& t : th) t.join();
    if (err) std::rethrow_exception(err);
}

// ---------------------------------------------------------------------------
// ring Z_Q[X]/(X^N+1): the reference's NTT in its bit-reversed EVAL order
// (ChineseRemainderTransformFTTNat, transformnat-impl.h:300-354, 492-552,
//  tables 705-760: table[brv(i)] = psi^i), Shoup products
// ---------------------------------------------------------------------------
struct Ring {
    uint32_t N = 0, lg = 0;
    uint64_t Q = 0;
    std::vector<uint32_t> w, ws, wi, wis;  // forward / inverse twiddles + Shoup companions
    uint32_t ninv = 0, ninvs = 0;

    static uint32_t shoup(uint64_t x, uint64_t Q) { return (uint32_t)((x << 32) / Q); }
    uint32_t mul(uint32_t a, uint32_t b, uint32_t bs) const {
        const uint64_t qt = ((uint64_t)a * bs) >> 32;
        uint64_t r = (uint64_t)a * b - qt * Q;
        return (uint32_t)(r >= Q ? r - Q : r);
    }
    uint32_t mulmod_full(uint32_t a, uint32_t b) const { return (uint32_t)((uint64_t)a * b % Q); }

    Ring(uint32_t N_, uint64_t Q_, uint64_t psi) : N(N_), Q(Q_) {
        while ((1u << lg) < N) ++lg;
        w.resize(N); ws.resize(N); wi.resize(N); wis.resize(N);
        const uint64_t psiI = modinv(psi, Q);
        uint64_t x = 1, xi = 1;
        for (uint32_t i = 0; i < N; ++i) {
            const uint32_t r = bit_reverse(i, lg);
            w[r] = (uint32_t)x; ws[r] = shoup(x, Q);
            wi[r] = (uint32_t)xi; wis[r] = shoup(xi, Q);
            x = mulmod(x, psi, Q);
            xi = mulmod(xi, psiI, Q);
        }
        ninv = (uint32_t)modinv(N, Q);
        ninvs = shoup(ninv, Q);
    }
    // COEFF -> EVAL (ForwardTransformToBitReverseInPlace)
    void fwd(uint32_t* a) const {
        for (uint32_t m = 1, t = N >> 1; m < N; m <<= 1, t >>= 1)
            for (uint32_t i = 0; i < m; ++i) {
                const uint32_t W = w[m + i], Ws = ws[m + i];
                for (uint32_t j = 2 * i * t; j < 2 * i * t + t; ++j) {
                    const uint32_t U = a[j], V = mul(a[j + t], W, Ws);
                    const uint32_t s = U + V;
                    a[j] = s >= Q ? s - (uint32_t)Q : s;
                    a[j + t] = U >= V ? U - V : U + (uint32_t)Q - V;
                }
            }
    }
    // EVAL -> COEFF (InverseTransformFromBitReverseInPlace, GS, times N^-1)
    void inv(uint32_t* a) const {
        for (uint32_t m = N >> 1, t = 1; m >= 1; m >>= 1, t <<= 1)
            for (uint32_t i = 0; i < m; ++i) {
                const uint32_t W = wi[m + i], Ws = wis[m + i];
                for (uint32_t j = 2 * i * t; j < 2 * i * t + t; ++j) {
                    const uint32_t U = a[j], V = a[j + t];
                    const uint32_t s = U + V;
                    a[j] = s >= Q ? s - (uint32_t)Q : s;
                    a[j + t] = mul(U >= V ? U - V : U + (uint32_t)Q - V, W, Ws);
                }
            }
        for (uint32_t j = 0; j < N; ++j) a[j] = mul(a[j], ninv, ninvs);
    }
};

// ---------------------------------------------------------------------------
// parameter checks
// ---------------------------------------------------------------------------
struct P {
    uint32_t method, k, n, N, dg, nk, baseG, baseKS, dks;
    uint64_t Q, q, qKS, root;
};

int unpack(const mkkg_params* p, P& o) {
    if (!p) return fail(MKACC_E_ARG, "null parameters");
    const mkacc_params& a = p->acc;
    o.method = a.method;
    o.k = a.k; o.n = a.n; o.N = a.N; o.Q = a.Q; o.q = a.q; o.baseG = a.baseG;
    if (o.method > MKACC_METHOD_MKNTRU_LWE) return fail(MKACC_E_ARG, "bad method");
    if (!o.k || !o.n || !o.N || (o.N & (o.N - 1)) || o.N < 8) return fail(MKACC_E_ARG, "bad k, n or N");
    if (o.Q < 3 || o.Q >= (1ull << 31) || !is_prime(o.Q) || (o.Q - 1) % (2ull * o.N))
        return fail(MKACC_E_ARG, "Q must be a prime < 2^31 with Q = 1 mod 2N");
    if (o.baseG < 2 || (o.baseG & (o.baseG - 1))) return fail(MKACC_E_ARG, "Gadget base should be a power of two.");
    const uint32_t digitsG = a.digitsG ? a.digitsG : digits_g(o.Q, o.baseG);
    if (digitsG < 2) return fail(MKACC_E_ARG, "digitsG must be at least 2");
    o.dg = digitsG - 1;
    o.nk = o.method == MKACC_METHOD_MKNTRU ? 2 : 1;
    o.root = a.root ? a.root : root_of_unity(2ull * o.N, o.Q);
    if (!is_primitive_root(o.root, 2ull * o.N, o.Q)) return fail(MKACC_E_ARG, "root is not a primitive 2N-th root");
    o.qKS = p->ks.qKS ? p->ks.qKS : o.q;
    o.baseKS = p->ks.baseKS;
    if (o.q < 4 || o.q >= (1ull << 16) || o.qKS < 4 || o.qKS >= (1ull << 16))
        return fail(MKACC_E_UNSUPPORTED, "key material supports q, qKS < 2^16 (every MK parameter set)");
    if (o.baseKS < 2 || o.baseKS > 256) return fail(MKACC_E_ARG, "baseKS must be in [2, 256]");
    if (p->ks.n_out && p->ks.n_out != o.n) return fail(MKACC_E_ARG, "ks.n_out must equal n");
    o.dks = ks_digit_count(o.qKS, o.baseKS);
    return MKACC_OK;
}

#define UNPACK(p, P_)                      \
    P P_;                                  \
    {                                      \
        const int rc_ = unpack((p), P_);   \
        if (rc_) return rc_;               \
    }

// ---------------------------------------------------------------------------
// Gauss-Jordan inverse mod q (replaces NTL inv(mat_ZZ_p), mntru-pke.cpp:60-62).
// Rows of [M | I] are held as 64-bit lazy sums: an update adds (q - f) * p_j
// with both factors < 2^16, so n updates stay far below 2^64.  Returns false
// if M is singular mod q.
// ---------------------------------------------------------------------------
bool invert_mod(const std::vector<uint32_t>& M, uint32_t n, uint32_t q, std::vector<uint32_t>& out) {
    const size_t W = 2 * (size_t)n;
    std::vector<uint64_t> A((size_t)n * W, 0);
    for (uint32_t r = 0; r < n; ++r) {
        for (uint32_t c = 0; c < n; ++c) A[r * W + c] = M[(size_t)r * n + c];
        A[r * W + n + r] = 1;
    }
    std::vector<uint32_t> prow(W);
    for (uint32_t c = 0; c < n; ++c) {
        uint32_t piv = n;
        for (uint32_t r = c; r < n; ++r)
            if (A[r * W + c] % q) { piv = r; break; }
        if (piv == n) return false;
        if (piv != c)
            for (size_t j = 0; j < W; ++j) std::swap(A[piv * W + j], A[c * W + j]);
        uint64_t* pr = &A[c * W];
        const uint64_t inv = modinv(pr[c] % q, q);
        for (size_t j = c; j < W; ++j) {
            const uint32_t v = (uint32_t)((pr[j] % q) * inv % q);
            pr[j] = v;
            prow[j] = v;
        }
        parallel_for((n + 31) / 32, [&](size_t blk) {
            const uint32_t r0 = (uint32_t)blk * 32, r1 = std::min(n, r0 + 32);
            for (uint32_t r = r0; r < r1; ++r) {
                if (r == c) continue;
                uint64_t* row = &A[r * W];
                const uint32_t f = (uint32_t)(row[c] % q);
                if (!f) continue;
                const uint32_t g = q - f;
                for (size_t j = c; j < W; ++j) row[j] += (uint64_t)(g * prow[j]);  // g*p < 2^32
            }
        });
    }
    out.resize((size_t)n * n);
    for (uint32_t r = 0; r < n; ++r)
        for (uint32_t c = 0; c < n; ++c) out[(size_t)r * n + c] = (uint32_t)(A[r * W + n + c] % q);
    return true;
}

// g_i = Gpow[i+1] = baseG^(i+1) mod Q (mk-cryptoparameters.cpp:27-33): a constant
// polynomial, so its EVAL form is the constant in every slot.
uint32_t gpow(const P& p, uint32_t i) {
    uint64_t v = 1;
    for (uint32_t t = 0; t <= i; ++t) v = v * p.baseG % p.Q;
    return (uint32_t)v;
}

void sample_poly_eval(const Ring& R, const Dgg& g, Rng& r, uint32_t* out) {
    for (uint32_t j = 0; j < R.N; ++j) out[j] = to_mod(g.sample(r), R.Q);
    R.fwd(out);
}

// KeyGenXZW / KDMKeyGenXZW (mk-acc-xzw.cpp:132-228, identical in
// mk-acc-xzw_B.cpp:135-220) for one (u, i) slot: out [dg][2][N] EVAL.
//   r   <- NTT(DggR)                                   (skrPoly)
//   f_t  = (NTT(e1) + g_t * r) * s^-1
//   d_t  = NTT(e0) + [m] g_t (KeyGen) or [m] g_t * s^-1 (KDM) + r[t] * CRS_t
// r[t] is the EVAL slot t of r (skrPoly[i] in the reference), a scalar.
//
// The r-defect: the r-terms cancel in HbProd only when r = 0, so a key whose r
// has a nonzero coefficient breaks the gates that use it.  The
// default policy keeps the reference's keys bit for bit and only counts such
// keys; MKKG_RDEFECT_RESAMPLE draws r again from the slot's own stream until it
// is zero (r conditioned on 0).  Returns whether the slot's first r was nonzero.
bool unienc_key(const P& p, const Ring& R, const Dgg& dgg, const Dgg& dggR, Rng& rng, const uint32_t* crs,
                const uint32_t* sinv, bool m, bool kdm, uint32_t* out, uint32_t policy) {
    const uint32_t N = p.N;
    const uint32_t Q = (uint32_t)p.Q;
    std::vector<uint32_t> r(N), e0(N), e1(N);
    bool drew_defect = false;   // the slot's first r had a nonzero coefficient
    for (int attempt = 0;; ++attempt) {
        for (uint32_t j = 0; j < N; ++j) r[j] = to_mod(dggR.sample(rng), R.Q);
        const bool defect = std::any_of(r.begin(), r.end(), [](uint32_t x) { return x != 0; });
        if (attempt == 0) drew_defect = defect;
        if (!defect || policy != MKKG_RDEFECT_RESAMPLE) break;
        if (attempt == 64) throw std::runtime_error("DggR kept drawing nonzero samples");
    }
    R.fwd(r.data());
    for (uint32_t t = 0; t < p.dg; ++t) {
        sample_poly_eval(R, dgg, rng, e0.data());
        sample_poly_eval(R, dgg, rng, e1.data());
        const uint32_t g = gpow(p, t);
        const uint32_t rt = r[t];
        uint32_t* d = out + (size_t)t * 2 * N;
        uint32_t* f = d + N;
        for (uint32_t j = 0; j < N; ++j) {
            const uint32_t fr = (uint32_t)(((uint64_t)e1[j] + (uint64_t)g * r[j]) % Q);
            f[j] = R.mulmod_full(fr, sinv[j]);
            uint64_t dv = e0[j];
            if (m) dv += kdm ? R.mulmod_full(g, sinv[j]) : g;
            dv += (uint64_t)rt * crs[(size_t)t * N + j] % Q;
            d[j] = (uint32_t)(dv % Q);
        }
    }
    return drew_defect;
}

}  // namespace

extern "C" {

int mkkg_abi_version(void) { return MKKG_ABI_VERSION; }

#ifndef MKKG_HEADER_ID
#define MKKG_HEADER_ID "unknown"
#endif
#ifndef MKKG_SOURCE_ID
#define MKKG_SOURCE_ID "unknown"
#endif
#ifndef MKKG_BUILD_FLAGS
#define MKKG_BUILD_FLAGS ""
#endif
const char* mkkg_build_info(void) {
    static const std::string info = "abi=" + std::to_string(MKKG_ABI_VERSION) +
                                    ";header=" MKKG_HEADER_ID ";source=" MKKG_SOURCE_ID ";flags=" MKKG_BUILD_FLAGS;
    return info.c_str();
}

int mkkg_entropy_replay(int enable) try {
    Entropy& e = entropy();
    std::lock_guard<std::mutex> lk(e.mu);
    if (!enable) {
        e.replay = false;
        return MKACC_OK;
    }
    if (const char* env = std::getenv("MKFHE_ENTROPY")) {
        uint32_t m[8];
        if (!parse_hex256(env, m))
            return fail(MKACC_E_ARG, "MKFHE_ENTROPY must be 64 hex digits; the replay journal was not enabled");
        // the imported master restarts the call counter, so it is imported only while no
        // seed-0 call has drawn from the journal: a restart after one would make later
        // seed-0 keys and ciphertexts reuse the call keys of earlier ones.  A repeated
        // opt-in with the journal's own master keeps the counter.
        if (e.init && e.calls != 0) {
            if (std::memcmp(e.master, m, sizeof m) != 0)
                return fail(MKACC_E_ARG, "MKFHE_ENTROPY is imported only before the first seed-0 call of the "
                                         "process; the journal keeps its master and counter");
        } else {
            std::memcpy(e.master, m, sizeof m);
            e.calls = 0;
            e.init = true;
        }
    } else {
        entropy_init_locked(e);
    }
    e.replay = true;
    return MKACC_OK;
} catch (const std::exception& e) {
    return fail(MKACC_E_ARG, std::string("mkkg_entropy_replay: ") + e.what());
}

int mkkg_entropy_get(uint32_t master[8], uint64_t* calls) try {
    if (!master) return fail(MKACC_E_ARG, "null argument");
    Entropy& e = entropy();
    std::lock_guard<std::mutex> lk(e.mu);
    if (!e.replay)
        return fail(MKACC_E_ARG, "the entropy master is not exportable: call mkkg_entropy_replay(1) first "
                                 "(whoever holds the master holds every seed-0 key of the process)");
    entropy_init_locked(e);
    std::memcpy(master, e.master, sizeof e.master);
    if (calls) *calls = e.calls;
    return MKACC_OK;
} catch (const std::exception& e) {
    return fail(MKACC_E_ARG, std::string("mkkg_entropy_get: ") + e.what());
}

int mkkg_entropy_set(const uint32_t master[8], uint64_t calls) try {
    Entropy& e = entropy();
    std::lock_guard<std::mutex> lk(e.mu);
    if (master) {
        std::memcpy(e.master, master, sizeof e.master);
    } else {
        std::random_device rd;
        for (auto& w : e.master) w = rd();
    }
    e.calls = calls;
    e.init = true;
    e.replay = true;
    return MKACC_OK;
} catch (const std::exception& e) {
    return fail(MKACC_E_ARG, std::string("mkkg_entropy_set: ") + e.what());
}
const char* mkkg_last_error(void) { return g_err.c_str(); }

int mkkg_paramset(const char* name, uint32_t method, mkkg_params* out) try {
    if (!name || !out) return fail(MKACC_E_ARG, "null argument");
    const ParamRow* row = find_paramset(name);
    if (!row) return fail(MKACC_E_ARG, std::string("unknown parameter set ") + name);
    if (method > MKACC_METHOD_MKNTRU_LWE) return fail(MKACC_E_ARG, "bad method");
    mkkg_params p{};
    p.acc.method = method;
    p.acc.k = row->numUser;
    p.acc.n = row->latticeParam;
    p.acc.N = row->cyclOrder / 2;
    p.acc.Q = previous_prime(first_prime(row->numberBits, row->cyclOrder), row->cyclOrder);
    p.acc.q = row->mod;
    p.acc.baseG = row->gadgetBase;
    p.acc.digitsG = digits_g(p.acc.Q, p.acc.baseG);
    p.acc.root = root_of_unity(2ull * p.acc.N, p.acc.Q);
    p.ks.qKS = row->modKS;
    p.ks.baseKS = row->baseKS;
    p.ks.n_out = row->latticeParam;
    p.sigma = row->stdDev;
    p.sigma_unienc = 0.25;
    p.sigma_r = 0.15;
    p.lwe_keydist = row->keyDist;
    // MKKeyGen samples s_u GAUSSIAN for MK-NTRU (binfhe-base-scheme.cpp:216)
    // and UNIFORM_TERNARY for MK-LWE (:297)
    p.ring_keydist = method == MKACC_METHOD_MKNTRU_LWE ? MKKG_DIST_TERNARY : MKKG_DIST_GAUSSIAN;
    *out = p;
    return MKACC_OK;
} catch (const std::exception& e) {
    return fail(MKACC_E_ARG, std::string("mkkg_paramset: ") + e.what());
}

size_t mkkg_evk_words(const mkkg_params* pp) {
    P p;
    if (unpack(pp, p)) return 0;
    return (size_t)p.k * p.nk * (p.n + 1) * p.dg * 2 * p.N;
}
size_t mkkg_pkey_words(const mkkg_params* pp) {
    P p;
    if (unpack(pp, p)) return 0;
    return (size_t)p.k * p.dg * p.N;
}
size_t mkkg_ksk_mntru_words(const mkkg_params* pp) {
    P p;
    if (unpack(pp, p)) return 0;
    return (size_t)p.k * p.N * p.dks * p.n;
}
size_t mkkg_ksk_mklwe_a_words(const mkkg_params* pp) {
    P p;
    if (unpack(pp, p)) return 0;
    return (size_t)p.k * p.N * p.baseKS * p.dks * p.n;
}
size_t mkkg_ksk_mklwe_b_words(const mkkg_params* pp) {
    P p;
    if (unpack(pp, p)) return 0;
    return (size_t)p.k * p.N * p.baseKS * p.dks;
}

// MNTRUEncryptionScheme::KeyGen / KeyGenGaussian (mntru-pke.cpp:124-156) with
// Get_invertible_Matrix (:19-106): entries uniform ternary, or N(0,1) assigned
// to a ZZ_p (truncated toward zero); resampled until invertible mod qKS.
int mkkg_mntru_keygen(const mkkg_params* pp, uint64_t seed, uint32_t* F, uint32_t* Finv) try {
    UNPACK(pp, p);
    if (!F || !Finv) return fail(MKACC_E_ARG, "null output");
    const Seed sd = resolve_seed(seed);
    const uint32_t n = p.n, q = (uint32_t)p.qKS;
    std::vector<uint32_t> M((size_t)n * n), Mi;
    for (uint32_t u = 0; u < p.k; ++u) {
        for (uint64_t attempt = 0;; ++attempt) {
            Rng r(sd, 1, u, attempt);
            for (auto& v : M) {
                const int64_t x = pp->lwe_keydist == MKKG_DIST_GAUSSIAN ? (int64_t)r.normal(1.0) : r.ternary();
                v = to_mod(x, q);
            }
            if (invert_mod(M, n, q, Mi)) break;
            if (attempt > 64) return fail(MKACC_E_ARG, "no invertible key matrix after 64 samples");
        }
        std::memcpy(F + (size_t)u * n * n, M.data(), M.size() * 4);
        std::memcpy(Finv + (size_t)u * n * n, Mi.data(), Mi.size() * 4);
    }
    return MKACC_OK;
} catch (const std::exception& e) {
    return fail(MKACC_E_ARG, std::string("mkkg_mntru_keygen: ") + e.what());
}

// MKLWEEncryptionScheme::KeyGenBinary (mklwe-pke.cpp:19-34)
int mkkg_mklwe_keygen(const mkkg_params* pp, uint64_t seed, uint32_t* s) try {
    UNPACK(pp, p);
    if (!s) return fail(MKACC_E_ARG, "null output");
    const Seed sd = resolve_seed(seed);
    for (uint32_t u = 0; u < p.k; ++u) {
        Rng r(sd, 2, u);
        for (uint32_t i = 0; i < p.n; ++i) s[(size_t)u * p.n + i] = (uint32_t)r.binary();
    }
    return MKACC_OK;
} catch (const std::exception& e) {
    return fail(MKACC_E_ARG, std::string("mkkg_mklwe_keygen: ") + e.what());
}

// m_CRS = dg polys NativePoly(m_dgg, COEFFICIENT) -> EVALUATION (mk-cryptoparameters.h:173-178)
int mkkg_crs(const mkkg_params* pp, uint64_t seed, uint32_t* crs) try {
    UNPACK(pp, p);
    if (!crs) return fail(MKACC_E_ARG, "null output");
    const Seed sd = resolve_seed(seed);
    const Ring R(p.N, p.Q, p.root);
    const Dgg g(pp->sigma_unienc);
    for (uint32_t i = 0; i < p.dg; ++i) {
        Rng r(sd, 3, i);
        sample_poly_eval(R, g, r, crs + (size_t)i * p.N);
    }
    return MKACC_OK;
} catch (const std::exception& e) {
    return fail(MKACC_E_ARG, std::string("mkkg_crs: ") + e.what());
}

// Get_invertible_NativeVector (binfhe-base-scheme.cpp:104-195): coefficients
// from N(0, 0.5) assigned to ZZ_p (truncated; GAUSSIAN) or uniform ternary,
// resampled until s is a unit mod (X^N+1, Q).
int mkkg_ring_secrets(const mkkg_params* pp, uint64_t seed, uint32_t* skN, uint32_t* skN_eval,
                      uint32_t* skNinv_eval) try {
    UNPACK(pp, p);
    if (!skN || !skN_eval || !skNinv_eval) return fail(MKACC_E_ARG, "null output");
    const Seed sd = resolve_seed(seed);
    const Ring R(p.N, p.Q, p.root);
    const uint32_t N = p.N;
    std::vector<uint32_t> c(N), e(N);
    for (uint32_t u = 0; u < p.k; ++u) {
        for (uint64_t attempt = 0;; ++attempt) {
            Rng r(sd, 4, u, attempt);
            for (uint32_t j = 0; j < N; ++j) {
                const int64_t x = pp->ring_keydist == MKKG_DIST_TERNARY ? r.ternary() : (int64_t)r.normal(0.5);
                c[j] = to_mod(x, p.Q);
            }
            e = c;
            R.fwd(e.data());
            if (std::find(e.begin(), e.end(), 0u) == e.end()) break;
            if (attempt > 1000) return fail(MKACC_E_ARG, "no invertible ring secret after 1000 samples");
        }
        std::memcpy(skN + (size_t)u * N, c.data(), N * 4);
        std::memcpy(skN_eval + (size_t)u * N, e.data(), N * 4);
        for (uint32_t j = 0; j < N; ++j) skNinv_eval[(size_t)u * N + j] = (uint32_t)modinv(e[j], p.Q);
    }
    return MKACC_OK;
} catch (const std::exception& e) {
    return fail(MKACC_E_ARG, std::string("mkkg_ring_secrets: ") + e.what());
}

// Pkey[u][i] = e_i - CRS[i] * s_u, e_i <- NTT(m_dgg) (binfhe-base-scheme.cpp:255-268)
int mkkg_pkey(const mkkg_params* pp, uint64_t seed, const uint32_t* crs, const uint32_t* skN_eval, uint32_t* pkey) try {
    UNPACK(pp, p);
    if (!crs || !skN_eval || !pkey) return fail(MKACC_E_ARG, "null argument");
    const Seed sd = resolve_seed(seed);
    const Ring R(p.N, p.Q, p.root);
    const Dgg g(pp->sigma_unienc);
    const uint32_t N = p.N;
    std::vector<uint32_t> e(N);
    for (uint32_t u = 0; u < p.k; ++u)
        for (uint32_t i = 0; i < p.dg; ++i) {
            Rng r(sd, 5, u, i);
            sample_poly_eval(R, g, r, e.data());
            uint32_t* out = pkey + ((size_t)u * p.dg + i) * N;
            for (uint32_t j = 0; j < N; ++j) {
                const uint32_t cs = R.mulmod_full(crs[(size_t)i * N + j], skN_eval[(size_t)u * N + j]);
                out[j] = e[j] >= cs ? e[j] - cs : e[j] + (uint32_t)p.Q - cs;
            }
        }
    return MKACC_OK;
} catch (const std::exception& e) {
    return fail(MKACC_E_ARG, std::string("mkkg_pkey: ") + e.what());
}

// KeyGenAcc (mk-acc-xzw.cpp:38-87 / mk-acc-xzw_B.cpp:38-101):
//   XZW:   ek[u][0][i] = Enc(s == 1), ek[u][1][i] = Enc(s == q-1); slot (0,0)
//          is KDM, plus ek[0][0][n] = KDM-Enc(1).  Unset slots are zero.
//   XZW_B: ek[u][0][i] = Enc(s == 1); slot (0,0) KDM, ek[0][0][n] = KDM-Enc(1).
int mkkg_acc_keygen(const mkkg_params* pp, uint64_t seed, const uint32_t* crs, const uint32_t* skNinv_eval,
                    const uint32_t* lwe_sk, uint32_t* evk) {
    return mkkg_acc_keygen_ex(pp, seed, crs, skNinv_eval, lwe_sk, evk, MKKG_RDEFECT_KEEP, nullptr);
}

int mkkg_acc_keygen_ex(const mkkg_params* pp, uint64_t seed, const uint32_t* crs, const uint32_t* skNinv_eval,
                       const uint32_t* lwe_sk, uint32_t* evk, uint32_t rdefect_policy, uint64_t* defective) try {
    UNPACK(pp, p);
    if (!crs || !skNinv_eval || !lwe_sk || !evk) return fail(MKACC_E_ARG, "null argument");
    if (rdefect_policy > MKKG_RDEFECT_RESAMPLE) return fail(MKACC_E_ARG, "unknown r-defect policy");
    std::atomic<uint64_t> ndef{0};
    const Seed sd = resolve_seed(seed);
    const Ring R(p.N, p.Q, p.root);
    const Dgg dgg(pp->sigma_unienc), dggR(pp->sigma_r);
    const size_t key_words = (size_t)p.dg * 2 * p.N;
    const uint32_t n1 = p.n + 1;
    // the secret's modulus: MNTRU keys are mod qKS, MKLWE binary
    const uint64_t neg = (p.method == MKACC_METHOD_MKNTRU_LWE ? p.q : p.qKS) - 1;
    const size_t slots = (size_t)p.k * p.nk * n1;
    parallel_for(slots, [&](size_t idx) {
        const uint32_t i = (uint32_t)(idx % n1);
        const uint32_t s_ = (uint32_t)((idx / n1) % p.nk);
        const uint32_t u = (uint32_t)(idx / n1 / p.nk);
        uint32_t* out = evk + idx * key_words;
        const uint32_t* sinv = skNinv_eval + (size_t)u * p.N;
        bool kdm = false, m = false, set = true;
        if (i == p.n) {
            set = (u == 0 && s_ == 0);  // ek00[n] of party 0 only
            kdm = m = true;
        } else {
            const uint32_t sv = lwe_sk[(size_t)u * p.n + i];
            kdm = (u == 0 && i == 0);
            m = s_ == 0 ? sv == 1 : sv == neg;
        }
        if (!set) {
            std::memset(out, 0, key_words * 4);
            return;
        }
        Rng r(sd, 6, idx);
        if (unienc_key(p, R, dgg, dggR, r, crs, sinv, m, kdm, out, rdefect_policy)) ndef.fetch_add(1);
    });
    if (defective) *defective = ndef.load();
    if (ndef.load() && rdefect_policy == MKKG_RDEFECT_REJECT)
        return fail(MKKG_E_RDEFECT, std::to_string(ndef.load()) +
                                        " bootstrapping key(s) drew a nonzero DggR sample r (the reference's "
                                        "KeyGenXZW defect, mk-acc-xzw.cpp:160-167): gates using them may decrypt wrong");
    return MKACC_OK;
} catch (const std::exception& e) {
    return fail(MKACC_E_ARG, std::string("mkkg_acc_keygen: ") + e.what());
}

// KeySwitchGen2 (mntru-pke.cpp:624-760), the j = 1 table KSK2[u][1] = KSK[u]:
//   E [N*dks][n] <- dggKS;  E[i*dks + t][0] += s_u[i] * baseKS^t  (mod qKS)
//   KSK[u] = centred(E) * centred(F_u^-1)  mod qKS
// Deviation: the reference fills all N*dks rows of E with copies of ONE
// sampled vector (`std::vector<NativeVector> E(N * digitCount,
// GenerateVector(n, qKS))`, mntru-pke.cpp:653), so the key-switching noise is
// e[0] * (sum of all digits) -- about 1.3e5 >> q/8 whenever that one e[0] is
// nonzero (21-45% of key sets at sigma 0.5-0.75), and every gate of such a key
// set decrypts at random.  Each row gets its own noise vector here.  The key's
// shape, its decryption relation and the KeySwitch2 that consumes it are the
// reference's.
int mkkg_ksk_mntru(const mkkg_params* pp, uint64_t seed, const uint32_t* skN, const uint32_t* Finv, uint32_t* ksk) try {
    UNPACK(pp, p);
    if (!skN || !Finv || !ksk) return fail(MKACC_E_ARG, "null argument");
    const Seed sd = resolve_seed(seed);
    const uint32_t n = p.n, rows = p.N * p.dks;
    const uint64_t qKS = p.qKS;
    const Dgg dgg(pp->sigma);
    for (uint32_t u = 0; u < p.k; ++u) {
        std::vector<int32_t> fc((size_t)n * n);
        for (size_t t = 0; t < fc.size(); ++t) fc[t] = (int32_t)centered(Finv[(size_t)u * n * n + t], qKS);
        const uint32_t* su = skN + (size_t)u * p.N;
        parallel_for((rows + 63) / 64, [&](size_t blk) {
            std::vector<int32_t> e(n);
            std::vector<int32_t> acc(n);
            for (uint32_t row = (uint32_t)blk * 64; row < std::min<uint32_t>(rows, (uint32_t)blk * 64 + 64); ++row) {
                Rng r(sd, 7, u, row);
                for (uint32_t l = 0; l < n; ++l) e[l] = dgg.sample(r);
                const uint32_t i = row / p.dks, t = row % p.dks;
                uint64_t pw = 1;
                for (uint32_t x = 0; x < t; ++x) pw *= p.baseKS;  // coef_w_pwr *= baseKS (no reduction, < 2^40)
                const uint64_t s_q = switch_mod((uint32_t)(su[i] % p.Q), p.Q, qKS);  // s[u].SwitchModulus(qKS)
                const uint32_t e0 = to_mod((int64_t)e[0] + (int64_t)(s_q * pw % qKS), qKS);
                const int64_t c0 = centered(e0, qKS);
                // rows l >= 1: |e| <= ceil(11.9 sigma) and |F^-1| < 2^15 -> int32 sums are exact
                std::fill(acc.begin(), acc.end(), 0);
                for (uint32_t l = 1; l < n; ++l) {
                    const int32_t el = e[l];
                    if (!el) continue;
                    const int32_t* fr = &fc[(size_t)l * n];
                    for (uint32_t j = 0; j < n; ++j) acc[j] += el * fr[j];
                }
                uint32_t* out = ksk + ((size_t)u * rows + row) * n;
                for (uint32_t j = 0; j < n; ++j) out[j] = to_mod((int64_t)acc[j] + c0 * fc[j], qKS);
            }
        });
    }
    return MKACC_OK;
} catch (const std::exception& e) {
    return fail(MKACC_E_ARG, std::string("mkkg_ksk_mntru: ") + e.what());
}

// MKLWEEncryptionScheme::KeySwitchGen (mklwe-pke.cpp:176-258):
//   A[u][i][j][t] <- dgg(sigma)^n,  B = dggKS + svN[i] * j * baseKS^t + <A, s_u>  (mod qKS)
int mkkg_ksk_mklwe(const mkkg_params* pp, uint64_t seed, const uint32_t* skN, const uint32_t* s, uint32_t* A,
                   uint32_t* B) try {
    UNPACK(pp, p);
    if (!skN || !s || !A || !B) return fail(MKACC_E_ARG, "null argument");
    const Seed sd = resolve_seed(seed);
    const uint32_t n = p.n;
    const uint64_t qKS = p.qKS;
    const Dgg dgg(pp->sigma);
    parallel_for((size_t)p.k * p.N, [&](size_t ui) {
        const uint32_t u = (uint32_t)(ui / p.N), i = (uint32_t)(ui % p.N);
        const uint32_t svN = switch_mod(skN[(size_t)u * p.N + i], p.Q, qKS);
        const uint32_t* sv = s + (size_t)u * n;
        Rng r(sd, 8, ui);
        for (uint32_t j = 0; j < p.baseKS; ++j) {
            uint64_t dig = 1;
            for (uint32_t t = 0; t < p.dks; ++t, dig *= p.baseKS) {
                const size_t row = ((ui * p.baseKS + j) * p.dks + t);
                uint32_t* a = A + row * n;
                int64_t acc = 0;
                for (uint32_t l = 0; l < n; ++l) {
                    const int32_t x = dgg.sample(r);
                    a[l] = to_mod(x, qKS);
                    acc += (int64_t)a[l] * (int64_t)switch_mod(sv[l] % qKS, p.q, qKS);
                }
                const uint64_t m = (uint64_t)svN * ((j * dig) % qKS) % qKS;
                B[row] = to_mod((int64_t)dgg.sample(r) + (int64_t)m + acc % (int64_t)qKS, qKS);
            }
        }
    });
    return MKACC_OK;
} catch (const std::exception& e) {
    return fail(MKACC_E_ARG, std::string("mkkg_ksk_mklwe: ") + e.what());
}

namespace {
// c_i = (e + [i == 0] delta) * F_i^-1 (mod q): Encrypt / ctGateGen
void mntru_encrypt_one(const P& p, const Dgg& dgg, Rng& r, const uint32_t* Finv, uint32_t delta, uint32_t* ct) {
    const uint32_t n = p.n;
    const uint64_t q = p.q;
    std::vector<int64_t> acc(n);
    std::vector<int32_t> e(n);
    for (uint32_t u = 0; u < p.k; ++u) {
        for (uint32_t l = 0; l < n; ++l) e[l] = dgg.sample(r);  // GetDgg().GenerateVector(n, mod)
        std::fill(acc.begin(), acc.end(), 0);
        const uint32_t* fi = Finv + (size_t)u * n * n;
        for (uint32_t l = 0; l < n; ++l) {
            int64_t el = e[l];
            if (u == 0 && l == 0) el = (int64_t)to_mod(el, q) + delta;  // e[0].ModAddFastEq(delta)
            if (!el) continue;
            const uint32_t* fr = fi + (size_t)l * n;
            for (uint32_t j = 0; j < n; ++j) acc[j] += el * (int64_t)switch_mod(fr[j], p.qKS, q);
        }
        for (uint32_t j = 0; j < n; ++j) ct[(size_t)u * n + j] = to_mod(acc[j], q);
    }
}
}  // namespace

// MNTRUEncryptionScheme::Encrypt (mntru-pke.cpp:158-206): e[0] += (m % p) * (q / p)
int mkkg_mntru_encrypt(const mkkg_params* pp, uint64_t seed, const uint32_t* Finv, const uint32_t* m, uint32_t pt,
                       size_t count, uint32_t* ct) try {
    UNPACK(pp, p);
    if (!Finv || !m || !ct) return fail(MKACC_E_ARG, "null argument");
    if (pt < 2) return fail(MKACC_E_ARG, "plaintext modulus must be >= 2");
    if (count >= kMaxPerCall) return fail(MKACC_E_ARG, "at most 2^24 - 1 encryptions per call");
    const Seed sd = resolve_seed(seed);
    const Dgg dgg(pp->sigma);
    parallel_for(count, [&](size_t c) {
        Rng r(sd, 9, c);
        const uint32_t delta = (uint32_t)((m[c] % pt) * (p.q / pt));
        mntru_encrypt_one(p, dgg, r, Finv, delta, ct + c * p.k * p.n);
    });
    return MKACC_OK;
} catch (const std::exception& e) {
    return fail(MKACC_E_ARG, std::string("mkkg_mntru_encrypt: ") + e.what());
}

// ctGateGen(sk, NAND) (binfhe-base-scheme.cpp:340-376): e[0] += 5q/8
int mkkg_mntru_ctgate(const mkkg_params* pp, uint64_t seed, const uint32_t* Finv, uint32_t* ct_nand) try {
    UNPACK(pp, p);
    if (!Finv || !ct_nand) return fail(MKACC_E_ARG, "null argument");
    const Seed sd = resolve_seed(seed);
    const Dgg dgg(pp->sigma);
    Rng r(sd, 10);
    mntru_encrypt_one(p, dgg, r, Finv, (uint32_t)(5 * p.q / 8), ct_nand);
    return MKACC_OK;
} catch (const std::exception& e) {
    return fail(MKACC_E_ARG, std::string("mkkg_mntru_ctgate: ") + e.what());
}

// Decrypt / Decrypt2 / DecryptNAND (mntru-pke.cpp:208-357):
//   inner = sum_u <c_u, F_u[:,0]> mod q, then the variant's offset and scale.
int mkkg_mntru_decrypt(const mkkg_params* pp, const uint32_t* F, const uint32_t* ct, uint64_t mod, uint32_t pt,
                       uint32_t variant, size_t count, uint32_t* m) try {
    UNPACK(pp, p);
    if (!F || !ct || !m) return fail(MKACC_E_ARG, "null argument");
    if (pt < 2 || variant > MKKG_DECRYPT_NAND) return fail(MKACC_E_ARG, "bad plaintext modulus or variant");
    if (!mod) mod = p.q;
    const uint32_t n = p.n;
    std::vector<uint32_t> col((size_t)p.k * n);
    for (uint32_t u = 0; u < p.k; ++u)
        for (uint32_t l = 0; l < n; ++l)
            col[(size_t)u * n + l] = switch_mod(F[((size_t)u * n + l) * n], p.qKS, mod);  // F_col0.SwitchModulus(mod)
    for (size_t c = 0; c < count; ++c) {
        uint64_t inner = 0;
        for (uint32_t u = 0; u < p.k; ++u) {
            uint64_t sum = 0;
            for (uint32_t l = 0; l < n; ++l) sum += (uint64_t)ct[(c * p.k + u) * n + l] * col[(size_t)u * n + l];
            inner = (inner + sum % mod) % mod;
        }
        uint64_t scale = pt, off = mod / pt;
        if (variant == MKKG_DECRYPT2) off = mod / (2 * pt);
        if (variant == MKKG_DECRYPT_NAND) { scale = pt / 2; off = mod / (pt / 2 * 2); }
        inner = (inner + off) % mod;
        m[c] = (uint32_t)(scale * inner / mod);
    }
    return MKACC_OK;
} catch (const std::exception& e) {
    return fail(MKACC_E_ARG, std::string("mkkg_mntru_decrypt: ") + e.what());
}

// MKLWEEncryptionScheme::Encrypt (mklwe-pke.cpp:36-64): a_u <- DGG(sigma = 1)
// (a default-constructed generator), b = (m % p)(q/p) + dgg(sigma) + sum <a_u, s_u>
int mkkg_mklwe_encrypt(const mkkg_params* pp, uint64_t seed, const uint32_t* s, const uint32_t* m, uint32_t pt,
                       size_t count, uint32_t* a, uint32_t* b) try {
    UNPACK(pp, p);
    if (!s || !m || !a || !b) return fail(MKACC_E_ARG, "null argument");
    if (pt < 2) return fail(MKACC_E_ARG, "plaintext modulus must be >= 2");
    if (count >= kMaxPerCall) return fail(MKACC_E_ARG, "at most 2^24 - 1 encryptions per call");
    const Seed sd = resolve_seed(seed);
    const Dgg err(pp->sigma), dga(1.0);
    const uint64_t q = p.q;
    parallel_for(count, [&](size_t c) {
        Rng r(sd, 11, c);
        int64_t bb = (int64_t)((m[c] % pt) * (q / pt)) + err.sample(r);
        for (uint32_t u = 0; u < p.k; ++u)
            for (uint32_t i = 0; i < p.n; ++i) {
                const uint32_t av = to_mod(dga.sample(r), q);
                a[(c * p.k + u) * p.n + i] = av;
                bb += (int64_t)av * switch_mod(s[(size_t)u * p.n + i] % p.qKS, p.qKS, q);
            }
        b[c] = to_mod(bb, q);
    });
    return MKACC_OK;
} catch (const std::exception& e) {
    return fail(MKACC_E_ARG, std::string("mkkg_mklwe_encrypt: ") + e.what());
}

// Decrypt (mklwe-pke.cpp:66-113): r = b - sum <a_u, s_u> + q/(2p); floor(p r / q)
// DecryptNAND (:115-158):          r = b - sum <a_u, s_u> + q/p;     floor(p/2 r / q)
int mkkg_mklwe_decrypt(const mkkg_params* pp, const uint32_t* s, const uint32_t* a, const uint32_t* b, uint64_t mod,
                       uint32_t pt, uint32_t variant, size_t count, uint32_t* m) try {
    UNPACK(pp, p);
    if (!s || !a || !b || !m) return fail(MKACC_E_ARG, "null argument");
    if (pt < 2 || (variant != MKKG_DECRYPT && variant != MKKG_DECRYPT_NAND))
        return fail(MKACC_E_ARG, "bad plaintext modulus or variant");
    if (!mod) mod = p.q;
    for (size_t c = 0; c < count; ++c) {
        uint64_t inner = 0;
        for (uint32_t u = 0; u < p.k; ++u) {
            for (uint32_t i = 0; i < p.n; ++i)
                inner += (uint64_t)a[(c * p.k + u) * p.n + i] * switch_mod(s[(size_t)u * p.n + i] % p.qKS, p.qKS, mod);
            inner %= mod;
        }
        uint64_t r = (b[c] % mod + mod - inner) % mod;
        if (variant == MKKG_DECRYPT) {
            r = (r + mod / (2 * pt)) % mod;
            m[c] = (uint32_t)(pt * r / mod);
        } else {
            r = (r + mod / pt) % mod;
            m[c] = (uint32_t)((pt / 2) * r / mod);
        }
    }
    return MKACC_OK;
} catch (const std::exception& e) {
    return fail(MKACC_E_ARG, std::string("mkkg_mklwe_decrypt: ") + e.what());
}

}  // extern "C"

// ---------------------------------------------------------------------------
// key wire format (include/mkfhe_keys.h)
// ---------------------------------------------------------------------------
namespace {

constexpr char kMagic[8] = {'M', 'K', 'F', 'H', 'E', 'K', 'E', 'Y'};
constexpr uint32_t kFileVersion = 1;
constexpr int kParamWords = 18;

uint64_t fnv1a(const void* p, size_t n, uint64_t h = 0xCBF29CE484222325ull) {
    const unsigned char* b = static_cast<const unsigned char*>(p);
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 0x100000001B3ull;
    return h;
}
uint64_t dbits(double d) {
    uint64_t u;
    std::memcpy(&u, &d, 8);
    return u;
}
double bitsd(uint64_t u) {
    double d;
    std::memcpy(&d, &u, 8);
    return d;
}
void pack_params(const mkkg_params& p, uint64_t (&w)[kParamWords]) {
    const uint64_t v[kParamWords] = {p.acc.method, p.acc.k, p.acc.n, p.acc.N, p.acc.Q, p.acc.q, p.acc.baseG,
                                     p.acc.digitsG, p.acc.root, p.ks.qKS, p.ks.baseKS, p.ks.n_out,
                                     dbits(p.sigma), dbits(p.sigma_unienc), dbits(p.sigma_r), p.lwe_keydist,
                                     p.ring_keydist, 0};
    for (int i = 0; i < kParamWords; ++i) w[i] = v[i];
}
void unpack_params(const uint64_t (&w)[kParamWords], mkkg_params& p) {
    p = mkkg_params{};
    p.acc.method = (uint32_t)w[0]; p.acc.k = (uint32_t)w[1]; p.acc.n = (uint32_t)w[2]; p.acc.N = (uint32_t)w[3];
    p.acc.Q = w[4]; p.acc.q = w[5]; p.acc.baseG = (uint32_t)w[6]; p.acc.digitsG = (uint32_t)w[7]; p.acc.root = w[8];
    p.ks.qKS = w[9]; p.ks.baseKS = (uint32_t)w[10]; p.ks.n_out = (uint32_t)w[11];
    p.sigma = bitsd(w[12]); p.sigma_unienc = bitsd(w[13]); p.sigma_r = bitsd(w[14]);
    p.lwe_keydist = (uint32_t)w[15]; p.ring_keydist = (uint32_t)w[16];
}

struct File {
    FILE* f = nullptr;
    uint64_t size = 0;   // bytes, for reads: every size a file supplies is checked against it
    explicit File(const char* path, const char* mode) : f(path ? std::fopen(path, mode) : nullptr) {
        if (f && mode[0] == 'r') {
            if (fseeko(f, 0, SEEK_END) == 0) {
                const off_t e = ftello(f);
                size = e > 0 ? (uint64_t)e : 0;
            }
            if (fseeko(f, 0, SEEK_SET) != 0) {
                std::fclose(f);
                f = nullptr;
            }
        }
    }
    ~File() {
        if (f) std::fclose(f);
    }
    File(const File&) = delete;
    File& operator=(const File&) = delete;
    bool get(void* p, size_t n) { return std::fread(p, 1, n, f) == n; }
    bool put(const void* p, size_t n) { return std::fwrite(p, 1, n, f) == n; }
    // bytes left after the current position
    uint64_t left() const {
        const off_t at = ftello(f);
        return at < 0 || (uint64_t)at > size ? 0 : size - (uint64_t)at;
    }
};

constexpr uint64_t kSectionHead = 16 + 8;   // name, words
constexpr uint64_t kSectionTail = 8;        // checksum

// A parameter block must describe a context this library can serve (the checks
// of every key routine, unpack) before any reader sizes a buffer from it.
int check_file_params(const mkkg_params& p, uint32_t kind) {
    if (kind < MKKG_FILE_MNTRU_SK || kind > MKKG_FILE_CIPHERTEXT) return fail(MKACC_E_ARG, "unknown key file kind");
    if (p.acc.k > 1024 || p.acc.n > (1u << 16) || p.acc.N > (1u << 16))
        return fail(MKACC_E_ARG, "key file parameter block out of range");
    for (double d : {p.sigma, p.sigma_unienc, p.sigma_r})
        if (!std::isfinite(d) || d < 0 || d > 1e9) return fail(MKACC_E_ARG, "key file parameter block: bad sigma");
    P chk;
    if (unpack(&p, chk)) return fail(MKACC_E_ARG, "key file parameter block is not a valid MK parameter set");
    return MKACC_OK;
}

// header; leaves the file positioned at the first section
int read_header(File& fl, uint32_t* kind, mkkg_params* p, uint32_t* count) {
    if (!fl.f) return fail(MKACC_E_ARG, "cannot open key file");
    char magic[8];
    uint32_t ver = 0, knd = 0, cnt = 0;
    uint64_t w[kParamWords];
    if (!fl.get(magic, 8) || std::memcmp(magic, kMagic, 8)) return fail(MKACC_E_ARG, "not an MKFHEKEY file");
    if (!fl.get(&ver, 4) || ver != kFileVersion) return fail(MKACC_E_ARG, "unsupported key file version");
    if (!fl.get(&knd, 4) || !fl.get(w, sizeof(w)) || !fl.get(&cnt, 4)) return fail(MKACC_E_ARG, "truncated key file");
    mkkg_params prm;
    unpack_params(w, prm);
    if (int rc = check_file_params(prm, knd)) return rc;
    if (cnt > fl.left() / (kSectionHead + kSectionTail)) return fail(MKACC_E_ARG, "truncated key file (section count)");
    if (kind) *kind = knd;
    if (p) *p = prm;
    if (count) *count = cnt;
    return MKACC_OK;
}

// find section `name`; on success the file is positioned at its data and *words is
// set, bounded by the bytes the file still holds (data + checksum)
int seek_section(File& fl, const char* name, uint64_t* words) {
    uint32_t count = 0;
    int rc = read_header(fl, nullptr, nullptr, &count);
    if (rc) return rc;
    for (uint32_t s = 0; s < count; ++s) {
        char nm[16];
        uint64_t w = 0;
        if (!fl.get(nm, 16) || !fl.get(&w, 8)) return fail(MKACC_E_ARG, "truncated key file");
        const uint64_t left = fl.left();
        if (left < kSectionTail || w > (left - kSectionTail) / 4)
            return fail(MKACC_E_ARG, "truncated key file (section larger than the file)");
        if (!std::strncmp(nm, name, 16)) {
            *words = w;
            return MKACC_OK;
        }
        if (fseeko(fl.f, (off_t)(w * 4 + kSectionTail), SEEK_CUR)) return fail(MKACC_E_ARG, "truncated key file");
    }
    return fail(MKACC_E_ARG, std::string("key file has no section ") + name);
}

}  // namespace

extern "C" {

int mkkg_file_write(const char* path, uint32_t kind, const mkkg_params* p, const mkkg_section* sections,
                    uint32_t count) try {
    if (!path || !p || (count && !sections)) return fail(MKACC_E_ARG, "null argument");
    File fl(path, "wb");
    if (!fl.f) return fail(MKACC_E_ARG, std::string("cannot create ") + path);
    uint64_t w[kParamWords];
    pack_params(*p, w);
    bool ok = fl.put(kMagic, 8) && fl.put(&kFileVersion, 4) && fl.put(&kind, 4) && fl.put(w, sizeof(w)) &&
              fl.put(&count, 4);
    for (uint32_t s = 0; ok && s < count; ++s) {
        const mkkg_section& sec = sections[s];
        if (sec.words && !sec.data) return fail(MKACC_E_ARG, "section without data");
        char nm[16] = {0};
        std::strncpy(nm, sec.name, 15);
        const uint64_t h = fnv1a(sec.data, sec.words * 4);
        ok = fl.put(nm, 16) && fl.put(&sec.words, 8) && fl.put(sec.data, sec.words * 4) && fl.put(&h, 8);
    }
    if (!ok) return fail(MKACC_E_ARG, std::string("write failed: ") + path);
    return MKACC_OK;
} catch (const std::exception& e) {
    return fail(MKACC_E_ARG, std::string("mkkg_file_write: ") + e.what());
}

int mkkg_file_info(const char* path, uint32_t* kind, mkkg_params* p, uint32_t* count) try {
    File fl(path, "rb");
    return read_header(fl, kind, p, count);
} catch (const std::exception& e) {
    return fail(MKACC_E_ARG, std::string("mkkg_file_info: ") + e.what());
}

uint64_t mkkg_file_section_words(const char* path, const char* name) {
    if (!name) return 0;
    File fl(path, "rb");
    uint64_t w = 0;
    return seek_section(fl, name, &w) ? 0 : w;
}

int mkkg_file_read_section(const char* path, const char* name, uint32_t* out, uint64_t words) try {
    if (!name || (words && !out)) return fail(MKACC_E_ARG, "null argument");
    File fl(path, "rb");
    uint64_t w = 0;
    int rc = seek_section(fl, name, &w);
    if (rc) return rc;
    if (w != words) return fail(MKACC_E_ARG, std::string("section ") + name + " has a different size");
    uint64_t h = 0;
    if (!fl.get(out, words * 4) || !fl.get(&h, 8)) return fail(MKACC_E_ARG, "truncated key file");
    if (h != fnv1a(out, words * 4)) return fail(MKACC_E_ARG, std::string("checksum mismatch in section ") + name);
    return MKACC_OK;
} catch (const std::exception& e) {
    return fail(MKACC_E_ARG, std::string("mkkg_file_read_section: ") + e.what());
}

int mkkg_ntt_forward(const mkkg_params* pp, const uint32_t* in, uint32_t* out, size_t count) try {
    UNPACK(pp, p);
    if (!in || !out) return fail(MKACC_E_ARG, "null argument");
    const Ring R(p.N, p.Q, p.root);
    for (size_t c = 0; c < count; ++c) {
        uint32_t* o = out + c * p.N;
        for (uint32_t j = 0; j < p.N; ++j) {
            if (in[c * p.N + j] >= p.Q) return fail(MKACC_E_RANGE, "input word >= Q");
            o[j] = in[c * p.N + j];
        }
        R.fwd(o);
    }
    return MKACC_OK;
} catch (const std::exception& e) {
    return fail(MKACC_E_ARG, std::string("mkkg_ntt_forward: ") + e.what());
}

int mkkg_ntt_inverse(const mkkg_params* pp, const uint32_t* in, uint32_t* out, size_t count) try {
    UNPACK(pp, p);
    if (!in || !out) return fail(MKACC_E_ARG, "null argument");
    const Ring R(p.N, p.Q, p.root);
    for (size_t c = 0; c < count; ++c) {
        uint32_t* o = out + c * p.N;
        for (uint32_t j = 0; j < p.N; ++j) {
            if (in[c * p.N + j] >= p.Q) return fail(MKACC_E_RANGE, "input word >= Q");
            o[j] = in[c * p.N + j];
        }
        R.inv(o);
    }
    return MKACC_OK;
} catch (const std::exception& e) {
    return fail(MKACC_E_ARG, std::string("mkkg_ntt_inverse: ") + e.what());
}

}  // extern "C"
