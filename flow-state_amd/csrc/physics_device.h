// Device helpers shared by the physics kernels (energy, local moves, MH accept):
// numpy-order minimum-image distances, the shifted LJ pair term and the numpy
// PCG64 stream.  Evaluation order follows the reference line by line (cited per
// helper) so that results track numpy to the ulp.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <string.h>

#include "../../include/flowstate.h"

#pragma clang fp contract(off)

namespace fs {

// np.round(d / L) (round half to even) without the division: q = d * (1/L) is within
// a few ulps of the correctly rounded quotient, so rint(q) can only differ when q is
// within that distance of a half-integer; those (rare) lanes take the exact division.
// |d| <= 2L on every call site, so 1e-12 is many ulps of q.
__device__ __forceinline__ double rint_div(double d, double L, double invL) {
    const double q = d * invL;
    const double k = rint(q);
    if (__builtin_expect(fabs(fabs(q - k) - 0.5) < 1e-12, 0)) return rint(d / L);
    return k;
}

// ---------------------------------------------------------------------------
// Squared-distance thresholds.  The reference compares r = sqrt(s) (float32: the
// correctly rounded float sqrt of the float32 sdot; float64: sqrt of the ddot) with
// r_cut (inclusive) and r_core; correctly rounded sqrt is monotone, so each comparison
// is exactly one comparison of s with a host-computed threshold, and the sqrt is only
// taken for pairs inside the cutoff (about 1 % of pairs at rho = 0.03).  Likewise the
// minimum-image round: for |d| <= L, rint(d / L) is sign(d) if fl(|d| / L) > 0.5
// (round-half-even keeps 0.5 at 0), else 0, i.e. one comparison with h = the largest
// double with fl(h / L) <= 0.5.
struct PairThresh {
    double cut64, core64;  // s <= cut64 <=> sqrt(s) <= r_cut; s <= core64 <=> sqrt(s) < r_core
    double hx, hy;         // min-image half-box thresholds
    float cut32, core32;   // the same for the float32 path
    // float32 path: for a float d, (double)|d| > hx <=> |d| > hx32 and (double)|d| <= Lx <=>
    // |d| <= Lx32 (each the largest float not above the double), so the common minimum-image
    // case needs no float64 compare
    float hx32, hy32, Lx32, Ly32;
};

template <class P>
static inline uint64_t fs_bisect_u64(P pred, uint64_t lo, uint64_t hi) {  // pred(lo), !pred(hi)
    while (hi - lo > 1) {
        const uint64_t m = lo + (hi - lo) / 2;
        if (pred(m)) lo = m; else hi = m;
    }
    return lo;
}

static inline double fs_u2d(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
static inline float fs_u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

// largest non-negative double / float x with pred(x); -1 if pred(0) is false
template <class P>
static inline double fs_max_true_f64(P pred) {
    if (!pred(0.0)) return -1.0;
    return fs_u2d(fs_bisect_u64([&](uint64_t u) { return pred(fs_u2d(u)); }, 0, 0x7ff0000000000000ull));
}
template <class P>
static inline float fs_max_true_f32(P pred) {
    if (!pred(0.0f)) return -1.0f;
    return fs_u2f((uint32_t)fs_bisect_u64([&](uint64_t u) { return pred(fs_u2f((uint32_t)u)); }, 0, 0x7f800000ull));
}

static inline PairThresh fs_pair_thresh(const fs_phys &p) {
    PairThresh t;
    t.cut64 = fs_max_true_f64([&](double s) { return sqrt(s) <= p.r_cut; });
    t.core64 = fs_max_true_f64([&](double s) { return sqrt(s) < p.r_core; });
    t.cut32 = fs_max_true_f32([&](float s) { return (double)(float)sqrt((double)s) <= p.r_cut; });
    t.core32 = fs_max_true_f32([&](float s) { return (double)(float)sqrt((double)s) < p.r_core; });
    t.hx = fs_max_true_f64([&](double a) { return a / p.Lx <= 0.5; });
    t.hy = fs_max_true_f64([&](double a) { return a / p.Ly <= 0.5; });
    t.hx32 = fs_max_true_f32([&](float a) { return (double)a <= t.hx; });
    t.hy32 = fs_max_true_f32([&](float a) { return (double)a <= t.hy; });
    t.Lx32 = fs_max_true_f32([&](float a) { return (double)a <= p.Lx; });
    t.Ly32 = fs_max_true_f32([&](float a) { return (double)a <= p.Ly; });
    return t;
}

// d - L * rint(d / L) as simulation_box.py:35-39 computes it
__device__ __forceinline__ double wrap_min_image(double d, double L, double h, double invL) {
    const double a = fabs(d);
    if (a <= L) return a > h ? d - copysign(L, d) : d;
    return d - L * rint_div(d, L, invL);
}

// squared minimum-image distances (simulation_box.py:31-56) with numpy's promotion rules.
// float32 state: float32 delta, wrapped in float64 (box lengths are np.float64), back to
// float32, then the float32 sdot t0*t0 + t1*t1 as OpenBLAS computes it -- plain operators
// under fp contract(off): HIP's __f*_rn helpers carry the `contract` flag, which would let
// the backend fuse the sdot into an FMA.  float64 state: the ddot with its FMA.
// The distance itself is the correctly rounded sqrt of s (r_of_sq): for float32 the double
// sqrt rounded once more to float is exact-rounded (53 >= 2*24+2 bits), whereas the
// device f32 sqrt instruction is only faithful.
__device__ __forceinline__ float sqdist_f32(float ax, float ay, float bx, float by, double Lx, double Ly,
                                            const PairThresh &T, double iLx, double iLy) {
    const float d0 = ax - bx, d1 = ay - by;
    const float t0 = (float)wrap_min_image((double)d0, Lx, T.hx, iLx);
    const float t1 = (float)wrap_min_image((double)d1, Ly, T.hy, iLy);
    const float s0 = t0 * t0, s1 = t1 * t1;
    return s0 + s1;
}
// the same for float32 coordinates without a float64 compare or branch in the common case
// (|d| <= L): the wrap subtraction stays in float64 (exact there, rounded once), and the
// rare |d| > L takes wrap_min_image's general path
__device__ __forceinline__ float wrap32(float d, double L, float h32, float L32, double h, double invL) {
    const float a = fabsf(d);
    float t = a > h32 ? (float)((double)d - copysign(L, (double)d)) : d;
    if (__builtin_expect(a > L32, 0)) t = (float)wrap_min_image((double)d, L, h, invL);
    return t;
}
__device__ __forceinline__ float sqdist32(float ax, float ay, float bx, float by, double Lx, double Ly,
                                         const PairThresh &T, double iLx, double iLy) {
    const float t0 = wrap32(ax - bx, Lx, T.hx32, T.Lx32, T.hx, iLx);
    const float t1 = wrap32(ay - by, Ly, T.hy32, T.Ly32, T.hy, iLy);
    const float s0 = t0 * t0, s1 = t1 * t1;
    return s0 + s1;
}
__device__ __forceinline__ double sqdist_f64(double ax, double ay, double bx, double by, double Lx, double Ly,
                                             const PairThresh &T, double iLx, double iLy) {
    const double t0 = wrap_min_image(ax - bx, Lx, T.hx, iLx);
    const double t1 = wrap_min_image(ay - by, Ly, T.hy, iLy);
    const double s0 = t0 * t0;
    return fma(t1, t1, s0);
}
__device__ __forceinline__ double r_of_sq(float s) { return (double)(float)__dsqrt_rn((double)s); }
__device__ __forceinline__ double r_of_sq(double s) { return __dsqrt_rn(s); }

// x^6 rounded once from a double-double product (tracks the correctly rounded pow)
__device__ __forceinline__ double pow6(double x) {
    const double x2 = x * x, x2e = fma(x, x, -x2);
    const double x3 = x2 * x, x3e = fma(x2, x, -x3) + x2e * x;
    const double x6 = x3 * x3, x6e = fma(x3, x3, -x6) + 2.0 * x3 * x3e;
    return x6 + x6e;
}

__device__ __forceinline__ void lj_pair(double r, double r_cut, double e_cut, double &e, double &w) {
    if (r <= r_cut) {  // potential.py:11 inclusive
        const double sr6 = pow6(1.0 / r);
        const double sr12 = sr6 * sr6;
        e = 4.0 * (sr12 - sr6) - e_cut;
        w = 48.0 * (sr12 - 0.5 * sr6);
    } else {
        e = 0.0;
        w = 0.0;
    }
}

// ---------------------------------------------------------------- PCG64
struct u128 {
    uint64_t hi, lo;
};

__device__ __forceinline__ u128 mul_add(u128 a, u128 m, u128 inc) {
    u128 r;
    r.lo = a.lo * m.lo;
    r.hi = __umul64hi(a.lo, m.lo) + a.lo * m.hi + a.hi * m.lo;
    const uint64_t lo = r.lo + inc.lo;
    r.hi += inc.hi + (lo < r.lo ? 1 : 0);
    r.lo = lo;
    return r;
}

__device__ __forceinline__ double pcg64_next_double(uint64_t *s) {
    const u128 M = {0x2360ED051FC65DA4ull, 0x4385DF649FCCF645ull};
    u128 st = {s[0], s[1]}, inc = {s[2], s[3]};
    st = mul_add(st, M, inc);
    s[0] = st.hi;
    s[1] = st.lo;
    const uint64_t x = st.hi ^ st.lo;
    const unsigned rot = (unsigned)(st.hi >> 58);
    const uint64_t out = (x >> rot) | (x << ((64 - rot) & 63));
    return (double)(out >> 11) * (1.0 / 9007199254740992.0);
}

// numpy PCG64 with the 32-bit half buffer (numpy/random/src/pcg64/pcg64.h
// pcg64_next32: has_uint32 / uinteger), as Generator.integers consumes it
struct Pcg64 {
    uint64_t s[4];
    uint32_t has, buf;
};

__device__ __forceinline__ uint64_t pcg64_next64(uint64_t *s) {
    const u128 M = {0x2360ED051FC65DA4ull, 0x4385DF649FCCF645ull};
    u128 st = {s[0], s[1]}, inc = {s[2], s[3]};
    st = mul_add(st, M, inc);
    s[0] = st.hi;
    s[1] = st.lo;
    const uint64_t x = st.hi ^ st.lo;
    const unsigned rot = (unsigned)(st.hi >> 58);
    return (x >> rot) | (x << ((64 - rot) & 63));
}

__device__ __forceinline__ double pcg64_double(Pcg64 &g) {
    return (double)(pcg64_next64(g.s) >> 11) * (1.0 / 9007199254740992.0);
}

__device__ __forceinline__ uint32_t pcg64_next32(Pcg64 &g) {
    if (g.has) {
        g.has = 0;
        return g.buf;
    }
    const uint64_t v = pcg64_next64(g.s);
    g.has = 1;
    g.buf = (uint32_t)(v >> 32);
    return (uint32_t)v;
}

// Generator.integers(n), 1 <= n <= 2^32 (random_bounded_uint64_fill ->
// buffered_bounded_lemire_uint32); n == 1 draws nothing
__device__ __forceinline__ uint32_t pcg64_integers(Pcg64 &g, uint32_t n) {
    const uint32_t rng = n - 1u;
    if (rng == 0u) return 0u;
    const uint32_t excl = rng + 1u;
    uint64_t m = (uint64_t)pcg64_next32(g) * excl;
    uint32_t left = (uint32_t)m;
    if (left < excl) {
        const uint32_t thr = (0xFFFFFFFFu - rng) % excl;
        while (left < thr) {
            m = (uint64_t)pcg64_next32(g) * excl;
            left = (uint32_t)m;
        }
    }
    return (uint32_t)(m >> 32);
}

// one well's term V0_i * (1 - transition) of double_well_potential (potential.py:98-112)
__device__ __forceinline__ double dw_term(double x, double y, int well, double Lx, double Ly, double V0, double r0,
                                          double k, double iLx, double iLy) {
    const double cx = (well == 0) ? Lx / 4.0 : 3.0 * Lx / 4.0, cy = Ly / 2.0;
    double dx = x - cx, dy = y - cy;
    dx -= Lx * rint_div(dx, Lx, iLx);
    dy -= Ly * rint_div(dy, Ly, iLy);
    const double r = sqrt(dx * dx + dy * dy);
    const double tr = 0.5 * (1.0 + tanh(k * (r - r0)));
    return V0 * (1.0 - tr);
}

// numpy floor remainder (npy_divmod) for SimulationBox.apply_pbc (simulation_box.py:19-29)
__device__ __forceinline__ double np_remainder(double a, double b) {
    // fast paths (b > 0): fmod is exact, so these equal the general branch bit for bit
    if (a > 0.0 && a < b) return a;
    if (a < 0.0 && a > -b) return a + b;
    if (a >= b && a < 2.0 * b) return a - b;  // Sterbenz: exact
    double mod = fmod(a, b);
    if (mod != 0.0) {
        if ((b < 0) != (mod < 0)) mod += b;
    } else {
        mod = copysign(0.0, b);
    }
    return mod;
}

}  // namespace fs
