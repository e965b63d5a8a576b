// Fused circular rational-quadratic spline with its backward, for the training path
// (Algorithm 2).  One thread per spline element (sample x
// feature); the knots are rebuilt from the unnormalised parameters in registers in
// both passes, so the backward stores nothing but the inputs.
//
// Forward: unconstrained_rational_quadratic_spline, circular-tail branch
// (NF/normflows/utils/splines.py:16-88) + rational_quadratic_spline (:91-222): identity
// and log-det 0 outside [-B, B]; inside: softmax -> min-width affine -> cumsum
// (double accumulation, as torch CPU) -> [-B, B] with pinned ends; derivatives
// 1e-3 + softplus; searchsorted with the eps on the last knot; the rational-quadratic
// map (forward) or its quadratic-root inverse, and the log|det|.
// Backward: reverse-mode by hand.  Forward direction: through theta = (x - cw_b)/w_b.
// Inverse direction: the root theta* solves F(theta) = y, so its adjoint reaches y and
// the knot values through -F_q / F_theta (implicit function theorem).  Knot adjoints go
// back through the pinned cumsum (suffix sums), the min-width affine and softmax;
// derivative adjoints through softplus (threshold 20, as torch).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <stdlib.h>

#include <atomic>

#include "fs_internal.h"

#pragma clang fp contract(off)

namespace fs {

constexpr float kMin = 1e-3f;  // DEFAULT_MIN_BIN_WIDTH / HEIGHT / DERIVATIVE (splines.py:6-8)

template <int K>
struct Knots {
    float c[K + 1];  // cumulative knots, pinned ends
    float p[K];      // softmax probabilities
};

template <int K>
__device__ __forceinline__ void build_knots(const float *u, float B, Knots<K> &kn) {
    float m = u[0];
#pragma unroll
    for (int k = 1; k < K; ++k) m = fmaxf(m, u[k]);
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < K; ++k) {
        kn.p[k] = expf(u[k] - m);
        s += kn.p[k];
    }
#pragma unroll
    for (int k = 0; k < K; ++k) kn.p[k] = kn.p[k] / s;
    const float c1 = 1.f - kMin * (float)K;
    double cs = 0.0;
    kn.c[0] = -B;
#pragma unroll
    for (int k = 0; k < K - 1; ++k) {
        cs += (double)(kMin + c1 * kn.p[k]);
        kn.c[k + 1] = (2.f * B) * (float)cs + (-B);
    }
    kn.c[K] = B;
}

__device__ __forceinline__ float softplus(float v) { return v > 20.f ? v : log1pf(expf(v)); }
__device__ __forceinline__ float softplus_grad(float v) {
    if (v > 20.f) return 1.f;
    const float z = expf(v);
    return z / (z + 1.f);
}

// knots c[b], c[b+1] of bin b by a register scan (a dynamically indexed array would live
// in scratch memory)
template <int K>
__device__ __forceinline__ void pick_bin(const float *c, int b, float &lo, float &hi) {
    lo = c[0];
    hi = c[1];
#pragma unroll
    for (int k = 1; k < K; ++k) {
        if (k == b) {
            lo = c[k];
            hi = c[k + 1];
        }
    }
}

// values of the bin that contains x (searchsorted over `knots`, eps on the last one)
template <int K>
__device__ __forceinline__ int find_bin(float x, const float *knots) {
    int b = -1;
#pragma unroll
    for (int k = 0; k <= K; ++k) {
        const float kv = (k == K) ? knots[K] + 1e-6f : knots[k];
        b += (x >= kv) ? 1 : 0;
    }
    return b < 0 ? 0 : (b > K - 1 ? K - 1 : b);
}

// one element from its built knots (wc: width knots, hc: height knots); x inside [-B, B]
template <int K, bool INV>
__device__ __forceinline__ void rqs_eval_knots(float xv, const float *wc, const float *hc, const float *dd,
                                               float &out, float &lad, int32_t *nan_flag) {
    const int b = find_bin<K>(xv, INV ? hc : wc);
    const float d0 = kMin + softplus(dd[b]), d1 = kMin + softplus(dd[b + 1]);
    float icw, cw1, ich, ch1;
    pick_bin<K>(wc, b, icw, cw1);
    pick_bin<K>(hc, b, ich, ch1);
    const float ibw = cw1 - icw, ih = ch1 - ich;
    const float s = ih / ibw;
    float th;
    if (INV) {
        const float sdd = d0 + d1 - 2.f * s;
        const float a = (xv - ich) * sdd + ih * (s - d0);
        const float bb = ih * d0 - (xv - ich) * sdd;
        const float c = -s * (xv - ich);
        const float disc = fabsf(bb * bb - 4.f * a * c);
        if (disc != disc && nan_flag) atomicOr(nan_flag, 1);
        th = (2.f * c) / (-bb - sqrtf(disc));
    } else {
        th = (xv - icw) / ibw;
    }
    const float t = th * (1.f - th);
    const float den = s + (d0 + d1 - 2.f * s) * t;
    const float A = d1 * th * th + 2.f * s * t + d0 * (1.f - th) * (1.f - th);
    const float l = logf(s * s * A) - 2.f * logf(den);
    if (INV) {
        out = th * ibw + icw;
        lad = -l;
    } else {
        out = ich + ih * (s * th * th + d0 * t) / den;
        lad = l;
    }
}

// one element: x inside [-B, B] (callers route the outside identity themselves)
template <int K, bool INV>
__device__ __forceinline__ void rqs_point(float xv, const float *uw, const float *uh, const float *dd, float B,
                                          float &out, float &lad, int32_t *nan_flag) {
    Knots<K> W, Hh;
    build_knots<K>(uw, B, W);
    build_knots<K>(uh, B, Hh);
    rqs_eval_knots<K, INV>(xv, W.c, Hh.c, dd, out, lad, nan_flag);
}

template <int K, bool INV>
__global__ __launch_bounds__(256) void rqs_forward_kernel(int64_t M, const float *__restrict__ x, const float *__restrict__ uw,
                                   const float *__restrict__ uh, const float *__restrict__ ud, float B,
                                   float *__restrict__ out, float *__restrict__ lad, int32_t *__restrict__ nan_flag) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M) return;
    const float xv = x[i];
    if (!(xv >= -B && xv <= B)) {
        out[i] = xv;
        lad[i] = 0.f;
        return;
    }
    rqs_point<K, INV>(xv, uw + i * K, uh + i * K, ud + i * (K + 1), B, out[i], lad[i], nan_flag);
}

// knot adjoints (g_c over c[0..K]) -> unnormalised-parameter adjoints
template <int K>
__device__ __forceinline__ void knots_backward(const Knots<K> &kn, const float *gc, float B, float *gu) {
    const float c1 = 1.f - kMin * (float)K;
    // c[k] = 2B * C[k] - B (k = 1..K-1), C[k] = sum_{j<k} w_j; c[0], c[K] pinned
    float gw[K];
    float suffix = 0.f;
#pragma unroll
    for (int j = K - 1; j >= 0; --j) {
        gw[j] = suffix;                                  // sum over k = j+1 .. K-1 of g_C[k]
        if (j >= 1) suffix += (2.f * B) * gc[j];         // add k = j for the next (smaller) j
    }
    float dot = 0.f;
#pragma unroll
    for (int j = 0; j < K; ++j) dot += kn.p[j] * (c1 * gw[j]);
#pragma unroll
    for (int j = 0; j < K; ++j) gu[j] = kn.p[j] * (c1 * gw[j] - dot);
}

// the adjoint core of one element inside [-B, B] from its built knots: gx and the
// adjoints of the bin's knots (gcw / gch over c[0..K]) and derivative logits (gud)
template <int K, bool INV>
__device__ __forceinline__ void rqs_bwd_core(float xv, const float *wc, const float *hc, const float *dd, float go,
                                             float gl, float &gx, float *gcw, float *gch, float *gud) {
    const int b = find_bin<K>(xv, INV ? hc : wc);
    const float e0 = dd[b], e1 = dd[b + 1];
    const float d0 = kMin + softplus(e0), d1 = kMin + softplus(e1);
    float icw, cw1, ich, ch1;
    pick_bin<K>(wc, b, icw, cw1);
    pick_bin<K>(hc, b, ich, ch1);
    const float ibw = cw1 - icw, ih = ch1 - ich;
    const float s = ih / ibw;
    float th;
    if (INV) {
        const float sdd = d0 + d1 - 2.f * s;
        const float a = (xv - ich) * sdd + ih * (s - d0);
        const float bb = ih * d0 - (xv - ich) * sdd;
        const float c = -s * (xv - ich);
        const float disc = fabsf(bb * bb - 4.f * a * c);
        th = (2.f * c) / (-bb - sqrtf(disc));
    } else {
        th = (xv - icw) / ibw;
    }
    const float t = th * (1.f - th);
    const float omt = 1.f - th;
    const float Nn = s * th * th + d0 * t;
    const float den = s + (d0 + d1 - 2.f * s) * t;
    const float A = d1 * th * th + 2.f * s * t + d0 * omt * omt;
    const float dnum = s * s * A;
    float g_th = 0.f, g_s = 0.f, g_t = 0.f, g_d0 = 0.f, g_d1 = 0.f;
    float g_icw = 0.f, g_ibw = 0.f, g_ich = 0.f, g_ih = 0.f, g_x = 0.f;
    // log-det part: l = log(dnum) - 2 log(den); forward lad = l, inverse lad = -l
    const float gll = INV ? -gl : gl;
    {
        const float g_dnum = gll / dnum;
        const float g_den = -2.f * gll / den;
        const float g_A = g_dnum * s * s;
        g_s += g_dnum * 2.f * s * A + g_A * 2.f * t;
        g_d1 += g_A * th * th;
        g_d0 += g_A * omt * omt;
        g_th += g_A * (2.f * d1 * th - 2.f * d0 * omt);
        g_t += g_A * 2.f * s;
        g_s += g_den * (1.f - 2.f * t);
        g_d0 += g_den * t;
        g_d1 += g_den * t;
        g_t += g_den * (d0 + d1 - 2.f * s);
    }
    if (INV) {
        // out = theta * w_b + cw_b
        g_th += go * ibw;
        g_icw += go;
        g_ibw += go * th;
        g_th += g_t * (1.f - 2.f * th);
        // theta* solves F(theta) = y, F = ch_b + h_b * N / den
        const float N_th = 2.f * s * th + d0 * (1.f - 2.f * th);
        const float den_th = (d0 + d1 - 2.f * s) * (1.f - 2.f * th);
        const float F_th = ih * (N_th * den - Nn * den_th) / (den * den);
        const float F_s = ih * (th * th * den - Nn * (1.f - 2.f * t)) / (den * den);
        const float F_d0 = ih * (t * den - Nn * t) / (den * den);
        const float F_d1 = -ih * Nn * t / (den * den);
        const float wgt = g_th / F_th;
        g_x += wgt;
        g_ich -= wgt;
        g_ih -= wgt * Nn / den;
        g_s -= wgt * F_s;
        g_d0 -= wgt * F_d0;
        g_d1 -= wgt * F_d1;
    } else {
        // out = ch_b + h_b * N / den
        const float g_num = go / den;
        const float g_den = -go * (ih * Nn) / (den * den);
        g_ich += go;
        g_ih += g_num * Nn;
        const float g_N = g_num * ih;
        g_s += g_N * th * th;
        g_th += g_N * 2.f * s * th;
        g_d0 += g_N * t;
        g_t += g_N * d0;
        g_s += g_den * (1.f - 2.f * t);
        g_d0 += g_den * t;
        g_d1 += g_den * t;
        g_t += g_den * (d0 + d1 - 2.f * s);
        g_th += g_t * (1.f - 2.f * th);
        // theta = (x - cw_b) / w_b
        g_x += g_th / ibw;
        g_icw -= g_th / ibw;
        g_ibw -= g_th * th / ibw;
    }
    // s = h_b / w_b
    g_ih += g_s / ibw;
    g_ibw -= g_s * s / ibw;
    gx = g_x;
#pragma unroll
    for (int k = 0; k <= K; ++k) {
        gcw[k] = (k == b) ? (g_icw - g_ibw) : ((k == b + 1) ? g_ibw : 0.f);
        gch[k] = (k == b) ? (g_ich - g_ih) : ((k == b + 1) ? g_ih : 0.f);
    }
#pragma unroll
    for (int k = 0; k <= K; ++k) {
        float g = 0.f;
        if (k == b) g = g_d0 * softplus_grad(e0);
        if (k == b + 1) g = g_d1 * softplus_grad(e1);
        gud[k] = g;
    }
}

// adjoints of one element inside [-B, B]: gx, guw[K], guh[K], gud[K+1]
template <int K, bool INV>
__device__ __forceinline__ void rqs_point_bwd(float xv, const float *uw, const float *uh, const float *dd, float B,
                                              float go, float gl, float &gx, float *guw, float *guh, float *gud) {
    Knots<K> W, Hh;
    build_knots<K>(uw, B, W);
    build_knots<K>(uh, B, Hh);
    float gcw[K + 1], gch[K + 1];
    rqs_bwd_core<K, INV>(xv, W.c, Hh.c, dd, go, gl, gx, gcw, gch, gud);
    knots_backward<K>(W, gcw, B, guw);
    knots_backward<K>(Hh, gch, B, guh);
}

template <int K, bool INV>
__global__ __launch_bounds__(256) void rqs_backward_kernel(int64_t M, const float *__restrict__ x, const float *__restrict__ uw,
                                    const float *__restrict__ uh, const float *__restrict__ ud, float B,
                                    const float *__restrict__ g_out, const float *__restrict__ g_lad,
                                    float *__restrict__ gx, float *__restrict__ guw, float *__restrict__ guh,
                                    float *__restrict__ gud) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M) return;
    const float xv = x[i];
    const float go = g_out ? g_out[i] : 0.f, gl = g_lad ? g_lad[i] : 0.f;
    if (!(xv >= -B && xv <= B)) {
        gx[i] = go;
#pragma unroll
        for (int k = 0; k < K; ++k) {
            guw[i * K + k] = 0.f;
            guh[i * K + k] = 0.f;
        }
#pragma unroll
        for (int k = 0; k <= K; ++k) gud[i * (K + 1) + k] = 0.f;
        return;
    }
    float a[K], b[K], d[K + 1];
    rqs_point_bwd<K, INV>(xv, uw + i * K, uh + i * K, ud + i * (K + 1), B, go, gl, gx[i], a, b, d);
#pragma unroll
    for (int k = 0; k < K; ++k) {
        guw[i * K + k] = a[k];
        guh[i * K + k] = b[k];
    }
#pragma unroll
    for (int k = 0; k <= K; ++k) gud[i * (K + 1) + k] = d[k];
}


// ---------------------------------------------------------------------------
// One coupling layer of the training path around its conditioner: the feature gather,
// periodic features (nn.py:120-137), the conditional and unconditional splines, the
// half-roll and the log-det sums (coupling.py:71-134, wrapper.py:269-275) in one launch
// per side of the conditioner instead of ~30 torch kernels.  One wave per sample row,
// lane = feature j (j += 64); log-det sums are wave reductions read from lane 0.
struct CouplingArgs {
    int64_t rows;
    int D, n, split;
    const int64_t *id, *tr;
    float bound, scale, sq;
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return __shfl(v, 0);
}

template <int K>
__device__ __forceinline__ void cond_params(const float *p, float sq, float *w, float *h) {
#pragma unroll
    for (int k = 0; k < K; ++k) {
        w[k] = p[k] / sq;  // params[..., :K] / sqrt(H) (coupling.py:340-342)
        h[k] = p[K + k] / sq;
    }
}

#ifndef FS_CPL_ROWS
#define FS_CPL_ROWS 1  // A/B at batch 256 (profiles/r02/train/cpl_rows_ab.log): 1 row ~1 % ahead of 2 or 4
#endif
// sample rows (one wave each) per workgroup of the coupling kernels
constexpr int kCplRows = FS_CPL_ROWS;

// density direction forward (Coupling.forward), after the conditioner: both splines,
// rolled output, lq_out = lq_in + (sum lad_cond + sum lad_uncond)
struct DensityFwdArgs {
    const float *x, *params, *uw, *uh, *ud, *lq_in;
    float *out, *lq_out;
};

template <int K>
__device__ __forceinline__ void density_fwd_row(const CouplingArgs &c, const DensityFwdArgs &d, int64_t row,
                                                float *rb = nullptr) {
    const int lane = threadIdx.x & 63;
    const float *xr = d.x + row * c.D;
    float sc = 0.f, su = 0.f;
    for (int j = lane; j < c.n; j += 64) {
        const int pi = (int)c.id[j], pt = (int)c.tr[j];
        const float xi = xr[pi], xt = xr[pt];
        float yt = xt, lt = 0.f;
        if (xt >= -c.bound && xt <= c.bound) {
            const float *p = d.params + (row * c.n + j) * (3 * K + 1);
            float w[K], h[K];
            cond_params<K>(p, c.sq, w, h);
            rqs_point<K, false>(xt, w, h, p + 2 * K, c.bound, yt, lt, nullptr);
        }
        float yi = xi, li = 0.f;
        if (xi >= -c.bound && xi <= c.bound)
            rqs_point<K, false>(xi, d.uw + j * K, d.uh + j * K, d.ud + j * (K + 1), c.bound, yi, li, nullptr);
        d.out[row * c.D + (pt + c.D - c.split) % c.D] = yt;
        d.out[row * c.D + (pi + c.D - c.split) % c.D] = yi;
        if (rb) {  // the row for the next layer's features in the same launch
            rb[(pt + c.D - c.split) % c.D] = yt;
            rb[(pi + c.D - c.split) % c.D] = yi;
        }
        sc += lt;
        su += li;
    }
    sc = wave_sum(sc);
    su = wave_sum(su);
    if (lane == 0) d.lq_out[row] = (d.lq_in ? d.lq_in[row] : 0.f) + (sc + su);
}

template <int K>
__global__ __launch_bounds__(256) void coupling_density_fwd_kernel(CouplingArgs c, DensityFwdArgs d) {
    const int64_t row = (int64_t)blockIdx.x * kCplRows + (threadIdx.x >> 6);
    if (row < c.rows) density_fwd_row<K>(c, d, row);
}

// its adjoints: gx (both halves, spline part), g_params [rows][n][3K+1], g_u the per-row
// unconditional adjoints [rows][n][3K+1] (summed over rows by the caller)
// two waves per row: wave part 0 takes the conditional spline's adjoints, part 1 the
// unconditional one's (each lane one feature), so the row's work is spread twice as wide.
// gor: the row of g_out (nullable: no output gradient)
template <int K>
__device__ __forceinline__ void density_bwd_row(const CouplingArgs &c, const float *__restrict__ x,
                                                const float *__restrict__ params, const float *__restrict__ uw,
                                                const float *__restrict__ uh, const float *__restrict__ ud,
                                                const float *gor, const float *__restrict__ g_lq, float *gx,
                                                float *g_params, float *g_u, int64_t row, int part) {
    const int lane = threadIdx.x & 63;
    const float *xr = x + row * c.D;
    const float gl = g_lq ? g_lq[row] : 0.f;
    constexpr int P = 3 * K + 1;
    for (int j = lane; j < c.n; j += 64) {
        const int pi = (int)c.id[j], pt = (int)c.tr[j];
        const float xi = xr[pi], xt = xr[pt];
        const float got = gor ? gor[(pt + c.D - c.split) % c.D] : 0.f;
        const float goi = gor ? gor[(pi + c.D - c.split) % c.D] : 0.f;
        float *gp = g_params + (row * c.n + j) * P;
        // g_u row: [uw n*K | uh n*K | ud n*(K+1)], the parameters' own layouts back to back
        float *guw = g_u + row * c.n * P + j * K;
        float *guh = guw + c.n * K;
        float *gud = g_u + row * c.n * P + 2 * c.n * K + j * (K + 1);
        float gw[K], gh[K], gd[K + 1];
        if (part == 1) {
        } else if (xt >= -c.bound && xt <= c.bound) {
            const float *p = params + (row * c.n + j) * P;
            float w[K], h[K];
            cond_params<K>(p, c.sq, w, h);
            float g;
            rqs_point_bwd<K, false>(xt, w, h, p + 2 * K, c.bound, got, gl, g, gw, gh, gd);
            gx[row * c.D + pt] = g;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                gp[k] = gw[k] / c.sq;
                gp[K + k] = gh[k] / c.sq;
            }
#pragma unroll
            for (int k = 0; k <= K; ++k) gp[2 * K + k] = gd[k];
        } else {
            gx[row * c.D + pt] = got;
#pragma unroll
            for (int k = 0; k < P; ++k) gp[k] = 0.f;
        }
        if (part == 0) {
        } else if (xi >= -c.bound && xi <= c.bound) {
            float g;
            rqs_point_bwd<K, false>(xi, uw + j * K, uh + j * K, ud + j * (K + 1), c.bound, goi, gl, g, gw, gh, gd);
            gx[row * c.D + pi] = g;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                guw[k] = gw[k];
                guh[k] = gh[k];
            }
#pragma unroll
            for (int k = 0; k <= K; ++k) gud[k] = gd[k];
        } else {
            gx[row * c.D + pi] = goi;
#pragma unroll
            for (int k = 0; k < K; ++k) {
                guw[k] = 0.f;
                guh[k] = 0.f;
            }
#pragma unroll
            for (int k = 0; k <= K; ++k) gud[k] = 0.f;
        }
    }
}

template <int K>
__global__ __launch_bounds__(256) void coupling_density_bwd_kernel(
    CouplingArgs c, const float *__restrict__ x, const float *__restrict__ params, const float *__restrict__ uw,
    const float *__restrict__ uh, const float *__restrict__ ud, const float *__restrict__ g_out,
    const float *__restrict__ g_lq, float *gx, float *g_params, float *g_u) {
    const int wv = threadIdx.x >> 6;
    const int64_t row = (int64_t)blockIdx.x * kCplRows + (wv >> 1);
    if (row >= c.rows) return;
    density_bwd_row<K>(c, x, params, uw, uh, ud, g_out ? g_out + row * c.D : nullptr, g_lq, gx, g_params, g_u, row,
                       wv & 1);
}

// density direction, before the conditioner: t = [cos(s x_id), sin(s x_id)]
__device__ __forceinline__ void features_row(const CouplingArgs &c, const float *__restrict__ x, float *t, int64_t row,
                                             const float *xr = nullptr) {
    const int lane = threadIdx.x & 63;
    if (!xr) xr = x + row * c.D;
    for (int j = lane; j < c.n; j += 64) {
        const float v = c.scale * xr[c.id[j]];
        t[row * 2 * c.n + j] = cosf(v);
        t[row * 2 * c.n + c.n + j] = sinf(v);
    }
}

__global__ __launch_bounds__(256) void coupling_features_fwd_kernel(CouplingArgs c, const float *__restrict__ x,
                                                                    float *t) {
    const int64_t row = (int64_t)blockIdx.x * kCplRows + (threadIdx.x >> 6);
    if (row < c.rows) features_row(c, x, t, row);
}

// adjoint of the periodic features t = [cos(s x_id), sin(s x_id)]: gx at the identity
// positions, 0 at the transform positions (+ gx_add, the splines' gradient of the same x)
__device__ __forceinline__ void features_bwd_row(const CouplingArgs &c, const float *__restrict__ x,
                                                 const float *__restrict__ g_t, float *gx,
                                                 const float *__restrict__ gx_add, int64_t row, float *rb = nullptr) {
    const int lane = threadIdx.x & 63;
    for (int j = lane; j < c.n; j += 64) {
        const int pi = (int)c.id[j], pt = (int)c.tr[j];
        const float v = c.scale * x[row * c.D + pi];
        const float gc = g_t[row * 2 * c.n + j] * -sinf(v), gs = g_t[row * 2 * c.n + c.n + j] * cosf(v);
        const float ai = gx_add ? gx_add[row * c.D + pi] : 0.f, at = gx_add ? gx_add[row * c.D + pt] : 0.f;
        const float gi = (gc * c.scale + gs * c.scale) + ai;
        gx[row * c.D + pi] = gi;
        gx[row * c.D + pt] = at;
        if (rb) {
            rb[pi] = gi;
            rb[pt] = at;
        }
    }
}

__global__ __launch_bounds__(256) void coupling_features_bwd_kernel(CouplingArgs c, const float *__restrict__ x,
                                                                    const float *__restrict__ g_t, float *gx,
                                                                    const float *__restrict__ gx_add) {
    const int64_t row = (int64_t)blockIdx.x * kCplRows + (threadIdx.x >> 6);
    if (row >= c.rows) return;
    features_bwd_row(c, x, g_t, gx, gx_add, row);
}

// The backward between two layers of the density pass in one launch (fs_coupling_bwd_step):
// layer l's features adjoint (its input gradient, = the output gradient of layer l - 1,
// kept in LDS and also written to gx) and then layer l - 1's spline adjoints on that row,
// each exactly as fs_coupling_features_bwd then fs_coupling_density_bwd compute them.
constexpr int kCplMaxDB = 256;

template <int K>
__global__ __launch_bounds__(256) void coupling_bwd_step_kernel(CouplingArgs cf, const float *__restrict__ xf,
                                                                const float *__restrict__ g_t, float *gxf,
                                                                const float *__restrict__ gx_add, CouplingArgs c,
                                                                const float *__restrict__ x,
                                                                const float *__restrict__ params,
                                                                const float *__restrict__ uw,
                                                                const float *__restrict__ uh,
                                                                const float *__restrict__ ud,
                                                                const float *__restrict__ g_lq, float *gx,
                                                                float *g_params, float *g_u) {
    __shared__ float rbuf[kCplRows][kCplMaxDB];
    const int wv = threadIdx.x >> 6;
    float *rb = rbuf[wv >> 1];
    const int64_t row = (int64_t)blockIdx.x * kCplRows + (wv >> 1);
    const bool live = row < c.rows;
    if (live && (wv & 1) == 0) features_bwd_row(cf, xf, g_t, gxf, gx_add, row, rb);
    __syncthreads();
    if (!live) return;
    density_bwd_row<K>(c, x, params, uw, uh, ud, rb, g_lq, gx, g_params, g_u, row, wv & 1);
}

// sampling direction (Coupling.inverse), forward only: roll, unconditional inverse spline
// of the identity half, features of its output; out holds the new identity values and
// the untouched transform half; lad_u[row] = its log-det sum
struct SamplePreArgs {
    const float *z, *uw, *uh, *ud;
    float *t, *out, *lad_u;
    int32_t *nan_flag;
};

template <int K>
__device__ __forceinline__ void sample_pre_row(const CouplingArgs &c, const SamplePreArgs &s, int64_t row,
                                               const float *zr = nullptr) {
    const int lane = threadIdx.x & 63;
    if (!zr) zr = s.z + row * c.D;
    float su = 0.f;
    for (int j = lane; j < c.n; j += 64) {
        const int pi = (int)c.id[j], pt = (int)c.tr[j];
        const float xi = zr[(pi + c.split) % c.D];
        float yi = xi, li = 0.f;
        if (xi >= -c.bound && xi <= c.bound)
            rqs_point<K, true>(xi, s.uw + j * K, s.uh + j * K, s.ud + j * (K + 1), c.bound, yi, li, s.nan_flag);
        const float v = c.scale * yi;
        s.t[row * 2 * c.n + j] = cosf(v);
        s.t[row * 2 * c.n + c.n + j] = sinf(v);
        s.out[row * c.D + pi] = yi;
        s.out[row * c.D + pt] = zr[(pt + c.split) % c.D];
        su += li;
    }
    su = wave_sum(su);
    if (lane == 0) s.lad_u[row] = su;
}

template <int K>
__global__ __launch_bounds__(256) void coupling_sample_pre_kernel(CouplingArgs c, SamplePreArgs s) {
    const int64_t row = (int64_t)blockIdx.x * kCplRows + (threadIdx.x >> 6);
    if (row < c.rows) sample_pre_row<K>(c, s, row);
}

// ... then the conditional inverse spline of the transform half in place;
// lq_out = lq_in - (lad_u + sum lad_cond)
struct SamplePostArgs {
    const float *params, *lad_u, *lq_in;
    float *out, *lq_out;
    int32_t *nan_flag;
};

template <int K>
__device__ __forceinline__ void sample_post_row(const CouplingArgs &c, const SamplePostArgs &s, int64_t row,
                                                float *rb = nullptr) {
    const int lane = threadIdx.x & 63;
    float sc = 0.f;
    for (int j = lane; j < c.n; j += 64) {
        const int pt = (int)c.tr[j];
        if (rb) {
            const int pi = (int)c.id[j];
            rb[pi] = s.out[row * c.D + pi];  // written by this layer's pre launch
        }
        const float xt = s.out[row * c.D + pt];
        float yt = xt, lt = 0.f;
        if (xt >= -c.bound && xt <= c.bound) {
            const float *p = s.params + (row * c.n + j) * (3 * K + 1);
            float w[K], h[K];
            cond_params<K>(p, c.sq, w, h);
            rqs_point<K, true>(xt, w, h, p + 2 * K, c.bound, yt, lt, s.nan_flag);
        }
        s.out[row * c.D + pt] = yt;
        if (rb) rb[pt] = yt;
        sc += lt;
    }
    sc = wave_sum(sc);
    if (lane == 0) s.lq_out[row] = (s.lq_in ? s.lq_in[row] : 0.f) - (s.lad_u[row] + sc);
}

template <int K>
__global__ __launch_bounds__(256) void coupling_sample_post_kernel(CouplingArgs c, SamplePostArgs s) {
    const int64_t row = (int64_t)blockIdx.x * kCplRows + (threadIdx.x >> 6);
    if (row < c.rows) sample_post_row<K>(c, s, row);
}

// The training step's two passes side by side (fs_coupling_pair_pre / _post): workgroups
// [0, nb0) run the sampling pass's layer (rows of cs), the rest the density pass's layer
// (rows of cd), each row exactly as the single-pass kernels compute it.
template <int K>
__global__ __launch_bounds__(256) void coupling_pair_pre_kernel(CouplingArgs cs, SamplePreArgs s, CouplingArgs cd,
                                                                const float *__restrict__ x, float *t, unsigned nb0) {
    const bool dens = blockIdx.x >= nb0;
    const int64_t row = (int64_t)(dens ? blockIdx.x - nb0 : blockIdx.x) * kCplRows + (threadIdx.x >> 6);
    if (!dens) {
        if (row < cs.rows) sample_pre_row<K>(cs, s, row);
    } else if (row < cd.rows) {
        features_row(cd, x, t, row);
    }
}

template <int K>
__global__ __launch_bounds__(256) void coupling_pair_post_kernel(CouplingArgs cs, SamplePostArgs s, CouplingArgs cd,
                                                                 DensityFwdArgs d, unsigned nb0) {
    const bool dens = blockIdx.x >= nb0;
    const int64_t row = (int64_t)(dens ? blockIdx.x - nb0 : blockIdx.x) * kCplRows + (threadIdx.x >> 6);
    if (!dens) {
        if (row < cs.rows) sample_post_row<K>(cs, s, row);
    } else if (row < cd.rows) {
        density_fwd_row<K>(cd, d, row);
    }
}

// One launch between two layers of the training step's passes (fs_coupling_pair_step):
// the post launch of layer l (sampling: conditional inverse spline; density: both splines,
// roll, log-det) and, on the row it just produced (kept in LDS), the pre launch of the
// next layer (sampling: roll + unconditional inverse spline + features; density: the
// features).  Each row exactly as fs_coupling_pair_post then fs_coupling_pair_pre compute
// it; one launch and one HBM round trip of the rows fewer per layer.
constexpr int kCplMaxD = 256;

template <int K>
__global__ __launch_bounds__(256) void coupling_pair_step_kernel(CouplingArgs cs, SamplePostArgs s, CouplingArgs cs2,
                                                                 SamplePreArgs s2, CouplingArgs cd, DensityFwdArgs d,
                                                                 CouplingArgs cd2, float *t_d2, unsigned nb0) {
    __shared__ float rbuf[kCplRows][kCplMaxD];
    float *rb = rbuf[threadIdx.x >> 6];
    const bool dens = blockIdx.x >= nb0;
    const int64_t row = (int64_t)(dens ? blockIdx.x - nb0 : blockIdx.x) * kCplRows + (threadIdx.x >> 6);
    const bool live = dens ? row < cd.rows : row < cs.rows;
    if (live) {
        if (!dens)
            sample_post_row<K>(cs, s, row, rb);
        else
            density_fwd_row<K>(cd, d, row, rb);
    }
    __syncthreads();  // the row's LDS copy, written by every lane of its wave
    if (!live) return;
    if (!dens)
        sample_pre_row<K>(cs2, s2, row, rb);
    else
        features_row(cd2, d.out, t_d2, row, rb);
}

// ---------------------------------------------------------------------------
// The same two launches with each row's splines spread over more waves
// (fs_set_coupling_waves, default on).  A spline's cost is mostly building its two knot
// sets (softmax + cumulative sum over K, each element a precise division), one lane per
// feature in a serial chain; here wave h of a pair builds one set (h = 0 widths, h = 1
// heights), the pair swaps the knots through LDS and finishes the element from them.
// Every value comes from the same device functions on the same operands, so the
// results are bit-identical to coupling_pair_step_kernel / coupling_bwd_step_kernel
// (tests/test_gpu_train.py).

// knots c[0..K] of wave slot w (lane-major in kx: conflict-free)
template <int K>
__device__ __forceinline__ void knots_put(float *kx, int w, const float *c) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k <= K; ++k) kx[(w * (K + 1) + k) * 64 + lane] = c[k];
}

template <int K>
__device__ __forceinline__ void knots_get(const float *kx, int w, float *c) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int k = 0; k <= K; ++k) c[k] = kx[(w * (K + 1) + k) * 64 + lane];
}

// this wave's knot set (own) and its partner's (slot w ^ 1) as (width, height) knots
template <int K>
__device__ __forceinline__ void knots_pair(float *kx, int w, int h, const float *own, float *wc, float *hc) {
    knots_put<K>(kx, w, own);
    __syncthreads();
    float oc[K + 1];
    knots_get<K>(kx, w ^ 1, oc);
#pragma unroll
    for (int k = 0; k <= K; ++k) {
        wc[k] = h == 0 ? own[k] : oc[k];
        hc[k] = h == 0 ? oc[k] : own[k];
    }
}

// sample_post_row on a wave pair (h: this wave's knot set); the lower wave stores
template <int K>
__device__ __forceinline__ void sample_post_row2(const CouplingArgs &c, const SamplePostArgs &s, int64_t row, float *rb,
                                                 float *kx, int h) {
    const int lane = threadIdx.x & 63;
    float sc = 0.f;
    for (int j0 = 0; j0 < c.n; j0 += 64) {  // uniform trip count: the pair meets at its barriers
        const int j = j0 + lane;
        const bool on = j < c.n;
        const int jj = on ? j : 0;
        const int pt = (int)c.tr[jj];
        if (h == 0 && on) {
            const int pi = (int)c.id[jj];
            rb[pi] = s.out[row * c.D + pi];  // written by this layer's pre launch
        }
        const float xt = s.out[row * c.D + pt];
        const float *p = s.params + (row * c.n + jj) * (3 * K + 1);
        Knots<K> kn;
        {
            float u[K];
#pragma unroll
            for (int k = 0; k < K; ++k) u[k] = p[h * K + k] / c.sq;  // cond_params' half
            build_knots<K>(u, c.bound, kn);
        }
        float wc[K + 1], hc[K + 1];
        knots_pair<K>(kx, h, h, kn.c, wc, hc);
        float yt = xt, lt = 0.f;
        if (on && xt >= -c.bound && xt <= c.bound)
            rqs_eval_knots<K, true>(xt, wc, hc, p + 2 * K, yt, lt, h == 0 ? s.nan_flag : nullptr);
        if (h == 0 && on) {
            s.out[row * c.D + pt] = yt;
            rb[pt] = yt;
        }
        sc += on ? lt : 0.f;
        __syncthreads();  // the partner has read this round's knots
    }
    sc = wave_sum(sc);
    if (h == 0 && lane == 0) s.lq_out[row] = (s.lq_in ? s.lq_in[row] : 0.f) - (s.lad_u[row] + sc);
}

// sample_pre_row on a wave pair: the lower wave stores the cosines and the row, the upper
// one the sines
template <int K>
__device__ __forceinline__ void sample_pre_row2(const CouplingArgs &c, const SamplePreArgs &s, int64_t row,
                                                const float *zr, float *kx, int h) {
    const int lane = threadIdx.x & 63;
    float su = 0.f;
    for (int j0 = 0; j0 < c.n; j0 += 64) {
        const int j = j0 + lane;
        const bool on = j < c.n;
        const int jj = on ? j : 0;
        const int pi = (int)c.id[jj], pt = (int)c.tr[jj];
        const float xi = zr[(pi + c.split) % c.D];
        Knots<K> kn;
        build_knots<K>((h == 0 ? s.uw : s.uh) + jj * K, c.bound, kn);
        float wc[K + 1], hc[K + 1];
        knots_pair<K>(kx, h, h, kn.c, wc, hc);
        float yi = xi, li = 0.f;
        if (on && xi >= -c.bound && xi <= c.bound)
            rqs_eval_knots<K, true>(xi, wc, hc, s.ud + jj * (K + 1), yi, li, h == 0 ? s.nan_flag : nullptr);
        const float v = c.scale * yi;
        if (on) {
            if (h == 0) {
                s.t[row * 2 * c.n + j] = cosf(v);
                s.out[row * c.D + pi] = yi;
                s.out[row * c.D + pt] = zr[(pt + c.split) % c.D];
            } else {
                s.t[row * 2 * c.n + c.n + j] = sinf(v);
            }
        }
        su += on ? li : 0.f;
        __syncthreads();
    }
    su = wave_sum(su);
    if (h == 0 && lane == 0) s.lad_u[row] = su;
}

// density_fwd_row on a wave pair: wave 0 the conditional spline of the transform half,
// wave 1 the unconditional one of the identity half; the log-det sums meet in red
template <int K>
__device__ __forceinline__ float density_fwd_row2(const CouplingArgs &c, const DensityFwdArgs &d, int64_t row, float *rb,
                                                  float *red, int h) {
    const int lane = threadIdx.x & 63;
    const float *xr = d.x + row * c.D;
    float sl = 0.f;
    for (int j = lane; j < c.n; j += 64) {
        if (h == 0) {
            const int pt = (int)c.tr[j];
            const float xt = xr[pt];
            float yt = xt, lt = 0.f;
            if (xt >= -c.bound && xt <= c.bound) {
                const float *p = d.params + (row * c.n + j) * (3 * K + 1);
                float w[K], hh[K];
                cond_params<K>(p, c.sq, w, hh);
                rqs_point<K, false>(xt, w, hh, p + 2 * K, c.bound, yt, lt, nullptr);
            }
            d.out[row * c.D + (pt + c.D - c.split) % c.D] = yt;
            rb[(pt + c.D - c.split) % c.D] = yt;
            sl += lt;
        } else {
            const int pi = (int)c.id[j];
            const float xi = xr[pi];
            float yi = xi, li = 0.f;
            if (xi >= -c.bound && xi <= c.bound)
                rqs_point<K, false>(xi, d.uw + j * K, d.uh + j * K, d.ud + j * (K + 1), c.bound, yi, li, nullptr);
            d.out[row * c.D + (pi + c.D - c.split) % c.D] = yi;
            rb[(pi + c.D - c.split) % c.D] = yi;
            sl += li;
        }
    }
    sl = wave_sum(sl);
    if (h == 1 && lane == 0) red[0] = sl;
    return sl;
}

template <int K>
__global__ __launch_bounds__(128) void coupling_pair_step2_kernel(CouplingArgs cs, SamplePostArgs s, CouplingArgs cs2,
                                                                  SamplePreArgs s2, CouplingArgs cd, DensityFwdArgs d,
                                                                  CouplingArgs cd2, float *t_d2, unsigned nb0) {
    __shared__ float rb[kCplMaxD];
    __shared__ float kx[2 * (K + 1) * 64];
    __shared__ float red[1];
    const int h = (int)(threadIdx.x >> 6);
    const bool dens = blockIdx.x >= nb0;
    const int64_t row = (int64_t)(dens ? blockIdx.x - nb0 : blockIdx.x);
    if (!dens) {
        if (row >= cs.rows) return;  // whole workgroup: no barrier is left waiting
        sample_post_row2<K>(cs, s, row, rb, kx, h);
        __syncthreads();  // the row in LDS
        sample_pre_row2<K>(cs2, s2, row, rb, kx, h);
        return;
    }
    if (row >= cd.rows) return;
    const float sl = density_fwd_row2<K>(cd, d, row, rb, red, h);
    __syncthreads();  // the row in LDS, the unconditional log-det sum in red
    const int lane = threadIdx.x & 63;
    if (h == 0 && lane == 0) d.lq_out[row] = (d.lq_in ? d.lq_in[row] : 0.f) + (sl + red[0]);  // density_fwd_row's order
    for (int j = lane; j < cd2.n; j += 64) {  // features_row, cosines on wave 0, sines on wave 1
        const float v = cd2.scale * rb[cd2.id[j]];
        if (h == 0)
            t_d2[row * 2 * cd2.n + j] = cosf(v);
        else
            t_d2[row * 2 * cd2.n + cd2.n + j] = sinf(v);
    }
}

// density_bwd_row on four waves: part = wave >> 1 (0: the conditional spline's adjoints,
// 1: the unconditional one's, as in density_bwd_row), h = wave & 1 the knot set it builds
// and back-propagates (0 widths, 1 heights); the core adjoints are computed by both waves
// of a part from the swapped knots
template <int K>
__device__ __forceinline__ void density_bwd_row4(const CouplingArgs &c, const float *__restrict__ x,
                                                 const float *__restrict__ params, const float *__restrict__ uw,
                                                 const float *__restrict__ uh, const float *__restrict__ ud,
                                                 const float *gor, const float *__restrict__ g_lq, float *gx,
                                                 float *g_params, float *g_u, int64_t row, float *kx) {
    const int lane = threadIdx.x & 63, wv = (int)(threadIdx.x >> 6), part = wv >> 1, h = wv & 1;
    const float *xr = x + row * c.D;
    const float gl = g_lq ? g_lq[row] : 0.f;
    constexpr int P = 3 * K + 1;
    for (int j0 = 0; j0 < c.n; j0 += 64) {
        const int j = j0 + lane;
        const bool on = j < c.n;
        const int jj = on ? j : 0;
        const int pi = (int)c.id[jj], pt = (int)c.tr[jj];
        const int pos = part == 0 ? pt : pi;
        const float xv = xr[pos];
        const float go = gor ? gor[(pos + c.D - c.split) % c.D] : 0.f;
        const float *p = params + (row * c.n + jj) * P;
        Knots<K> kn;
        if (part == 0) {
            float u[K];
#pragma unroll
            for (int k = 0; k < K; ++k) u[k] = p[h * K + k] / c.sq;  // cond_params' half
            build_knots<K>(u, c.bound, kn);
        } else {
            build_knots<K>((h == 0 ? uw : uh) + jj * K, c.bound, kn);
        }
        float wc[K + 1], hc[K + 1];
        knots_pair<K>(kx, wv, h, kn.c, wc, hc);
        const bool inside = xv >= -c.bound && xv <= c.bound;
        float *gp = g_params + (row * c.n + jj) * P;
        // g_u row: [uw n*K | uh n*K | ud n*(K+1)], the parameters' own layouts back to back
        float *guw = g_u + row * c.n * P + jj * K;
        float *guh = guw + c.n * K;
        float *gud = g_u + row * c.n * P + 2 * c.n * K + jj * (K + 1);
        if (on && inside) {
            float g, gcw[K + 1], gch[K + 1], gd[K + 1];
            rqs_bwd_core<K, false>(xv, wc, hc, part == 0 ? p + 2 * K : ud + jj * (K + 1), go, gl, g, gcw, gch, gd);
            float gsel[K + 1], gk[K];
#pragma unroll
            for (int k = 0; k <= K; ++k) gsel[k] = h == 0 ? gcw[k] : gch[k];
            knots_backward<K>(kn, gsel, c.bound, gk);
            if (part == 0) {
#pragma unroll
                for (int k = 0; k < K; ++k) gp[h * K + k] = gk[k] / c.sq;
                if (h == 0) {
                    gx[row * c.D + pt] = g;
#pragma unroll
                    for (int k = 0; k <= K; ++k) gp[2 * K + k] = gd[k];
                }
            } else {
                float *gu = h == 0 ? guw : guh;
#pragma unroll
                for (int k = 0; k < K; ++k) gu[k] = gk[k];
                if (h == 0) {
                    gx[row * c.D + pi] = g;
#pragma unroll
                    for (int k = 0; k <= K; ++k) gud[k] = gd[k];
                }
            }
        } else if (on) {
            if (part == 0) {
#pragma unroll
                for (int k = 0; k < K; ++k) gp[h * K + k] = 0.f;
                if (h == 0) {
                    gx[row * c.D + pt] = go;
#pragma unroll
                    for (int k = 0; k <= K; ++k) gp[2 * K + k] = 0.f;
                }
            } else {
                float *gu = h == 0 ? guw : guh;
#pragma unroll
                for (int k = 0; k < K; ++k) gu[k] = 0.f;
                if (h == 0) {
                    gx[row * c.D + pi] = go;
#pragma unroll
                    for (int k = 0; k <= K; ++k) gud[k] = 0.f;
                }
            }
        }
        __syncthreads();  // the partners have read this round's knots
    }
}

template <int K>
__global__ __launch_bounds__(256) void coupling_bwd_step4_kernel(CouplingArgs cf, const float *__restrict__ xf,
                                                                 const float *__restrict__ g_t, float *gxf,
                                                                 const float *__restrict__ gx_add, CouplingArgs c,
                                                                 const float *__restrict__ x,
                                                                 const float *__restrict__ params,
                                                                 const float *__restrict__ uw,
                                                                 const float *__restrict__ uh,
                                                                 const float *__restrict__ ud,
                                                                 const float *__restrict__ g_lq, float *gx,
                                                                 float *g_params, float *g_u) {
    __shared__ float rb[kCplMaxDB];
    __shared__ float kx[4 * (K + 1) * 64];
    const int64_t row = blockIdx.x;
    if (row >= c.rows) return;  // whole workgroup
    if (threadIdx.x < 64) features_bwd_row(cf, xf, g_t, gxf, gx_add, row, rb);
    __syncthreads();
    density_bwd_row4<K>(c, x, params, uw, uh, ud, rb, g_lq, gx, g_params, g_u, row, kx);
}

}  // namespace fs

using namespace fs;

#define FS_RQS_K(X) X(5) X(8) X(15) X(32)

hipError_t fs_rqs_forward_impl(int64_t M, int K, int inverse, const float *x, const float *uw, const float *uh,
                               const float *ud, float B, float *out, float *lad, int32_t *nan_flag,
                               hipStream_t st) {
    if (M <= 0) return hipSuccess;
    const dim3 grid((unsigned)((M + 255) / 256)), block(256);
#define FS_F(KK)                                                                                          \
    if (K == KK) {                                                                                        \
        if (inverse)                                                                                      \
            hipLaunchKernelGGL((rqs_forward_kernel<KK, true>), grid, block, 0, st, M, x, uw, uh, ud, B, out, \
                               lad, nan_flag);                                                            \
        else                                                                                              \
            hipLaunchKernelGGL((rqs_forward_kernel<KK, false>), grid, block, 0, st, M, x, uw, uh, ud, B, out, \
                               lad, nan_flag);                                                            \
        return hipGetLastError();                                                                         \
    }
    FS_RQS_K(FS_F)
#undef FS_F
    return hipErrorInvalidValue;
}

hipError_t fs_rqs_backward_impl(int64_t M, int K, int inverse, const float *x, const float *uw, const float *uh,
                                const float *ud, float B, const float *g_out, const float *g_lad, float *gx,
                                float *guw, float *guh, float *gud, hipStream_t st) {
    if (M <= 0) return hipSuccess;
    const dim3 grid((unsigned)((M + 255) / 256)), block(256);
#define FS_B(KK)                                                                                              \
    if (K == KK) {                                                                                            \
        if (inverse)                                                                                          \
            hipLaunchKernelGGL((rqs_backward_kernel<KK, true>), grid, block, 0, st, M, x, uw, uh, ud, B, g_out, \
                               g_lad, gx, guw, guh, gud);                                                     \
        else                                                                                                  \
            hipLaunchKernelGGL((rqs_backward_kernel<KK, false>), grid, block, 0, st, M, x, uw, uh, ud, B, g_out, \
                               g_lad, gx, guw, guh, gud);                                                     \
        return hipGetLastError();                                                                             \
    }
    FS_RQS_K(FS_B)
#undef FS_B
    return hipErrorInvalidValue;
}

// the training step's coupling launches on two / four waves per row (1, default, or
// FS_COUPLING_WAVES / fs_set_coupling_waves) or one / two (0); bit-identical either way
static std::atomic<int> g_cpl_waves{-1};
static bool coupling_waves() {
    int v = g_cpl_waves.load(std::memory_order_relaxed);
    if (v < 0) {
        const char *e = getenv("FS_COUPLING_WAVES");
        int expect = -1;
        g_cpl_waves.compare_exchange_strong(expect, (e && e[0] == '0') ? 0 : 1);
        v = g_cpl_waves.load(std::memory_order_relaxed);
    }
    return v != 0;
}

int32_t fs_set_coupling_waves_impl(int32_t on) {
    const int32_t prev = coupling_waves() ? 1 : 0;
    if (on >= 0) g_cpl_waves.store(on ? 1 : 0, std::memory_order_relaxed);
    return prev;
}

static fs::CouplingArgs coupling_args(const fs_coupling *c) {
    fs::CouplingArgs a;
    a.rows = c->rows;
    a.D = c->D;
    a.n = c->D / 2;
    a.split = c->D / 2;
    a.id = c->identity_features;
    a.tr = c->transform_features;
    a.bound = (float)c->tail_bound;
    a.scale = (float)(M_PI / c->tail_bound);  // scale * ident with the Python-float scale (nn.py:133)
    a.sq = (float)sqrt((double)c->hidden);     // np.sqrt(num_hidden_channels) (coupling.py:340)
    return a;
}

#define FS_COUPLING_LAUNCH(KERNEL, ...)                                                         \
    const fs::CouplingArgs a = coupling_args(cp);                                               \
    if (a.rows <= 0) return hipSuccess;                                                         \
    const dim3 grid((unsigned)((a.rows + kCplRows - 1) / kCplRows)), block(64 * kCplRows);                                  \
    switch (cp->K) {                                                                            \
    case 5: hipLaunchKernelGGL((KERNEL<5>), grid, block, 0, st, a, __VA_ARGS__); break;         \
    case 8: hipLaunchKernelGGL((KERNEL<8>), grid, block, 0, st, a, __VA_ARGS__); break;         \
    case 15: hipLaunchKernelGGL((KERNEL<15>), grid, block, 0, st, a, __VA_ARGS__); break;       \
    case 32: hipLaunchKernelGGL((KERNEL<32>), grid, block, 0, st, a, __VA_ARGS__); break;       \
    default: return hipErrorInvalidValue;                                                       \
    }                                                                                           \
    return hipGetLastError();

hipError_t fs_coupling_density_fwd_impl(const fs_coupling *cp, const float *x, const float *params, const float *uw,
                                        const float *uh, const float *ud, const float *lq_in, float *out, float *lq_out,
                                        hipStream_t st) {
    const DensityFwdArgs d{x, params, uw, uh, ud, lq_in, out, lq_out};
    FS_COUPLING_LAUNCH(coupling_density_fwd_kernel, d)
}

hipError_t fs_coupling_density_bwd_impl(const fs_coupling *cp, const float *x, const float *params, const float *uw,
                                        const float *uh, const float *ud, const float *g_out, const float *g_lq,
                                        float *gx, float *g_params, float *g_u, hipStream_t st) {
    static_assert(2 * kCplRows <= 4, "launch bounds: two waves per row");
    const fs::CouplingArgs a = coupling_args(cp);
    if (a.rows <= 0) return hipSuccess;
    const unsigned grid = (unsigned)((a.rows + kCplRows - 1) / kCplRows);
#define FS_DB(KK)                                                                                                  \
    if (cp->K == KK) {                                                                                             \
        hipLaunchKernelGGL(coupling_density_bwd_kernel<KK>, dim3(grid), dim3(128 * kCplRows), 0, st, a, x, params, uw, \
                           uh, ud, g_out, g_lq, gx, g_params, g_u);                                                \
        return hipGetLastError();                                                                                  \
    }
    FS_DB(5) FS_DB(8) FS_DB(15) FS_DB(32)
#undef FS_DB
    return hipErrorInvalidValue;
}

hipError_t fs_coupling_bwd_step_impl(const fs_coupling *fp, const float *xf, const float *g_t, float *gxf,
                                     const float *gx_add, const fs_coupling *cp, const float *x, const float *params,
                                     const float *uw, const float *uh, const float *ud, const float *g_lq, float *gx,
                                     float *g_params, float *g_u, hipStream_t st) {
    const fs::CouplingArgs af = coupling_args(fp), a = coupling_args(cp);
    if (af.rows != a.rows || af.D != a.D || a.D > kCplMaxDB) return hipErrorInvalidValue;
    if (a.rows <= 0) return hipSuccess;
    const unsigned grid = (unsigned)((a.rows + kCplRows - 1) / kCplRows);
    const bool four = coupling_waves() && a.rows <= 0x7fffffff;
#define FS_DB(KK)                                                                                                  \
    if (cp->K == KK) {                                                                                             \
        if (four)                                                                                                  \
            hipLaunchKernelGGL(coupling_bwd_step4_kernel<KK>, dim3((unsigned)a.rows), dim3(256), 0, st, af, xf, g_t, \
                               gxf, gx_add, a, x, params, uw, uh, ud, g_lq, gx, g_params, g_u);                   \
        else                                                                                                       \
            hipLaunchKernelGGL(coupling_bwd_step_kernel<KK>, dim3(grid), dim3(128 * kCplRows), 0, st, af, xf, g_t,  \
                               gxf, gx_add, a, x, params, uw, uh, ud, g_lq, gx, g_params, g_u);                   \
        return hipGetLastError();                                                                                  \
    }
    FS_DB(5) FS_DB(8) FS_DB(15) FS_DB(32)
#undef FS_DB
    return hipErrorInvalidValue;
}

hipError_t fs_coupling_sample_pre_impl(const fs_coupling *cp, const float *z, const float *uw, const float *uh,
                                       const float *ud, float *t, float *out, float *lad_u, int32_t *nan_flag,
                                       hipStream_t st) {
    const SamplePreArgs s{z, uw, uh, ud, t, out, lad_u, nan_flag};
    FS_COUPLING_LAUNCH(coupling_sample_pre_kernel, s)
}

hipError_t fs_coupling_sample_post_impl(const fs_coupling *cp, const float *params, const float *lad_u,
                                        const float *lq_in, float *out, float *lq_out, int32_t *nan_flag,
                                        hipStream_t st) {
    const SamplePostArgs s{params, lad_u, lq_in, out, lq_out, nan_flag};
    FS_COUPLING_LAUNCH(coupling_sample_post_kernel, s)
}
#undef FS_COUPLING_LAUNCH

#define FS_PAIR_LAUNCH(KERNEL, ...)                                                                     \
    const fs::CouplingArgs as = coupling_args(sp), ad = coupling_args(dp);                              \
    if (sp->K != dp->K || as.rows < 0 || ad.rows < 0) return hipErrorInvalidValue;                     \
    const unsigned nb0 = (unsigned)((as.rows + kCplRows - 1) / kCplRows);                              \
    const unsigned nb = nb0 + (unsigned)((ad.rows + kCplRows - 1) / kCplRows);                         \
    if (nb == 0) return hipSuccess;                                                                     \
    const dim3 block(64 * kCplRows);                                                                    \
    switch (sp->K) {                                                                                    \
    case 5: hipLaunchKernelGGL((KERNEL<5>), dim3(nb), block, 0, st, __VA_ARGS__, nb0); break;           \
    case 8: hipLaunchKernelGGL((KERNEL<8>), dim3(nb), block, 0, st, __VA_ARGS__, nb0); break;           \
    case 15: hipLaunchKernelGGL((KERNEL<15>), dim3(nb), block, 0, st, __VA_ARGS__, nb0); break;         \
    case 32: hipLaunchKernelGGL((KERNEL<32>), dim3(nb), block, 0, st, __VA_ARGS__, nb0); break;         \
    default: return hipErrorInvalidValue;                                                               \
    }                                                                                                   \
    return hipGetLastError();

hipError_t fs_coupling_pair_pre_impl(const fs_coupling *sp, const float *z, const float *uw, const float *uh,
                                     const float *ud, float *t, float *out, float *lad_u, int32_t *nan_flag,
                                     const fs_coupling *dp, const float *x, float *td, hipStream_t st) {
    const SamplePreArgs s{z, uw, uh, ud, t, out, lad_u, nan_flag};
    FS_PAIR_LAUNCH(coupling_pair_pre_kernel, as, s, ad, x, td)
}

hipError_t fs_coupling_pair_post_impl(const fs_coupling *sp, const float *params, const float *lad_u,
                                      const float *lq_in, float *out, float *lq_out, int32_t *nan_flag,
                                      const fs_coupling *dp, const float *x, const float *params_d, const float *uw,
                                      const float *uh, const float *ud, const float *lq_in_d, float *out_d,
                                      float *lq_out_d, hipStream_t st) {
    const SamplePostArgs s{params, lad_u, lq_in, out, lq_out, nan_flag};
    const DensityFwdArgs d{x, params_d, uw, uh, ud, lq_in_d, out_d, lq_out_d};
    FS_PAIR_LAUNCH(coupling_pair_post_kernel, as, s, ad, d)
}
#undef FS_PAIR_LAUNCH

hipError_t fs_coupling_pair_step_impl(const fs_coupling *sp, const float *params, const float *lad_u,
                                      const float *lq_in, float *out, float *lq_out, int32_t *nan_flag,
                                      const fs_coupling *sp2, const float *uw2, const float *uh2, const float *ud2,
                                      float *t2, float *out2, float *lad_u2, const fs_coupling *dp, const float *x,
                                      const float *params_d, const float *uw, const float *uh, const float *ud,
                                      const float *lq_in_d, float *out_d, float *lq_out_d, const fs_coupling *dp2,
                                      float *t_d2, hipStream_t st) {
    const SamplePostArgs s{params, lad_u, lq_in, out, lq_out, nan_flag};
    const SamplePreArgs s2{out, uw2, uh2, ud2, t2, out2, lad_u2, nan_flag};
    const DensityFwdArgs d{x, params_d, uw, uh, ud, lq_in_d, out_d, lq_out_d};
    const fs::CouplingArgs as2 = coupling_args(sp2), ad2 = coupling_args(dp2);
    if (sp2->K != sp->K || as2.rows != sp->rows || ad2.rows != dp->rows || sp->D > kCplMaxD || dp->D > kCplMaxD ||
        sp2->D != sp->D || dp2->D != dp->D)
        return hipErrorInvalidValue;
#define FS_PAIR_LAUNCH(KERNEL, ...)                                                                     \
    const fs::CouplingArgs as = coupling_args(sp), ad = coupling_args(dp);                              \
    if (sp->K != dp->K || as.rows < 0 || ad.rows < 0) return hipErrorInvalidValue;                     \
    const unsigned nb0 = (unsigned)((as.rows + kCplRows - 1) / kCplRows);                              \
    const unsigned nb = nb0 + (unsigned)((ad.rows + kCplRows - 1) / kCplRows);                         \
    if (nb == 0) return hipSuccess;                                                                     \
    const dim3 block(64 * kCplRows);                                                                    \
    switch (sp->K) {                                                                                    \
    case 5: hipLaunchKernelGGL((KERNEL<5>), dim3(nb), block, 0, st, __VA_ARGS__, nb0); break;           \
    case 8: hipLaunchKernelGGL((KERNEL<8>), dim3(nb), block, 0, st, __VA_ARGS__, nb0); break;           \
    case 15: hipLaunchKernelGGL((KERNEL<15>), dim3(nb), block, 0, st, __VA_ARGS__, nb0); break;         \
    case 32: hipLaunchKernelGGL((KERNEL<32>), dim3(nb), block, 0, st, __VA_ARGS__, nb0); break;         \
    default: return hipErrorInvalidValue;                                                               \
    }                                                                                                   \
    return hipGetLastError();
    if (coupling_waves() && sp->rows + dp->rows <= 0x7fffffff) {  // one row per two-wave workgroup
        const fs::CouplingArgs as = coupling_args(sp), ad = coupling_args(dp);
        if (sp->K != dp->K || as.rows < 0 || ad.rows < 0) return hipErrorInvalidValue;
        const unsigned nb0 = (unsigned)as.rows, nb = nb0 + (unsigned)ad.rows;
        if (nb == 0) return hipSuccess;
        switch (sp->K) {
        case 5: hipLaunchKernelGGL(coupling_pair_step2_kernel<5>, dim3(nb), dim3(128), 0, st, as, s, as2, s2, ad, d, ad2, t_d2, nb0); break;
        case 8: hipLaunchKernelGGL(coupling_pair_step2_kernel<8>, dim3(nb), dim3(128), 0, st, as, s, as2, s2, ad, d, ad2, t_d2, nb0); break;
        case 15: hipLaunchKernelGGL(coupling_pair_step2_kernel<15>, dim3(nb), dim3(128), 0, st, as, s, as2, s2, ad, d, ad2, t_d2, nb0); break;
        case 32: hipLaunchKernelGGL(coupling_pair_step2_kernel<32>, dim3(nb), dim3(128), 0, st, as, s, as2, s2, ad, d, ad2, t_d2, nb0); break;
        default: return hipErrorInvalidValue;
        }
        return hipGetLastError();
    }
    FS_PAIR_LAUNCH(coupling_pair_step_kernel, as, s, as2, s2, ad, d, ad2, t_d2)
#undef FS_PAIR_LAUNCH
}

hipError_t fs_coupling_features_fwd_impl(const fs_coupling *cp, const float *x, float *t, hipStream_t st) {
    const fs::CouplingArgs a = coupling_args(cp);
    if (a.rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(coupling_features_fwd_kernel, dim3((unsigned)((a.rows + kCplRows - 1) / kCplRows)), dim3(64 * kCplRows), 0, st, a, x, t);
    return hipGetLastError();
}

hipError_t fs_coupling_features_bwd_impl(const fs_coupling *cp, const float *x, const float *g_t, float *gx,
                                         const float *gx_add, hipStream_t st) {
    const fs::CouplingArgs a = coupling_args(cp);
    if (a.rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(coupling_features_bwd_kernel, dim3((unsigned)((a.rows + kCplRows - 1) / kCplRows)), dim3(64 * kCplRows), 0, st, a, x, g_t,
                       gx, gx_add);
    return hipGetLastError();
}
