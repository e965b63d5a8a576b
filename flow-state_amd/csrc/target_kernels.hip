// Algorithm 2's target energy: DoubleWellLJ._energy (NF/normflows/Energy/SimpleLJ.py:15-39,
// 63-128), the score reverse_kld evaluates on flow samples (core.py:105-142), and its
// gradient with respect to the samples (what reverse_kld's backward needs when
// ALPHA != 1, main_algorithm_2.py:316-318).
//
// One wave per sample row; lane p owns particle p (p += 64 beyond 64 particles).  The
// wrapped coordinates d = x - 2B rint(x / 2B) are staged in LDS; each lane walks every
// other particle, so its gradient needs no atomics: the energy counts the pairs j > p
// (plus the pair with the extra particle at the origin that SimpleLJ prepends), the
// gradient all of them.  The arithmetic follows the reference's float32 torch ops one by
// one (scalars rounded to float32 as torch does, correctly rounded sqrt, the pow terms
// rounded once from double); the sums over pairs and particles accumulate in double and
// round once (torch's float32 reduction order is not reproducible anyway).
//
// Kept from the reference: no minimum image between particles (only each particle is
// wrapped into the box), the linear core below r = 0.82 (inclusive), the LJ part divided
// by the temperature and the double well not, the double well on the raw (unwrapped)
// coordinates, and torch's gradient quirks: a pair with (1/r)^11 overflowing float32
// (coinciding particles included) makes both particles' gradients NaN (the unselected
// pow branch of torch.where multiplies its zero gradient by inf), and so does a
// particle exactly at a well centre (sqrt's backward at 0).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "fs_internal.h"

#pragma clang fp contract(off)

namespace fs {

struct TargetArgs {
    float two_b;    // fl32(2 * bound): x / (bound * 2) and 2 * bound * round(...)
    float inv_t;    // 1 / temperature (LJ gradient)
    float temp;     // temperature: the LJ energy is divided by it (SimpleLJ.py:39)
    float cx[2];    // well centres fl32(-bound / 2), fl32(bound / 2) at y = 0
    float v0[2];
    float r0, k;
    int num_wells;
    int want_grad;
};

__device__ __forceinline__ float sqrt_rn_f(float s) { return (float)__dsqrt_rn((double)s); }

__global__ void __launch_bounds__(256) target_energy_kernel(const float *__restrict__ x, int64_t B, int N,
                                                            TargetArgs a, float *__restrict__ E,
                                                            float *__restrict__ gx) {
    extern __shared__ float sm[];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t b = (int64_t)blockIdx.x * 4 + wid;
    const bool valid = b < B;
    float *sx = sm + wid * 2 * N;
    float *sy = sx + N;
    const float *xr = x + (valid ? b : 0) * 2 * N;
    if (valid)
        for (int p = lane; p < N; p += 64) {
            const float px = xr[2 * p], py = xr[2 * p + 1];
            sx[p] = px - a.two_b * rintf(px / a.two_b);
            sy[p] = py - a.two_b * rintf(py / a.two_b);
        }
    __syncthreads();
    if (!valid) return;
    const float bk = 0.82f;
    double e_lj = 0.0, e_dw = 0.0;
    for (int p = lane; p < N; p += 64) {
        const float xi = sx[p], yi = sy[p];
        double gxi = 0.0, gyi = 0.0;
        // pairs with the origin particle (j = -1) and with every other particle
        for (int j = -1; j < N; ++j) {
            if (j == p) continue;
            const float xj = j < 0 ? 0.0f : sx[j], yj = j < 0 ? 0.0f : sy[j];
            const float dx = xi - xj, dy = yi - yj;
            const float s = dx * dx + dy * dy;
            const float r = sqrt_rn_f(s);
            float e;
            double fp;  // dE/dr
            if (r <= bk) {
                e = -80.0f * (r - bk) + 30.0f;
                fp = -80.0;
            } else {
                const float ir = 1.0f / r;
                const double t = ir, t2 = t * t, t3 = t2 * t, t6 = t3 * t3;
                e = 4.0f * ((float)(t6 * t6) - (float)t6);
                fp = 4.0 * (-12.0 * t6 * t6 * t + 6.0 * t6 * t);
            }
            if (j < 0 || j > p) e_lj += (double)e;
            if (a.want_grad) {
                // torch.where's unselected pow branch: its zero gradient times (1/r)^11 is
                // NaN once that overflows float32 (r = 0 included, 1/r = inf)
                const float ir = 1.0f / r;
                const double t = ir, t2 = t * t, t5 = t2 * t2 * t;
                if (isinf((float)(t5 * t5 * t))) {
                    gxi = gyi = NAN;
                } else {
                    const double f = fp / (double)r;
                    gxi += f * (double)dx;
                    gyi += f * (double)dy;
                }
            }
        }
        // double well on the raw coordinates (SimpleLJ.py:63-115)
        const float px = xr[2 * p], py = xr[2 * p + 1];
        const float L = a.two_b;
        float vp = 0.0f;
        double gdx = 0.0, gdy = 0.0;
        for (int w = 0; w < a.num_wells; ++w) {
            float dx = px - a.cx[w], dy = py - 0.0f;
            dx = dx - L * rintf(dx / L);
            dy = dy - L * rintf(dy / L);
            const float r = sqrt_rn_f(dx * dx + dy * dy);
            const float th = tanhf(a.k * (r - a.r0));
            const float tr = 0.5f * (1.0f + th);
            vp = vp + a.v0[w] * (1.0f - tr);
            if (a.want_grad && r == 0.0f) {
                gdx = gdy = NAN;  // sqrt's backward at 0 (inf) times d(dx^2)/ddx = 0
            } else if (a.want_grad) {
                const double dvdr = (double)a.v0[w] * -0.5 * (double)a.k * (1.0 - (double)th * (double)th);
                gdx += dvdr * (double)dx / (double)r;
                gdy += dvdr * (double)dy / (double)r;
            }
        }
        e_dw += (double)vp;
        if (a.want_grad) {
            float *g = gx + b * 2 * N;
            g[2 * p] = (float)(gxi * (double)a.inv_t + gdx);
            g[2 * p + 1] = (float)(gyi * (double)a.inv_t + gdy);
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        e_lj += __shfl_xor(e_lj, off);
        e_dw += __shfl_xor(e_dw, off);
    }
    if (lane == 0) E[b] = (float)e_lj / a.temp + (float)e_dw;
}

// The energy alone (reverse_kld's score in the training step, where nothing needs dE/dx):
// one workgroup per row, the N + 1 points (the origin first) staged in LDS and the
// (N + 1) N / 2 unordered pairs spread over all 256 threads as (i, i + d mod (N + 1)),
// d <= (N + 1) / 2, instead of one wave walking every ordered pair.  Each pair's energy is
// the same float32 arithmetic as above; only the order of the double sums differs.
__global__ void __launch_bounds__(256) target_energy_only_kernel(const float *__restrict__ x, int N, TargetArgs a,
                                                                 float *__restrict__ E) {
    extern __shared__ float sm[];
    __shared__ double red[2][256];
    const int t = threadIdx.x;
    const int64_t b = blockIdx.x;
    const int M = N + 1;
    float *sx = sm, *sy = sm + M;
    const float *xr = x + b * 2 * N;
    for (int p = t; p < M; p += 256) {
        if (p == 0) {
            sx[0] = 0.0f;
            sy[0] = 0.0f;
        } else {
            const float px = xr[2 * (p - 1)], py = xr[2 * (p - 1) + 1];
            sx[p] = px - a.two_b * rintf(px / a.two_b);
            sy[p] = py - a.two_b * rintf(py / a.two_b);
        }
    }
    __syncthreads();
    const float bk = 0.82f;
    const int D = M / 2;
    const bool even = (M & 1) == 0;
    double e_lj = 0.0, e_dw = 0.0;
    for (int q = t; q < M * D; q += 256) {
        const int i = q / D, d = q - i * D + 1;
        if (even && d == D && i >= D) continue;  // the antipodal pairs once
        const int j = i + d < M ? i + d : i + d - M;
        const float dx = sx[i] - sx[j], dy = sy[i] - sy[j];
        const float r = sqrt_rn_f(dx * dx + dy * dy);
        float e;
        if (r <= bk) {
            e = -80.0f * (r - bk) + 30.0f;
        } else {
            const float ir = 1.0f / r;
            const double u = ir, u2 = u * u, u3 = u2 * u, u6 = u3 * u3;
            e = 4.0f * ((float)(u6 * u6) - (float)u6);
        }
        e_lj += (double)e;
    }
    for (int p = t; p < N; p += 256) {
        const float px = xr[2 * p], py = xr[2 * p + 1];
        const float L = a.two_b;
        float vp = 0.0f;
        for (int w = 0; w < a.num_wells; ++w) {
            float dx = px - a.cx[w], dy = py - 0.0f;
            dx = dx - L * rintf(dx / L);
            dy = dy - L * rintf(dy / L);
            const float r = sqrt_rn_f(dx * dx + dy * dy);
            const float th = tanhf(a.k * (r - a.r0));
            const float tr = 0.5f * (1.0f + th);
            vp = vp + a.v0[w] * (1.0f - tr);
        }
        e_dw += (double)vp;
    }
    red[0][t] = e_lj;
    red[1][t] = e_dw;
    __syncthreads();
#pragma unroll
    for (int w = 128; w > 0; w >>= 1) {
        if (t < w) {
            red[0][t] = red[0][t] + red[0][t + w];
            red[1][t] = red[1][t] + red[1][t + w];
        }
        __syncthreads();
    }
    if (t == 0) E[b] = (float)red[0][0] / a.temp + (float)red[1][0];
}

}  // namespace fs

hipError_t fs_target_energy_impl(const float *x, int64_t B, int N, double bound, double temperature, int num_wells,
                                 double v0a, double v0b, double r0, double k, float *E, float *gx, hipStream_t st) {
    if (B <= 0) return hipSuccess;
    fs::TargetArgs a;
    a.two_b = (float)(2.0 * bound);
    a.inv_t = (float)(1.0 / temperature);
    a.temp = (float)temperature;
    a.cx[0] = (float)(-bound / 2.0);
    a.cx[1] = (float)(bound / 2.0);
    a.v0[0] = (float)v0a;
    a.v0[1] = (float)v0b;
    a.r0 = (float)r0;
    a.k = (float)k;
    a.num_wells = num_wells;
    a.want_grad = gx != nullptr;
    if (!gx) {
        const size_t lds1 = (size_t)2 * (N + 1) * sizeof(float);
        hipLaunchKernelGGL(fs::target_energy_only_kernel, dim3((unsigned)B), dim3(256), lds1, st, x, N, a, E);
        return hipGetLastError();
    }
    const size_t lds = (size_t)4 * 2 * N * sizeof(float);
    hipLaunchKernelGGL(fs::target_energy_kernel, dim3((unsigned)((B + 3) / 4)), dim3(256), lds, st, x, B, N, a, E,
                       gx);
    return hipGetLastError();
}
