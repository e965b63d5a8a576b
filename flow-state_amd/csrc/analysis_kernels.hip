// Analysis reductions of the Algorithm-1 driver on MI355X:
//   * classify_particles + the per-configuration part of calculate_well_statistics
//     (hybrid_NF_MCMC/utils.py:61-141): well A / B / outside per particle, the
//     all-in-A / all-in-B flag and np.mean(config[:, 0]) per configuration;
//   * the pair-distance histogram and the g(r) mean of calculate_pair_correlation
//     (utils.py:530-574).
// numpy's scalar promotion is reproduced: with a float32 array every Python float
// (centres, box, radius**2, 2*bound) is rounded to float32 first (NEP 50 weak
// scalars, comparisons included) and the arithmetic stays float32; with float64
// it is float64.  Sums follow numpy's pairwise order in the array's dtype.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "fs_internal.h"

#pragma clang fp contract(off)

namespace fs {

// numpy pairwise_sum (loops_utils.h) of load(0..n-1), accumulating in T: blocks of
// <= 128 use 8 partial sums (sequential below 8); larger blocks split at n2 = n/2
// rounded down to a multiple of 8 and add the halves.  The recursion runs on an
// explicit stack (depth <= log2(n/128) + 1).
template <typename T, typename Load>
__device__ T pairwise_leaf(Load load, int64_t off, int64_t n) {
    if (n < 8) {
        T res = T(0);
        for (int64_t i = 0; i < n; ++i) res += load(off + i);
        return res;
    }
    T r[8];
    for (int j = 0; j < 8; ++j) r[j] = load(off + j);
    int64_t i = 8;
    for (; i < n - (n % 8); i += 8)
        for (int j = 0; j < 8; ++j) r[j] += load(off + i + j);
    T res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += load(off + i);
    return res;
}

template <typename T, typename Load>
__device__ T pairwise_sum_dev(Load load, int64_t n) {
    struct Frame {
        int64_t off, n;
        T left;
        int stage;  // 0 new, 1 left half pending, 2 right half pending
    };
    auto half = [](int64_t k) { return k / 2 - (k / 2) % 8; };
    Frame st[48];
    int sp = 0;
    st[0] = {0, n, T(0), 0};
    while (true) {
        Frame &f = st[sp];
        if (f.n > 128) {
            f.stage = 1;
            st[sp + 1] = {f.off, half(f.n), T(0), 0};
            ++sp;
            continue;
        }
        T val = pairwise_leaf<T>(load, f.off, f.n);
        while (true) {  // hand the finished block to its parents
            if (sp == 0) return val;
            --sp;
            Frame &p = st[sp];
            if (p.stage == 1) {
                p.left = val;
                p.stage = 2;
                const int64_t n2 = half(p.n);
                st[sp + 1] = {p.off + n2, p.n - n2, T(0), 0};
                ++sp;
                break;
            }
            val = p.left + val;
        }
    }
}

// classify_particles' per-particle test (utils.py:104-141) in the array dtype T:
// box = halfbox*2 for both axes, centres (box/4, box/2) and (3box/4, box/2), radius
// r0*1.1, each a Python float rounded into T (numpy 2 weak scalars)
template <typename T>
struct WellTest {
    T bx, by, lcx, lcy, rcx, rcy, rad2;
    __device__ WellTest(double half_box, double r0) {
        const double box = half_box * 2.0, radius = r0 * 1.1;
        bx = (T)box;
        by = (T)box;
        lcx = (T)(box / 4.0);
        lcy = (T)(box / 2.0);
        rcx = (T)(3.0 * box / 4.0);
        rcy = (T)(box / 2.0);
        rad2 = (T)(radius * radius);  // radius ** 2 (Python float), compared in T
    }
    __device__ bool in_circle(T x, T y, T cx, T cy) const {
        T dx = x - cx, dy = y - cy;
        dx -= bx * (T)rint(dx / bx);
        dy -= by * (T)rint(dy / by);
        const T dx2 = dx * dx, dy2 = dy * dy;
        return (dx2 + dy2) <= rad2;
    }
    // 0 = 'A' (left), 1 = 'B' (right), 2 = 'Outside'
    __device__ int classify(T x, T y) const {
        if (in_circle(x, y, lcx, lcy)) return 0;
        return in_circle(x, y, rcx, rcy) ? 1 : 2;
    }
};

// one wave per configuration, lane loop over particles
template <typename T>
__global__ void __launch_bounds__(256) classify_kernel(const T *__restrict__ pos, int64_t M, int N, double half_box,
                                                       double r0, uint8_t *__restrict__ cls,
                                                       uint8_t *__restrict__ state, double *__restrict__ avg_x) {
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t m = (int64_t)blockIdx.x * 4 + wid;
    if (m >= M) return;
    const WellTest<T> w(half_box, r0);
    const T *q = pos + m * (int64_t)N * 2;
    bool allA = true, allB = true;
    for (int i = lane; i < N; i += 64) {
        const int k = w.classify(q[2 * i], q[2 * i + 1]);
        if (cls) cls[m * N + i] = (uint8_t)k;
        allA &= k == 0;
        allB &= k == 1;
    }
    allA = __all(allA);
    allB = __all(allB);
    if (lane == 0) {
        if (state) state[m] = allA ? 1 : (allB ? 2 : 0);
        if (avg_x) {  // np.mean(config[:, 0]) in the array dtype: pairwise sum / N
            const T s = pairwise_sum_dev<T>([&](int64_t i) { return q[2 * i]; }, N);
            avg_x[m] = (double)(s / (T)N);
        }
    }
}

// calculate_well_statistics' all-in-A / all-in-B counts (utils.py:73-86) for the
// batched engine's live chain states: state f64 [C][N][2] holding each chain's
// values, classified in that chain's reference dtype (float32 after an accepted big
// move, monte_carlo.py:296), one wave per chain.
__global__ void __launch_bounds__(256) well_stats_kernel(const double *__restrict__ pos,
                                                         const uint8_t *__restrict__ is_f32, int64_t C, int N,
                                                         double half_box, double r0,
                                                         long long *__restrict__ counts) {
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t c = (int64_t)blockIdx.x * 4 + wid;
    if (c >= C) return;
    const double *q = pos + c * (int64_t)N * 2;
    bool allA = true, allB = true;
    if (is_f32 && is_f32[c]) {
        const WellTest<float> w(half_box, r0);
        for (int i = lane; i < N; i += 64) {
            const int k = w.classify((float)q[2 * i], (float)q[2 * i + 1]);
            allA &= k == 0;
            allB &= k == 1;
        }
    } else {
        const WellTest<double> w(half_box, r0);
        for (int i = lane; i < N; i += 64) {
            const int k = w.classify(q[2 * i], q[2 * i + 1]);
            allA &= k == 0;
            allB &= k == 1;
        }
    }
    allA = __all(allA);
    allB = __all(allB);
    if (lane == 0) {
        counts[3 * c] += allA;
        counts[3 * c + 1] += (!allA && allB);
        counts[3 * c + 2] += 1;
    }
}

// pair-distance histogram of one configuration per wave (utils.py:546-556): all
// ordered pairs i != j, distance != 0, bins [e_k, e_k+1) with the last bin closed
template <typename T>
__global__ void __launch_bounds__(256) pair_hist_kernel(const T *__restrict__ pos, int64_t M, int N, double bound,
                                                        const double *__restrict__ edges, int nb,
                                                        int32_t *__restrict__ counts) {
    __shared__ int32_t h[4][128];
    __shared__ T sx[4][256], sy[4][256];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int64_t m = (int64_t)blockIdx.x * 4 + wid;
    if (m >= M) return;
    for (int k = lane; k < nb; k += 64) h[wid][k] = 0;
    const T *q = pos + m * (int64_t)N * 2;
    for (int i = lane; i < N; i += 64) {
        sx[wid][i] = q[2 * i];
        sy[wid][i] = q[2 * i + 1];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const T tb = (T)(2.0 * bound);
    const double e0 = edges[0], elast = edges[nb];
    for (int i = lane; i < N; i += 64) {
        const T xi = sx[wid][i], yi = sy[wid][i];
        for (int j = 0; j < N; ++j) {
            T dx = xi - sx[wid][j], dy = yi - sy[wid][j];
            dx = dx - tb * (T)rint(dx / tb);
            dy = dy - tb * (T)rint(dy / tb);
            const T s0 = dx * dx, s1 = dy * dy;
            const T s = s0 + s1;
            const double d = (double)(T)sqrt(s);
            if (d == 0.0 || d < e0 || d > elast) continue;
            // searchsorted: k with edges[k] <= d < edges[k+1], last bin right-inclusive
            int lo = 0, hi = nb;
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (edges[mid] <= d) lo = mid;
                else hi = mid;
            }
            atomicAdd(&h[wid][lo], 1);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    for (int k = lane; k < nb; k += 64) counts[m * nb + k] = h[wid][k];
}

// g(r) = mean over configurations of counts / denom (utils.py:558-566): the
// per-configuration ratio in float64, then pandas' mean = pairwise sum / M
__global__ void rdf_mean_kernel(const int32_t *__restrict__ counts, int64_t M, int nb, const double *__restrict__ denom,
                                double *__restrict__ g) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= nb) return;
    const double dk = denom[k];
    const double s =
        pairwise_sum_dev<double>([&](int64_t m) { return (double)counts[m * nb + k] / dk; }, M);
    g[k] = s / (double)M;
}

}  // namespace fs

using namespace fs;

hipError_t fs_classify_wells_impl(const void *pos, int f32, int64_t M, int N, double half_box, double r0,
                                  uint8_t *cls, uint8_t *state, double *avg_x, hipStream_t st) {
    if (M <= 0) return hipSuccess;
    const dim3 grid((unsigned)((M + 3) / 4));
    if (f32)
        hipLaunchKernelGGL(classify_kernel<float>, grid, dim3(256), 0, st, (const float *)pos, M, N, half_box, r0, cls,
                           state, avg_x);
    else
        hipLaunchKernelGGL(classify_kernel<double>, grid, dim3(256), 0, st, (const double *)pos, M, N, half_box, r0,
                           cls, state, avg_x);
    return hipGetLastError();
}

hipError_t fs_well_stats_impl(const double *pos, const uint8_t *is_f32, int64_t C, int N, double half_box, double r0,
                              int64_t *counts, hipStream_t st) {
    if (C <= 0) return hipSuccess;
    hipLaunchKernelGGL(well_stats_kernel, dim3((unsigned)((C + 3) / 4)), dim3(256), 0, st, pos, is_f32, C, N, half_box,
                       r0, (long long *)counts);
    return hipGetLastError();
}

hipError_t fs_pair_hist_impl(const void *pos, int f32, int64_t M, int N, double bound, const double *edges, int nb,
                             int32_t *counts, hipStream_t st) {
    if (M <= 0) return hipSuccess;
    const dim3 grid((unsigned)((M + 3) / 4));
    if (f32)
        hipLaunchKernelGGL(pair_hist_kernel<float>, grid, dim3(256), 0, st, (const float *)pos, M, N, bound, edges, nb,
                           counts);
    else
        hipLaunchKernelGGL(pair_hist_kernel<double>, grid, dim3(256), 0, st, (const double *)pos, M, N, bound, edges,
                           nb, counts);
    return hipGetLastError();
}

hipError_t fs_rdf_mean_impl(const int32_t *counts, int64_t M, int nb, const double *denom, double *g, hipStream_t st) {
    if (nb <= 0) return hipSuccess;
    hipLaunchKernelGGL(rdf_mean_kernel, dim3((unsigned)((nb + 63) / 64)), dim3(64), 0, st, counts, M, nb, denom, g);
    return hipGetLastError();
}
