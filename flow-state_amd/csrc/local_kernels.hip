// Batched local Metropolis moves on MI355X: MonteCarlo.particle_displacement
// (monte_carlo.py:146-189) + metropolis_acceptance_particle_move (:191-223),
// adjust_displacement (:375-403) and the sample() snapshots (:416-444) that the
// Algorithm-1 driver interleaves with them (main_algorithm_1.py:203-210, 245-252,
// 384-390).
//
// Layout: a group of LPC lanes owns one chain (LPC = 64/32/16/8 for N <= 64/32/16/8);
// lane j holds particle j's coordinates in registers for the whole launch, so a
// launch of n moves touches HBM only to load and store the state.  Every lane of a
// group runs the chain's PCG64 redundantly (group-uniform values, no broadcast).
// Per move each lane evaluates its two pair terms (particle p before / after the
// displacement against particle j); the per-particle sums use numpy's pairwise
// order over the np.delete-compacted index (loops_utils.h): 8 partial sums with
// 8-lane shuffles for the tree, then the tail — so E, W and the accept decisions
// track the reference to the ulp.  The double-well terms are spread over lanes
// 0..3 (before/after x well 0/1).  Chains are independent: no grid-level sync,
// each group exits after its n moves.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "fs_internal.h"
#include "physics_device.h"

#pragma clang fp contract(off)

namespace fs {

struct LocalArgs {
    fs_phys p;
    int64_t C;
    int N;
    double *state;
    const uint8_t *is_f32;
    double *E, *W;
    uint64_t *pcg, *pcg_buf;
    double *max_disp;
    int64_t *attempts, *accepted, *prev;
    int64_t n_moves, step0;
    int adjust_every;
    double target;
    int sample_every;
    int64_t n_samp;
    double *samples_xy, *samples_ew;
    uint8_t *accept_log;
    unsigned long long *n_accept;
};

constexpr int kLocalWaves = 4;

// adjust_displacement (monte_carlo.py:375-403) on one chain's registers
__device__ __forceinline__ void adjust_md(double &md, int64_t att, int64_t acc, int64_t &prev_att, int64_t &prev_acc,
                                          double target) {
    if (att > prev_att) {
        const int64_t da = att - prev_att, dc = acc - prev_acc;
        const double frac = da > 0 ? (double)dc / (double)da : 0.0;  // Python int / int
        const double factor = frac / target;
        double nm = md * factor;
        const double ratio = nm / md;
        if (ratio > 1.5) nm = md * 1.5;
        else if (ratio < 0.5) nm = md * 0.5;
        md = nm;
        prev_att = att;
        prev_acc = acc;
    }
}

__global__ void adjust_kernel(int64_t C, double *max_disp, const int64_t *attempts, const int64_t *accepted,
                              int64_t *prev, double target) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    double md = max_disp[c];
    int64_t pa = prev[2 * c], pc = prev[2 * c + 1];
    adjust_md(md, attempts[c], accepted[c], pa, pc, target);
    max_disp[c] = md;
    prev[2 * c] = pa;
    prev[2 * c + 1] = pc;
}

// group broadcast of lane `src` (group-relative); a whole-wave group uses v_readlane
// with a wave-uniform index, smaller groups a ds_bpermute shuffle
template <int LPC>
__device__ __forceinline__ double bcast(double v, int src) {
    if constexpr (LPC == 64) {
        const uint64_t u = __double_as_longlong(v);
        const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)u, src);
        const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), src);
        return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
    } else {
        return __shfl(v, src, LPC);
    }
}

template <int LPC>
__device__ __forceinline__ uint64_t uniform_u64(uint64_t v) {
    if constexpr (LPC == 64) {  // one chain per wave: keep the chain's scalars in SGPRs
        const uint32_t lo = __builtin_amdgcn_readfirstlane((int)(uint32_t)v);
        const uint32_t hi = __builtin_amdgcn_readfirstlane((int)(uint32_t)(v >> 32));
        return ((uint64_t)hi << 32) | lo;
    } else {
        return v;
    }
}

// select element q (group-uniform, runtime) of a small register array
template <int PPL>
__device__ __forceinline__ double pick(const double (&v)[PPL], int q) {
    double r = v[0];
#pragma unroll
    for (int i = 1; i < PPL; ++i)
        if (q == i) r = v[i];
    return r;
}

// LPC lanes per chain, PPL particles per lane (particle j = gl + LPC * q): LPC*PPL >= N.
// Several chains per wave amortise the per-move work that does not scale with N
// (the PCG64 stream, broadcasts, the reduction tree, the double well, the accept).
template <int LPC, int PPL>
__global__ void __launch_bounds__(64 * kLocalWaves, LPC == 64 ? 4 : 2) local_moves_kernel(LocalArgs a) {
    constexpr int G = 64 / LPC;          // chains per wave
    constexpr int SLOTS = LPC * PPL;     // LDS slots per chain and array
    __shared__ double lds[kLocalWaves][4][G * SLOTS];
    __shared__ double res[kLocalWaves][G][4];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = lane / LPC, gl = lane % LPC;
    const int sb = g * SLOTS;            // this chain's slot base
    const int64_t c = ((int64_t)blockIdx.x * kLocalWaves + wid) * G + g;
    if (c >= a.C) return;  // whole groups leave; only group-internal shuffles below
    const int N = a.N;
    const fs_phys &P = a.p;
    const bool f32 = a.is_f32 && a.is_f32[c];
    double xj[PPL], yj[PPL];
#pragma unroll
    for (int q = 0; q < PPL; ++q) {
        const int j = gl + LPC * q;
        xj[q] = j < N ? a.state[(c * N + j) * 2] : 0.0;
        yj[q] = j < N ? a.state[(c * N + j) * 2 + 1] : 0.0;
    }
    Pcg64 rng;
#pragma unroll
    for (int i = 0; i < 4; ++i) rng.s[i] = uniform_u64<LPC>(a.pcg[4 * c + i]);
    rng.has = (uint32_t)uniform_u64<LPC>(a.pcg_buf[2 * c]);
    rng.buf = (uint32_t)uniform_u64<LPC>(a.pcg_buf[2 * c + 1]);
    double E = a.E[c], W = a.W ? a.W[c] : 0.0, md = a.max_disp[c];
    int64_t att = a.attempts[c], acc_n = a.accepted[c];
    int64_t prev_att = a.prev ? a.prev[2 * c] : 0, prev_acc = a.prev ? a.prev[2 * c + 1] : 0;
    const double sr6c = pow6(1.0 / P.r_cut);
    const double e_cut = 4.0 * (sr6c * sr6c - sr6c);
    const double iLx = 1.0 / P.Lx, iLy = 1.0 / P.Ly;
    const int n = N - 1;
    const int nfull = n - (n % 8);
    const uint64_t gmask = (LPC == 64) ? ~0ull : (((1ull << LPC) - 1ull) << (g * LPC));
    // double-well role of this lane: 0/1 = old position well 0/1, 2/3 = new position
    const int dw_well = gl & 1;
    const bool dw_lane = gl < 4 && dw_well < P.num_wells;
    const double dw_V0 = P.V0[dw_well];
    int64_t samp = 0;
    unsigned long long n_acc_local = 0;

    for (int64_t t = 0; t < a.n_moves; ++t) {
        const int64_t step = a.step0 + t + 1;
        att += 1;
        const int p = (int)pcg64_integers(rng, (uint32_t)N);
        const int pq = p / LPC, pl = p % LPC;
        const double ox = bcast<LPC>(pick<PPL>(xj, pq), pl), oy = bcast<LPC>(pick<PPL>(yj, pq), pl);
        const double d0 = (pcg64_double(rng) - 0.5) * md;
        const double d1 = (pcg64_double(rng) - 0.5) * md;
        double nx, ny;
        if (f32) {  // float32 row += float64 array, then float32 % np.float64 stored back
            nx = (double)(float)np_remainder((double)(float)(ox + d0), P.Lx);
            ny = (double)(float)np_remainder((double)(float)(oy + d1), P.Ly);
        } else {
            nx = np_remainder(ox + d0, P.Lx);
            ny = np_remainder(oy + d1, P.Ly);
        }
        // pair terms of particle p against this lane's particles (np.delete order: j - (j > p))
        bool ho = false, hn = false;
#pragma unroll
        for (int q = 0; q < PPL; ++q) {
            const int j = gl + LPC * q;
            if (j < N && j != p) {
                double ro, rn;
                if (f32) {
                    const float fx = (float)xj[q], fy = (float)yj[q];
                    ro = dist_f32((float)ox, (float)oy, fx, fy, P.Lx, P.Ly, iLx, iLy);
                    rn = dist_f32((float)nx, (float)ny, fx, fy, P.Lx, P.Ly, iLx, iLy);
                } else {
                    ro = dist_f64(ox, oy, xj[q], yj[q], P.Lx, P.Ly, iLx, iLy);
                    rn = dist_f64(nx, ny, xj[q], yj[q], P.Lx, P.Ly, iLx, iLy);
                }
                ho |= ro < P.r_core;
                hn |= rn < P.r_core;
                double eo, wo, en, wn;
                lj_pair(ro, P.r_cut, e_cut, eo, wo);
                lj_pair(rn, P.r_cut, e_cut, en, wn);
                const int tt = sb + j - (j > p ? 1 : 0);
                lds[wid][0][tt] = eo;
                lds[wid][1][tt] = wo;
                lds[wid][2][tt] = en;
                lds[wid][3][tt] = wn;
            }
        }
        const bool hit_old = (__ballot(ho) & gmask) != 0;
        const bool hit_new = (__ballot(hn) & gmask) != 0;
        double dw = 0.0;
        if (dw_lane)
            dw = dw_term(gl < 2 ? ox : nx, gl < 2 ? oy : ny, dw_well, P.Lx, P.Ly, dw_V0, P.r0, P.k, iLx, iLy);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // numpy pairwise sums of the four compacted rows: eno, viro, enn, virn
        double sums[4];
        if (n < 8) {
            double r = 0.0;
            if (gl < 4)
                for (int k = 0; k < n; ++k) r += lds[wid][gl][sb + k];
#pragma unroll
            for (int q = 0; q < 4; ++q) sums[q] = bcast<LPC>(r, q);
        } else if constexpr (LPC == 64) {
            // lanes 8*arr + k: partial sum k of array arr, tree by xor-shuffles, tail on lane 8*arr
            double r = 0.0;
            if (gl < 32) {
                const int arr = gl >> 3, k = gl & 7;
                r = lds[wid][arr][k];
                for (int b = 8; b < nfull; b += 8) r += lds[wid][arr][b + k];
            }
            r += __shfl_xor(r, 1, 64);
            r += __shfl_xor(r, 2, 64);
            r += __shfl_xor(r, 4, 64);
            if (gl < 32 && (gl & 7) == 0)
                for (int i = nfull; i < n; ++i) r += lds[wid][gl >> 3][i];
#pragma unroll
            for (int q = 0; q < 4; ++q) sums[q] = bcast<LPC>(r, 8 * q);
        } else {
            for (int ak = gl; ak < 32; ak += LPC) {  // LPC >= 8
                const int arr = ak >> 3, k = ak & 7;
                double r = lds[wid][arr][sb + k];
                for (int b = 8; b < nfull; b += 8) r += lds[wid][arr][sb + b + k];
                r += __shfl_xor(r, 1, LPC);
                r += __shfl_xor(r, 2, LPC);
                r += __shfl_xor(r, 4, LPC);
                if (k == 0) {
                    for (int i = nfull; i < n; ++i) r += lds[wid][arr][sb + i];
                    res[wid][g][arr] = r;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int q = 0; q < 4; ++q) sums[q] = res[wid][g][q];
        }
        double eno = sums[0], viro = sums[1], enn = sums[2], virn = sums[3];
        if (P.num_wells > 0) {  // V = 0; V += term(well 0); V += term(well 1)  (potential.py:96-112)
            double vo = 0.0 + bcast<LPC>(dw, 0), vn = 0.0 + bcast<LPC>(dw, 2);
            if (P.num_wells > 1) {
                vo += bcast<LPC>(dw, 1);
                vn += bcast<LPC>(dw, 3);
            }
            eno += vo;
            enn += vn;
        }
        if (hit_old) eno = viro = INFINITY;  // energy_calculator.py:69-73
        if (hit_new) enn = virn = INFINITY;
        bool accept;
        if (enn <= eno) accept = true;
        else if (isinf(enn)) accept = false;
        else accept = pcg64_double(rng) < exp(-P.beta * (enn - eno));
        if (accept) {
            acc_n += 1;
            E += enn - eno;
            W += virn - viro;
            n_acc_local += 1;
            if (gl == pl) {
#pragma unroll
                for (int q = 0; q < PPL; ++q)
                    if (q == pq) {
                        xj[q] = nx;
                        yj[q] = ny;
                    }
            }
        }
        if (a.accept_log && gl == 0) a.accept_log[c * a.n_moves + t] = accept ? 1 : 0;
        if (a.adjust_every > 0 && step % a.adjust_every == 0) adjust_md(md, att, acc_n, prev_att, prev_acc, a.target);
        if (a.sample_every > 0 && step % a.sample_every == 0 && samp < a.n_samp) {
            if (a.samples_xy) {
#pragma unroll
                for (int q = 0; q < PPL; ++q) {
                    const int j = gl + LPC * q;
                    if (j < N) {
                        double *o = a.samples_xy + ((c * a.n_samp + samp) * N + j) * 2;
                        o[0] = xj[q];
                        o[1] = yj[q];
                    }
                }
            }
            if (a.samples_ew && gl == 0) {
                a.samples_ew[(c * a.n_samp + samp) * 2] = E;
                a.samples_ew[(c * a.n_samp + samp) * 2 + 1] = W;
            }
            ++samp;
        }
    }
#pragma unroll
    for (int q = 0; q < PPL; ++q) {
        const int j = gl + LPC * q;
        if (j < N) {
            a.state[(c * N + j) * 2] = xj[q];
            a.state[(c * N + j) * 2 + 1] = yj[q];
        }
    }
    if (gl == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i) a.pcg[4 * c + i] = rng.s[i];
        a.pcg_buf[2 * c] = rng.has;
        a.pcg_buf[2 * c + 1] = rng.buf;
        a.E[c] = E;
        if (a.W) a.W[c] = W;
        a.max_disp[c] = md;
        a.attempts[c] = att;
        a.accepted[c] = acc_n;
        if (a.prev) {
            a.prev[2 * c] = prev_att;
            a.prev[2 * c + 1] = prev_acc;
        }
        if (a.n_accept && n_acc_local) atomicAdd(a.n_accept, n_acc_local);
    }
}

}  // namespace fs

using namespace fs;

int64_t fs_local_samples_per_chain(int64_t step0, int64_t n_moves, int32_t sample_every) {
    if (sample_every <= 0 || n_moves <= 0) return 0;
    return (step0 + n_moves) / sample_every - step0 / sample_every;
}

hipError_t fs_local_moves_impl(const fs_phys *p, int64_t C, int N, double *state, const uint8_t *is_f32,
                               double *E, double *W, uint64_t *pcg, uint64_t *pcg_buf, double *max_disp,
                               int64_t *attempts, int64_t *accepted, int64_t *prev, int64_t n_moves, int64_t step0,
                               int adjust_every, double target, int sample_every, double *samples_xy,
                               double *samples_ew, uint8_t *accept_log, unsigned long long *n_accept,
                               hipStream_t st) {
    if (C <= 0 || n_moves <= 0) return hipSuccess;
    LocalArgs a{*p,       C,         N,        state,      is_f32,     E,          W,
                pcg,      pcg_buf,   max_disp, attempts,   accepted,   prev,       n_moves,
                step0,    adjust_every, target, sample_every, fs_local_samples_per_chain(step0, n_moves, sample_every),
                samples_xy, samples_ew, accept_log, n_accept};
    // lanes per chain x particles per lane (FS_LOCAL_LAYOUT=LPCxPPL overrides, for A/B runs)
    // measured at 65536 chains x 1000 moves: 8 lanes per chain is fastest at every N
    // (N=64: 1.90 G moves/s with 8x8 vs 1.11 G with 64x1; N=32: 2.68 G; N=16: 3.50 G)
    int lpc = 8;
    int ppl = N > 32 ? 8 : N > 16 ? 4 : N > 8 ? 2 : 1;
    if (const char *e = getenv("FS_LOCAL_LAYOUT")) {
        int l = 0, q = 0;
        if (sscanf(e, "%dx%d", &l, &q) == 2 && l * q >= N) {
            lpc = l;
            ppl = q;
        }
    }
    const int64_t chains_per_block = (int64_t)kLocalWaves * (64 / lpc);
    const dim3 grid((unsigned)((C + chains_per_block - 1) / chains_per_block)), block(64 * kLocalWaves);
#define FS_LCASE(L, Q)                                                                \
    if (lpc == L && ppl == Q) {                                                       \
        hipLaunchKernelGGL((local_moves_kernel<L, Q>), grid, block, 0, st, a);        \
        return hipGetLastError();                                                     \
    }
    FS_LCASE(8, 1) FS_LCASE(8, 2) FS_LCASE(8, 4) FS_LCASE(8, 8) FS_LCASE(64, 1) FS_LCASE(16, 4)
#undef FS_LCASE
    return hipErrorInvalidValue;
}

hipError_t fs_adjust_displacement_impl(int64_t C, double *max_disp, const int64_t *attempts, const int64_t *accepted,
                                       int64_t *prev, double target, hipStream_t st) {
    if (C <= 0) return hipSuccess;
    hipLaunchKernelGGL(adjust_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, st, C, max_disp, attempts,
                       accepted, prev, target);
    return hipGetLastError();
}
