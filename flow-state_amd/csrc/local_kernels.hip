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

#include <map>
#include <mutex>
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
    PairThresh T;  // squared-distance / min-image thresholds (physics_device.h)
    const uint8_t *gate;  // nullable: the launch does nothing when *gate == 0
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
    if constexpr (LPC == 1) {
        return v;
    } else if constexpr (LPC == 64) {
        const uint64_t u = __double_as_longlong(v);
        const uint32_t lo = __builtin_amdgcn_readlane((int)(uint32_t)u, src);
        const uint32_t hi = __builtin_amdgcn_readlane((int)(uint32_t)(u >> 32), src);
        return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
    } else {
        return __shfl(v, src, LPC);
    }
}

// Within-group exchanges with a compile-time pattern: groups of 2 or 4 lanes sit inside one
// DPP quad, so quad_perm moves them through the VALU (a few cycles) instead of an LDS-path
// ds_bpermute round trip; other group sizes fall back to the shuffles.
template <int CTRL>
__device__ __forceinline__ uint64_t dpp_u64(uint64_t v) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)v, CTRL, 0xF, 0xF, false);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)(uint32_t)(v >> 32), CTRL, 0xF, 0xF, false);
    return ((uint64_t)hi << 32) | lo;
}

// lane SRC of the group
template <int LPC, int SRC>
__device__ __forceinline__ double bcast_c(double v) {
    if constexpr (LPC == 1) {
        return v;
    } else if constexpr (LPC == 2 || LPC == 4) {  // quad_perm [SRC x4] / [SRC, SRC, 2+SRC, 2+SRC]
        constexpr int ctrl = LPC == 4 ? SRC * 0x55 : (SRC == 0 ? 0xA0 : 0xF5);
        return __longlong_as_double((long long)dpp_u64<ctrl>((uint64_t)__double_as_longlong(v)));
    } else {
        return bcast<LPC>(v, SRC);
    }
}

// lane (lane ^ O) of the group
template <int LPC, int O>
__device__ __forceinline__ uint64_t xor_c(uint64_t v) {
    if constexpr (LPC == 2 || LPC == 4) {  // quad_perm [1,0,3,2] / [2,3,0,1]
        return dpp_u64<O == 1 ? 0xB1 : 0x4E>(v);
    } else {
        return __shfl_xor(v, O, LPC);
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
// LPC = 1 / 2 (few particles, few chains: the reference's N = 3 regime) keep a chain in
// one or two lanes, each lane taking RPL of the four sum rows and double-well roles, so a
// move has no or one shuffle level on its dependent path; the sums are the same
// additions in the same order, so every layout gives the same bits.
// position of the k-th set bit of m (k < popcount(m))
__device__ __forceinline__ int nth_set_bit(uint64_t m, int k) {
    for (int i = 0; i < k; ++i) m &= m - 1;
    return __builtin_ctzll(m);
}

// SORT (small launches, r06): twice the waves per workgroup, the workgroup's float64-state
// chains packed into its first waves and its float32-state chains from the next wave
// boundary on, so no wave runs both dtypes' branches (a chain's state turns float32 after an
// accepted big move, monte_carlo.py:289-292; a wave holding both ran each move's position and
// distance code twice).  Each chain still runs the same code on its own lanes: the same bits.
template <int LPC, int PPL, bool SORT = false>
__global__ void __launch_bounds__(64 * kLocalWaves * (SORT ? 2 : 1), LPC == 64 ? 4 : 2)
    local_moves_kernel(LocalArgs a) {
    constexpr int G = 64 / LPC;          // chains per wave
    constexpr int SLOTS = LPC * PPL;     // LDS slots per chain and array
    constexpr int WPB = kLocalWaves * (SORT ? 2 : 1);
    __shared__ double lds[WPB][4][G * SLOTS];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = lane / LPC, gl = lane % LPC;
    const int sb = g * SLOTS;            // this chain's slot base
    int64_t c;
    if constexpr (SORT) {
        static_assert(kLocalWaves * G <= 64, "a sorted workgroup's chains fit one ballot");
        constexpr int CPB = kLocalWaves * G;  // chains per workgroup
        const int64_t cb = (int64_t)blockIdx.x * CPB;
        const bool v = lane < CPB && cb + lane < a.C;
        const bool f = v && a.is_f32 && a.is_f32[cb + lane];
        const uint64_t m32 = __ballot(f), m64 = __ballot(v) & ~m32;
        const int n64 = __builtin_popcountll(m64), n32 = __builtin_popcountll(m32);
        const int base32 = (n64 + G - 1) / G * G;
        const int slot = wid * G + g;
        int idx = -1;
        if (slot < n64) idx = nth_set_bit(m64, slot);
        else if (slot >= base32 && slot - base32 < n32) idx = nth_set_bit(m32, slot - base32);
        if (idx < 0) return;  // whole groups leave
        c = cb + idx;
    } else {
        c = ((int64_t)blockIdx.x * kLocalWaves + wid) * G + g;
        if (c >= a.C) return;  // whole groups leave; only group-internal shuffles below
    }
    if (a.gate && *a.gate == 0) return;  // (launch-uniform)
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
    // double-well roles / sum rows of this lane: gl + LPC k (role 0/1 = old position well
    // 0/1, 2/3 = new position; rows eno, viro, enn, virn)
    constexpr int RPL = LPC >= 4 ? 1 : 4 / LPC;
    int64_t samp = 0;
    unsigned long long n_acc_local = 0;
    // (step0 + t + 1) mod adjust_every / sample_every, carried as counters: one 64-bit
    // remainder per launch instead of one per move
    int ra = a.adjust_every > 0 ? (int)((a.step0 + 1) % a.adjust_every) : 1;
    int rsm = a.sample_every > 0 ? (int)((a.step0 + 1) % a.sample_every) : 1;

    for (int64_t t = 0; t < a.n_moves; ++t) {
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
        // pair terms of particle p against this lane's particles (np.delete order: j - (j > p)).
        // Only terms inside the cutoff are non-zero (about 1 % at rho = 0.03): they alone are
        // written to LDS, at their compacted index, and flagged in a 64-bit mask per row
        bool ho = false, hn = false;
        uint64_t mo = 0, mn = 0;
#pragma unroll
        for (int q = 0; q < PPL; ++q) {
            const int j = gl + LPC * q;
            if (j < N && j != p) {
                const int t = j - (j > p ? 1 : 0);
                bool io, in;
                double ro = 0.0, rn = 0.0;
                if (f32) {
                    const float fx = (float)xj[q], fy = (float)yj[q];
                    const float so = sqdist_f32((float)ox, (float)oy, fx, fy, P.Lx, P.Ly, a.T, iLx, iLy);
                    const float sn = sqdist_f32((float)nx, (float)ny, fx, fy, P.Lx, P.Ly, a.T, iLx, iLy);
                    ho |= so <= a.T.core32;
                    hn |= sn <= a.T.core32;
                    io = so <= a.T.cut32;
                    in = sn <= a.T.cut32;
                    if (io) ro = r_of_sq(so);
                    if (in) rn = r_of_sq(sn);
                } else {
                    const double so = sqdist_f64(ox, oy, xj[q], yj[q], P.Lx, P.Ly, a.T, iLx, iLy);
                    const double sn = sqdist_f64(nx, ny, xj[q], yj[q], P.Lx, P.Ly, a.T, iLx, iLy);
                    ho |= so <= a.T.core64;
                    hn |= sn <= a.T.core64;
                    io = so <= a.T.cut64;
                    in = sn <= a.T.cut64;
                    if (io) ro = r_of_sq(so);
                    if (in) rn = r_of_sq(sn);
                }
                if (io) {
                    double e, w;
                    lj_pair(ro, P.r_cut, e_cut, e, w);
                    lds[wid][0][sb + t] = e;
                    lds[wid][1][sb + t] = w;
                    mo |= 1ull << t;
                }
                if (in) {
                    double e, w;
                    lj_pair(rn, P.r_cut, e_cut, e, w);
                    lds[wid][2][sb + t] = e;
                    lds[wid][3][sb + t] = w;
                    mn |= 1ull << t;
                }
            }
        }
        if constexpr (LPC >= 2) {
            mo |= xor_c<LPC, 1>(mo);
            mn |= xor_c<LPC, 1>(mn);
        }
        if constexpr (LPC >= 4) {
            mo |= xor_c<LPC, 2>(mo);
            mn |= xor_c<LPC, 2>(mn);
        }
#pragma unroll
        for (int o = 4; o < LPC; o <<= 1) {
            mo |= __shfl_xor(mo, o, LPC);
            mn |= __shfl_xor(mn, o, LPC);
        }
        const bool hit_old = (__ballot(ho) & gmask) != 0;
        const bool hit_new = (__ballot(hn) & gmask) != 0;
        double dw[RPL];
#pragma unroll
        for (int k = 0; k < RPL; ++k) {
            const int role = gl + LPC * k, well = role & 1;
            dw[k] = 0.0;
            if (role < 4 && well < P.num_wells)
                dw[k] = dw_term(role < 2 ? ox : nx, role < 2 ? oy : ny, well, P.Lx, P.Ly, P.V0[well], P.r0, P.k, iLx,
                                iLy);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // numpy pairwise sums of the four compacted rows (eno, viro, enn, virn), lane gl + LPC u
        // summing row gl + LPC u over its flagged terms only: the terms left out are +0.0 and
        // no term or partial sum is -0.0, so adding them changes nothing (x + 0 == x)
        double rs[RPL];
#pragma unroll
        for (int u = 0; u < RPL; ++u) {
            const int rw = gl + LPC * u;
            double r = 0.0;
            if (rw < 4) {
                const uint64_t m = rw < 2 ? mo : mn;
                const double *row = &lds[wid][rw][sb];
                if (n < 8) {
                    for (uint64_t b = m; b; b &= b - 1) r += row[__builtin_ctzll(b)];
                } else {
                    const uint64_t body = nfull >= 64 ? ~0ull : ((1ull << nfull) - 1);
                    double acc[8];
#pragma unroll
                    for (int k = 0; k < 8; ++k) {  // partial k: terms k, k+8, k+16, ... in order
                        acc[k] = 0.0;
                        for (uint64_t b = m & body & (0x0101010101010101ull << k); b; b &= b - 1)
                            acc[k] += row[__builtin_ctzll(b)];
                    }
                    r = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
                    for (uint64_t b = m & ~body; b; b &= b - 1) r += row[__builtin_ctzll(b)];
                }
            }
            rs[u] = r;
        }
        // row / role q lives in lane q % LPC of the group, slot q / LPC
#define FS_FROM(v, q) bcast_c<LPC, (q) % LPC>(pick<RPL>(v, (q) / LPC))
        double eno = FS_FROM(rs, 0), viro = FS_FROM(rs, 1), enn = FS_FROM(rs, 2), virn = FS_FROM(rs, 3);
        if (P.num_wells > 0) {  // V = 0; V += term(well 0); V += term(well 1)  (potential.py:96-112)
            double vo = 0.0 + FS_FROM(dw, 0), vn = 0.0 + FS_FROM(dw, 2);
            if (P.num_wells > 1) {
                vo += FS_FROM(dw, 1);
                vn += FS_FROM(dw, 3);
            }
#undef FS_FROM
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
        if (a.adjust_every > 0 && ra == 0) adjust_md(md, att, acc_n, prev_att, prev_acc, a.target);
        const bool take = a.sample_every > 0 && rsm == 0;
        if (a.adjust_every > 0) ra = ra + 1 == a.adjust_every ? 0 : ra + 1;
        if (a.sample_every > 0) rsm = rsm + 1 == a.sample_every ? 0 : rsm + 1;
        if (take && samp < a.n_samp) {
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

// the dynamic-LDS limit a launch of `bytes` needs (above the default 64 KiB), raised once
// per kernel and device (the limit plus the kernel's static LDS must stay within 160 KiB)
static hipError_t local_dyn_lds_once(const void *kfn, unsigned bytes) {
    static std::mutex mu;
    static std::map<std::pair<const void *, int>, unsigned> done;
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev); e != hipSuccess) return e;
    std::lock_guard<std::mutex> g(mu);
    unsigned &have = done[{kfn, dev}];
    if (have >= bytes) return hipSuccess;
    hipError_t e = hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e == hipSuccess) have = bytes;
    return e;
}

hipError_t fs_local_moves_impl(const fs_phys *p, int64_t C, int N, double *state, const uint8_t *is_f32,
                               double *E, double *W, uint64_t *pcg, uint64_t *pcg_buf, double *max_disp,
                               int64_t *attempts, int64_t *accepted, int64_t *prev, int64_t n_moves, int64_t step0,
                               int adjust_every, double target, int sample_every, double *samples_xy,
                               double *samples_ew, uint8_t *accept_log, unsigned long long *n_accept,
                               hipStream_t st, const uint8_t *gate) {
    if (C <= 0 || n_moves <= 0) return hipSuccess;
    LocalArgs a{*p,       C,         N,        state,      is_f32,     E,          W,
                pcg,      pcg_buf,   max_disp, attempts,   accepted,   prev,       n_moves,
                step0,    adjust_every, target, sample_every, fs_local_samples_per_chain(step0, n_moves, sample_every),
                samples_xy, samples_ew, accept_log, n_accept, fs_pair_thresh(*p), gate};
    // lanes per chain x particles per lane (FS_LOCAL_LAYOUT=LPCxPPL overrides, for A/B runs).
    // Measured at 65536 chains x 1000 moves (sparse in-cutoff sums): N=64 8x8 2.41 G moves/s
    // (16x4 1.88 G, 64x1 1.06 G, 4x16 1.69 G: register-limited); N=32 4x8 4.04 G (8x4 3.20 G);
    // N=16 4x4 5.52 G (8x2 4.78 G).  More chains per wave amortise the per-move work.
    // N = 3 (the reference's Algorithm-1 runs), 1000 moves: 10 chains 8x1 2.47 ms, 4x1 2.29,
    // 2x4 3.94, 1x4 5.80 (the double-well and sum work, serial in fewer lanes, outweighs the
    // shuffles it saves); 65536 chains 8x1 10.2 ms, 4x1 5.71, 2x4 5.28, 1x4 5.52
    // (profiles/r05/r05m_local_layouts.log).  Chains stay packed 64 / LPC per wave even when
    // that leaves SIMDs idle: spreading 10 or 256 chains one per wave (one wave per CU or four)
    // was 1.1-2.3x slower than one packed wave, though a packed wave runs the union of its
    // chains' branches (profiles/r05/r05ap_cpw_sweep.log, r05aq_wpb_sweep.log).
    int lpc = N > 32 ? 8 : N > 8 ? 4 : 8;
    int ppl = N > 32 ? 8 : N > 16 ? 8 : N > 8 ? 4 : 1;
    if (N <= 4) {
        lpc = C >= 16384 ? 2 : 4;
        ppl = C >= 16384 ? 4 : 1;
    }
    if (const char *e = getenv("FS_LOCAL_LAYOUT")) {
        int l = 0, q = 0;
        if (sscanf(e, "%dx%d", &l, &q) == 2 && l * q >= N) {
            lpc = l;
            ppl = q;
        }
    }
    const int64_t chains_per_block = (int64_t)kLocalWaves * (64 / lpc);
    const dim3 grid((unsigned)((C + chains_per_block - 1) / chains_per_block));
    // dtype-sorted workgroups for launches of at most 8 workgroups (FS_LOCAL_SORT=0 / 1 turns
    // them off / on everywhere, for A/B runs and tests)
    const char *se = getenv("FS_LOCAL_SORT");
    const bool sort = is_f32 && lpc >= 4 && (se && (se[0] == '0' || se[0] == '1') ? se[0] == '1' : grid.x <= 8);
    // A launch of a few workgroups (the reference's 10 runs: one) is latency-bound on its
    // waves' dependent chains, and a workgroup of another stream's kernel placed on its CU
    // (the Algorithm-1 pipeline runs density passes beside it) takes issue slots from it.
    // Such launches claim 128 KiB of LDS per workgroup, so no workgroup of the wide path's
    // trunk or final phase (33 KiB each) is placed on their CUs (FS_LOCAL_EXCLUSIVE=0 turns
    // this off; 1 forces it).  r06, Algorithm-1 regime through the pipeline: 3114 -> 3214
    // attempts/s (profiles/r06/r06zk_*).  Placing the work on another XCD than the density
    // passes' (a workgroup offset) changed nothing (r06zo_*), and density passes on one or two
    // other streams do not slow such a launch (r06zw_*, r06zx_*): what had slowed the regime's
    // launches (2.71 against 2.3 ms per 1000 moves) was waves holding both float32- and
    // float64-state chains, which the dtype-sorted workgroups above remove.
    static const int excl_env = [] {
        const char *e = getenv("FS_LOCAL_EXCLUSIVE");
        return e && (e[0] == '0' || e[0] == '1') ? e[0] - '0' : -1;
    }();
    const bool excl = excl_env == 1 || (excl_env < 0 && grid.x <= 8);
#define FS_LLAUNCH(L, Q, S)                                                                       \
    {                                                                                             \
        unsigned dyn = 0;                                                                         \
        if (excl) {                                                                               \
            dyn = 131072u - (unsigned)sizeof(double) * kLocalWaves * (S ? 2 : 1) * 4 * 64 * Q;    \
            if (hipError_t e = local_dyn_lds_once((const void *)local_moves_kernel<L, Q, S>, dyn); \
                e != hipSuccess)                                                                  \
                return e;                                                                         \
        }                                                                                         \
        hipLaunchKernelGGL((local_moves_kernel<L, Q, S>), grid, dim3(64 * kLocalWaves * (S ? 2 : 1)), dyn, st, \
                           a);                                                                    \
        return hipGetLastError();                                                                 \
    }
#define FS_LCASE(L, Q) \
    if (lpc == L && ppl == Q) FS_LLAUNCH(L, Q, false)
#define FS_LCASE_S(L, Q)                    \
    if (lpc == L && ppl == Q) {             \
        if (sort) FS_LLAUNCH(L, Q, true)    \
        FS_LLAUNCH(L, Q, false)             \
    }
    FS_LCASE_S(8, 1) FS_LCASE(8, 2) FS_LCASE(8, 4) FS_LCASE_S(8, 8) FS_LCASE(64, 1) FS_LCASE(16, 4) FS_LCASE(4, 16)
    FS_LCASE(4, 8) FS_LCASE_S(4, 4) FS_LCASE(1, 4) FS_LCASE(1, 8) FS_LCASE(2, 4) FS_LCASE_S(4, 1)
#undef FS_LCASE_S
#undef FS_LCASE
#undef FS_LLAUNCH
    return hipErrorInvalidValue;
}

// dst chain c := src chain c for every chain when *gate != 0 (one thread per chain; the
// Algorithm-1 pipeline's fix-up after a big move that some chain accepted)
__global__ void chains_copy_if_kernel(const uint8_t *gate, int64_t C, int N, fs_local_chains src,
                                      fs_local_chains dst) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C || *gate == 0) return;
    for (int j = 0; j < 2 * N; ++j) dst.state[c * 2 * N + j] = src.state[c * 2 * N + j];
    if (src.state_is_f32) dst.state_is_f32[c] = src.state_is_f32[c];
    dst.E[c] = src.E[c];
    if (src.W) dst.W[c] = src.W[c];
    for (int i = 0; i < 4; ++i) dst.pcg[4 * c + i] = src.pcg[4 * c + i];
    dst.pcg_buf[2 * c] = src.pcg_buf[2 * c];
    dst.pcg_buf[2 * c + 1] = src.pcg_buf[2 * c + 1];
    dst.max_disp[c] = src.max_disp[c];
    dst.attempts[c] = src.attempts[c];
    dst.accepted[c] = src.accepted[c];
    if (src.prev_counts) {
        dst.prev_counts[2 * c] = src.prev_counts[2 * c];
        dst.prev_counts[2 * c + 1] = src.prev_counts[2 * c + 1];
    }
}

hipError_t fs_chains_copy_if_impl(const uint8_t *gate, int64_t C, int N, const fs_local_chains *src,
                                  const fs_local_chains *dst, hipStream_t st) {
    if (C <= 0) return hipSuccess;
    hipLaunchKernelGGL(chains_copy_if_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, st, gate, C, N, *src,
                       *dst);
    return hipGetLastError();
}

hipError_t fs_adjust_displacement_impl(int64_t C, double *max_disp, const int64_t *attempts, const int64_t *accepted,
                                       int64_t *prev, double target, hipStream_t st) {
    if (C <= 0) return hipSuccess;
    hipLaunchKernelGGL(adjust_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, st, C, max_disp, attempts,
                       accepted, prev, target);
    return hipGetLastError();
}
