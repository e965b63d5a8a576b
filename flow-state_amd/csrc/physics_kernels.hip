// MI355X kernels for the physics / acceptance side of the NF-MH step:
//   * LJ + double-well total energy (energy_calculator.py:121-203) — one wave per
//     chain, lane i = particle i = pair-row i, coordinates staged in LDS, fp64
//     pair arithmetic in the reference's evaluation order (numpy pairwise row
//     sums, Python-float row accumulation) so results track numpy to the ulp;
//     hard-core flag by wave ballot; optional r <= r_cut neighbour masks;
//   * numpy SeedSequence + PCG64 (monte_carlo.py:92-95) and Generator.random();
//   * the nf_big_move accept / reject + state update (monte_carlo.py:235-303)
//     with a wave ballot / popcount accept counter and a ballot-driven
//     wave-cooperative copy of the accepted configurations;
//   * histogram2d / well-occupancy reductions (hybrid_NF_MCMC/utils.py:61-141, 488-495).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include <type_traits>

#include "flow_layout.h"
#include "fs_internal.h"
#include "physics_device.h"

#pragma clang fp contract(off)

namespace fs {

// ---------------------------------------------------------------- energy
// numpy pairwise sum of n <= 128 values held in LDS (serial, one lane)
__device__ double pairwise_lds(const double *a, int n) {
    if (n < 8) {
        double res = 0.0;
        for (int i = 0; i < n; ++i) res += a[i];
        return res;
    }
    double r[8];
    for (int j = 0; j < 8; ++j) r[j] = a[j];
    int i = 8;
    for (; i < n - (n % 8); i += 8)
        for (int j = 0; j < 8; ++j) r[j] += a[i + j];
    double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
    for (; i < n; ++i) res += a[i];
    return res;
}

// Two chains per wave (one per 32-lane half).  Lane l of a half owns pair rows l and
// N-2-l, so every lane evaluates N pair terms (the triangle is folded); each row is
// still summed in numpy's pairwise order and the rows are accumulated in row order.
template <bool F32>
__global__ void __launch_bounds__(256) energy_kernel(fs_phys p, PairThresh T, const void *__restrict__ pos, int64_t C,
                                                     int N, double *__restrict__ E, double *__restrict__ W,
                                                     uint8_t *__restrict__ ov, uint64_t *__restrict__ nbr,
                                                     const uint8_t *__restrict__ is_f32) {
    using CT = typename std::conditional<F32, float, double>::type;  // coordinates in LDS, stored dtype
    __shared__ CT sx[4][2][64], sy[4][2][64];
    __shared__ double se[4][2][64], sw[4][2][64], sv[4][2][64];
    const int wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int hh = lane >> 5, hl = lane & 31;
    const int64_t c = ((int64_t)blockIdx.x * 4 + wid) * 2 + hh;
    if (c >= C) return;  // a whole half leaves; only wave-level barriers below
    // float64 storage holding a chain whose reference state is float32 (after an accepted
    // big move, monte_carlo.py:296): the float32 distance path on the exact float values
    const bool as_f32 = F32 || (is_f32 && is_f32[c]);
    CT *X = sx[wid][hh], *Y = sy[wid][hh];
    for (int q = hl; q < N; q += 32) {
        if (F32) {
            const float *src = (const float *)pos + c * 2 * N;
            X[q] = src[2 * q];
            Y[q] = src[2 * q + 1];
        } else {
            const double *src = (const double *)pos + c * 2 * N;
            X[q] = src[2 * q];
            Y[q] = src[2 * q + 1];
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const double sr6c = pow6(1.0 / p.r_cut);
    const double e_cut = 4.0 * (sr6c * sr6c - sr6c);
    const double iLx = 1.0 / p.Lx, iLy = 1.0 / p.Ly;
    bool hit = false;
    // Row i (pairs j > i, t = j - i - 1) in two passes.  Pass 1: the squared minimum-image
    // distances, the hard-core flag and the in-cutoff mask (PairThresh: one comparison each).
    // Pass 2: lennard_jones_energy_virial (potential.py:3-29) of the in-cutoff pairs only
    // (about 1 % at rho = 0.03), added in numpy's pairwise order of the whole row
    // (loops_utils.h pairwise_sum, n <= 128): a term's accumulator is fixed by its position t,
    // and the skipped terms are +0.0 while no term or partial sum is -0.0, so x + 0 == x
    // leaves every sum as the full row's.  Evaluating the LJ term inside pass 1 made a wave
    // run the sqrt / reciprocal / pow6 chain on every pair some lane had inside the cutoff
    // (~half of them for 64 lanes).
    auto sqc = [&](CT xi, CT yi, int j) -> double {
        if (as_f32)
            return F32 ? sqdist32((float)xi, (float)yi, (float)X[j], (float)Y[j], p.Lx, p.Ly, T, iLx, iLy)
                       : sqdist_f32((float)xi, (float)yi, (float)X[j], (float)Y[j], p.Lx, p.Ly, T, iLx, iLy);
        return sqdist_f64(xi, yi, X[j], Y[j], p.Lx, p.Ly, T, iLx, iLy);
    };
    auto term = [&](int i, int j, double &e, double &w) {
        const double s = sqc(X[i], Y[i], j);
        lj_pair(as_f32 ? r_of_sq((float)s) : r_of_sq(s), p.r_cut, e_cut, e, w);
    };
    // pass 2 of row i over its in-cutoff mask: the row's energy / virial sums
    auto row_sums = [&](int i, uint64_t mask) {
        const int n = N - 1 - i;
        double re = 0.0, rw = 0.0;
        if (n < 8) {
            for (uint64_t b = mask; b; b &= b - 1) {
                double e, w;
                term(i, i + 1 + __builtin_ctzll(b), e, w);
                re += e;
                rw += w;
            }
        } else {
            const int nfull = n - (n % 8);
            const uint64_t body = nfull >= 64 ? ~0ull : (((uint64_t)1 << nfull) - 1);
            double ae[8], aw[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) ae[k] = aw[k] = 0.0;
            for (uint64_t b = mask & body; b; b &= b - 1) {
                const int t = __builtin_ctzll(b);
                double e, w;
                term(i, i + 1 + t, e, w);
#pragma unroll
                for (int k = 0; k < 8; ++k)
                    if ((t & 7) == k) {
                        ae[k] += e;
                        aw[k] += w;
                    }
            }
            re = ((ae[0] + ae[1]) + (ae[2] + ae[3])) + ((ae[4] + ae[5]) + (ae[6] + ae[7]));
            rw = ((aw[0] + aw[1]) + (aw[2] + aw[3])) + ((aw[4] + aw[5]) + (aw[6] + aw[7]));
            for (uint64_t b = mask & ~body; b; b &= b - 1) {
                double e, w;
                term(i, i + 1 + __builtin_ctzll(b), e, w);
                re += e;
                rw += w;
            }
        }
        if (i + 1 < 64) mask <<= (i + 1);  // neighbour mask: bit j of word i
        else mask = 0;
        se[wid][hh][i] = re;
        sw[wid][hh][i] = rw;
        if (nbr) nbr[c * N + i] = mask;
    };
    // pass 1 of both rows of this lane in one loop (r06): rows ra = l and rb = N-2-l have
    // N-1-l and l+1 pairs, so each lane runs N pairs and the wave N iterations, where one
    // loop per row ran the longest row of each (N-1 + N/2 iterations)
    const int ra = hl, rb = N - 2 - hl;
    const int na = ra <= N - 2 ? N - 1 - ra : 0, nb = rb > ra ? N - 1 - rb : 0;
    const CT xa = na ? X[ra] : CT(0), ya = na ? Y[ra] : CT(0), xb = nb ? X[rb] : CT(0), yb = nb ? Y[rb] : CT(0);
    uint64_t ma = 0, mb = 0;  // bit t: pair (i, i + 1 + t) inside the cutoff
    for (int k = 0; k < na + nb; ++k) {
        const bool in_a = k < na;
        const int t = in_a ? k : k - na;
        const double s = sqc(in_a ? xa : xb, in_a ? ya : yb, (in_a ? ra : rb) + 1 + t);
        const bool core = as_f32 ? (float)s <= T.core32 : s <= T.core64;
        const bool cut = as_f32 ? (float)s <= T.cut32 : s <= T.cut64;
        hit |= core;
        const uint64_t bit = cut ? (uint64_t)1 << t : 0;
        if (in_a) ma |= bit;
        else mb |= bit;
    }
    if (na) row_sums(ra, ma);
    if (nb) row_sums(rb, mb);
    if (nbr && hl == 0 && N >= 1) nbr[c * N + N - 1] = 0;  // the last row has no j > i
    // external double well per particle (potential.py:89-112)
    for (int q = hl; q < N; q += 32) {
        double v = 0.0;
        const double cy = p.Ly / 2.0;
        for (int k = 0; k < p.num_wells && k < 2; ++k) {
            const double cx = (k == 0) ? p.Lx / 4.0 : 3.0 * p.Lx / 4.0;
            double dx = X[q] - cx, dy = Y[q] - cy;
            dx -= p.Lx * rint_div(dx, p.Lx, iLx);
            dy -= p.Ly * rint_div(dy, p.Ly, iLy);
            const double r = sqrt(dx * dx + dy * dy);
            const double tr = 0.5 * (1.0 + tanh(p.k * (r - p.r0)));
            v += p.V0[k] * (1.0 - tr);
        }
        sv[wid][hh][q] = v;
    }
    const uint64_t half = hh ? 0xffffffff00000000ull : 0x00000000ffffffffull;
    const bool any_hit = (__ballot(hit) & half) != 0;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (hl == 0) {
        double te = 0.0, tw = 0.0;
        for (int k = 0; k < N - 1; ++k) {  // Python-float accumulation over rows
            te += se[wid][hh][k];
            tw += sw[wid][hh][k];
        }
        if (p.num_wells > 0) te += pairwise_lds(sv[wid][hh], N);
        if (any_hit) {
            te = INFINITY;
            tw = INFINITY;
        }
        E[c] = te;
        if (W) W[c] = tw;
        if (ov) ov[c] = any_hit ? 1 : 0;
    }
}

// ---------------------------------------------------------------- PCG64
__device__ __forceinline__ uint32_t ss_hashmix(uint32_t v, uint32_t &hc) {
    v ^= hc;
    hc *= 0x931e8875u;
    v *= hc;
    v ^= v >> 16;
    return v;
}

__device__ __forceinline__ uint32_t ss_mix(uint32_t x, uint32_t y) {
    uint32_t r = 0xca01f9ddu * x - 0x4973f715u * y;
    r ^= r >> 16;
    return r;
}

// numpy SeedSequence(seed).generate_state(4, uint64) -> pcg64_set_seed
__global__ void pcg64_seed_kernel(const uint64_t *__restrict__ seeds, int64_t C, uint64_t *__restrict__ state) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    uint64_t seed = seeds[c];
    uint32_t ent[2] = {0u, 0u};
    int n_ent = 0;
    if (seed == 0) ent[n_ent++] = 0;
    while (seed) {
        ent[n_ent++] = (uint32_t)seed;
        seed >>= 32;
    }
    uint32_t pool[4];
    uint32_t hc = 0x43b0d7e5u;
    for (int i = 0; i < 4; ++i) pool[i] = ss_hashmix(i < n_ent ? ent[i] : 0u, hc);
    for (int s = 0; s < 4; ++s)
        for (int d = 0; d < 4; ++d)
            if (s != d) pool[d] = ss_mix(pool[d], ss_hashmix(pool[s], hc));
    uint32_t w[8];
    uint32_t hb = 0x8b51f9ddu;
    for (int i = 0; i < 8; ++i) {
        uint32_t v = pool[i & 3];
        v ^= hb;
        hb *= 0x58f38dedu;
        v *= hb;
        v ^= v >> 16;
        w[i] = v;
    }
    uint64_t val[4];
    for (int i = 0; i < 4; ++i) val[i] = (uint64_t)w[2 * i] | ((uint64_t)w[2 * i + 1] << 32);
    const u128 M = {0x2360ED051FC65DA4ull, 0x4385DF649FCCF645ull};
    const u128 initstate = {val[0], val[1]};
    u128 inc = {(val[2] << 1) | (val[3] >> 63), (val[3] << 1) | 1ull};
    u128 st = {0, 0};
    st = mul_add(st, M, inc);
    const uint64_t lo = st.lo + initstate.lo;
    st.hi += initstate.hi + (lo < st.lo ? 1 : 0);
    st.lo = lo;
    st = mul_add(st, M, inc);
    state[4 * c + 0] = st.hi;
    state[4 * c + 1] = st.lo;
    state[4 * c + 2] = inc.hi;
    state[4 * c + 3] = inc.lo;
}

__global__ void pcg64_random_kernel(uint64_t *__restrict__ state, int64_t C, double *__restrict__ out) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    out[c] = pcg64_next_double(state + 4 * c);
}

// ---------------------------------------------------------------- MH accept
__global__ void __launch_bounds__(256) mh_accept_kernel(fs_phys p, int64_t C, int N, double *E_old, double *W_old,
                                                        double *nll_old, const double *E_new, const double *W_new,
                                                        const float *log_q_new, uint64_t *pcg, double *state,
                                                        uint8_t *state_is_f32, const float *config,
                                                        uint8_t *accept, int64_t *attempts, int64_t *accepted,
                                                        unsigned long long *n_accept, int flags,
                                                        const float *log_q_old, const double *E_cur,
                                                        const double *W_cur) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const bool valid = c < C;
    int acc = 0;
    if (valid) {
        const double en = E_new[c];
        const double nll_new = -(double)log_q_new[c];  // - log_prob(new).item()
        const double dE = en - E_old[c];
        // hybrid: old NLL of the current (locally moved) state, monte_carlo.py:251-261
        const double no = log_q_old ? -(double)log_q_old[c] : nll_old[c];
        const double dN = nll_new - no;
        const double ratio_log = (flags & FS_MH_CORRECT_SIGN) ? (-p.beta * dE + dN) : (-p.beta * dE - dN);
        const double ratio = exp(ratio_log);
        if (ratio >= 1.0) {
            acc = 1;
        } else {
            const double u = pcg64_next_double(pcg + 4 * c);
            acc = u < ratio ? 1 : 0;  // NaN ratio -> draw and reject
        }
        accept[c] = (uint8_t)acc;
        if (attempts) attempts[c] += 1;
        if (acc) {
            E_old[c] = en;
            if (W_old && W_new) W_old[c] = W_new[c];
            nll_old[c] = nll_new;
            if (accepted) accepted[c] += 1;
            if (state_is_f32) state_is_f32[c] = 1;
        } else {
            if (log_q_old) nll_old[c] = no;
            if (E_cur) {  // reject recomputes the total energy (monte_carlo.py:299-301)
                E_old[c] = E_cur[c];
                if (W_old && W_cur) W_old[c] = W_cur[c];
            }
        }
    }
    uint64_t m = __ballot(acc);
    if (lane == 0 && n_accept && m) atomicAdd(n_accept, (unsigned long long)__popcll(m));
    if (state && config) {  // wave-cooperative coalesced copy of each accepted configuration
        const int64_t base = c - lane;
        const int D = 2 * N;
        while (m) {
            const int b = __ffsll((unsigned long long)m) - 1;
            m &= m - 1;
            const int64_t cc = base + b;
            for (int t = lane; t < D; t += 64) state[cc * D + t] = (double)config[cc * D + t];
        }
    }
}

// SimulationBox.minimum_image / compute_distance (simulation_box.py:31-56) for n pairs
// (a[i * sa], b[i]), sa = 0 broadcasts one first position (compute_distances, :58-65):
// delta = the wrapped displacement in the positions' dtype (float32: wrapped in float64
// against the np.float64 box lengths, rounded back), r = np.linalg.norm(delta) (the
// float32 sdot / float64 ddot, correctly rounded sqrt), both widened to float64.
template <bool F32>
__global__ void __launch_bounds__(256) min_image_kernel(fs_phys p, PairThresh T, const void *__restrict__ a, int64_t sa,
                                 const void *__restrict__ b, int64_t n, double *__restrict__ delta,
                                 double *__restrict__ r) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double iLx = 1.0 / p.Lx, iLy = 1.0 / p.Ly;
    double t0, t1, rr;
    if (F32) {
        const float *A = (const float *)a + 2 * i * sa, *B = (const float *)b + 2 * i;
        const float u0 = (float)wrap_min_image((double)(A[0] - B[0]), p.Lx, T.hx, iLx);
        const float u1 = (float)wrap_min_image((double)(A[1] - B[1]), p.Ly, T.hy, iLy);
        t0 = u0;
        t1 = u1;
        rr = r_of_sq(sqdist_f32(A[0], A[1], B[0], B[1], p.Lx, p.Ly, T, iLx, iLy));
    } else {
        const double *A = (const double *)a + 2 * i * sa, *B = (const double *)b + 2 * i;
        t0 = wrap_min_image(A[0] - B[0], p.Lx, T.hx, iLx);
        t1 = wrap_min_image(A[1] - B[1], p.Ly, T.hy, iLy);
        rr = r_of_sq(sqdist_f64(A[0], A[1], B[0], B[1], p.Lx, p.Ly, T, iLx, iLy));
    }
    if (delta) {
        delta[2 * i] = t0;
        delta[2 * i + 1] = t1;
    }
    if (r) r[i] = rr;
}

// EnergyCalculator.calculate_particle_energy_virial (energy_calculator.py:48-108): the
// energy / virial of particle part[c] of chain c with the np.delete-compacted others
// (pair t <-> particle t + (t >= part)), +inf for both if any r < 0.5, else np.sum of the
// LJ terms (numpy's pairwise order) + the particle's double-well term.  One thread per
// chain (an API call, not the local-move hot loop, which has its own kernel).
template <bool F32>
__global__ void __launch_bounds__(64) particle_energy_kernel(fs_phys p, PairThresh T, const void *__restrict__ pos, int64_t C, int N,
                                       const int32_t *__restrict__ part, double *__restrict__ E,
                                       double *__restrict__ W) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const int pi = part[c];
    const double iLx = 1.0 / p.Lx, iLy = 1.0 / p.Ly;
    const double sr6c = pow6(1.0 / p.r_cut);
    const double e_cut = 4.0 * (sr6c * sr6c - sr6c);
    auto X = [&](int j) {
        return F32 ? (double)((const float *)pos)[(c * N + j) * 2] : ((const double *)pos)[(c * N + j) * 2];
    };
    auto Y = [&](int j) {
        return F32 ? (double)((const float *)pos)[(c * N + j) * 2 + 1] : ((const double *)pos)[(c * N + j) * 2 + 1];
    };
    bool hit = false;
    auto term = [&](int t, double &e, double &w) {
        const int j = t + (t >= pi ? 1 : 0);
        e = 0.0;
        w = 0.0;
        if (F32) {
            const float s = sqdist_f32((float)X(pi), (float)Y(pi), (float)X(j), (float)Y(j), p.Lx, p.Ly, T, iLx, iLy);
            hit |= s <= T.core32;
            if (s <= T.cut32) lj_pair(r_of_sq(s), p.r_cut, e_cut, e, w);
        } else {
            const double s = sqdist_f64(X(pi), Y(pi), X(j), Y(j), p.Lx, p.Ly, T, iLx, iLy);
            hit |= s <= T.core64;
            if (s <= T.cut64) lj_pair(r_of_sq(s), p.r_cut, e_cut, e, w);
        }
    };
    const int n = N - 1;
    double re = 0.0, rw = 0.0;
    if (n < 8) {
        for (int t = 0; t < n; ++t) {
            double e, w;
            term(t, e, w);
            re += e;
            rw += w;
        }
    } else {
        double ae[8], aw[8];
        for (int j = 0; j < 8; ++j) term(j, ae[j], aw[j]);
        const int nfull = n - (n % 8);
        for (int t0 = 8; t0 < nfull; t0 += 8)
            for (int j = 0; j < 8; ++j) {
                double e, w;
                term(t0 + j, e, w);
                ae[j] += e;
                aw[j] += w;
            }
        re = ((ae[0] + ae[1]) + (ae[2] + ae[3])) + ((ae[4] + ae[5]) + (ae[6] + ae[7]));
        rw = ((aw[0] + aw[1]) + (aw[2] + aw[3])) + ((aw[4] + aw[5]) + (aw[6] + aw[7]));
        for (int t = nfull; t < n; ++t) {
            double e, w;
            term(t, e, w);
            re += e;
            rw += w;
        }
    }
    if (hit) {
        E[c] = INFINITY;
        W[c] = INFINITY;
        return;
    }
    double v = 0.0;
    for (int k = 0; k < p.num_wells && k < 2; ++k)
        v += dw_term(X(pi), Y(pi), k, p.Lx, p.Ly, p.V0[k], p.r0, p.k, iLx, iLy);
    E[c] = p.num_wells > 0 ? re + v : re;
    W[c] = rw;
}

// Energy-only Metropolis of supplied proposals against a reference energy, without moving
// the chain: judge_normalizing_flow (monte_carlo.py:305-329, reference = the chain's
// energy) and bulk_judge_normalizing_flow (:331-370, M proposals per chain against one
// reference energy), both through metropolis_acceptance_particle_move (:191-223):
// E_new <= E_ref accepts and E_new = +-inf rejects without a draw, otherwise
// Generator.random() < exp(-beta (E_new - E_ref)) (a NaN energy draws and rejects).
// One thread per chain walks its M proposals in order (one PCG64 stream).
__global__ void __launch_bounds__(256) metropolis_judge_kernel(double beta, int64_t C, int64_t M,
                                                               const double *__restrict__ E_ref,
                                                               const double *__restrict__ E_new,
                                                               uint64_t *__restrict__ pcg, uint8_t *__restrict__ accept,
                                                               int64_t *__restrict__ n_accept) {
    const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const double eo = E_ref[c];
    int64_t n = 0;
    for (int64_t m = 0; m < M; ++m) {
        const double en = E_new[c * M + m];
        int acc;
        if (en <= eo) {
            acc = 1;
        } else if (isinf(en)) {
            acc = 0;
        } else {
            const double bf = exp(-beta * (en - eo));
            acc = pcg64_next_double(pcg + 4 * c) < bf ? 1 : 0;
        }
        if (accept) accept[c * M + m] = (uint8_t)acc;
        n += acc;
    }
    if (n_accept) n_accept[c] = n;
}

// (float32)(particles - half_width): the NF coordinates of the current state
// (monte_carlo.py:251-257)
__global__ void center_kernel(const double *__restrict__ state, int64_t n, double hw, float *__restrict__ out) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t < n) out[t] = (float)(state[t] - hw);
}

// ---------------------------------------------------------------- reductions
__global__ void hist2d_kernel(const double *__restrict__ pos, int64_t C, int N, double shift,
                              const double *__restrict__ edges, int nb, unsigned long long *__restrict__ hist) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= C * N) return;
    const double x = pos[2 * t] - shift, y = pos[2 * t + 1] - shift;
    // np.searchsorted(edges, v, side='right'), right edge folded into the last bin
    auto bin_of = [&](double v) {
        int lo = 0, hi = nb + 1;  // edges has nb+1 entries
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (edges[mid] <= v) lo = mid + 1;
            else hi = mid;
        }
        int b = lo;  // in [0, nb+1]
        if (v == edges[nb]) b -= 1;
        return b - 1;  // -1 or nb => outlier
    };
    const int bx = bin_of(x), by = bin_of(y);
    if (bx < 0 || bx >= nb || by < 0 || by >= nb) return;
    atomicAdd(&hist[bx * nb + by], 1ull);
}

// The same histogram with a private LDS copy per workgroup (uint32 counters, edges in LDS),
// one workgroup per CU walking the points grid-stride, and one global atomic per non-empty
// bin at the end: the points of many chains land in the same bins (the wells, the lattice),
// which serialises global atomics.  nb <= kHistLdsBins (LDS budget).
constexpr int kHistLdsBins = 120;
__global__ void __launch_bounds__(1024) hist2d_lds_kernel(const double *__restrict__ pos, int64_t n, double shift,
                                                          const double *__restrict__ edges, int nb,
                                                          unsigned long long *__restrict__ hist) {
    __shared__ unsigned int h[kHistLdsBins * kHistLdsBins];
    __shared__ double e[kHistLdsBins + 1];
    for (int i = threadIdx.x; i < nb * nb; i += blockDim.x) h[i] = 0u;
    for (int i = threadIdx.x; i <= nb; i += blockDim.x) e[i] = edges[i];
    __syncthreads();
    auto bin_of = [&](double v) {  // np.searchsorted(edges, v, 'right') - 1, last edge inclusive
        int lo = 0, hi = nb + 1;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (e[mid] <= v) lo = mid + 1;
            else hi = mid;
        }
        int b = lo;
        if (v == e[nb]) b -= 1;
        return b - 1;
    };
    for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x) {
        const int bx = bin_of(pos[2 * t] - shift), by = bin_of(pos[2 * t + 1] - shift);
        if (bx >= 0 && bx < nb && by >= 0 && by < nb) atomicAdd(&h[bx * nb + by], 1u);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nb * nb; i += blockDim.x)
        if (h[i]) atomicAdd(&hist[i], (unsigned long long)h[i]);
}

}  // namespace fs

using namespace fs;

hipError_t fs_energy_impl(const fs_phys *p, const void *pos, int pos_is_f32, int64_t C, int N, double *E,
                          double *W, uint8_t *overlap, uint64_t *nbr, hipStream_t st, const uint8_t *chain_is_f32) {
    if (C <= 0) return hipSuccess;
    const dim3 grid((unsigned)((C + 7) / 8));
    const PairThresh T = fs_pair_thresh(*p);
    if (pos_is_f32)
        hipLaunchKernelGGL(energy_kernel<true>, grid, dim3(256), 0, st, *p, T, pos, C, N, E, W, overlap, nbr,
                           nullptr);
    else
        hipLaunchKernelGGL(energy_kernel<false>, grid, dim3(256), 0, st, *p, T, pos, C, N, E, W, overlap, nbr,
                           chain_is_f32);
    return hipGetLastError();
}

hipError_t fs_mh_accept_impl(const fs_phys *p, int64_t C, int N, double *E_old, double *W_old, double *nll_old,
                             const double *E_new, const double *W_new, const float *log_q_new, uint64_t *pcg,
                             double *state, uint8_t *state_is_f32, const float *config, uint8_t *accept,
                             int64_t *attempts, int64_t *accepted, unsigned long long *n_accept, int flags,
                             hipStream_t st, const float *log_q_old, const double *E_cur, const double *W_cur) {
    if (C <= 0) return hipSuccess;
    hipLaunchKernelGGL(mh_accept_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, st, *p, C, N, E_old,
                       W_old, nll_old, E_new, W_new, log_q_new, pcg, state, state_is_f32, config, accept,
                       attempts, accepted, n_accept, flags, log_q_old, E_cur, W_cur);
    return hipGetLastError();
}

hipError_t fs_min_image_impl(const fs_phys *p, const void *a, int64_t sa, const void *b, int f32, int64_t n,
                            double *delta, double *r, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    const PairThresh T = fs_pair_thresh(*p);
    const dim3 grid((unsigned)((n + 255) / 256));
    if (f32)
        hipLaunchKernelGGL(min_image_kernel<true>, grid, dim3(256), 0, st, *p, T, a, sa, b, n, delta, r);
    else
        hipLaunchKernelGGL(min_image_kernel<false>, grid, dim3(256), 0, st, *p, T, a, sa, b, n, delta, r);
    return hipGetLastError();
}

hipError_t fs_particle_energy_impl(const fs_phys *p, const void *pos, int f32, int64_t C, int N, const int32_t *part,
                                   double *E, double *W, hipStream_t st) {
    if (C <= 0) return hipSuccess;
    const PairThresh T = fs_pair_thresh(*p);
    const dim3 grid((unsigned)((C + 63) / 64));
    if (f32)
        hipLaunchKernelGGL(particle_energy_kernel<true>, grid, dim3(64), 0, st, *p, T, pos, C, N, part, E, W);
    else
        hipLaunchKernelGGL(particle_energy_kernel<false>, grid, dim3(64), 0, st, *p, T, pos, C, N, part, E, W);
    return hipGetLastError();
}

hipError_t fs_metropolis_judge_impl(double beta, int64_t C, int64_t M, const double *E_ref, const double *E_new,
                                   uint64_t *pcg, uint8_t *accept, int64_t *n_accept, hipStream_t st) {
    if (C <= 0) return hipSuccess;
    hipLaunchKernelGGL(metropolis_judge_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, st, beta, C, M,
                       E_ref, E_new, pcg, accept, n_accept);
    return hipGetLastError();
}

hipError_t fs_pcg64_seed_impl(const uint64_t *seeds, int64_t C, uint64_t *state, hipStream_t st) {
    if (C <= 0) return hipSuccess;
    hipLaunchKernelGGL(pcg64_seed_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, st, seeds, C, state);
    return hipGetLastError();
}

hipError_t fs_pcg64_random_impl(uint64_t *state, int64_t C, double *out, hipStream_t st) {
    if (C <= 0) return hipSuccess;
    hipLaunchKernelGGL(pcg64_random_kernel, dim3((unsigned)((C + 255) / 256)), dim3(256), 0, st, state, C, out);
    return hipGetLastError();
}

hipError_t fs_hist2d_impl(const double *pos, int64_t C, int N, double shift, const double *edges, int nb,
                          int64_t *hist, hipStream_t st) {
    const int64_t n = C * N;
    if (n <= 0) return hipSuccess;
    if (nb <= kHistLdsBins) {
        int dev = 0, cus = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        const int64_t want = (n + 1023) / 1024;
        const unsigned blocks = (unsigned)(want < cus ? (want > 0 ? want : 1) : cus);
        hipLaunchKernelGGL(hist2d_lds_kernel, dim3(blocks), dim3(1024), 0, st, pos, n, shift, edges, nb,
                           (unsigned long long *)hist);
    } else {
        hipLaunchKernelGGL(hist2d_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, pos, C, N, shift,
                           edges, nb, (unsigned long long *)hist);
    }
    return hipGetLastError();
}


hipError_t fs_center_impl(const double *state, int64_t n, double hw, float *out, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(center_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, state, n, hw, out);
    return hipGetLastError();
}
