// Device pieces shared by the f32-MFMA flow kernel (flow_kernels.hip) and the
// split-bf16 flow kernel (flow_split_kernels.hip): argument block, barriers, the
// rational-quadratic spline arithmetic (float32, no contraction: every torch op
// rounds separately, splines.py:16-222) and the Philox base-draw generator.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "flow_layout.h"

namespace fs {

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr float kMinW = 1e-3f;  // splines.py:6-8
constexpr float kMinH = 1e-3f;
constexpr float kMinD = 1e-3f;
constexpr double kMinWd = 1e-3;  // the same minima, exact (knots_from_logits)
constexpr double kMinHd = 1e-3;

enum { MODE_DENSITY = 0, MODE_SAMPLE = 1, MODE_PROPOSE = 2 };

struct FlowArgs {
    const float *packed;
    const float *in;      // [B][D] (density / sample); unused by propose
    float *out;           // [B][D] logical-order result, nullable
    float *scalar_out;    // [B] log_q (density + base) or log_det, nullable
    float *config;        // propose: fl32(x + B) box coordinates, nullable
    float *centered;      // propose: fl32(config - half_width), nullable
    int32_t *err;         // bit0: NaN discriminant, nullable
    int64_t nrows;
    uint64_t seed, counter;
    int64_t row_offset;   // global index of row 0 (multi-GPU sharding of the proposal stream)
    int64_t rows_per_counter;  // propose: > 0 = rows are (step, chain) = (row / rpc, row % rpc)
                               // blocks of consecutive steps' proposals; 0 = one counter
    double half_width;
    int N, L, nb, K;
    int add_base;
    float B, twoB, negB;  // fl32(tail_bound), fl32(2*tail_bound), -fl32(tail_bound)
    double Bd, twoBd;     // tail_bound, 2*tail_bound (the knots' double-precision affine)
    float scale_pf;       // fl32(pi / tail_bound)          (wrapper.py:151-154, nn.py:125-126)
    float sqrtH;          // fl32(sqrt(H))                 (coupling.py:340-342)
    float base_lp;        // fl32(-D * log(fl32(2B)))      (Uniform.py:70)
};

// Phase timers for tools/flow_phases.py (built only into libflowstate_prof.so,
// -DFS_PROF): per wave, s_memtime deltas accumulated per phase of the pass.
enum { PH_INPUT, PH_PF, PH_INIT_GEMM, PH_EPI, PH_RES_GEMM, PH_BARRIER, PH_TAIL_GEMM, PH_FINAL_GEMM, PH_SPLINE,
       PH_UNCOND, PH_COUNT };
#ifdef FS_PROF
__device__ unsigned long long g_prof[16];
struct Prof {
    uint64_t t, acc[PH_COUNT];
    __device__ Prof() : t(__builtin_amdgcn_s_memtime()) {
        for (int i = 0; i < PH_COUNT; ++i) acc[i] = 0;
    }
    __device__ __forceinline__ void mark(int ph) {
        const uint64_t n = __builtin_amdgcn_s_memtime();
        acc[ph] += n - t;
        t = n;
    }
    __device__ void flush() {
        if ((threadIdx.x & 63) == 0)
            for (int i = 0; i < PH_COUNT; ++i) atomicAdd(&g_prof[i], (unsigned long long)acc[i]);
    }
};
#else
struct Prof {
    __device__ __forceinline__ void mark(int) {}
    __device__ __forceinline__ void flush() {}
};
#endif

// Barrier of the 4 waves of a row group: LDS arrival counter (monotonic; phase
// counts this wave's arrivals x 4), workgroup-scope release / acquire.
__device__ __forceinline__ void group_barrier(int *ctr, int &phase) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    if ((threadIdx.x & 63) == 0) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    phase += 4;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < phase)
        __builtin_amdgcn_s_sleep(1);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Lane-per-chain view of the two chain halves of a transposed 32-row tile: after the
// swap, lane c (chain c) holds rows 8g + j in lo[4g + j] and rows 8g + 4 + j in hi[4g + j].
// (inline asm with both operands read-write: with the builtin, hipcc 7.2 emitted swaps
// whose second result it then treated as the unswapped input, handing several rows the
// same register.  The compiler's hazard recognizer does not look into inline asm, so the
// asm carries its own wait states: 24 before the first swap for a VGPR just written by a
// 16-pass XDL op (the accumulators come straight from the MFMA chain; without them
// row 0 of the second chain half read the value before the last MFMA), two before the
// others for a VALU-written operand.)
__device__ __forceinline__ void lanes_to_chains(f32x16 &t0, f32x16 &t1) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        float a = t0[i], b = t1[i];
        if (i == 0)
            asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
        else
            asm volatile("v_nop\n\tv_nop\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
        t0[i] = a;
        t1[i] = b;
    }
}

// row m of a swapped tile pair
__device__ __forceinline__ float tile_row(const f32x16 &lo, const f32x16 &hi, int m) {
    return ((m >> 2) & 1) ? hi[4 * (m >> 3) + (m & 3)] : lo[4 * (m >> 3) + (m & 3)];
}

// accumulator element i of tile rt -> row
__device__ __forceinline__ int acc_row(int rt, int i, int h) {
    return 32 * rt + 8 * (i >> 2) + 4 * h + (i & 3);
}

// ---------------------------------------------------------------------------
// Spline pieces (float32, no contraction: each torch op rounds separately)
// ---------------------------------------------------------------------------
#pragma clang fp contract(off)

__device__ __forceinline__ float softplus_t(float x) {  // F.softplus(beta=1, threshold=20)
    return x > 20.f ? x : log1pf(expf(x));
}

// softmax -> min-width affine -> cumsum -> scale to [-B, B] with pinned ends
// (splines.py:117-127 / :131-143).  The reference rounds each op to float32 (its
// cumsum accumulates in double, torch CPU); here the normalisation, the affines and
// the cumsum run in double from the float32 exponentials, and each knot is rounded to
// float32 once.  A float32 1/sum is a scale error shared by every width, which the
// cumsum carries up to 2B (~1 ulp of B at the top knot) - the largest error term of
// the float32 spline; in double the knots are within ~0.5 ulp of the exact ones, so
// the pass is closer to the exact function than the reference's own float32
// (tools/acc_layers.py, tools/acc_uncond.py).  K is a compile-time constant so every
// array below stays in registers.
template <int K>
__device__ __forceinline__ void knots_from_logits(const float (&u)[K], float (&kn)[K + 1], double minb,
                                                  const FlowArgs &a) {
    float m = u[0];
#pragma unroll
    for (int k = 1; k < K; ++k) m = fmaxf(m, u[k]);
    float e[K];
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < K; ++k) {  // logits carry log2(e) (folded at pack time): one v_exp_f32 each
        e[k] = __builtin_amdgcn_exp2f(u[k] - m);
        s += (double)e[k];
    }
    const double sc = (1.0 - minb * (double)K) / s;
    double cs = 0.0;
    kn[0] = a.negB;
#pragma unroll
    for (int k = 0; k < K - 1; ++k) {
        cs += __builtin_fma((double)e[k], sc, minb);
        kn[k + 1] = (float)__builtin_fma(a.twoBd, cs, -a.Bd);
    }
    kn[K] = a.B;
}

// rational_quadratic_spline forward (splines.py:202-222) / inverse (:162-201)
template <bool INV>
__device__ __forceinline__ void rqs_eval(float x, float icw, float ibw, float ich, float ih, float d0,
                                         float d1, float &y, float &lad, bool &nan_disc) {
    const float idl = ih / ibw;
    const float sdd = (d0 + d1) - 2.f * idl;
    if (INV) {
        const float xm = x - ich;
        const float a = xm * sdd + ih * (idl - d0);
        const float b = ih * d0 - xm * sdd;
        const float c = -idl * xm;
        const float disc = fabsf(b * b - (4.f * a) * c);
        nan_disc = disc != disc;
        const float root = (2.f * c) / (-b - sqrtf(disc));
        y = root * ibw + icw;
        const float tomt = root * (1.f - root);
        const float den = idl + sdd * tomt;
        const float omr = 1.f - root;
        const float dnum = (idl * idl) * ((d1 * (root * root) + (2.f * idl) * tomt) + d0 * (omr * omr));
        lad = -(logf(dnum) - 2.f * logf(den));
    } else {
        const float theta = (x - icw) / ibw;
        const float tomt = theta * (1.f - theta);
        const float num = ih * (idl * (theta * theta) + d0 * tomt);
        const float den = idl + sdd * tomt;
        y = ich + num / den;
        const float omt = 1.f - theta;
        const float dnum = (idl * idl) * ((d1 * (theta * theta) + (2.f * idl) * tomt) + d0 * (omt * omt));
        lad = logf(dnum) - 2.f * logf(den);
        nan_disc = false;
    }
}

// Unconditional spline over the identity features f = wid, wid + 8, ... (lane = chain);
// wid is the wave's index in the fused kernel and the virtual wave of the wide path.
template <int K, bool INV>
__device__ __forceinline__ float uncond_spline_w(const float *__restrict__ U, float *CO, int cs, int N,
                                                 int D, int off, const FlowArgs &a, bool &nan_any, int wid) {
    const int lane = threadIdx.x & 63;
    constexpr int K1 = K + 1;
    float ld = 0.f;
    for (int f = wid; f < N; f += kWaves) {
        const float *T = U + (size_t)f * 3 * K1;
        const int p = (2 * f + off) % D;
        const float x = CO[lane * cs + p];
        const bool inside = (x >= a.negB) && (x <= a.B);
        const float *kn = INV ? T + K1 : T;
        int bin = -1;
#pragma unroll
        for (int k = 0; k < K; ++k) bin += (x >= kn[k]) ? 1 : 0;
        bin = bin < 0 ? 0 : (bin > K - 1 ? K - 1 : bin);
        const float icw = T[bin], cw1 = T[bin + 1];
        const float ich = T[K1 + bin], ch1 = T[K1 + bin + 1];
        const float d0 = T[2 * K1 + bin], d1 = T[2 * K1 + bin + 1];
        float y, l;
        bool nd;
        rqs_eval<INV>(x, icw, cw1 - icw, ich, ch1 - ich, d0, d1, y, l, nd);
        if (inside) {
            CO[lane * cs + p] = y;
            ld += l;
            nan_any |= nd;
        }
    }
    return ld;
}

template <int K, bool INV>
__device__ __forceinline__ float uncond_spline(const float *__restrict__ U, float *CO, int cs, int N,
                                               int D, int off, const FlowArgs &a, bool &nan_any) {
    return uncond_spline_w<K, INV>(U, CO, cs, N, D, off, a, nan_any, (int)(threadIdx.x >> 6));
}

#pragma clang fp contract(on)


// Counter-based uniform draws for the base distribution (UniformParticle.sample,
// Energy/Uniform.py:20-36): Philox4x32-10 keyed by seed, counter (row, step, i/4).
__device__ __forceinline__ uint4 philox4x32(uint4 c, uint2 k) {
#pragma unroll
    for (int i = 0; i < 10; ++i) {
        const uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
        const uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
        c = make_uint4(hi1 ^ c.y ^ k.x, lo1, hi0 ^ c.w ^ k.y, lo0);
        k.x += 0x9E3779B9u;
        k.y += 0xBB67AE85u;
    }
    return c;
}

}  // namespace fs
