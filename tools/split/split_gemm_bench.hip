// Microbenchmark: a chain of ResidualNet-shaped GEMMs (H=256, 64 chains per
// workgroup) with f32 operands emulated by P bf16 planes on the gfx950 bf16
// matrix cores (v_mfma_f32_32x32x16_bf16), against the f32 MFMA baseline.
//   x_{g+1} = relu(a_g * (W_g x_g) + c_g)   (eval-BN + ReLU epilogue)
// Layout: transposed GEMM (C^T = W X^T): A operand = weight fragments streamed from
// L2 (pre-split, pre-packed), B operand = activation planes in LDS ([64][256+8] bf16
// per plane), accumulator lane = chain, registers = output features.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 split_gemm_bench.hip -o split_gemm_bench
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <vector>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

#define CHECK(x)                                                                         \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

__device__ unsigned long long g_clk[2];
constexpr int H = 256, ROWS = 64, WAVES = 8, KS = H / 16, XSB = 2 * H + 16;  // bytes per plane row

// products (p, q): weight plane p x activation plane q, p + q < P; small terms first
template <int P>
struct Prods;
template <>
struct Prods<1> {
    static constexpr int n = 1;
    static constexpr int p[1] = {0}, q[1] = {0};
};
template <>
struct Prods<2> {
    static constexpr int n = 3;
    static constexpr int p[3] = {0, 1, 0}, q[3] = {1, 0, 0};
};
template <>
struct Prods<3> {
    static constexpr int n = 6;
    static constexpr int p[6] = {0, 1, 2, 0, 1, 0}, q[6] = {2, 1, 0, 1, 0, 0};
};

__device__ __forceinline__ uint32_t bf_bits_hi(uint32_t packed) { return packed & 0xffff0000u; }
__device__ __forceinline__ uint32_t bf_bits_lo(uint32_t packed) { return packed << 16; }

// split two f32 into P packed bf16x2 words (RNE at every level)
template <int P>
__device__ __forceinline__ void split2(float v0, float v1, uint32_t (&o)[P]) {
#pragma unroll
    for (int p = 0; p < P; ++p) {
        f32x2 v = {v0, v1};
        bf16x2 b = __builtin_convertvector(v, bf16x2);
        const uint32_t u = __builtin_bit_cast(uint32_t, b);
        o[p] = u;
        if (p + 1 < P) {
            v0 = v0 - __builtin_bit_cast(float, bf_bits_lo(u));
            v1 = v1 - __builtin_bit_cast(float, bf_bits_hi(u));
        }
    }
}

template <int P>
__global__ void __launch_bounds__(512, 2)
    chain_split(const uint4 *__restrict__ Wp, const float *__restrict__ ac, const float *__restrict__ xin,
                float *__restrict__ out, int ngemm) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int64_t row0 = (int64_t)blockIdx.x * ROWS;
    // input -> planes
    for (int e = tid; e < ROWS * H / 2; e += 512) {
        const int rr = e / (H / 2), c2 = e % (H / 2);
        const float v0 = xin[(row0 + rr) * H + 2 * c2], v1 = xin[(row0 + rr) * H + 2 * c2 + 1];
        uint32_t o[P];
        split2<P>(v0, v1, o);
#pragma unroll
        for (int p = 0; p < P; ++p) *(uint32_t *)(smem + p * ROWS * XSB + rr * XSB + 4 * c2) = o[p];
    }
    __syncthreads();
    using PR = Prods<P>;
    f32x16 acc[2];
    for (int g = 0; g < ngemm; ++g) {
        const uint4 *Wg = Wp + ((int64_t)(g * WAVES + wid) * KS) * P * 64 + lane;
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[ct][i] = 0.f;
        uint4 wr[3][P];
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int p = 0; p < P; ++p) wr[s][p] = Wg[(s * P + p) * 64];
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            if (s + 2 < KS)
#pragma unroll
                for (int p = 0; p < P; ++p) wr[(s + 2) % 3][p] = Wg[((s + 2) * P + p) * 64];
            bf16x8 xb[2][P];
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                for (int q = 0; q < P; ++q)
                    xb[ct][q] = *(const bf16x8 *)(smem + q * ROWS * XSB + (32 * ct + r) * XSB + 2 * (16 * s + 8 * h));
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                for (int k = 0; k < PR::n; ++k)
                    acc[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                        __builtin_bit_cast(bf16x8, wr[s % 3][PR::p[k]]), xb[ct][PR::q[k]], acc[ct], 0, 0, 0);
        }
        __syncthreads();
        // epilogue: features f = 32*wid + 8*(i>>2) + 4h + (i&3); chain = 32ct + r
        const float *A = ac + (int64_t)g * 2 * H;
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
            const int f0 = 32 * wid + 8 * gq + 4 * h;
            const f32x4 a4 = *(const f32x4 *)(A + f0), c4 = *(const f32x4 *)(A + H + f0);
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                float v[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = fmaxf(fmaf(acc[ct][4 * gq + j], a4[j], c4[j]), 0.f);
                uint32_t o0[P], o1[P];
                split2<P>(v[0], v[1], o0);
                split2<P>(v[2], v[3], o1);
#pragma unroll
                for (int p = 0; p < P; ++p)
                    *(uint2 *)(smem + p * ROWS * XSB + (32 * ct + r) * XSB + 2 * f0) = make_uint2(o0[p], o1[p]);
                if (g == ngemm - 1)
#pragma unroll
                    for (int j = 0; j < 4; ++j) out[(row0 + 32 * ct + r) * H + f0 + j] = v[j];
            }
        }
        __syncthreads();
    }
}

// v2: weight ring of depth RD carried across GEMM boundaries (the next GEMM's first
// k-steps are issued before the barriers), activation fragments one k-step ahead,
// epilogue arithmetic + split before the first barrier, only the LDS stores between
// the two barriers.
template <int P, int RD, bool NOEPI = false>
__global__ void __launch_bounds__(512, 2)
    chain_split2(const uint4 *__restrict__ Wp, const float *__restrict__ ac, const float *__restrict__ xin,
                 float *__restrict__ out, int ngemm) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int64_t row0 = (int64_t)blockIdx.x * ROWS;
    for (int e = tid; e < ROWS * H / 2; e += 512) {
        const int rr = e / (H / 2), c2 = e % (H / 2);
        const float v0 = xin[(row0 + rr) * H + 2 * c2], v1 = xin[(row0 + rr) * H + 2 * c2 + 1];
        uint32_t o[P];
        split2<P>(v0, v1, o);
#pragma unroll
        for (int p = 0; p < P; ++p) *(uint32_t *)(smem + p * ROWS * XSB + rr * XSB + 4 * c2) = o[p];
    }
    using PR = Prods<P>;
    const uint64_t t0c = __builtin_amdgcn_s_memtime(), t0w = wall_clock64();
    const char *xbase = smem + r * XSB + 16 * h;
    auto ldx = [&](int s, bf16x8 (&xb)[2][P]) {
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int q = 0; q < P; ++q) xb[ct][q] = *(const bf16x8 *)(xbase + q * ROWS * XSB + 32 * ct * XSB + 32 * s);
    };
    uint4 wr[RD][P];
    auto ldw = [&](int g, int s, uint4 (&w)[P]) {
        const uint4 *Wg = Wp + ((int64_t)(g * WAVES + wid) * KS + s) * P * 64 + lane;
#pragma unroll
        for (int p = 0; p < P; ++p) w[p] = Wg[p * 64];
    };
#pragma unroll
    for (int s = 0; s < RD; ++s) ldw(0, s, wr[s]);
    __syncthreads();
    f32x16 acc[2];
    for (int g = 0; g < ngemm; ++g) {
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[ct][i] = 0.f;
        bf16x8 xb[2][2][P];
        ldx(0, xb[0]);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
            if (s + 1 < KS) ldx(s + 1, xb[(s + 1) & 1]);
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                for (int k = 0; k < PR::n; ++k)
                    acc[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                        __builtin_bit_cast(bf16x8, wr[s % RD][PR::p[k]]), xb[s & 1][ct][PR::q[k]], acc[ct], 0, 0, 0);
            // refill this ring slot: k-step s + RD of this GEMM, or the next GEMM's first steps
            const int sn = s + RD;
            if (sn < KS)
                ldw(g, sn, wr[s % RD]);
            else if (g + 1 < ngemm)
                ldw(g + 1, sn - KS, wr[s % RD]);
        }
        if (NOEPI && g + 1 < ngemm) continue;
        const float *A = ac + (int64_t)g * 2 * H;
        uint2 pk[4][2][P];
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
            const int f0 = 32 * wid + 8 * gq + 4 * h;
            const f32x4 a4 = *(const f32x4 *)(A + f0), c4 = *(const f32x4 *)(A + H + f0);
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                float v[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = fmaxf(fmaf(acc[ct][4 * gq + j], a4[j], c4[j]), 0.f);
                uint32_t o0[P], o1[P];
                split2<P>(v[0], v[1], o0);
                split2<P>(v[2], v[3], o1);
#pragma unroll
                for (int p = 0; p < P; ++p) pk[gq][ct][p] = make_uint2(o0[p], o1[p]);
                if (g == ngemm - 1)
#pragma unroll
                    for (int j = 0; j < 4; ++j) out[(row0 + 32 * ct + r) * H + f0 + j] = v[j];
            }
        }
        __syncthreads();
#pragma unroll
        for (int gq = 0; gq < 4; ++gq)
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                for (int p = 0; p < P; ++p)
                    *(uint2 *)(smem + p * ROWS * XSB + (32 * ct + r) * XSB + 2 * (32 * wid + 8 * gq + 4 * h)) =
                        pk[gq][ct][p];
        __syncthreads();
    }
    if (tid == 0 && blockIdx.x == 0) {
        const uint64_t t1c = __builtin_amdgcn_s_memtime(), t1w = wall_clock64();
        g_clk[0] = t1c - t0c;
        g_clk[1] = t1w - t0w;
    }
}

// v3 (= v2 with the load placement pinned by sched_barrier): weight ring of depth RD carried across GEMM boundaries (the next GEMM's first
// k-steps are issued before the barriers), activation fragments one k-step ahead,
// epilogue arithmetic + split before the first barrier, only the LDS stores between
// the two barriers.
template <int P, int RD, bool NOEPI = false>
__global__ void __launch_bounds__(512, 2)
    chain_split3(const uint4 *__restrict__ Wp, const float *__restrict__ ac, const float *__restrict__ xin,
                 float *__restrict__ out, int ngemm) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int64_t row0 = (int64_t)blockIdx.x * ROWS;
    for (int e = tid; e < ROWS * H / 2; e += 512) {
        const int rr = e / (H / 2), c2 = e % (H / 2);
        const float v0 = xin[(row0 + rr) * H + 2 * c2], v1 = xin[(row0 + rr) * H + 2 * c2 + 1];
        uint32_t o[P];
        split2<P>(v0, v1, o);
#pragma unroll
        for (int p = 0; p < P; ++p) *(uint32_t *)(smem + p * ROWS * XSB + rr * XSB + 4 * c2) = o[p];
    }
    using PR = Prods<P>;
    const uint64_t t0c = __builtin_amdgcn_s_memtime(), t0w = wall_clock64();
    const char *xbase = smem + r * XSB + 16 * h;
    auto ldx = [&](int s, bf16x8 (&xb)[2][P]) {
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int q = 0; q < P; ++q) xb[ct][q] = *(const bf16x8 *)(xbase + q * ROWS * XSB + 32 * ct * XSB + 32 * s);
    };
    uint4 wr[RD][P];
    auto ldw = [&](int g, int s, uint4 (&w)[P]) {
        const uint4 *Wg = Wp + ((int64_t)(g * WAVES + wid) * KS + s) * P * 64 + lane;
#pragma unroll
        for (int p = 0; p < P; ++p) w[p] = Wg[p * 64];
    };
#pragma unroll
    for (int s = 0; s < RD; ++s) ldw(0, s, wr[s]);
    __syncthreads();
    f32x16 acc[2];
    for (int g = 0; g < ngemm; ++g) {
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[ct][i] = 0.f;
        bf16x8 xb[2][2][P];
        ldx(0, xb[0]);
        ldx(1, xb[1]);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                for (int k = 0; k < PR::n; ++k)
                    acc[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                        __builtin_bit_cast(bf16x8, wr[s % RD][PR::p[k]]), xb[s & 1][ct][PR::q[k]], acc[ct], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            if (s + 2 < KS) ldx(s + 2, xb[s & 1]);
            const int sn = s + RD;
            if (sn < KS)
                ldw(g, sn, wr[s % RD]);
            else if (g + 1 < ngemm)
                ldw(g + 1, sn - KS, wr[s % RD]);
            __builtin_amdgcn_sched_barrier(0);
        }
        if (NOEPI && g + 1 < ngemm) continue;
        const float *A = ac + (int64_t)g * 2 * H;
        uint2 pk[4][2][P];
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
            const int f0 = 32 * wid + 8 * gq + 4 * h;
            const f32x4 a4 = *(const f32x4 *)(A + f0), c4 = *(const f32x4 *)(A + H + f0);
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                float v[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = fmaxf(fmaf(acc[ct][4 * gq + j], a4[j], c4[j]), 0.f);
                uint32_t o0[P], o1[P];
                split2<P>(v[0], v[1], o0);
                split2<P>(v[2], v[3], o1);
#pragma unroll
                for (int p = 0; p < P; ++p) pk[gq][ct][p] = make_uint2(o0[p], o1[p]);
                if (g == ngemm - 1)
#pragma unroll
                    for (int j = 0; j < 4; ++j) out[(row0 + 32 * ct + r) * H + f0 + j] = v[j];
            }
        }
        __syncthreads();
#pragma unroll
        for (int gq = 0; gq < 4; ++gq)
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                for (int p = 0; p < P; ++p)
                    *(uint2 *)(smem + p * ROWS * XSB + (32 * ct + r) * XSB + 2 * (32 * wid + 8 * gq + 4 * h)) =
                        pk[gq][ct][p];
        __syncthreads();
    }
    if (tid == 0 && blockIdx.x == 0) {
        const uint64_t t1c = __builtin_amdgcn_s_memtime(), t1w = wall_clock64();
        g_clk[0] = t1c - t0c;
        g_clk[1] = t1w - t0w;
    }
}

// v4 (experiment: loads switched off) (= v2 with the load placement pinned by sched_barrier): weight ring of depth RD carried across GEMM boundaries (the next GEMM's first
// k-steps are issued before the barriers), activation fragments one k-step ahead,
// epilogue arithmetic + split before the first barrier, only the LDS stores between
// the two barriers.
template <int P, int RD, bool NOEPI, bool NOW, bool NOX>
__global__ void __launch_bounds__(512, 2)
    chain_split4(const uint4 *__restrict__ Wp, const float *__restrict__ ac, const float *__restrict__ xin,
                 float *__restrict__ out, int ngemm) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int64_t row0 = (int64_t)blockIdx.x * ROWS;
    for (int e = tid; e < ROWS * H / 2; e += 512) {
        const int rr = e / (H / 2), c2 = e % (H / 2);
        const float v0 = xin[(row0 + rr) * H + 2 * c2], v1 = xin[(row0 + rr) * H + 2 * c2 + 1];
        uint32_t o[P];
        split2<P>(v0, v1, o);
#pragma unroll
        for (int p = 0; p < P; ++p) *(uint32_t *)(smem + p * ROWS * XSB + rr * XSB + 4 * c2) = o[p];
    }
    using PR = Prods<P>;
    const uint64_t t0c = __builtin_amdgcn_s_memtime(), t0w = wall_clock64();
    const char *xbase = smem + r * XSB + 16 * h;
    auto ldx = [&](int s, bf16x8 (&xb)[2][P]) {
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int q = 0; q < P; ++q) xb[ct][q] = *(const bf16x8 *)(xbase + q * ROWS * XSB + 32 * ct * XSB + 32 * s);
    };
    uint4 wr[RD][P];
    auto ldw = [&](int g, int s, uint4 (&w)[P]) {
        const uint4 *Wg = Wp + ((int64_t)(g * WAVES + wid) * KS + s) * P * 64 + lane;
#pragma unroll
        for (int p = 0; p < P; ++p) w[p] = Wg[p * 64];
    };
#pragma unroll
    for (int s = 0; s < RD; ++s) ldw(0, s, wr[s]);
    __syncthreads();
    f32x16 acc[2];
    for (int g = 0; g < ngemm; ++g) {
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[ct][i] = 0.f;
        bf16x8 xb[2][2][P];
        ldx(0, xb[0]);
        ldx(1, xb[1]);
#pragma unroll
        for (int s = 0; s < KS; ++s) {
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                for (int k = 0; k < PR::n; ++k)
                    acc[ct] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                        __builtin_bit_cast(bf16x8, wr[s % RD][PR::p[k]]), xb[s & 1][ct][PR::q[k]], acc[ct], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
            if (!NOX && s + 2 < KS) ldx(s + 2, xb[s & 1]);
            const int sn = s + RD;
            if (NOW) {
            } else if (sn < KS)
                ldw(g, sn, wr[s % RD]);
            else if (g + 1 < ngemm)
                ldw(g + 1, sn - KS, wr[s % RD]);
            __builtin_amdgcn_sched_barrier(0);
        }
        if (NOEPI && g + 1 < ngemm) continue;
        const float *A = ac + (int64_t)g * 2 * H;
        uint2 pk[4][2][P];
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
            const int f0 = 32 * wid + 8 * gq + 4 * h;
            const f32x4 a4 = *(const f32x4 *)(A + f0), c4 = *(const f32x4 *)(A + H + f0);
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                float v[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = fmaxf(fmaf(acc[ct][4 * gq + j], a4[j], c4[j]), 0.f);
                uint32_t o0[P], o1[P];
                split2<P>(v[0], v[1], o0);
                split2<P>(v[2], v[3], o1);
#pragma unroll
                for (int p = 0; p < P; ++p) pk[gq][ct][p] = make_uint2(o0[p], o1[p]);
                if (g == ngemm - 1)
#pragma unroll
                    for (int j = 0; j < 4; ++j) out[(row0 + 32 * ct + r) * H + f0 + j] = v[j];
            }
        }
        __syncthreads();
#pragma unroll
        for (int gq = 0; gq < 4; ++gq)
#pragma unroll
            for (int ct = 0; ct < 2; ++ct)
#pragma unroll
                for (int p = 0; p < P; ++p)
                    *(uint2 *)(smem + p * ROWS * XSB + (32 * ct + r) * XSB + 2 * (32 * wid + 8 * gq + 4 * h)) =
                        pk[gq][ct][p];
        __syncthreads();
    }
    if (tid == 0 && blockIdx.x == 0) {
        const uint64_t t1c = __builtin_amdgcn_s_memtime(), t1w = wall_clock64();
        g_clk[0] = t1c - t0c;
        g_clk[1] = t1w - t0w;
    }
}

// f32 MFMA baseline with the same structure (A = weights f32 fragments, B = X^T f32 from LDS)
__global__ void __launch_bounds__(512, 2)
    chain_f32(const f32x4 *__restrict__ Wp, const float *__restrict__ ac, const float *__restrict__ xin,
              float *__restrict__ out, int ngemm) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float *X = (float *)smem;
    constexpr int XS = H + 4;
    const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63, r = lane & 31, h = lane >> 5;
    const int64_t row0 = (int64_t)blockIdx.x * ROWS;
    for (int e = tid; e < ROWS * H; e += 512) X[(e / H) * XS + e % H] = xin[row0 * H + e];
    __syncthreads();
    f32x16 acc[2];
    constexpr int KG = H / 8;
    for (int g = 0; g < ngemm; ++g) {
        const f32x4 *Wg = Wp + ((int64_t)(g * WAVES + wid) * KG) * 64 + lane;
#pragma unroll
        for (int ct = 0; ct < 2; ++ct)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[ct][i] = 0.f;
        f32x4 wr[4];
#pragma unroll
        for (int s = 0; s < 3; ++s) wr[s] = Wg[s * 64];
#pragma unroll
        for (int s = 0; s < KG; ++s) {
            if (s + 3 < KG) wr[(s + 3) % 4] = Wg[(s + 3) * 64];
            f32x4 xb[2];
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) xb[ct] = *(const f32x4 *)(X + (32 * ct + r) * XS + 8 * s + 4 * h);
#pragma unroll
            for (int j = 0; j < 4; ++j)
#pragma unroll
                for (int ct = 0; ct < 2; ++ct)
                    acc[ct] = __builtin_amdgcn_mfma_f32_32x32x2f32(wr[s % 4][j], xb[ct][j], acc[ct], 0, 0, 0);
        }
        __syncthreads();
        const float *A = ac + (int64_t)g * 2 * H;
#pragma unroll
        for (int gq = 0; gq < 4; ++gq) {
            const int f0 = 32 * wid + 8 * gq + 4 * h;
            const f32x4 a4 = *(const f32x4 *)(A + f0), c4 = *(const f32x4 *)(A + H + f0);
#pragma unroll
            for (int ct = 0; ct < 2; ++ct) {
                f32x4 v;
#pragma unroll
                for (int j = 0; j < 4; ++j) v[j] = fmaxf(fmaf(acc[ct][4 * gq + j], a4[j], c4[j]), 0.f);
                *(f32x4 *)(X + (32 * ct + r) * XS + f0) = v;
                if (g == ngemm - 1) *(f32x4 *)(out + (row0 + 32 * ct + r) * H + f0) = v;
            }
        }
        __syncthreads();
    }
}

static uint16_t bf16_rne(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    u += 0x7FFF + ((u >> 16) & 1);
    return (uint16_t)(u >> 16);
}
static float bf16_f(uint16_t b) {
    uint32_t u = (uint32_t)b << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

int main(int argc, char **argv) {
    const int nwg = argc > 1 ? atoi(argv[1]) : 1024;
    const int ngemm = argc > 2 ? atoi(argv[2]) : 64;
    const int64_t C = (int64_t)nwg * ROWS;
    srand(1);
    auto urand = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
    std::vector<float> W((size_t)ngemm * H * H), ac((size_t)ngemm * 2 * H), x((size_t)C * H);
    for (auto &w : W) w = urand() / 16.f;
    for (int g = 0; g < ngemm; ++g)
        for (int f = 0; f < H; ++f) {
            ac[g * 2 * H + f] = 0.8f + 0.6f * (urand() + 1) / 2;  // a ~ BN scale
            ac[g * 2 * H + H + f] = 0.3f * urand();
        }
    for (auto &v : x) v = fabsf(urand());
    // packed f32 fragments: [g][t][kg][lane][4]: lane (r, h) -> W[32t + r][8kg + 4h + j]
    std::vector<float> Wf((size_t)ngemm * 8 * (H / 8) * 64 * 4);
    for (int g = 0; g < ngemm; ++g)
        for (int t = 0; t < 8; ++t)
            for (int kg = 0; kg < H / 8; ++kg)
                for (int l = 0; l < 64; ++l)
                    for (int j = 0; j < 4; ++j)
                        Wf[((((size_t)g * 8 + t) * (H / 8) + kg) * 64 + l) * 4 + j] =
                            W[(size_t)g * H * H + (32 * t + (l & 31)) * H + 8 * kg + 4 * (l >> 5) + j];
    float *dW32, *dac, *dx, *dout;
    CHECK(hipMalloc(&dW32, Wf.size() * 4));
    CHECK(hipMalloc(&dac, ac.size() * 4));
    CHECK(hipMalloc(&dx, x.size() * 4));
    CHECK(hipMalloc(&dout, x.size() * 4));
    CHECK(hipMemcpy(dW32, Wf.data(), Wf.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dac, ac.data(), ac.size() * 4, hipMemcpyHostToDevice));
    CHECK(hipMemcpy(dx, x.data(), x.size() * 4, hipMemcpyHostToDevice));
    // CPU reference for workgroup 0 in double
    std::vector<double> ref((size_t)ROWS * H), cur((size_t)ROWS * H);
    for (int i = 0; i < ROWS * H; ++i) cur[i] = x[i];
    for (int g = 0; g < ngemm; ++g) {
        for (int rr = 0; rr < ROWS; ++rr)
            for (int f = 0; f < H; ++f) {
                double s = 0;
                for (int k = 0; k < H; ++k) s += (double)W[(size_t)g * H * H + f * H + k] * cur[rr * H + k];
                // f32 epilogue on the f64 sum: matches the device's fmaf after rounding the sum
                const double v = s * ac[g * 2 * H + f] + ac[g * 2 * H + H + f];
                ref[rr * H + f] = v > 0 ? v : 0;
            }
        cur = ref;
    }
    std::vector<float> got((size_t)ROWS * H);
    auto report = [&](const char *name, float ms) {
        CHECK(hipMemcpy(got.data(), dout, got.size() * 4, hipMemcpyDeviceToHost));
        double mx = 0, rmax = 0;
        for (int i = 0; i < ROWS * H; ++i) {
            mx = fmax(mx, fabs(got[i] - ref[i]));
            rmax = fmax(rmax, fabs(ref[i]));
        }
        const double flop = 2.0 * C * H * H * ngemm;
        printf("{\"kernel\": \"%s\", \"ms\": %.3f, \"f32_equiv_tflops\": %.1f, \"max_abs_err\": %.3e, \"rel_to_max\": %.3e}\n",
               name, ms, flop / (ms * 1e-3) / 1e12, mx, mx / rmax);
        fflush(stdout);
    };
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    auto timeit = [&](auto launch) {
        launch();
        CHECK(hipDeviceSynchronize());
        CHECK(hipEventRecord(e0));
        for (int it = 0; it < 3; ++it) launch();
        CHECK(hipEventRecord(e1));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        return ms / 3;
    };
    {
        const int lds = ROWS * (H + 4) * 4;
        CHECK(hipFuncSetAttribute((const void *)chain_f32, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        float ms = timeit([&] {
            hipLaunchKernelGGL(chain_f32, dim3(nwg), dim3(512), lds, 0, (const f32x4 *)dW32, dac, dx, dout, ngemm);
        });
        report("f32_mfma", ms);
    }
    auto run_split = [&](auto kern, int P, const char *name) {
        std::vector<uint16_t> Wb((size_t)ngemm * 8 * KS * P * 64 * 8);
        for (int g = 0; g < ngemm; ++g)
            for (int t = 0; t < 8; ++t)
                for (int s = 0; s < KS; ++s)
                    for (int l = 0; l < 64; ++l)
                        for (int j = 0; j < 8; ++j) {
                            float v = W[(size_t)g * H * H + (32 * t + (l & 31)) * H + 16 * s + 8 * (l >> 5) + j];
                            for (int p = 0; p < P; ++p) {
                                const uint16_t b = bf16_rne(v);
                                Wb[(((((size_t)g * 8 + t) * KS + s) * P + p) * 64 + l) * 8 + j] = b;
                                v -= bf16_f(b);
                            }
                        }
        void *dWb;
        CHECK(hipMalloc(&dWb, Wb.size() * 2));
        CHECK(hipMemcpy(dWb, Wb.data(), Wb.size() * 2, hipMemcpyHostToDevice));
        const int lds = P * ROWS * XSB;
        CHECK(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
        float ms = timeit([&] {
            hipLaunchKernelGGL(kern, dim3(nwg), dim3(512), lds, 0, (const uint4 *)dWb, dac, dx, dout, ngemm);
        });
        report(name, ms);
        unsigned long long clk[2];
        CHECK(hipMemcpyFromSymbol(clk, HIP_SYMBOL(g_clk), sizeof(clk)));
        int wr = 0;
        CHECK(hipDeviceGetAttribute(&wr, hipDeviceAttributeWallClockRate, 0));
        if (clk[1]) printf("   block0: %llu shader clks over %.1f us -> %.2f GHz\n", clk[0], clk[1] * 1e3 / wr, clk[0] / (clk[1] * 1e3 / wr) / 1e3);
        CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_clk), (unsigned long long[2]){0, 0}, sizeof(clk)));
        CHECK(hipFree(dWb));
    };
    run_split(chain_split3<3, 4>, 3, "bf16x6_v3_rd4");
    run_split(chain_split4<3, 4, true, true, false>, 3, "bf16x6_noepi_noW");
    run_split(chain_split4<3, 4, true, false, true>, 3, "bf16x6_noepi_noX");
    run_split(chain_split4<3, 4, true, true, true>, 3, "bf16x6_noepi_noW_noX");
    run_split(chain_split4<1, 4, true, true, true>, 1, "bf16x1_noepi_noW_noX");
    return 0;
}
