// Split-bf16 variant of the coupling-flow pass (fs_flow_dims.precision = 1 or 2).
//
// Same algorithm and the same reference semantics as flow_pass_kernel
// (flow_kernels.hip): one workgroup of 8 waves carries 64 chains through all L
// circular-RQS coupling layers; only the conditioner GEMMs change.  gfx950's f32
// MFMA runs at the f32 vector rate (64 FLOP/clk/SIMD), its bf16 MFMA at 16x that.
// Every f32 operand x is carried as P bf16 planes x = x_0 + x_1 (+ x_2), each the
// RNE bf16 of what the previous planes left, and a product is the sum of the
// plane products a_p b_q with p + q < P (6 MFMAs at P = 3, 3 at P = 2).  At P = 3
// the dropped terms are O(2^-24) relative, the f32 rounding level: the GEMM
// error matches the exact-f32 MFMA (tools/split/split_gemm_bench.hip: 2.0e-7 vs
// 1.8e-7 relative to an f64 GEMM chain).  P = 2 keeps 16 significant bits per
// operand (3.4e-6 there).
//
// Layout (transposed GEMMs, C^T = W . X^T): the weights are the A operand,
// streamed from L2 as pre-split 1 KiB fragments (SplitLayout); the activations
// are the B operand, P bf16 planes in LDS with one row per chain; an accumulator
// lane is a chain and its 16 registers are output rows.  Consequences:
//   * epilogues store 4 consecutive output features of one chain per
//     ds_write_b64 (no scattered 2-byte stores);
//   * the final layer's 32-row tiles of two chain halves become lane-per-chain
//     with 16 v_permlane32_swap, no LDS transpose;
//   * each wave owns one 32-row output tile x both chain halves at H = 256, so a
//     weight fragment feeds 2 x (products) MFMAs.
// Transform features are owned per wave in contiguous runs of ceil(N/8); the
// d_K "tail" of a wave's own features is one small GEMM of its own, so no
// cross-wave ordering is needed in the final phase.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "flow_device.h"
#include "flow_layout.h"
#include "fs_internal.h"

namespace fs {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#ifndef FS_SPLIT_RD
#define FS_SPLIT_RD 2  // weight-fragment ring depth (k-steps), a multiple of FS_SPLIT_XB
#endif
#ifndef FS_SPLIT_XB
#define FS_SPLIT_XB 1  // activation-fragment buffers (k-steps read ahead)
#endif


// (H, K) instantiations of the split kernel
#define FS_SPLIT_INSTANCES FS_SCASE(256, 32) FS_SCASE(256, 15) FS_SCASE(128, 32) FS_SCASE(128, 15) FS_SCASE(64, 8) FS_SCASE(32, 5)

// plane products (weight plane p, activation plane q), small terms first
template <int P>
struct SplitProds;
template <>
struct SplitProds<2> {
    static constexpr int n = 3;
    static constexpr int p[3] = {0, 1, 0}, q[3] = {1, 0, 0};
};
template <>
struct SplitProds<3> {
    static constexpr int n = 6;
    static constexpr int p[6] = {0, 1, 2, 0, 1, 0}, q[6] = {2, 1, 0, 1, 0, 0};
};

// two f32 -> P packed bf16x2 words (v_cvt_pk_bf16_f32: RNE; remainders exact in f32)
template <int P>
__device__ __forceinline__ void split2(float v0, float v1, uint32_t (&o)[P]) {
#pragma unroll
    for (int p = 0; p < P; ++p) {
        const f32x2v v = {v0, v1};
        const uint32_t u = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2v));
        o[p] = u;
        if (p + 1 < P) {
            v0 = v0 - __builtin_bit_cast(float, u << 16);
            v1 = v1 - __builtin_bit_cast(float, u & 0xffff0000u);
        }
    }
}

// Work of a wave in an H-output GEMM: CTW output tiles from tile0, RTW chain halves from rt0.
template <int H>
struct SplitWork {
    static constexpr int NT = H / 32;
    static constexpr int RTW = NT >= 8 ? 2 : 1;
    static constexpr int CTW = NT >= 8 ? NT / 8 : 1;
    static constexpr int NUNITS = NT >= 8 ? 8 : 2 * NT;  // active waves
    __device__ static int tile0(int wid) { return NT >= 8 ? wid * CTW : wid % NT; }
    __device__ static int rt0(int wid) { return NT >= 8 ? 0 : wid / NT; }
};

template <int P, int CTW, int RD>
struct SRing {
    u32x4 w[RD][CTW][P];
};

__device__ __forceinline__ u32x4 ld_frag(__amdgpu_buffer_rsrc_t W, int soff) {
    return __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(W, (int)(threadIdx.x & 63) * 16, soff, 0));
}

template <int P, int CTW, int RD>
__device__ __forceinline__ void sring_slot(u32x4 (&w)[CTW][P], __amdgpu_buffer_rsrc_t W, int sec, int kst, int tile0,
                                           int s) {
#pragma unroll
    for (int ct = 0; ct < CTW; ++ct)
#pragma unroll
        for (int p = 0; p < P; ++p) w[ct][p] = ld_frag(W, sec + (((tile0 + ct) * kst + s) * P + p) * 1024);
}

// weight fragments of k-steps 0..RD-1 (independent of the activations: issued
// before the barriers that precede the GEMM)
template <int P, int CTW, int RD>
__device__ __forceinline__ void sring_prologue(SRing<P, CTW, RD> &R, __amdgpu_buffer_rsrc_t W, int sec, int kst,
                                               int tile0) {
#pragma unroll
    for (int u = 0; u < RD; ++u)
        if (u < kst) sring_slot<P, CTW, RD>(R.w[u], W, sec, kst, tile0, u);
}

// Per-feature vectors of an epilogue (folded BatchNorm scale a and shift c) for a wave's
// tiles: lane half h holds features 32 tile + 8 g + 4 h + 0..3.  (Loading them inside
// the preceding GEMM instead, to hide their L2 latency, costs 32 live VGPRs there and
// spills: +27 % pass time.  Without the loads at all the epilogue phase shrinks only
// from 12.2 % to 9.3 % of wave time: its cost is the VALU split and the LDS stores.)
template <int CTW>
struct EpiVec {
    f32x4 a[CTW][4], c[CTW][4];
};

template <int CTW>
__device__ __forceinline__ void load_epi(EpiVec<CTW> &e, const float *__restrict__ av, const float *__restrict__ cv,
                                         int tile0) {
    const int h = (threadIdx.x >> 5) & 1;
#pragma unroll
    for (int ct = 0; ct < CTW; ++ct)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int f0 = 32 * (tile0 + ct) + 8 * g + 4 * h;
            e.c[ct][g] = *(const f32x4 *)(cv + f0);
            if (av) e.a[ct][g] = *(const f32x4 *)(av + f0);
        }
}

// acc[ct][rt] (+)= W[tile0 + ct] . X^T[chain half rt0 + rt] over kst k-steps.
// X planes: XP + q * plane + chain * xsb (bytes).  Weight ring slot = s % RD, the
// activation fragments of step s + XB are read right after the MFMAs of step s.
template <int P, int CTW, int RTW, int RD, bool ACC>
__device__ __forceinline__ void sgemm(const char *XP, int plane, int xsb, __amdgpu_buffer_rsrc_t W, int sec, int kst,
                                      int tile0, int rt0, SRing<P, CTW, RD> &R, f32x16 (&acc)[CTW][RTW]) {
    using PR = SplitProds<P>;
    const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
    if (!ACC)
#pragma unroll
        for (int ct = 0; ct < CTW; ++ct)
#pragma unroll
            for (int rt = 0; rt < RTW; ++rt)
#pragma unroll
                for (int i = 0; i < 16; ++i) acc[ct][rt][i] = 0.f;
    const char *xb0 = XP + (32 * rt0 + r) * xsb + 16 * h;
    constexpr int XB = FS_SPLIT_XB;
    bf16x8 xb[XB][RTW][P];
    auto ldx = [&](int s, bf16x8 (&x)[RTW][P]) {
#pragma unroll
        for (int rt = 0; rt < RTW; ++rt)
#pragma unroll
            for (int q = 0; q < P; ++q) x[rt][q] = *(const bf16x8 *)(xb0 + q * plane + 32 * rt * xsb + 32 * s);
    };
#pragma unroll
    for (int i = 0; i < XB; ++i)
        if (i < kst) ldx(i, xb[i]);
    for (int s0 = 0; s0 < kst; s0 += RD) {
#pragma unroll
        for (int u = 0; u < RD; ++u) {
            const int s = s0 + u;
            if (s < kst) {
#pragma unroll
                for (int ct = 0; ct < CTW; ++ct)
#pragma unroll
                    for (int rt = 0; rt < RTW; ++rt)
#pragma unroll
                        for (int k = 0; k < PR::n; ++k)
                            acc[ct][rt] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                                __builtin_bit_cast(bf16x8, R.w[u][ct][PR::p[k]]), xb[u % XB][rt][PR::q[k]],
                                acc[ct][rt], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
                if (s + XB < kst) ldx(s + XB, xb[u % XB]);
                if (s + RD < kst) sring_slot<P, CTW, RD>(R.w[u], W, sec, kst, tile0, s + RD);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
}

// 16 activations of a transposed tile (lane = chain 32 rt + r, register i = output
// row 8 (i >> 2) + 4 h + (i & 3)) -> P planes, 4 rows per 8-byte word pair
template <int P>
__device__ __forceinline__ void pack_tile(const float (&v)[16], uint2 (&pk)[4][P]) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        uint32_t o0[P], o1[P];
        split2<P>(v[4 * g], v[4 * g + 1], o0);
        split2<P>(v[4 * g + 2], v[4 * g + 3], o1);
#pragma unroll
        for (int p = 0; p < P; ++p) pk[g][p] = make_uint2(o0[p], o1[p]);
    }
}

template <int P>
__device__ __forceinline__ void store_tile(char *XP, int plane, int xsb, int tile, int rt, const uint2 (&pk)[4][P]) {
    const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
    char *row = XP + (32 * rt + r) * xsb + 2 * (32 * tile + 4 * h);
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int p = 0; p < P; ++p) *(uint2 *)(row + p * plane + 16 * g) = pk[g][p];
}

// ResNet epilogue of a wave's tiles into the activation planes: relu(a * acc + c)
// (eval BatchNorm folded, the block's deferred biases re-associated into c, resnet.py:37-50)
// when RELU, else acc + c (the final layer's input).  a, c: prefetched by the GEMM before.
template <int P, int H, int CTW, int RTW, bool RELU>
__device__ __forceinline__ void split_epilogue(char *XP, int plane, int xsb, int tile0, int rt0,
                                               const EpiVec<CTW> &e, const f32x16 (&acc)[CTW][RTW]) {
#pragma unroll
    for (int ct = 0; ct < CTW; ++ct) {
        float a[16], c[16];
#pragma unroll
        for (int g = 0; g < 4; ++g)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                a[4 * g + j] = RELU ? e.a[ct][g][j] : 1.f;
                c[4 * g + j] = e.c[ct][g][j];
            }
#pragma unroll
        for (int rt = 0; rt < RTW; ++rt) {
            float v[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] = RELU ? fmaxf(fmaf(acc[ct][rt][i], a[i], c[i]), 0.f) : acc[ct][rt][i] + c[i];
            uint2 pk[4][P];
            pack_tile<P>(v, pk);
            store_tile<P>(XP, plane, xsb, tile0 + ct, rt0 + rt, pk);
        }
    }
}

#pragma clang fp contract(off)

// Accumulator pair (both chain halves) preset to the final-layer biases of the tile's
// rows (row 8 (i >> 2) + 4 h + (i & 3) in register i): the bias add rides on the MFMAs.
__device__ __forceinline__ void preset_bias(f32x16 (&acc)[1][2], const float *__restrict__ b) {
    const int h = (threadIdx.x >> 5) & 1;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const f32x4 v = *(const f32x4 *)(b + 8 * g + 4 * h);
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[0][0][4 * g + j] = acc[0][1][4 * g + j] = v[j];
    }
}

// Final layer + conditional spline of transform feature j (lane = chain).
template <int P, int K, bool INV, int RD>
__device__ __forceinline__ float split_cond_spline(const char *XP, int plane, int xsb, __amdgpu_buffer_rsrc_t W,
                                                   int sec, int kst, const float *__restrict__ bf, float *CO, int cs,
                                                   int p, float ud_tail, const FlowArgs &a, bool &nan_any, Prof &pf) {
    const int lane = threadIdx.x & 63;
    const float x = CO[lane * cs + p];
    const bool inside = (x >= a.negB) && (x <= a.B);
    SRing<P, 1, RD> R;
    float icw, cw1, ich, ch1;
    int bin = 0;
    {
        float cw[K + 1], ch[K + 1];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
            f32x16 acc[1][2];
            sring_prologue<P, 1, RD>(R, W, sec, kst, t);
            preset_bias(acc, bf + 32 * t);
            sgemm<P, 1, 2, RD, true>(XP, plane, xsb, W, sec, kst, t, 0, R, acc);
            lanes_to_chains(acc[0][0], acc[0][1]);
            pf.mark(PH_FINAL_GEMM);
            float u[K];
#pragma unroll
            for (int k = 0; k < K; ++k) u[k] = tile_row(acc[0][0], acc[0][1], k);
            if (t == 0)
                knots_from_logits<K>(u, cw, kMinWd, a);
            else
                knots_from_logits<K>(u, ch, kMinHd, a);
            pf.mark(PH_SPLINE);
        }
        icw = cw[0], cw1 = cw[1], ich = ch[0], ch1 = ch[1];
#pragma unroll
        for (int k = 1; k < K; ++k) {
            if (x >= (INV ? ch[k] : cw[k])) {
                bin = k;
                icw = cw[k];
                cw1 = cw[k + 1];
                ich = ch[k];
                ch1 = ch[k + 1];
            }
        }
    }
    float ud0 = 0.f, ud1 = ud_tail;  // d_K unless bin + 1 < K
    {
        f32x16 acc[1][2];
        sring_prologue<P, 1, RD>(R, W, sec, kst, 2);
        preset_bias(acc, bf + 64);
        sgemm<P, 1, 2, RD, true>(XP, plane, xsb, W, sec, kst, 2, 0, R, acc);
        lanes_to_chains(acc[0][0], acc[0][1]);
        pf.mark(PH_FINAL_GEMM);
#pragma unroll
        for (int k = 0; k < K; ++k) {
            const float dk = tile_row(acc[0][0], acc[0][1], k);
            if (k == bin) ud0 = dk;
            if (k == bin + 1) ud1 = dk;
        }
    }
    const float d0 = kMinD + softplus_t(ud0);
    const float d1 = kMinD + softplus_t(ud1);
    float y, l;
    bool nd;
    rqs_eval<INV>(x, icw, cw1 - icw, ich, ch1 - ich, d0, d1, y, l, nd);
    pf.mark(PH_SPLINE);
    if (inside) {
        CO[lane * cs + p] = y;
        nan_any |= nd;
        return l;
    }
    return 0.f;
}

#pragma clang fp contract(on)

template <int H, int K, int MODE, int P>
__global__ void __launch_bounds__(kThreads, 2) flow_split_kernel(FlowArgs a) {
    using WK = SplitWork<H>;
    constexpr int CTW = WK::CTW, RTW = WK::RTW, RD = FS_SPLIT_RD;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int N = a.N, D = 2 * N;
    const SplitLds LL = split_lds(N, H, P);
    const SplitLayout SL = split_layout(N, H, a.nb, a.K, P == 3 ? 1 : 2);
    const PackLayout PL = pack_layout(N, H, a.nb, a.K);
    // wave index as a scalar: every weight-fragment offset derived from it is an SGPR
    // (buffer-load soffset), never a per-lane value the compiler would waterfall
    const int tid = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    char *XP = smem;
    const int plane = LL.plane, xsb = LL.xsb;
    float *CO = (float *)(smem + LL.coord);
    float *TL = (float *)(smem + LL.tail);
    float *LDP = (float *)(smem + LL.ld);
    const int cs = LL.cstride, ts = LL.tstride;
    const int64_t row0 = (int64_t)blockIdx.x * kRows;
    const bool row_valid = row0 + lane < a.nrows;
    const bool active = wid < WK::NUNITS;
    const int tile0 = WK::tile0(wid), rt0 = WK::rt0(wid);
    const int j0 = wid * SL.nfw, j1 = min(N, j0 + SL.nfw);

    // ---- inputs -> CO (as flow_pass_kernel)
    if (MODE == MODE_PROPOSE) {
        const int nq = (D + 3) / 4;
        for (int e = tid; e < kRows * nq; e += kThreads) {
            const int rr = e / nq, q = e - rr * nq;
            // Philox key (global chain, step): several steps' proposals in one launch
            // (rows_per_counter > 0) draw exactly what one launch per step would
            const int64_t lr = row0 + rr, rpc = a.rows_per_counter;
            const uint64_t ctr = rpc > 0 ? a.counter + (uint64_t)(lr / rpc) : a.counter;
            const uint64_t gr = (uint64_t)(a.row_offset + (rpc > 0 ? lr % rpc : lr));
            uint4 c = make_uint4((uint32_t)gr, (uint32_t)(gr >> 32) ^ (uint32_t)(ctr >> 32), (uint32_t)ctr,
                                 (uint32_t)q);
            uint4 o = philox4x32(c, make_uint2((uint32_t)a.seed, (uint32_t)(a.seed >> 32)));
            const uint32_t w[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int i = 4 * q + t;
                if (i < D) {
                    const float u = (float)(w[t] >> 8) * 5.9604644775390625e-08f;  // [0,1)
                    CO[rr * cs + i] = u * a.twoB + a.negB;
                }
            }
        }
    } else {
        for (int e = tid; e < kRows * D; e += kThreads) {
            const int rr = e / D, i = e - rr * D;
            const int64_t gr = row0 + rr;
            CO[rr * cs + i] = (gr < a.nrows) ? a.in[gr * D + i] : 0.f;
        }
    }
    float ld = 0.f;
    bool nan_any = false;
    int off = 0;
    __syncthreads();
    Prof pf;

    for (int s = 0; s < a.L; ++s) {
        const int layer = (MODE == MODE_DENSITY) ? a.L - 1 - s : s;
        const float *Pl = a.packed + (int64_t)layer * SL.stride;
        const float *V = Pl + SL.vec;
        const __amdgpu_buffer_rsrc_t W =
            __builtin_amdgcn_make_buffer_rsrc((void *)Pl, (short)0, (int)(SL.stride * 4), 0x00020000);
        if (MODE != MODE_DENSITY) {
            off = (off + N) % D;  // Coupling.inverse rolls first (coupling.py:113-114)
            ld += uncond_spline<K, true>(Pl + SL.unc, CO, cs, N, D, off, a, nan_any);
            pf.mark(PH_UNCOND);
            __syncthreads();
            pf.mark(PH_BARRIER);
        }
        SRing<P, CTW, RD> R;
        if (active) sring_prologue<P, CTW, RD>(R, W, (int)(SL.win * 4), SL.kst_in, tile0);
        // periodic features [cos(s x_id) | sin(s x_id)] (nn.py:120-137) -> planes
        for (int f = wid; f < N; f += kWaves) {
            const float v = CO[lane * cs + (2 * f + off) % D];
            const float sv = a.scale_pf * v;
            uint32_t o[P];
            split2<P>(cosf(sv), sinf(sv), o);
#pragma unroll
            for (int p = 0; p < P; ++p) {
                *(uint16_t *)(XP + p * plane + lane * xsb + 2 * f) = (uint16_t)(o[p] & 0xffffu);
                *(uint16_t *)(XP + p * plane + lane * xsb + 2 * (N + f)) = (uint16_t)(o[p] >> 16);
            }
        }
        for (int c = D + wid; c < 16 * SL.kst_in; c += kWaves)
#pragma unroll
            for (int p = 0; p < P; ++p) *(uint16_t *)(XP + p * plane + lane * xsb + 2 * c) = 0;
        pf.mark(PH_PF);
        __syncthreads();
        pf.mark(PH_BARRIER);

        // ResidualNet (resnet.py:53-104), transposed; hr = residual stream without its
        // deferred biases (pack_vec_kernel re-associates them exactly as for the f32 kernel)
        f32x16 hr[CTW][RTW], acc[CTW][RTW];
        EpiVec<CTW> ev;
        if (active) sgemm<P, CTW, RTW, RD, false>(XP, plane, xsb, W, (int)(SL.win * 4), SL.kst_in, tile0, rt0, R, hr);
        pf.mark(PH_INIT_GEMM);
        for (int jb = 0; jb < a.nb; ++jb) {
            const float *VB = V + PL.v_blocks + (int64_t)4 * H * jb;
            const int w0 = (int)((SL.blocks + jb * SL.block_stride) * 4);
            const int w1 = w0 + (int)(SL.block_stride * 2);
            if (active) sring_prologue<P, CTW, RD>(R, W, w0, SL.kst_h, tile0);
            __syncthreads();  // every wave is done reading X
            pf.mark(PH_BARRIER);
            if (active) load_epi<CTW>(ev, VB, VB + H, tile0);
            if (active) split_epilogue<P, H, CTW, RTW, true>(XP, plane, xsb, tile0, rt0, ev, hr);
            pf.mark(PH_EPI);
            __syncthreads();
            pf.mark(PH_BARRIER);
            if (active) {
                sgemm<P, CTW, RTW, RD, false>(XP, plane, xsb, W, w0, SL.kst_h, tile0, rt0, R, acc);
                sring_prologue<P, CTW, RD>(R, W, w1, SL.kst_h, tile0);
            }
            pf.mark(PH_RES_GEMM);
            __syncthreads();
            pf.mark(PH_BARRIER);
            if (active) load_epi<CTW>(ev, VB + 2 * H, VB + 3 * H, tile0);
            if (active) split_epilogue<P, H, CTW, RTW, true>(XP, plane, xsb, tile0, rt0, ev, acc);
            pf.mark(PH_EPI);
            __syncthreads();
            pf.mark(PH_BARRIER);
            if (active) sgemm<P, CTW, RTW, RD, true>(XP, plane, xsb, W, w1, SL.kst_h, tile0, rt0, R, hr);  // h += Lin1(t)
            pf.mark(PH_RES_GEMM);
        }
        // X <- h + the deferred biases: the final layer's input
        __syncthreads();
        pf.mark(PH_BARRIER);
        if (active) load_epi<CTW>(ev, nullptr, V, tile0);
        if (active) split_epilogue<P, H, CTW, RTW, false>(XP, plane, xsb, tile0, rt0, ev, hr);
        pf.mark(PH_EPI);
        __syncthreads();
        pf.mark(PH_BARRIER);
        // tail: d_K of this wave's features j0 + m (rows m < nfw of the wave's tail tile)
        if (j0 < j1) {
            SRing<P, 1, RD> RT;
            f32x16 t[1][2];
            sring_prologue<P, 1, RD>(RT, W, (int)(SL.wt * 4), SL.kst_h, wid);
            sgemm<P, 1, 2, RD, false>(XP, plane, xsb, W, (int)(SL.wt * 4), SL.kst_h, wid, 0, RT, t);
            lanes_to_chains(t[0][0], t[0][1]);
#pragma unroll
            for (int m = 0; m < (kMaxN + 7) / 8; ++m)
                if (m < j1 - j0) TL[lane * ts + j0 + m] = tile_row(t[0][0], t[0][1], m) + V[PL.v_bt + j0 + m];
        }
        pf.mark(PH_TAIL_GEMM);
        // final layer + conditional spline, feature by feature (TL column j: written by this wave only)
        for (int j = j0; j < j1; ++j) {
            const int p = (2 * j + 1 + off) % D;
            ld += split_cond_spline<P, K, MODE != MODE_DENSITY, RD>(
                XP, plane, xsb, W, (int)((SL.wf + (int64_t)3 * j * SL.kst_h * 256 * P) * 4), SL.kst_h,
                V + PL.v_bf + 96 * j, CO, cs, p, TL[lane * ts + j], a, nan_any, pf);
        }
        if (MODE == MODE_DENSITY) {
            ld += uncond_spline<K, false>(Pl + SL.unc, CO, cs, N, D, off, a, nan_any);
            off = (off + N) % D;  // Coupling.forward rolls last (coupling.py:100-101)
            pf.mark(PH_UNCOND);
        }
        __syncthreads();
        pf.mark(PH_BARRIER);
    }
    pf.flush();

    // ---- outputs (as flow_pass_kernel)
    LDP[wid * kRows + lane] = ld;
    if (nan_any && row_valid && a.err) atomicOr(a.err, 1);
    __syncthreads();
    if (wid == 0) {
        float tot = 0.f;
#pragma unroll
        for (int w = 0; w < kWaves; ++w) tot += LDP[w * kRows + lane];
        float outv = tot;
        if (MODE == MODE_DENSITY && a.add_base) {
            bool inb = true;
            for (int i = 0; i < D; ++i) {
                const float z = CO[lane * cs + i];
                inb = inb && (z >= a.negB) && (z <= a.B);
            }
            outv = tot + (inb ? a.base_lp : -INFINITY);
        }
        if (MODE == MODE_PROPOSE && a.add_base) outv = a.base_lp - tot;  // FS_MH_SINGLE_PASS
        if (row_valid && a.scalar_out) a.scalar_out[row0 + lane] = outv;
    }
    for (int e = tid; e < kRows * D; e += kThreads) {
        const int rr = e / D, i = e - rr * D;
        const int64_t gr = row0 + rr;
        if (gr >= a.nrows) continue;
        const float v = CO[rr * cs + (i + off) % D];
        if (a.out) a.out[gr * D + i] = v;
        if (MODE == MODE_PROPOSE) {
            const float cfg = v + a.B;  // a_ + HALF_BOX in float32 (main_algorithm_1.py:343)
            if (a.config) a.config[gr * D + i] = cfg;
            if (a.centered) a.centered[gr * D + i] = (float)((double)cfg - a.half_width);
        }
    }
}

// ---------------------------------------------------------------------------
// Packing: f32 weights -> P bf16 planes in A-fragment order.
// kind 0: plain linear W[nout][kin]; 1: final layer main (tile = 3 feat + t: widths,
// heights (scaled by wh_scale, as the f32 image), d_0..d_{K-1}); 2: per-wave tail
// (tile = wave w, row m < nfw -> d_K of feature w nfw + m).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint16_t bf16_rne_bits(float f) {
    const uint32_t u = __builtin_bit_cast(uint32_t, f);
    return (uint16_t)((u + 0x7FFFu + ((u >> 16) & 1u)) >> 16);
}

__global__ void pack_split_linear_kernel(uint16_t *__restrict__ dst, const float *__restrict__ src, int kin, int kst,
                                         int ntiles, int nout, int kind, int K, float wh_scale, int P, int nfw, int N) {
    const int64_t total = (int64_t)ntiles * kst * 64 * 8;
    const int P3 = 3 * K + 1;
    for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int j = idx & 7;
        const int lane = (idx >> 3) & 63;
        const int64_t ts = idx >> 9;
        const int s = (int)(ts % kst);
        const int tile = (int)(ts / kst);
        const int k = 16 * s + 8 * (lane >> 5) + j;
        const int rr = lane & 31;
        int64_t row = -1;
        float sc = 1.f;
        if (kind == 0) {
            const int o = 32 * tile + rr;
            row = o < nout ? o : -1;
        } else if (kind == 1) {
            const int feat = tile / 3, t = tile % 3;
            if (rr < K) row = (int64_t)feat * P3 + t * K + rr;
            if (t < 2) sc = wh_scale;
        } else {
            const int feat = tile * nfw + rr;
            if (rr < nfw && feat < N) row = (int64_t)feat * P3 + 3 * K;
        }
        float v = (row >= 0 && k < kin) ? (sc == 1.f ? src[row * kin + k] : src[row * kin + k] * sc) : 0.f;
        uint16_t *o = dst + ((ts * P) * 64 + lane) * 8 + j;
        for (int p = 0; p < P; ++p) {
            const uint16_t b = bf16_rne_bits(v);
            o[(int64_t)p * 64 * 8] = b;
            v -= __builtin_bit_cast(float, (uint32_t)b << 16);
        }
    }
}

template <int H, int K, int MODE, int P>
static hipError_t launch_split_t(const FlowArgs &a, int N, hipStream_t st) {
    auto kfn = flow_split_kernel<H, K, MODE, P>;
    static std::atomic<unsigned long long> attr_set{0};  // per instantiation, bit d = device d
    if (hipError_t e = fs_set_max_lds_once((const void *)kfn, attr_set); e != hipSuccess) return e;
    const int64_t blocks = (a.nrows + kRows - 1) / kRows;
    hipLaunchKernelGGL(kfn, dim3((unsigned)blocks), dim3(kThreads), split_lds(N, H, P).total, st, a);
    return hipGetLastError();
}

template <int MODE, int P>
static hipError_t launch_split_mode(const FlowArgs &a, int N, int H, int K, hipStream_t st) {
#define FS_SCASE(HH, KK) \
    if (H == HH && K == KK) return launch_split_t<HH, KK, MODE, P>(a, N, st);
    FS_SPLIT_INSTANCES
#undef FS_SCASE
    return hipErrorInvalidValue;
}

}  // namespace fs

#ifndef FS_SPLIT_NO_HOST  // (tools/split/unit_split.hip includes the device code only)
using namespace fs;

#ifdef FS_PROF
// this translation unit's phase counters (tools/flow_phases.py --precision)
extern "C" int fs_prof_read_split(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), sizeof(unsigned long long) * 16) != hipSuccess) return 1;
    if (reset) {
        unsigned long long z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof(z)) != hipSuccess) return 1;
    }
    return 0;
}
#endif

bool fs_flow_split_supported(const fs_flow_dims *d, char *why, size_t n) {
    bool ok = false;
#define FS_SCASE(HH, KK) ok |= (d->H == HH && d->K == KK);
    FS_SPLIT_INSTANCES
#undef FS_SCASE
    if (!ok) {
        snprintf(why, n, "precision %d: unsupported (H=%d, K=%d); split instances are listed in FS_SPLIT_INSTANCES "
                 "(flow_split_kernels.hip)", d->precision, d->H, d->K);
        return false;
    }
    if (split_lds(d->N, d->H, split_planes(d->precision)).total > 163840) {
        snprintf(why, n, "precision %d: LDS budget exceeded for N=%d H=%d", d->precision, d->N, d->H);
        return false;
    }
    return true;
}

int64_t fs_flow_split_packed_bytes(const fs_flow_dims *d) {
    return split_layout(d->N, d->H, d->nb, d->K, d->precision).stride * d->L * 4;
}

hipError_t fs_flow_split_pack(const fs_flow_dims *d, const float *raw, float *packed, hipStream_t st) {
    const int N = d->N, H = d->H, nb = d->nb, K = d->K;
    const RawLayout Rw = raw_layout(N, H, nb, K);
    const SplitLayout SL = split_layout(N, H, nb, K, d->precision);
    const PackLayout PL = pack_layout(N, H, nb, K);
    hipError_t e = hipMemsetAsync(packed, 0, (size_t)SL.stride * d->L * 4, st);
    if (e != hipSuccess) return e;
    const float whs = (float)(1.4426950408889634 / sqrt((double)H));
    for (int l = 0; l < d->L; ++l) {
        const float *src = raw + (int64_t)l * Rw.stride;
        float *dst = packed + (int64_t)l * SL.stride;
        auto lin = [&](float *o, const float *w, int kin, int kst, int ntiles, int nout, int kind) {
            const int64_t tot = (int64_t)ntiles * kst * 512;
            int blocks = (int)((tot + 255) / 256);
            if (blocks > 4096) blocks = 4096;
            hipLaunchKernelGGL(pack_split_linear_kernel, dim3(blocks), dim3(256), 0, st, (uint16_t *)o, w, kin, kst,
                               ntiles, nout, kind, K, whs, SL.P, SL.nfw, N);
        };
        lin(dst + SL.win, src + Rw.win, 2 * N, SL.kst_in, H / 32, H, 0);
        for (int jb = 0; jb < nb; ++jb) {
            const float *B = src + Rw.blocks + (int64_t)jb * Rw.block_stride;
            float *o = dst + SL.blocks + (int64_t)jb * SL.block_stride;
            lin(o, B + RawLayout::w0(H), H, SL.kst_h, H / 32, H, 0);
            lin(o + SL.block_stride / 2, B + RawLayout::w1(H), H, SL.kst_h, H / 32, H, 0);
        }
        lin(dst + SL.wf, src + Rw.wf, H, SL.kst_h, 3 * N, 0, 1);
        lin(dst + SL.wt, src + Rw.wf, H, SL.kst_h, 8, N, 2);
        // vectors + unconditional knots: the f32 image's sections, shifted so that
        // PL.vec lands on SL.vec (SL.unc - SL.vec == PL.unc - PL.vec)
        e = fs_flow_pack_vec(dst + (SL.vec - PL.vec), src, d, st);
        if (e != hipSuccess) return e;
    }
    return hipGetLastError();
}

hipError_t fs_flow_split_pass(const FlowArgs &a, int mode, int precision, int N, int H, int K, hipStream_t st) {
    if (precision == 1) {
        if (mode == MODE_DENSITY) return launch_split_mode<MODE_DENSITY, 3>(a, N, H, K, st);
        if (mode == MODE_SAMPLE) return launch_split_mode<MODE_SAMPLE, 3>(a, N, H, K, st);
        return launch_split_mode<MODE_PROPOSE, 3>(a, N, H, K, st);
    }
    if (mode == MODE_DENSITY) return launch_split_mode<MODE_DENSITY, 2>(a, N, H, K, st);
    if (mode == MODE_SAMPLE) return launch_split_mode<MODE_SAMPLE, 2>(a, N, H, K, st);
    return launch_split_mode<MODE_PROPOSE, 2>(a, N, H, K, st);
}
#endif  // FS_SPLIT_NO_HOST
