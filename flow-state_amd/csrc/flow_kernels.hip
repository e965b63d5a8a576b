// MI355X (gfx950) kernels for the circular rational-quadratic-spline coupling
// flow of the NF-proposed MH hot path.
//
// One workgroup = 8 waves = 64 chains (rows) carried through ALL L coupling
// layers of a pass without touching HBM between layers:
//   * the chain coordinates live in LDS (CO), the roll of every coupling
//     (coupling.py:100-101, :113-114) is an index offset, never a copy;
//   * the conditioner ResidualNet (resnet.py:53-104) runs as v_mfma_f32_32x32x2_f32
//     GEMMs: activations X [64 x H] in LDS (16-byte-slot XOR swizzle, conflict-free
//     ds_read_b128 A fragments), weights streamed from L2 as pre-packed 1 KiB
//     fragments (one dwordx4 per lane feeds 4 MFMAs), the residual stream h in
//     the accumulator registers of the wave that owns its columns;
//   * bias / eval-BatchNorm / ReLU / residual add are fused GEMM epilogues;
//   * the final layer is computed feature by feature: widths and heights as two
//     transposed 32-column tiles turned lane-per-chain by v_permlane32_swap, then
//     only the two derivative logits each chain's bin needs (per-lane dot products
//     with gathered rows); one lane = one chain for softmax / cumsum / bin search /
//     rational-quadratic map / log-det (splines.py:16-222);
//   * the unconditional spline (coupling.py:176-265) uses knots precomputed at
//     pack time (they are batch independent).
// Reference sign/shape quirks are kept: circular-tail derivative pad that ties
// nothing (splines.py:35-37), searchsorted eps on the last knot, the /sqrt(H)
// scaling of widths and heights (coupling.py:340-342), -D*log(2B) base density.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include <atomic>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include "flow_device.h"
#include "flow_layout.h"
#include "fs_internal.h"

namespace fs {

// eval-BatchNorm (folded) + ReLU epilogue of a ResNet accumulator
#define FS_EPI(v, a, b) fmaxf(fmaf((v), (a), (b)), 0.f)
#define FS_GROUP_BARRIER(c, ph) group_barrier((c), (ph))
#ifndef FS_RPD
#define FS_RPD 3  // weight-fragment ring depth of the ResNet GEMMs
#endif

// (H, K) instantiations: A1 of main_algorithm_1.py:59-67 (H=256, K=32), A2 of
// main_algorithm_2.py:43-51 (H=128, K=15), and the small test/golden shapes.
#define FS_FLOW_INSTANCES \
    FS_CASE(256, 32) FS_CASE(256, 15) FS_CASE(128, 32) FS_CASE(128, 15) FS_CASE(64, 8) FS_CASE(32, 5) FS_CASE(32, 8)

// ---------------------------------------------------------------------------
// GEMM: acc[rt][ct] (32x32 tiles, rows 32*rt.., cols 32*(tile0+ct)..) =
//       X[64 x 8*kg] . Bpacked[tiles tile0..tile0+CT-1]
// Operands of k-group g live in ring slot g % PD; the loads of group g+PD are
// issued right after the MFMAs of group g (sched_barrier keeps hipcc from
// sinking them next to their use), so PD-1 groups of MFMAs (>= 1024 cycles)
// cover the L2 latency of every weight fragment at one wave per SIMD.
// ---------------------------------------------------------------------------
// B-operand ring: weight fragments of k-groups 0..PD-1 can be issued BEFORE the
// barrier that precedes a GEMM (they do not depend on the activation tile),
// so their L2 latency overlaps the epilogue of the previous GEMM.
template <int CT, int PD>
struct BRing {
    f32x4 rb[PD][CT];
};

__device__ __forceinline__ f32x4 ldb_frag(__amdgpu_buffer_rsrc_t W, int voff, int soff) {
    return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(W, voff, soff, 0));
}

template <int CT, int PD>
__device__ __forceinline__ void b_prologue(BRing<CT, PD> &br, __amdgpu_buffer_rsrc_t W, int sec, int kg, int ct0) {
    const int voff = (ct0 * kg * 64 + (int)(threadIdx.x & 63)) * 16;
#pragma unroll
    for (int s = 0; s < PD; ++s)
        if (s < kg)
#pragma unroll
            for (int ct = 0; ct < CT; ++ct) br.rb[s][ct] = ldb_frag(W, voff, sec + (ct * kg + s) * 1024);
}

// acc[rt][ct] = X[rows 32*(rt0+rt)..+31][0 : 8*kg] . B[tile ct0+ct]  (TR = false: a ResidualNet
// section, fragment values in kResPos order)
// W: buffer descriptor of the layer's packed parameters; sec: byte offset of
// this GEMM's fragment section (wave-uniform).  32-bit offsets only: no 64-bit
// pointer per ring slot to keep live.  Operands of k-group g live in ring slot
// g % PD; the loads of group g+PD are issued right after the MFMAs of group g
// (sched_barrier keeps hipcc from sinking them next to their use).
// ACC = true accumulates onto the incoming acc (the residual add of a ResidualBlock
// done by the matrix cores instead of 16 VALU adds per tile).  TR = true computes the
// transposed tile, acc^T = B^T . X^T (the packed weight fragment is a valid A operand
// as it stands): accumulator lane = chain, registers = output columns.
// The ResidualNet sections (initial layer, blocks) store each lane's four k values of a
// fragment in the order j = 0, 2, 1, 3 (pack kind 0): element j sits at kResPos[j].  The
// 32x32x2 GEMMs read all four either way; the 16-row trunk's lanes need j = (h, 2 + h),
// which this order makes one 8-byte load.  The final-layer sections keep 0, 1, 2, 3.
__device__ constexpr int kResPos[4] = {0, 2, 1, 3};

template <int XS, int RT, int CT, int PD, bool ACC = false, bool TR = false>
__device__ __forceinline__ void gemm_run(const float *__restrict__ X, __amdgpu_buffer_rsrc_t W, int sec, int kg,
                                         int rt0, int ct0, BRing<CT, PD> &br, f32x16 (&acc)[RT][CT]) {
    const int lane = threadIdx.x & 63;
    const int h = lane >> 5, r = lane & 31;
    if (!ACC)
#pragma unroll
        for (int rt = 0; rt < RT; ++rt)
#pragma unroll
            for (int ct = 0; ct < CT; ++ct)
#pragma unroll
                for (int i = 0; i < 16; ++i) acc[rt][ct][i] = 0.f;
    const float *xa = X + (32 * rt0 + r) * XS + 4 * h;
    const int voff = (ct0 * kg * 64 + lane) * 16;
    f32x4 ra[PD][RT];
#pragma unroll
    for (int s = 0; s < PD; ++s)
        if (s < kg)
#pragma unroll
            for (int rt = 0; rt < RT; ++rt) ra[s][rt] = *(const f32x4 *)(xa + rt * 32 * XS + 8 * s);
    for (int g0 = 0; g0 < kg; g0 += PD) {
#pragma unroll
        for (int s = 0; s < PD; ++s) {
            const int g = g0 + s;
            if (g < kg) {
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
                        for (int rt = 0; rt < RT; ++rt)
                            acc[rt][ct] = TR ? __builtin_amdgcn_mfma_f32_32x32x2f32(br.rb[s][ct][j], ra[s][rt][j],
                                                                                   acc[rt][ct], 0, 0, 0)
                                             : __builtin_amdgcn_mfma_f32_32x32x2f32(ra[s][rt][j],
                                                                                   br.rb[s][ct][kResPos[j]],
                                                                                   acc[rt][ct], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
                const int gn = g + PD;
                if (gn < kg) {
#pragma unroll
                    for (int rt = 0; rt < RT; ++rt) ra[s][rt] = *(const f32x4 *)(xa + rt * 32 * XS + 8 * gn);
#pragma unroll
                    for (int ct = 0; ct < CT; ++ct) br.rb[s][ct] = ldb_frag(W, voff, sec + (ct * kg + gn) * 1024);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
}

template <int XS, int RT, int CT, int PD, bool ACC = false, bool TR = false>
__device__ __forceinline__ void gemm64(const float *__restrict__ X, __amdgpu_buffer_rsrc_t W, int sec, int kg,
                                       int rt0, int ct0, f32x16 (&acc)[RT][CT]) {
    BRing<CT, PD> br;
    b_prologue<CT, PD>(br, W, sec, kg, ct0);
    gemm_run<XS, RT, CT, PD, ACC, TR>(X, W, sec, kg, rt0, ct0, br, acc);
}

// Transposed final-layer tile of both chain halves with the column biases preset in the
// accumulators (register i of lane half h = column 8 (i >> 2) + 4 h + (i & 3)), turned
// lane-per-chain by 16 v_permlane32_swap: row k of the result is tile_row(t[0][0], t[1][0], k).
template <int XS, int FPD = 4>
__device__ __forceinline__ void final_tile(const float *__restrict__ X, __amdgpu_buffer_rsrc_t W, int sec, int kg,
                                           int tile, const float *__restrict__ b, f32x16 (&t)[2][1]) {
    const int h = (threadIdx.x >> 5) & 1;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const f32x4 v = *(const f32x4 *)(b + 8 * g + 4 * h);
#pragma unroll
        for (int j = 0; j < 4; ++j) t[0][0][4 * g + j] = t[1][0][4 * g + j] = v[j];
    }
    gemm64<XS, 2, 1, FPD, true, true>(X, W, sec, kg, 0, tile, t);
    lanes_to_chains(t[0][0], t[1][0]);
}

// The same for K <= 16 with two transform features per tile: feature 2p in columns
// 0..15, feature 2p+1 in 16..31 (ba, bb: their bias rows), so the widths / heights GEMMs
// of a pair cost one tile each instead of two half-empty ones.
template <int XS, int FPD = 4>
__device__ __forceinline__ void final_tile_pair(const float *__restrict__ X, __amdgpu_buffer_rsrc_t W, int sec,
                                                int kg, int tile, const float *__restrict__ ba,
                                                const float *__restrict__ bb, f32x16 (&t)[2][1]) {
    const int h = (threadIdx.x >> 5) & 1;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const f32x4 v = *(const f32x4 *)((g < 2 ? ba + 8 * g : bb + 8 * (g - 2)) + 4 * h);
#pragma unroll
        for (int j = 0; j < 4; ++j) t[0][0][4 * g + j] = t[1][0][4 * g + j] = v[j];
    }
    gemm64<XS, 2, 1, FPD, true, true>(X, W, sec, kg, 0, tile, t);
    lanes_to_chains(t[0][0], t[1][0]);
}

// final_tile_pair for the 32 chains of X's first row tile, duplicated into both lane halves
// (lane l and l + 32: chain l)
template <int XS, int FPD = 4>
__device__ __forceinline__ void final_tile_pair32(const float *__restrict__ X, __amdgpu_buffer_rsrc_t W, int sec,
                                                  int kg, int tile, const float *__restrict__ ba,
                                                  const float *__restrict__ bb, f32x16 (&t)[2][1]) {
    const int h = (threadIdx.x >> 5) & 1;
    f32x16 t1[1][1];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const f32x4 v = *(const f32x4 *)((g < 2 ? ba + 8 * g : bb + 8 * (g - 2)) + 4 * h);
#pragma unroll
        for (int j = 0; j < 4; ++j) t1[0][0][4 * g + j] = v[j];
    }
    gemm64<XS, 1, 1, FPD, true, true>(X, W, sec, kg, 0, tile, t1);
    t[0][0] = t1[0][0];
    t[1][0] = t1[0][0];
    lanes_to_chains(t[0][0], t[1][0]);
}

// final_tile for the 32 chains of X's first row tile, duplicated into both lane halves
// (K > 16: one transform feature per tile; the wide path's 32-row final blocks)
template <int XS, int FPD = 4>
__device__ __forceinline__ void final_tile32(const float *__restrict__ X, __amdgpu_buffer_rsrc_t W, int sec, int kg,
                                             int tile, const float *__restrict__ b, f32x16 (&t)[2][1]) {
    const int h = (threadIdx.x >> 5) & 1;
    f32x16 t1[1][1];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        const f32x4 v = *(const f32x4 *)(b + 8 * g + 4 * h);
#pragma unroll
        for (int j = 0; j < 4; ++j) t1[0][0][4 * g + j] = v[j];
    }
    gemm64<XS, 1, 1, FPD, true, true>(X, W, sec, kg, 0, tile, t1);
    t[0][0] = t1[0][0];
    t[1][0] = t1[0][0];
    lanes_to_chains(t[0][0], t[1][0]);
}

#pragma clang fp contract(off)

// Derivative-row gathers of cond_spline: QB quads (16-byte pieces of rows bin and
// bin + 1) per batch, two batches in flight.
template <int QB>
struct DRows {
    f32x4 a[QB], b[QB];
};

template <int QB, int K>
__device__ __forceinline__ void drows_issue(DRows<QB> &g, __amdgpu_buffer_rsrc_t W, int voff, int dsec, int q0) {
#pragma unroll
    for (int i = 0; i < QB; ++i) {
        g.a[i] = ldb_frag(W, voff, dsec + (q0 + i) * (K + 1) * 16);
        g.b[i] = ldb_frag(W, voff + 16, dsec + (q0 + i) * (K + 1) * 16);
    }
}

// u0 += row_bin . h, u1 += row_bin+1 . h over QB quads; even and odd k accumulate in
// the two halves of a float2 (v_pk_fma_f32 straight on the loaded register pairs)
template <int QB>
__device__ __forceinline__ void drows_dot(const DRows<QB> &g, const float *xr, int q0, f32x2 &u0, f32x2 &u1) {
#pragma unroll
    for (int i = 0; i < QB; ++i) {
        const f32x4 hv = *(const f32x4 *)(xr + 4 * (q0 + i));
        u0 = __builtin_elementwise_fma(g.a[i].xy, hv.xy, u0);
        u1 = __builtin_elementwise_fma(g.b[i].xy, hv.xy, u1);
        u0 = __builtin_elementwise_fma(g.a[i].zw, hv.zw, u0);
        u1 = __builtin_elementwise_fma(g.b[i].zw, hv.zw, u1);
    }
}

// Final layer + conditional spline of transform feature j for the 64 chains of the
// wave (lane = chain).  Widths and heights: two transposed single-tile GEMMs (all K
// logits of each feed the softmax / cumsum).  Derivatives: the reference computes
// all K+1 logits (coupling.py:327-342) but the spline reads only d_bin and d_bin+1
// (splines.py:157-158), so each lane takes the dot products of its chain's hidden
// vector (its X row) with those two rows of the final layer, gathered from the
// [H/4][K+1][4] `wd` section.  That replaces the 32-column derivative tile and the
// d_K tail GEMM: 9 % of the pass's MFMA work.  The bin comes from the knots of the
// searched tile (cumwidths in the density direction, cumheights when inverting), so
// that tile runs first and the first gathers are in flight during the other tile's GEMM.
template <int XS, int H, int K, bool INV, int FPD = 4>
__device__ __forceinline__ float cond_spline(const float *__restrict__ X, __amdgpu_buffer_rsrc_t W, int sec,
                                             int kg, const float *__restrict__ bf, int dsec,
                                             const float *__restrict__ bd, float *CO, int cs, int p, int j,
                                             const FlowArgs &a, bool &nan_any, Prof &pf) {
    constexpr int NQ = H / 4;                   // quads of the hidden vector
    constexpr int QB = NQ >= 8 ? 4 : NQ / 2;    // quads per gather batch
    const int lane = threadIdx.x & 63;
    const float x = CO[lane * cs + p];
    const bool inside = (x >= a.negB) && (x <= a.B);
    constexpr int TS = INV ? 1 : 0;  // searched tile: 0 widths, 1 heights
    float ks[K + 1];
    {
        f32x16 acc[2][1];
        final_tile<XS, FPD>(X, W, sec, kg, 2 * j + TS, bf + 32 * TS, acc);
        pf.mark(PH_FINAL_GEMM);
        float u[K];
#pragma unroll
        for (int k = 0; k < K; ++k) u[k] = tile_row(acc[0][0], acc[1][0], k);
        knots_from_logits<K>(u, ks, INV ? kMinHd : kMinWd, a);
    }
    // searchsorted (splines.py:11-13): knots are non-decreasing, so the last k
    // with x >= knot[k] is the bin; the gathered knots ride along the scan
    // (register-resident, no dynamically indexed array)
    int bin = 0;
    float s0 = ks[0], s1 = ks[1];
#pragma unroll
    for (int k = 1; k < K; ++k) {
        if (x >= ks[k]) {
            bin = k;
            s0 = ks[k];
            s1 = ks[k + 1];
        }
    }
    // d_bin, d_bin+1 = bias + row . h  (bin + 1 <= K: row K is the circular-tail d_K)
    const int voff = bin * 16;
    DRows<QB> g0, g1;
    drows_issue<QB, K>(g0, W, voff, dsec, 0);  // in flight during the other tile's GEMM
    f32x2 ud0 = {bd[bin], 0.f}, ud1 = {bd[bin + 1], 0.f};
    pf.mark(PH_SPLINE);
    float o0, o1;
    {
        f32x16 acc[2][1];
        final_tile<XS, FPD>(X, W, sec, kg, 2 * j + 1 - TS, bf + 32 * (1 - TS), acc);
        pf.mark(PH_FINAL_GEMM);
        float u[K], ko[K + 1];
#pragma unroll
        for (int k = 0; k < K; ++k) u[k] = tile_row(acc[0][0], acc[1][0], k);
        knots_from_logits<K>(u, ko, INV ? kMinWd : kMinHd, a);
        o0 = ko[0];
        o1 = ko[1];
#pragma unroll
        for (int k = 1; k < K; ++k) {
            if (k == bin) {
                o0 = ko[k];
                o1 = ko[k + 1];
            }
        }
    }
    pf.mark(PH_SPLINE);
    const float *xr = X + lane * XS;
#pragma unroll 1
    for (int q0 = 0; q0 < NQ; q0 += 2 * QB) {
        drows_issue<QB, K>(g1, W, voff, dsec, q0 + QB);
        drows_dot<QB>(g0, xr, q0, ud0, ud1);
        if (q0 + 2 * QB < NQ) drows_issue<QB, K>(g0, W, voff, dsec, q0 + 2 * QB);
        drows_dot<QB>(g1, xr, q0 + QB, ud0, ud1);
    }
    pf.mark(PH_FINAL_GEMM);
    const float icw = INV ? o0 : s0, cw1 = INV ? o1 : s1;
    const float ich = INV ? s0 : o0, ch1 = INV ? s1 : o1;
    const float d0 = kMinD + softplus_t(ud0.x + ud0.y);
    const float d1 = kMinD + softplus_t(ud1.x + ud1.y);
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

// The conditional spline of one feature of one chain from its width / height logits (uS:
// the searched set, uO: the other): knots, bin, the derivative logits d_bin, d_bin+1 by
// dot products of the chain's hidden vector xr with the gathered rows of the final layer,
// the spline; co: the chain's coordinates (element p updated when inside and store).
template <int H, int K, bool INV>
__device__ __forceinline__ float spline_from_logits(const float (&uS)[K], const float (&uO)[K],
                                                    const float *__restrict__ xr, __amdgpu_buffer_rsrc_t W, int dsec,
                                                    const float *__restrict__ bd, float *co, int p, bool store,
                                                    const FlowArgs &a, bool &nan_any, Prof &pf) {
    constexpr int NQ = H / 4;
    constexpr int QB = NQ >= 8 ? 4 : NQ / 2;
    const float x = co[p];
    const bool inside = (x >= a.negB) && (x <= a.B);
    float ks[K + 1];
    knots_from_logits<K>(uS, ks, INV ? kMinHd : kMinWd, a);
    int bin = 0;
    float s0 = ks[0], s1 = ks[1];
#pragma unroll
    for (int k = 1; k < K; ++k) {
        if (x >= ks[k]) {
            bin = k;
            s0 = ks[k];
            s1 = ks[k + 1];
        }
    }
    const int voff = bin * 16;
    DRows<QB> g0, g1;
    drows_issue<QB, K>(g0, W, voff, dsec, 0);
    f32x2 ud0 = {bd[bin], 0.f}, ud1 = {bd[bin + 1], 0.f};
    float o0, o1;
    {
        float ko[K + 1];
        knots_from_logits<K>(uO, ko, INV ? kMinWd : kMinHd, a);
        o0 = ko[0];
        o1 = ko[1];
#pragma unroll
        for (int k = 1; k < K; ++k) {
            if (k == bin) {
                o0 = ko[k];
                o1 = ko[k + 1];
            }
        }
    }
    pf.mark(PH_SPLINE);
#pragma unroll 1
    for (int q0 = 0; q0 < NQ; q0 += 2 * QB) {
        drows_issue<QB, K>(g1, W, voff, dsec, q0 + QB);
        drows_dot<QB>(g0, xr, q0, ud0, ud1);
        if (q0 + 2 * QB < NQ) drows_issue<QB, K>(g0, W, voff, dsec, q0 + 2 * QB);
        drows_dot<QB>(g1, xr, q0 + QB, ud0, ud1);
    }
    pf.mark(PH_FINAL_GEMM);
    const float icw = INV ? o0 : s0, cw1 = INV ? o1 : s1;
    const float ich = INV ? s0 : o0, ch1 = INV ? s1 : o1;
    const float d0 = kMinD + softplus_t(ud0.x + ud0.y);
    const float d1 = kMinD + softplus_t(ud1.x + ud1.y);
    float y, l;
    bool nd;
    rqs_eval<INV>(x, icw, cw1 - icw, ich, ch1 - ich, d0, d1, y, l, nd);
    pf.mark(PH_SPLINE);
    if (inside) {
        if (store) co[p] = y;
        nan_any |= nd;
        return l;
    }
    return 0.f;
}

// cond_spline for a feature pair (K <= 16): both tiles of the pair first, then each
// feature's spline from its 16 columns (c0 = 0 or 16) of the lane-per-chain tiles.
// RM: lane -> chain mask (31: a 32-chain tile pair duplicated into both lane halves, whose
// upper half only computes)
template <int XS, int H, int K, bool INV, int RM = 63>
__device__ __forceinline__ float spline_from_tiles(const f32x16 (&tS)[2][1], const f32x16 (&tO)[2][1], int c0,
                                                   const float *__restrict__ X, __amdgpu_buffer_rsrc_t W, int dsec,
                                                   const float *__restrict__ bd, float *CO, int cs, int p,
                                                   const FlowArgs &a, bool &nan_any, Prof &pf) {
    const int lane = (int)threadIdx.x & RM;
    float uS[K], uO[K];
#pragma unroll
    for (int k = 0; k < K; ++k) {
        uS[k] = tile_row(tS[0][0], tS[1][0], c0 + k);
        uO[k] = tile_row(tO[0][0], tO[1][0], c0 + k);
    }
    return spline_from_logits<H, K, INV>(uS, uO, X + lane * XS, W, dsec, bd, CO + lane * cs, p,
                                         RM == 63 || (threadIdx.x & 32) == 0, a, nan_any, pf);
}

#pragma clang fp contract(on)
// ---------------------------------------------------------------------------
// The pass kernel (K = spline bins, compile time).
// ---------------------------------------------------------------------------
template <int H, int K, int MODE>
__global__ void __launch_bounds__(kThreads, 2) flow_pass_kernel(FlowArgs a) {
    // ResNet GEMM work split: NT column tiles x 2 row tiles over the 8 waves
    constexpr int NT = H / 32;
    constexpr int CTg = NT >= 4 ? NT / 4 : 1;          // ResNet: column tiles per wave of a row group
    constexpr int NUg = NT / CTg;                      // ResNet: active waves per row group
    constexpr int XS = (H < 2 * kMaxN ? 2 * kMaxN : H) + 4;  // == lds_layout().xs
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int N = a.N, D = 2 * N;
    const LdsLayout LL = lds_layout(N, H);
    const PackLayout PL = pack_layout(N, H, a.nb, a.K);
    const int tid = threadIdx.x, lane = tid & 63;
    const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (scalar feature / offset math)
    const int h = lane >> 5, r = lane & 31;
    float *X = (float *)(smem + LL.x);
    float *CO = (float *)(smem + LL.coord);
    float *LDP = (float *)(smem + LL.ld);
    const int cs = LL.cstride;
    const int64_t row0 = (int64_t)blockIdx.x * kRows;
    const bool row_valid = row0 + lane < a.nrows;

    // ---- inputs -> CO (logical order == physical order at offset 0)
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
    const int grp = wid >> 2, gw = wid & 3;
    const bool gact = gw < NUg;
    const int gct0 = gw * CTg;
    int *gbar = (int *)(smem + LL.ld + kWaves * kRows * 4);  // one arrival counter per row group
    int gphase = 0;
    if (tid < 4) gbar[tid] = 0;
    Prof pf;
    __syncthreads();
    pf.mark(PH_INPUT);

    for (int s = 0; s < a.L; ++s) {
        const int layer = (MODE == MODE_DENSITY) ? a.L - 1 - s : s;
        const float *P = a.packed + (int64_t)layer * PL.stride;
        const float *V = P + PL.vec;
        const __amdgpu_buffer_rsrc_t W =
            __builtin_amdgcn_make_buffer_rsrc((void *)P, (short)0, (int)(PL.stride * 4), 0x00020000);
        if (MODE != MODE_DENSITY) {
            off = (off + N) % D;  // Coupling.inverse rolls first (coupling.py:113-114)
            ld += uncond_spline<K, true>(P + PL.unc, CO, cs, N, D, off, a, nan_any);
            pf.mark(PH_UNCOND);
            __syncthreads();
            pf.mark(PH_BARRIER);
        }
        // periodic features [cos(s x_id) | sin(s x_id)] (nn.py:120-137) -> X
        for (int f = wid; f < N; f += kWaves) {
            const float v = CO[lane * cs + (2 * f + off) % D];
            const float sv = a.scale_pf * v;
            X[lane * XS + f] = cosf(sv);
            X[lane * XS + N + f] = sinf(sv);
        }
        for (int c = D + wid; c < 8 * PL.kg_in; c += kWaves) X[lane * XS + c] = 0.f;
        pf.mark(PH_PF);
        __syncthreads();
        pf.mark(PH_BARRIER);

        // ResidualNet on two independent row groups: waves 0-3 carry rows 0-31,
        // waves 4-7 rows 32-63, each group splitting the H/32 column tiles; the
        // groups synchronise only internally (LDS-counter barriers), so one group's
        // epilogue / barrier bubbles run under the other group's MFMAs.
        f32x16 hr[1][CTg], acc[1][CTg];
        // hr = the residual stream WITHOUT its biases: b_in and every block's b1 are
        // deferred (pack_vec_kernel folds a0 * their running sum into each block's c0 and
        // their total into s_h), b0 is folded into c1, and the residual add is the
        // accumulator input of the second GEMM.  The epilogues are 1 FMA + 1 max.
        if (gact) gemm64<XS, 1, CTg, FS_RPD>(X, W, (int)(PL.win * 4), PL.kg_in, grp, gct0, hr);  // initial_layer
        pf.mark(PH_INIT_GEMM);
        // per-column epilogue vectors {a0,c0',a1,c1'} of a block: loaded one block
        // ahead and always BEFORE the next GEMM's weight prologue, so the epilogue's
        // vmcnt wait never covers the prologue's (L2 / MALL latency) loads
        float ev[4][CTg];
        auto load_ev = [&](int jb, float (&e)[4][CTg]) {
            const float *VB = V + PL.v_blocks + (int64_t)4 * H * jb;
#pragma unroll
            for (int q = 0; q < 4; ++q)
#pragma unroll
                for (int ct = 0; ct < CTg; ++ct) e[q][ct] = VB[q * H + 32 * (gct0 + ct) + r];
        };
        if (a.nb > 0) load_ev(0, ev);
        BRing<CTg, FS_RPD> br;
        if (gact && a.nb > 0) b_prologue<CTg, FS_RPD>(br, W, (int)(PL.blocks * 4), PL.kg_h, gct0);
        for (int jb = 0; jb < a.nb; ++jb) {  // ResidualBlock (resnet.py:37-50), eval BN folded
            const int w0 = (int)((PL.blocks + jb * PL.block_stride) * 4);
            const int w1 = w0 + (int)(PL.block_stride * 2);
            pf.mark(PH_EPI);
            FS_GROUP_BARRIER(gbar + grp, gphase);
            pf.mark(PH_BARRIER);
            if (gact) {
#pragma unroll
                for (int ct = 0; ct < CTg; ++ct) {
                    const int col = 32 * (gct0 + ct) + r;
#pragma unroll
                    for (int i = 0; i < 16; ++i)
                        X[acc_row(grp, i, h) * XS + col] = FS_EPI(hr[0][ct][i], ev[0][ct], ev[1][ct]);
                }
            }
            pf.mark(PH_EPI);
            FS_GROUP_BARRIER(gbar + grp, gphase);
            pf.mark(PH_BARRIER);
            if (gact) {
                gemm_run<XS, 1, CTg, FS_RPD>(X, W, w0, PL.kg_h, grp, gct0, br, acc);
                b_prologue<CTg, FS_RPD>(br, W, w1, PL.kg_h, gct0);  // next GEMM's first weight groups
            }
            pf.mark(PH_RES_GEMM);
            FS_GROUP_BARRIER(gbar + grp, gphase);
            pf.mark(PH_BARRIER);
            if (gact) {
#pragma unroll
                for (int ct = 0; ct < CTg; ++ct) {
                    const int col = 32 * (gct0 + ct) + r;
#pragma unroll
                    for (int i = 0; i < 16; ++i)
                        X[acc_row(grp, i, h) * XS + col] = FS_EPI(acc[0][ct][i], ev[2][ct], ev[3][ct]);
                }
            }
            pf.mark(PH_EPI);
            FS_GROUP_BARRIER(gbar + grp, gphase);
            pf.mark(PH_BARRIER);
            float evn[4][CTg];
            if (jb + 1 < a.nb) load_ev(jb + 1, evn);
            if (gact) {
                gemm_run<XS, 1, CTg, FS_RPD, true>(X, W, w1, PL.kg_h, grp, gct0, br, hr);  // h += Lin1(t)
                if (jb + 1 < a.nb) b_prologue<CTg, FS_RPD>(br, W, w1 + (int)(PL.block_stride * 2), PL.kg_h, gct0);
            }
            if (jb + 1 < a.nb)
#pragma unroll
                for (int q = 0; q < 4; ++q)
#pragma unroll
                    for (int ct = 0; ct < CTg; ++ct) ev[q][ct] = evn[q][ct];
            pf.mark(PH_RES_GEMM);
        }
        FS_GROUP_BARRIER(gbar + grp, gphase);
        pf.mark(PH_BARRIER);
        if (gact) {  // X <- h (+ the deferred biases) for the final layer
#pragma unroll
            for (int ct = 0; ct < CTg; ++ct) {
                const int col = 32 * (gct0 + ct) + r;
                const float sh = V[col];
#pragma unroll
                for (int i = 0; i < 16; ++i) X[acc_row(grp, i, h) * XS + col] = hr[0][ct][i] + sh;
            }
        }
        pf.mark(PH_EPI);
        __syncthreads();
        pf.mark(PH_BARRIER);
        // final layer + conditional spline, feature by feature
        if constexpr (K <= 16) {  // feature pairs share the widths / heights tiles
            constexpr bool INV = MODE != MODE_DENSITY;
            constexpr int TS = INV ? 1 : 0;
            for (int pp = wid; pp < (N + 1) / 2; pp += kWaves) {
                const int ja = 2 * pp, jb = 2 * pp + 1;
                const bool hb = jb < N;
                const float *ba = V + PL.v_bf + 96 * ja;
                const float *bb = hb ? V + PL.v_bf + 96 * jb : ba + 16;  // zeros beyond K
                f32x16 tS[2][1], tO[2][1];
                final_tile_pair<XS>(X, W, (int)(PL.wf * 4), PL.kg_h, 2 * pp + TS, ba + 32 * TS, bb + 32 * TS, tS);
                final_tile_pair<XS>(X, W, (int)(PL.wf * 4), PL.kg_h, 2 * pp + 1 - TS, ba + 32 * (1 - TS),
                                    bb + 32 * (1 - TS), tO);
                pf.mark(PH_FINAL_GEMM);
                ld += spline_from_tiles<XS, H, K, INV>(tS, tO, 0, X, W, (int)((PL.wd + (int64_t)ja * H * (K + 1)) * 4),
                                                       V + PL.v_bd + ja * (K + 1), CO, cs, (2 * ja + 1 + off) % D, a,
                                                       nan_any, pf);
                if (hb)
                    ld += spline_from_tiles<XS, H, K, INV>(tS, tO, 16, X, W,
                                                           (int)((PL.wd + (int64_t)jb * H * (K + 1)) * 4),
                                                           V + PL.v_bd + jb * (K + 1), CO, cs, (2 * jb + 1 + off) % D,
                                                           a, nan_any, pf);
            }
        } else {
        for (int j = wid; j < N; j += kWaves) {
            const int p = (2 * j + 1 + off) % D;
            ld += cond_spline<XS, H, K, MODE != MODE_DENSITY>(
                X, W, (int)(PL.wf * 4), PL.kg_h, V + PL.v_bf + 96 * j, (int)((PL.wd + (int64_t)j * H * (K + 1)) * 4),
                V + PL.v_bd + j * (K + 1), CO, cs, p, j, a, nan_any, pf);
        }
        }
        if (MODE == MODE_DENSITY) {
            ld += uncond_spline<K, false>(P + PL.unc, CO, cs, N, D, off, a, nan_any);
            off = (off + N) % D;  // Coupling.forward rolls last (coupling.py:100-101)
            pf.mark(PH_UNCOND);
        }
        __syncthreads();
        pf.mark(PH_BARRIER);
    }
    pf.flush();

    // ---- outputs
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
        // single-pass log q (FS_MH_SINGLE_PASS): log q(x') = log q0(z) - sum of the sampling
        // direction's log|dx/dz| (base draws are inside the bound by construction)
        if (MODE == MODE_PROPOSE && a.add_base) outv = a.base_lp - tot;
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
// Wide path for small batches.  flow_pass_kernel carries 64 rows through every layer
// in one workgroup, so a batch of R rows occupies R/64 CUs: 4096 chains are a quarter
// of the chip, the Algorithm-2 refeed's 100 runs two CUs.  The wide path runs the same
// pass phase by phase over the whole batch, each phase one launch spread over as many
// workgroups as it has independent tiles:
//   input   rows -> CO (coordinates, [R][2N] physical order), log-det partials zeroed
//   start   per layer: (sampling) roll + unconditional spline, periodic features -> XA
//   trunk   the layer's ResidualNet per 32-row tile (the fused kernel's trunk for one row
//           group): one wave per 32-column tile, activations in LDS between the GEMMs
//           (BatchNorm folded, ReLU, residual stream in the accumulators)
//   final   per (64-row block, feature unit): the final layer + conditional spline of one
//           transform feature (a pair for K <= 16), (density) the unconditional spline of
//           the same-index identity feature; log-dets per feature to LDC / LDU
//   fold    (in the next start / output launch) each row's per-feature log-dets added to
//           LDW[row][w] in the order the fused kernel's wave w adds them
//   output  the 8 partials summed in wave order, base density, outputs.
// Every value is computed by the fused kernel's own device code (gemm_run, FS_EPI,
// cond_spline, uncond_spline_w, the Philox draws) with the same operands in the same
// order, so the results are bit-identical to flow_pass_kernel's
// (tests/test_gpu_wide.py); only the schedule differs.  The state between phases (a few
// MB at these sizes) stays in the L2 / MALL.
// ---------------------------------------------------------------------------
// Weight-fragment ring depths of the wide path: its launches start with the weights in
// no L2 (every phase streams them from the MALL / HBM), so more k-groups are in flight
// than in the fused kernel, whose weights stay L2-resident.  Latency only: the operand
// order and the results are the fused kernel's.
#ifndef FS_WIDE_PD
#define FS_WIDE_PD 16
#endif
#ifndef FS_WIDE_FPD
#define FS_WIDE_FPD 8
#endif
constexpr int kWidePD = FS_WIDE_PD, kWideFPD = FS_WIDE_FPD;

struct WideArgs {
    FlowArgs a;
    float *CO;     // [R][D]
    float *XA;     // [R][XS] periodic features (the trunk's input)
    float *XB;     // [R][XS] the final layer's input (the trunk's output)
    float *LDW;    // [R][8] log-det partial of virtual wave w (the fused kernel's wave w)
    float *LDC;    // [R][N] the last final phase's conditional log-det of transform feature j
    float *LDU;    // [R][N] (density) its unconditional log-det of identity feature f;
                   // (sampling) the unconditional log-dets of the even layers' start
    float *LDU2;   // [R][N] (sampling) ... of the odd layers' start
    int pending;   // the start / output launch first folds the previous final phase into LDW
    int64_t R;     // rows padded to 64
    int off;       // physical index of logical coordinate 0 in this phase
    int layer;
    int jb;
    float *XG;     // (column-split trunk) [R / 16][2][H][16] handed-off column slices
    unsigned *CNT;  // [2][R / 16] hand-off counters (launch parity x tile)
    int T;          // R / 16
    unsigned spin;  // (column-split trunk) polls before a hand-off wait gives up; 0: give up at
                    // once (the timeout test hook, fs_set_wide_handoff_spins)
};

template <int MODE>
__global__ void __launch_bounds__(256) wide_input_kernel(WideArgs w) {
    const FlowArgs &a = w.a;
    const int N = a.N, D = 2 * N;
    const int64_t row0 = (int64_t)blockIdx.x * kRows;
    if (w.CNT)  // the column-split trunk's counters start every pass at zero
        for (int e = (int)(blockIdx.x * blockDim.x + threadIdx.x); e < 2 * w.T; e += (int)(gridDim.x * blockDim.x))
            __hip_atomic_store(w.CNT + e, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    float *CO = w.CO + row0 * D;
    if (MODE == MODE_PROPOSE) {
        const int nq = (D + 3) / 4;
        for (int e = threadIdx.x; e < kRows * nq; e += blockDim.x) {
            const int rr = e / nq, q = e - rr * nq;
            const int64_t lr = row0 + rr, rpc = a.rows_per_counter;
            const uint64_t ctr = rpc > 0 ? a.counter + (uint64_t)(lr / rpc) : a.counter;
            const uint64_t gr = (uint64_t)(a.row_offset + (rpc > 0 ? lr % rpc : lr));
            uint4 c = make_uint4((uint32_t)gr, (uint32_t)(gr >> 32) ^ (uint32_t)(ctr >> 32), (uint32_t)ctr,
                                 (uint32_t)q);
            uint4 o = philox4x32(c, make_uint2((uint32_t)a.seed, (uint32_t)(a.seed >> 32)));
            const uint32_t v[4] = {o.x, o.y, o.z, o.w};
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int i = 4 * q + t;
                if (i < D) {
                    const float u = (float)(v[t] >> 8) * 5.9604644775390625e-08f;  // [0,1)
                    CO[rr * D + i] = u * a.twoB + a.negB;
                }
            }
        }
    } else {
        for (int e = threadIdx.x; e < kRows * D; e += blockDim.x) {
            const int rr = e / D, i = e - rr * D;
            const int64_t gr = row0 + rr;
            CO[rr * D + i] = (gr < a.nrows) ? a.in[gr * D + i] : 0.f;
        }
    }
    for (int e = threadIdx.x; e < kRows * kWaves; e += blockDim.x) w.LDW[row0 * kWaves + e] = 0.f;
}


// LDW[row][w] += the previous final phase's per-feature log-dets, in the order wave w of
// the fused kernel added them: its transform features (pairs 2pp, 2pp+1 for K <= 16) in
// ascending order, then (density) the sum over its identity features, added as one term.
template <int K, int MODE>
__device__ __forceinline__ float wide_fold(const WideArgs &w, int64_t row, int vw, float ld) {
    const int N = w.a.N;
    const float *lc = w.LDC + row * N;
    if constexpr (K <= 16) {
        for (int pp = vw; pp < (N + 1) / 2; pp += kWaves) {
            ld += lc[2 * pp];
            if (2 * pp + 1 < N) ld += lc[2 * pp + 1];
        }
    } else {
        for (int j = vw; j < N; j += kWaves) ld += lc[j];
    }
    if (MODE == MODE_DENSITY) {
        const float *lu = w.LDU + row * N;
        float su = 0.f;
        for (int f = vw; f < N; f += kWaves) su += lu[f];
        ld += su;
    }
    return ld;
}

// (sampling modes) the unconditional spline of virtual wave wid's identity features,
// then the periodic features of the layer -> XA.  One workgroup of 8 waves per 64 rows.
template <int H, int K, int MODE>
__global__ void __launch_bounds__(kThreads) wide_start_kernel(WideArgs w) {
    constexpr int XS = (H < 2 * kMaxN ? 2 * kMaxN : H) + 4;
    const FlowArgs &a = w.a;
    const int N = a.N, D = 2 * N;
    const PackLayout PL = pack_layout(N, H, a.nb, a.K);
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t row0 = (int64_t)blockIdx.x * kRows;
    float *CO = w.CO + row0 * D;
    float *X = w.XA + row0 * XS;
    const float *P = a.packed + (int64_t)w.layer * PL.stride;
    if (w.pending || MODE != MODE_DENSITY) {
        bool nan_any = false;
        float ld = w.LDW[(row0 + lane) * kWaves + wid];
        if (w.pending) ld = wide_fold<K, MODE>(w, row0 + lane, wid, ld);
        if (MODE != MODE_DENSITY) ld += uncond_spline_w<K, true>(P + PL.unc, CO, D, N, D, w.off, a, nan_any, wid);
        w.LDW[(row0 + lane) * kWaves + wid] = ld;
        if (nan_any && row0 + lane < a.nrows && a.err) atomicOr(a.err, 1);
    }
    for (int f = wid; f < N; f += kWaves) {
        const float v = CO[lane * D + (2 * f + w.off) % D];
        const float sv = a.scale_pf * v;
        X[lane * XS + f] = cosf(sv);
        X[lane * XS + N + f] = sinf(sv);
    }
    for (int c = D + wid; c < 8 * PL.kg_in; c += kWaves) X[lane * XS + c] = 0.f;
}

// The layer's whole ResidualNet for one 32-row tile: the initial layer and every residual
// block, one wave per 32-column tile (H/32 waves), the activations in LDS between GEMMs
// (the fused kernel's trunk for one row group: same GEMMs, epilogues, deferred biases and
// residual stream in the accumulators), reading the periodic features from XA and
// writing the final layer's input h + s_h to XB.
template <int H>
__global__ void __launch_bounds__(64 * (H / 32)) wide_trunk_kernel(WideArgs w) {
    constexpr int XS = (H < 2 * kMaxN ? 2 * kMaxN : H) + 4;
    __shared__ __attribute__((aligned(16))) float X[32 * XS];
    const FlowArgs &a = w.a;
    const int N = a.N;
    const PackLayout PL = pack_layout(N, H, a.nb, a.K);
    const int lane = threadIdx.x & 63, h = lane >> 5, r = lane & 31;
    const int tile = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int64_t rowt = (int64_t)blockIdx.x * 32;
    const int nq = 2 * PL.kg_in;  // 16-byte quads of the used feature columns
    for (int e = threadIdx.x; e < 32 * nq; e += blockDim.x) {
        const int rr = e / nq, q = e - rr * nq;
        *(f32x4 *)(X + rr * XS + 4 * q) = *(const f32x4 *)(w.XA + (rowt + rr) * XS + 4 * q);
    }
    __syncthreads();
    const float *P = a.packed + (int64_t)w.layer * PL.stride;
    const float *V = P + PL.vec;
    const __amdgpu_buffer_rsrc_t W =
        __builtin_amdgcn_make_buffer_rsrc((void *)P, (short)0, (int)(PL.stride * 4), 0x00020000);
    const int col = 32 * tile + r;
    f32x16 hr[1][1], acc[1][1];
    gemm64<XS, 1, 1, kWidePD>(X, W, (int)(PL.win * 4), PL.kg_in, 0, tile, hr);  // initial_layer
    for (int jb = 0; jb < a.nb; ++jb) {  // ResidualBlock (resnet.py:37-50), eval BN folded
        const float *VB = V + PL.v_blocks + (int64_t)4 * H * jb;
        const float e0 = VB[col], e1 = VB[H + col], e2 = VB[2 * H + col], e3 = VB[3 * H + col];
        const int w0 = (int)((PL.blocks + jb * PL.block_stride) * 4);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 16; ++i) X[acc_row(0, i, h) * XS + col] = FS_EPI(hr[0][0][i], e0, e1);
        __syncthreads();
        gemm64<XS, 1, 1, kWidePD>(X, W, w0, PL.kg_h, 0, tile, acc);
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 16; ++i) X[acc_row(0, i, h) * XS + col] = FS_EPI(acc[0][0][i], e2, e3);
        __syncthreads();
        gemm64<XS, 1, 1, kWidePD, true>(X, W, w0 + (int)(PL.block_stride * 2), PL.kg_h, 0, tile, hr);  // h += Lin1(t)
    }
    const float sh = V[col];
#pragma unroll
    for (int i = 0; i < 16; ++i) w.XB[(rowt + acc_row(0, i, h)) * XS + col] = hr[0][0][i] + sh;
}

// The same trunk on 16-row tiles, so that a batch fills twice as many CUs (4096 rows: 256
// workgroups instead of 128).  v_mfma_f32_16x16x4_f32 is the same exact fmaf chain as
// v_mfma_f32_32x32x2_f32 (tools/probes/mfma_order.hip: bit-identical on every output), so
// feeding it the k order of the 32-row tiles keeps the results bit-identical: per 8-wide
// k-group g the 32x32x2 chain takes k = 8g + (0, 4), (1, 5), (2, 6), (3, 7); here MFMA 0
// takes the k-slots (0, 4, 1, 5) and MFMA 1 (2, 6, 3, 7), i.e. lane (q, r) of a 16x16x4
// supplies k = 8g + 4 (q & 1) + (q >> 1) and then + 2.  Its weight values are the 32-row
// image's fragment: lane 32 (q & 1) + 16 c + r, elements (q >> 1) and 2 + (q >> 1), one
// 8-byte load each (c = this wave's 16-column half; kResPos puts the pair side by side in the
// ResidualNet sections).  The activation pair is one ds_read_b64 of
// a tile image whose quads are stored as columns (0, 2, 1, 3), bit 1 of the position
// flipped in rows 8-15, at a row stride of 8 mod 64 dwords (no bank conflicts).
__device__ __forceinline__ int t16_pos(int row, int col, int xs) {
    const int p = (col & ~3) | ((col & 1) << 1) | ((col >> 1) & 1);
    return row * xs + (p ^ (((row >> 3) & 1) << 1));
}

typedef float f32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x2 ldb_pair(__amdgpu_buffer_rsrc_t W, int voff, int soff) {
    return __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(W, voff, soff, 0));
}

// acc[c] (16 x 16, columns 32 tile + 16 c ..) = X[16 x 8 kg] . B[tile], ACC: onto acc
template <int XS16, int PD, bool ACC>
__device__ __forceinline__ void gemm16(const float *__restrict__ X, __amdgpu_buffer_rsrc_t W, int sec, int kg,
                                       int tile, f32x4 (&acc)[2]) {
    const int lane = threadIdx.x & 63, q = lane >> 4, r = lane & 15, h = lane >> 5, qo = q & 1;
    if (!ACC)
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int i = 0; i < 4; ++i) acc[c][i] = 0.f;
    const float *xa = X + r * XS16 + 4 * qo + ((2 * h) ^ (((r >> 3) & 1) << 1));
    const int vb = (32 * qo + r) * 16 + 8 * h;  // + 256 c: the second 16-column half
    const int fb = sec + tile * kg * 1024;
    // both operands in PD-deep rings: the weights from L2 / MALL, the activation pairs from
    // LDS (an LDS read issued right before its MFMAs would stall every k-group)
    f32x2 rb[PD][2], ra[PD];
#pragma unroll
    for (int s = 0; s < PD; ++s)
        if (s < kg) {
#pragma unroll
            for (int c = 0; c < 2; ++c) rb[s][c] = ldb_pair(W, vb + 256 * c, fb + s * 1024);
            ra[s] = *(const f32x2 *)(xa + 8 * s);
        }
    for (int g0 = 0; g0 < kg; g0 += PD) {
#pragma unroll
        for (int s = 0; s < PD; ++s) {
            const int g = g0 + s;
            if (g < kg) {
#pragma unroll
                for (int m = 0; m < 2; ++m)
#pragma unroll
                    for (int c = 0; c < 2; ++c)
                        acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[s][m], rb[s][c][m], acc[c], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
                const int gn = g + PD;
                if (gn < kg) {
                    ra[s] = *(const f32x2 *)(xa + 8 * gn);
#pragma unroll
                    for (int c = 0; c < 2; ++c) rb[s][c] = ldb_pair(W, vb + 256 * c, fb + gn * 1024);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
}

#ifndef FS_WIDE16_PD
#define FS_WIDE16_PD 24  // k-groups in flight (2 loads each): the weights stream from MALL / HBM
#endif

// wide_trunk_kernel on a 16-row tile: one wave per 32-column tile (two 16x16 halves), the
// same GEMMs, epilogues (FS_EPI), deferred biases and residual stream, bit for bit
template <int H>
struct Trunk16 {
    static constexpr int XS = (H < 2 * kMaxN ? 2 * kMaxN : H) + 4;  // XA / XB row stride
    static constexpr int XS16 = XS + 4;                             // the LDS image's (== 8 mod 64)
    static_assert(XS16 % 64 == 8, "trunk16 LDS row stride");
};

// the trunk of one 16-row tile whose features are in the LDS image X (t16_pos layout); a
// launch of NW > H / 32 waves leaves the extra ones to the barriers
template <int H, int NW = H / 32>
__device__ __forceinline__ void trunk16_run(float *X, const WideArgs &w, int64_t rowt) {
    constexpr int XS = Trunk16<H>::XS, XS16 = Trunk16<H>::XS16;
    const FlowArgs &a = w.a;
    const int N = a.N;
    const PackLayout PL = pack_layout(N, H, a.nb, a.K);
    const int lane = threadIdx.x & 63, q = lane >> 4, r = lane & 15;
    const int tile = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const bool act = NW == H / 32 || tile < H / 32;
    const float *P = a.packed + (int64_t)w.layer * PL.stride;
    const float *V = P + PL.vec;
    const __amdgpu_buffer_rsrc_t W =
        __builtin_amdgcn_make_buffer_rsrc((void *)P, (short)0, (int)(PL.stride * 4), 0x00020000);
    int col[2], pos[2][4];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        col[c] = act ? 32 * tile + 16 * c + r : 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) pos[c][i] = t16_pos(4 * q + i, col[c], XS16);
    }
    f32x4 hr[2], acc[2];
    if (act) gemm16<XS16, FS_WIDE16_PD, false>(X, W, (int)(PL.win * 4), PL.kg_in, tile, hr);  // initial_layer
    for (int jb = 0; jb < a.nb; ++jb) {  // ResidualBlock (resnet.py:37-50), eval BN folded
        const float *VB = V + PL.v_blocks + (int64_t)4 * H * jb;
        float e0[2], e1[2], e2[2], e3[2];
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            e0[c] = VB[col[c]];
            e1[c] = VB[H + col[c]];
            e2[c] = VB[2 * H + col[c]];
            e3[c] = VB[3 * H + col[c]];
        }
        const int w0 = (int)((PL.blocks + jb * PL.block_stride) * 4);
        __syncthreads();
        if (act)
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
                for (int i = 0; i < 4; ++i) X[pos[c][i]] = FS_EPI(hr[c][i], e0[c], e1[c]);
        __syncthreads();
        if (act) gemm16<XS16, FS_WIDE16_PD, false>(X, W, w0, PL.kg_h, tile, acc);
        __syncthreads();
        if (act)
#pragma unroll
            for (int c = 0; c < 2; ++c)
#pragma unroll
                for (int i = 0; i < 4; ++i) X[pos[c][i]] = FS_EPI(acc[c][i], e2[c], e3[c]);
        __syncthreads();
        if (act) gemm16<XS16, FS_WIDE16_PD, true>(X, W, w0 + (int)(PL.block_stride * 2), PL.kg_h, tile, hr);  // h += Lin1(t)
    }
    if (!act) return;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
        const float sh = V[col[c]];
#pragma unroll
        for (int i = 0; i < 4; ++i) w.XB[(rowt + 4 * q + i) * XS + col[c]] = hr[c][i] + sh;
    }
}

// The 16-row trunk with each 32-column tile split over two waves, one 16-column half each
// (wide_trunk16s_kernel, trunk16 = 3, the default).  trunk16_run's waves were parked on
// their weight loads and barriers ~40 % of the time with two waves per SIMD (r05 PMC:
// SQ_VALU_MFMA_BUSY 0.61 of SIMD cycles); halving each wave's tile doubles the waves per SIMD
// that hide those waits, and at H = 128 the merged kernel's 8 waves all run the trunk instead
// of 4.  A half's accumulator takes the same MFMAs in the same order as gemm16's acc[c]
// (per k-group m = 0 then 1), so the results are bit-identical.
// The weight half of gemm16h's ring prologue, issued before the epilogue and barrier that
// precede the GEMM (its loads do not depend on the activations).  (Loading the next block's
// epilogue vectors a GEMM early lost 2-3 %, r05j.)
template <int PD>
__device__ __forceinline__ void gemm16h_pre(__amdgpu_buffer_rsrc_t W, int sec, int kg, int tile, int c,
                                            f32x2 (&rb)[PD]) {
    const int lane = threadIdx.x & 63, q = lane >> 4, r = lane & 15, h = lane >> 5, qo = q & 1;
    const int vb = (32 * qo + r) * 16 + 8 * h + 256 * c;
    const int fb = sec + tile * kg * 1024;
#pragma unroll
    for (int s = 0; s < PD; ++s)
        if (s < kg) rb[s] = ldb_pair(W, vb, fb + s * 1024);
}

template <int XS16, int PD, int XB, bool ACC>
__device__ __forceinline__ void gemm16h(const float *__restrict__ X, __amdgpu_buffer_rsrc_t W, int sec, int kg,
                                        int tile, int c, f32x4 &acc, f32x2 (&rb)[PD]) {
    static_assert(PD % XB == 0, "activation ring depth divides the weight ring's");
    const int lane = threadIdx.x & 63, q = lane >> 4, r = lane & 15, h = lane >> 5, qo = q & 1;
    if (!ACC)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = 0.f;
    const float *xa = X + r * XS16 + 4 * qo + ((2 * h) ^ (((r >> 3) & 1) << 1));
    const int vb = (32 * qo + r) * 16 + 8 * h + 256 * c;
    const int fb = sec + tile * kg * 1024;
    // rb: gemm16h_pre's loads of k-groups 0 .. PD - 1; the activations (LDS, short latency)
    // run XB k-groups ahead
    f32x2 ra[XB];
#pragma unroll
    for (int s = 0; s < XB; ++s)
        if (s < kg) ra[s] = *(const f32x2 *)(xa + 8 * s);
    for (int g0 = 0; g0 < kg; g0 += PD) {
#pragma unroll
        for (int s = 0; s < PD; ++s) {
            const int g = g0 + s;
            if (g < kg) {
#pragma unroll
                for (int m = 0; m < 2; ++m)
                    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ra[s % XB][m], rb[s][m], acc, 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
                if (g + XB < kg) ra[s % XB] = *(const f32x2 *)(xa + 8 * (g + XB));
                if (g + PD < kg) rb[s] = ldb_pair(W, vb, fb + (g + PD) * 1024);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
}

// k-groups in flight per half-tile wave: weights (one 8-byte load each) and activation
// reads from LDS.  Shallow rings run faster than deep ones (A1-N16 propose pass, 16 and 4096
// rows: 24/24 5.6-5.75 ms, 24/4 5.4-5.7, 16/4 5.3-5.4, 12/4 and 8/4 5.27-5.30;
// profiles/r05/r05q_trunk16h_rings.log).  With the ring this shallow, issuing the next GEMM's
// weights before the epilogue barrier gains ~2 % (8/4: 5.18 ms at 4096 rows, r05s); at 24/24
// it had lost 18 % (r05j).
#ifndef FS_WIDE16H_PD
#define FS_WIDE16H_PD 8
#endif
#ifndef FS_WIDE16H_XB
#define FS_WIDE16H_XB 4
#endif


// trunk16_run with wave w computing half (w & 1) of column tile w >> 1 (2 H / 32 trunk waves).
// The activation image is double-buffered (X: the features, then every other epilogue; Y: the
// rest), so an epilogue never overwrites the image the GEMM before it read: one barrier per
// epilogue (its writes before the next GEMM's reads) instead of two.
template <int H, int NW = 2 * (H / 32)>
__device__ __forceinline__ void trunk16h_run(float *X, float *Y, const WideArgs &w, int64_t rowt) {
    constexpr int XS = Trunk16<H>::XS, XS16 = Trunk16<H>::XS16;
    const FlowArgs &a = w.a;
    const int N = a.N;
    const PackLayout PL = pack_layout(N, H, a.nb, a.K);
    const int lane = threadIdx.x & 63, q = lane >> 4, r = lane & 15;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int tile = wv >> 1, c = wv & 1;
    const bool act = NW == 2 * (H / 32) || wv < 2 * (H / 32);
    const float *P = a.packed + (int64_t)w.layer * PL.stride;
    const float *V = P + PL.vec;
    const __amdgpu_buffer_rsrc_t W =
        __builtin_amdgcn_make_buffer_rsrc((void *)P, (short)0, (int)(PL.stride * 4), 0x00020000);
    const int col = act ? 32 * tile + 16 * c + r : 0;
    int pos[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) pos[i] = t16_pos(4 * q + i, col, XS16);
    f32x4 hr, acc;
    f32x2 rb[FS_WIDE16H_PD];
    if (act) {
        gemm16h_pre<FS_WIDE16H_PD>(W, (int)(PL.win * 4), PL.kg_in, tile, c, rb);
        gemm16h<XS16, FS_WIDE16H_PD, FS_WIDE16H_XB, false>(X, W, (int)(PL.win * 4), PL.kg_in, tile, c, hr, rb);  // initial_layer
    }
    for (int jb = 0; jb < a.nb; ++jb) {  // ResidualBlock (resnet.py:37-50), eval BN folded
        const float *VB = V + PL.v_blocks + (int64_t)4 * H * jb;
        const float e0 = VB[col], e1 = VB[H + col], e2 = VB[2 * H + col], e3 = VB[3 * H + col];
        const int w0 = (int)((PL.blocks + jb * PL.block_stride) * 4), w1 = w0 + (int)(PL.block_stride * 2);
        // Y was last read by the previous block's first GEMM (or never): every wave has passed
        // the barrier after it, so these writes need no barrier before them
        if (act) {
            gemm16h_pre<FS_WIDE16H_PD>(W, w0, PL.kg_h, tile, c, rb);  // ahead of the barrier
#pragma unroll
            for (int i = 0; i < 4; ++i) Y[pos[i]] = FS_EPI(hr[i], e0, e1);
        }
        __syncthreads();
        if (act) {
            gemm16h<XS16, FS_WIDE16H_PD, FS_WIDE16H_XB, false>(Y, W, w0, PL.kg_h, tile, c, acc, rb);
            gemm16h_pre<FS_WIDE16H_PD>(W, w1, PL.kg_h, tile, c, rb);
        }
        // X was last read by the GEMM before the barrier above (initial layer / second GEMM)
        if (act)
#pragma unroll
            for (int i = 0; i < 4; ++i) X[pos[i]] = FS_EPI(acc[i], e2, e3);
        __syncthreads();
        if (act) {
            gemm16h<XS16, FS_WIDE16H_PD, FS_WIDE16H_XB, true>(X, W, w1, PL.kg_h, tile, c, hr, rb);  // h += Lin1(t)
        }
    }
    if (!act) return;
    const float sh = V[col];
#pragma unroll
    for (int i = 0; i < 4; ++i) w.XB[(rowt + 4 * q + i) * XS + col] = hr[i] + sh;
}

template <int H>
__global__ void __launch_bounds__(64 * (H / 32)) wide_trunk16_kernel(WideArgs w) {
    constexpr int XS = Trunk16<H>::XS, XS16 = Trunk16<H>::XS16;
    __shared__ __attribute__((aligned(16))) float X[16 * XS16];
    const PackLayout PL = pack_layout(w.a.N, H, w.a.nb, w.a.K);
    const int64_t rowt = (int64_t)blockIdx.x * 16;
    const int nq = 2 * PL.kg_in;  // 16-byte quads of the used feature columns
    for (int e = threadIdx.x; e < 16 * nq; e += blockDim.x) {
        const int rr = e / nq, qq = e - rr * nq;
        const f32x4 v = *(const f32x4 *)(w.XA + (rowt + rr) * XS + 4 * qq);
        f32x4 o;  // positions of columns (0, 1, 2, 3): (0, 2, 1, 3), bit 1 flipped in rows 8-15
        if (rr < 8) {
            o[0] = v[0]; o[1] = v[2]; o[2] = v[1]; o[3] = v[3];
        } else {
            o[0] = v[1]; o[1] = v[3]; o[2] = v[0]; o[3] = v[2];
        }
        *(f32x4 *)(X + rr * XS16 + 4 * qq) = o;
    }
    __syncthreads();
    trunk16_run<H>(X, w, rowt);
}

// One feature of uncond_spline_w at the value x: its log-det returned and the new value in
// v (0 and x outside the tail bound).
template <int K, bool INV>
__device__ __forceinline__ float uncond_eval(const float *__restrict__ U, float x, const FlowArgs &a,
                                             bool &nan_any, int f, float &v) {
    constexpr int K1 = K + 1;
    const float *T = U + (size_t)f * 3 * K1;
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
        v = y;
        nan_any |= nd;
        return l;
    }
    v = x;
    return 0.f;
}

// ... on one row (co: its coordinates, p: the feature's physical index), updated in place
template <int K, bool INV>
__device__ __forceinline__ float uncond_at(const float *__restrict__ U, float *co, int p, const FlowArgs &a,
                                           bool &nan_any, int f) {
    const float x = co[p];
    float v;
    const float l = uncond_eval<K, INV>(U, x, a, nan_any, f, v);
    if ((x >= a.negB) && (x <= a.B)) co[p] = v;
    return l;
}

// ... on the lane's row of a 64-row block
template <int K, bool INV>
__device__ __forceinline__ float uncond_one(const float *__restrict__ U, float *CO, int cs, int D, int off,
                                            const FlowArgs &a, bool &nan_any, int f) {
    const int lane = threadIdx.x & 63;
    return uncond_at<K, INV>(U, CO + lane * cs, (2 * f + off) % D, a, nan_any, f);
}

// (sampling modes) the start spread over features: workgroup (block, j) runs feature
// f = wid + 8 j of virtual wave wid (one feature per wave instead of its 8): the
// unconditional inverse spline (CO updated in place, the log-det to this layer's LDU /
// LDU2 slot) and the periodic features of f.  The virtual wave's log-det sum over its
// features (uncond_spline_w's order) is added to LDW by the next start / output launch,
// before that layer's conditional terms, so LDW sees the fused kernel's additions in its
// order: ..., su(l - 1), cond(l - 1), su(l), ...  Workgroups j = 0 do that fold for the
// previous layer (its slot is the other buffer) and the feature padding.
template <int H, int K, int MODE>
__global__ void __launch_bounds__(kThreads) wide_start_s_kernel(WideArgs w) {
    constexpr int XS = (H < 2 * kMaxN ? 2 * kMaxN : H) + 4;
    const FlowArgs &a = w.a;
    const int N = a.N, D = 2 * N;
    const PackLayout PL = pack_layout(N, H, a.nb, a.K);
    const int lane = threadIdx.x & 63;
    const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int j = (int)blockIdx.y;
    const int64_t row0 = (int64_t)blockIdx.x * kRows, row = row0 + lane;
    float *CO = w.CO + row0 * D;
    float *X = w.XA + row0 * XS;
    const float *P = a.packed + (int64_t)w.layer * PL.stride;
    float *lu_cur = (w.layer & 1) ? w.LDU2 : w.LDU;
    if (j == 0 && w.pending) {
        const float *lu_prev = (w.layer & 1) ? w.LDU : w.LDU2;
        float ld = w.LDW[row * kWaves + wid];
        float su = 0.f;
        for (int f = wid; f < N; f += kWaves) su += lu_prev[row * N + f];
        ld += su;
        w.LDW[row * kWaves + wid] = wide_fold<K, MODE>(w, row, wid, ld);
    }
    const int f = wid + kWaves * j;
    if (f < N) {
        bool nan_any = false;
        lu_cur[row * N + f] = uncond_one<K, true>(P + PL.unc, CO, D, D, w.off, a, nan_any, f);
        if (nan_any && row < a.nrows && a.err) atomicOr(a.err, 1);
        const float v = CO[lane * D + (2 * f + w.off) % D];
        const float sv = a.scale_pf * v;
        X[lane * XS + f] = cosf(sv);
        X[lane * XS + N + f] = sinf(sv);
    }
    if (j == 0)
        for (int c = D + wid; c < 8 * PL.kg_in; c += kWaves) X[lane * XS + c] = 0.f;
}

// The start of a layer for the 16 rows of one trunk tile, then that tile's trunk: the
// periodic features go straight into the trunk's LDS image, which saves the start launch
// and the XA round trip.  Sampling modes write CO, LDU / LDU2 and LDW as
// wide_start_s_kernel does, density LDW as wide_start_kernel: the same device code on the
// same operands, so the pass stays bit-identical (tests/test_gpu_wide.py).
template <int H, bool HALF = false>
constexpr int trunk16s_waves() {  // twice the trunk's waves (the start's splines) up to 8; HALF: two per tile
    return HALF ? 2 * (H / 32) : (2 * (H / 32) < 8 ? 2 * (H / 32) : (H / 32 > 8 ? H / 32 : 8));
}

template <int H, int K, int MODE, bool HALF = false>
__global__ void __launch_bounds__((64 * trunk16s_waves<H, HALF>())) wide_trunk16s_kernel(WideArgs w) {
    constexpr int XS16 = Trunk16<H>::XS16;
    __shared__ __attribute__((aligned(16))) float X[16 * XS16];
    __shared__ float TU[MODE != MODE_DENSITY ? kMaxN * 3 * (K + 1) : 1];  // unconditional spline tables
    __shared__ __attribute__((aligned(16))) float Y[HALF ? 16 * XS16 : 4];  // trunk16h_run's second image
    const FlowArgs &a = w.a;
    const int N = a.N, D = 2 * N;
    const PackLayout PL = pack_layout(N, H, a.nb, a.K);
    const int64_t rowt = (int64_t)blockIdx.x * 16;
    if (w.pending)  // the previous final phase folded into LDW (wide_fold's order)
        for (int e = threadIdx.x; e < 16 * kWaves; e += blockDim.x) {
            const int64_t row = rowt + (e >> 3);
            const int vw = e & (kWaves - 1);
            float ld = w.LDW[row * kWaves + vw];
            if (MODE != MODE_DENSITY) {
                const float *lu_prev = (w.layer & 1) ? w.LDU : w.LDU2;
                float su = 0.f;
                for (int f = vw; f < N; f += kWaves) su += lu_prev[row * N + f];
                ld += su;
            }
            w.LDW[row * kWaves + vw] = wide_fold<K, MODE>(w, row, vw, ld);
        }
    const float *P = a.packed + (int64_t)w.layer * PL.stride;
    float *lu_cur = (w.layer & 1) ? w.LDU2 : w.LDU;
    // every thread's coordinates first (independent loads in flight together), the
    // sampling modes' spline tables staged in LDS (one coalesced pass), then the features
    constexpr int NW = trunk16s_waves<H, HALF>(), NT = 64 * NW, IT = (16 * kMaxN + NT - 1) / NT;
    float xv[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int e = (int)threadIdx.x + it * NT;
        if (e < 16 * N) xv[it] = w.CO[(rowt + (e & 15)) * D + (2 * (e >> 4) + w.off) % D];
    }
    const float *U = P + PL.unc;
    if (MODE != MODE_DENSITY) {
        const int nu = N * 3 * (K + 1);
        for (int e = threadIdx.x; e < nu; e += NT) TU[e] = U[e];
        __syncthreads();
    }
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int e = (int)threadIdx.x + it * NT;
        if (e >= 16 * N) break;
        const int rr = e & 15, f = e >> 4;
        const int64_t row = rowt + rr;
        float v = xv[it];
        if (MODE != MODE_DENSITY) {
            bool nan_any = false;
            const float x = v;
            lu_cur[row * N + f] = uncond_eval<K, true>(TU, x, a, nan_any, f, v);
            if ((x >= a.negB) && (x <= a.B)) w.CO[row * D + (2 * f + w.off) % D] = v;
            if (nan_any && row < a.nrows && a.err) atomicOr(a.err, 1);
        }
        const float sv = a.scale_pf * v;
        X[t16_pos(rr, f, XS16)] = cosf(sv);
        X[t16_pos(rr, N + f, XS16)] = sinf(sv);
    }
    const int npad = 8 * PL.kg_in - D;  // zero feature columns up to the k-group edge
    for (int e = threadIdx.x; e < 16 * npad; e += blockDim.x) {
        const int rr = e / npad;
        X[t16_pos(rr, D + e - rr * npad, XS16)] = 0.f;
    }
    __syncthreads();
    if constexpr (HALF)
        trunk16h_run<H, NW>(X, Y, w, rowt);
    else
        trunk16_run<H, NW>(X, w, rowt);
}

// ---------------------------------------------------------------------------
// Column-split trunk for small batches (trunk16 = 4): a 16-row tile's columns spread over G
// workgroups (CUs), each running 2 H / 32 / G of trunk16h_run's half-tile waves (the same
// MFMA chain per column, so bit-identical).  A CU's MFMA rate bounds the half-tile trunk
// however few rows there are (one tile takes as long per layer as 256 tiles on 256 CUs,
// profiles/r05/r05n_*); here every epilogue's column slice goes to the tile's other G - 1
// workgroups through an in-launch hand-off instead.  Its form is the guide's first Valid-forms
// row (MI355X_MICROARCH.md, inter-workgroup visibility): every slice stored sc1
// (write-through), each storing wave's vmcnt(0), a workgroup barrier, then ONE lane's
// agent-scope atomic add on the tile's counter; the consumer's lane 0 polls it with sc1
// loads, a barrier, then every load of the handed-off bytes is an sc1 buffer load.  The poll
// is bounded: a timeout sets err bit 2 and the workgroup stops waiting, so the grid always
// drains.  (The guide's tagged-granule form, each value an 8-byte {value, tag} sc1 store and
// every consumer thread re-reading its granules until the tags match, ran slower: 4.6-4.7
// against 4.2-4.3 ms per A1 N=16 pass at 16-64 rows, profiles/r05/r05ah_gsplit_granule.log.)
// Slices in XG[tile][step & 1][H][16] (column-major: a lane's four rows are one
// 16-byte store); counters CNT[launch & 1][tile], the other parity reset here for the next
// launch (the input kernel resets both).  Only workgroup 0 of a tile writes the start's
// side outputs (LDW, LDU, CO), the coordinates after the first hand-off, when every
// workgroup of the tile has read them.
#ifndef FS_GSPLIT
#define FS_GSPLIT 4  // workgroups (CUs) per 16-row tile
#endif
#ifndef FS_GSPLIT_XCD
#define FS_GSPLIT_XCD 1  // a tile's workgroups dealt to one XCD (0: consecutive blocks; A/B switch)
#endif
#ifndef FS_GSPLIT_AUTO_WG
#define FS_GSPLIT_AUTO_WG 128  // the default trunk's limit on column-split workgroups: up to 512
                               // rows.  A1 N=16 with a tile's workgroups on one XCD (r06,
                               // profiles/r06/r06e_gsplit_rows.log): 16-256 rows 3.8-4.0 ms per
                               // pass against 5.0-5.1 on the half-tile trunk, 384 rows 4.1 against
                               // 4.9, 512 rows 4.4 against 4.9 (r05, consecutive blocks: 512 rows
                               // 6.3-6.5 against 5.3, so the limit was 256 rows)
#endif
constexpr unsigned kGSpinMax = 1u << 20;  // default polls (sc1 load + s_sleep) before a hand-off gives up

template <int H>
constexpr bool gsplit_ok() {
    return 2 * (H / 32) % FS_GSPLIT == 0 && 2 * (H / 32) >= FS_GSPLIT;
}

template <int H, int K, int MODE, int G>
__global__ void __launch_bounds__(64 * (2 * (H / 32) / G)) wide_trunk16g_kernel(WideArgs w) {
    constexpr int XS = Trunk16<H>::XS, XS16 = Trunk16<H>::XS16;
    constexpr int NW = 2 * (H / 32) / G, NT = 64 * NW;  // waves / threads per workgroup
    constexpr int CPG = H / G;                          // columns per workgroup
    static_assert(NW >= 1 && NW * G == 2 * (H / 32), "G divides the trunk's half-tile waves");
    __shared__ __attribute__((aligned(16))) float X[16 * XS16];
    __shared__ __attribute__((aligned(16))) float Y[16 * XS16];
    __shared__ float TU[MODE != MODE_DENSITY ? kMaxN * 3 * (K + 1) : 1];
    __shared__ int dead_s;
    const FlowArgs &a = w.a;
    const int N = a.N, D = 2 * N;
    const PackLayout PL = pack_layout(N, H, a.nb, a.K);
#if FS_GSPLIT_XCD
    // a tile's G workgroups at equal blockIdx.x % 8 (one XCD under round-robin dealing; speed
    // only): b = (t % 8) + 8 (g + G (t / 8)); slots of tiles past T exit at once
    const int xb = (int)blockIdx.x & 7, yb = (int)blockIdx.x >> 3;
    const int g = yb % G, t = (yb / G) * 8 + xb;
    if (t >= w.T) return;
#else
    const int t = (int)blockIdx.x / G, g = (int)blockIdx.x - t * G;
#endif
    const int64_t rowt = (int64_t)t * 16;
    const int launch = MODE == MODE_DENSITY ? a.L - 1 - w.layer : w.layer;
    unsigned *cnt = w.CNT + (launch & 1) * w.T + t;
    if (threadIdx.x == 0) {
        dead_s = 0;
        if (g == 0)
            __hip_atomic_store(w.CNT + ((launch + 1) & 1) * w.T + t, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (g == 0 && w.pending)  // the previous final phase folded into LDW (wide_fold's order)
        for (int e = threadIdx.x; e < 16 * kWaves; e += NT) {
            const int64_t row = rowt + (e >> 3);
            const int vw = e & (kWaves - 1);
            float ld = w.LDW[row * kWaves + vw];
            if (MODE != MODE_DENSITY) {
                const float *lu_prev = (w.layer & 1) ? w.LDU : w.LDU2;
                float su = 0.f;
                for (int f = vw; f < N; f += kWaves) su += lu_prev[row * N + f];
                ld += su;
            }
            w.LDW[row * kWaves + vw] = wide_fold<K, MODE>(w, row, vw, ld);
        }
    const float *P = a.packed + (int64_t)w.layer * PL.stride;
    float *lu_cur = (w.layer & 1) ? w.LDU2 : w.LDU;
    constexpr int IT = (16 * kMaxN + NT - 1) / NT;
    float xv[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int e = (int)threadIdx.x + it * NT;
        if (e < 16 * N) xv[it] = w.CO[(rowt + (e & 15)) * D + (2 * (e >> 4) + w.off) % D];
    }
    const float *U = P + PL.unc;
    if (MODE != MODE_DENSITY) {
        const int nu = N * 3 * (K + 1);
        for (int e = threadIdx.x; e < nu; e += NT) TU[e] = U[e];
        __syncthreads();
    }
    float nv[IT], nl[IT];  // workgroup 0's deferred side outputs (sampling modes)
#pragma unroll
    for (int it = 0; it < IT; ++it) {
        const int e = (int)threadIdx.x + it * NT;
        if (e >= 16 * N) break;
        const int rr = e & 15, f = e >> 4;
        float v = xv[it];
        if (MODE != MODE_DENSITY) {
            bool nan_any = false;
            const float x = v;
            nl[it] = uncond_eval<K, true>(TU, x, a, nan_any, f, v);
            nv[it] = v;
            if (nan_any && g == 0 && rowt + rr < a.nrows && a.err) atomicOr(a.err, 1);
        }
        const float sv = a.scale_pf * v;
        X[t16_pos(rr, f, XS16)] = cosf(sv);
        X[t16_pos(rr, N + f, XS16)] = sinf(sv);
    }
    const int npad = 8 * PL.kg_in - D;
    for (int e = threadIdx.x; e < 16 * npad; e += NT) {
        const int rr = e / npad;
        X[t16_pos(rr, D + e - rr * npad, XS16)] = 0.f;
    }
    __syncthreads();
    auto flush_start = [&]() {
        if (MODE != MODE_DENSITY && g == 0)
#pragma unroll
            for (int it = 0; it < IT; ++it) {
                const int e = (int)threadIdx.x + it * NT;
                if (e >= 16 * N) break;
                const int64_t row = rowt + (e & 15);
                const int f = e >> 4;
                lu_cur[row * N + f] = nl[it];
                const float x = xv[it];
                if ((x >= a.negB) && (x <= a.B)) w.CO[row * D + (2 * f + w.off) % D] = nv[it];
            }
    };

    // the trunk (trunk16h_run on this workgroup's waves)
    const int lane = threadIdx.x & 63, q = lane >> 4, r = lane & 15;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int hw = g * NW + wv, tile = hw >> 1, c = hw & 1;
    const float *V = P + PL.vec;
    const __amdgpu_buffer_rsrc_t W =
        __builtin_amdgcn_make_buffer_rsrc((void *)P, (short)0, (int)(PL.stride * 4), 0x00020000);
    const __amdgpu_buffer_rsrc_t XGr =
        __builtin_amdgcn_make_buffer_rsrc((void *)(w.XG + (int64_t)t * 2 * H * 16), (short)0, 2 * H * 16 * 4, 0x00020000);
    const int col = 32 * tile + 16 * c + r;
    int pos[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) pos[i] = t16_pos(4 * q + i, col, XS16);
    // own slice (already in img at pos) out, the other workgroups' slices in
    auto hand_off = [&](int step, float *img, const f32x4 &v) {
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), XGr,
                                               (((step & 1) * H + col) * 16 + 4 * q) * 4, 0, 16);  // sc1
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // every wave's slice stored and drained, img's own columns written
        if (threadIdx.x == 0) {
            __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (!dead_s) {
                const unsigned target = (unsigned)(G * (step + 1));
                unsigned spins = 0;
                while (w.spin == 0 || __hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
                    __builtin_amdgcn_s_sleep(1);
                    if (++spins > w.spin) {
                        dead_s = 1;
                        if (a.err) atomicOr(a.err, 4);
                        break;
                    }
                }
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (compiler only: loads stay below)
        __syncthreads();
        if (step == 0) flush_start();
        for (int e = threadIdx.x; e < (H - CPG) * 4; e += NT) {
            const int cc = e >> 2, qq = e & 3;
            const int colf = cc < g * CPG ? cc : cc + CPG;
            const f32x4 f = __builtin_bit_cast(
                f32x4, __builtin_amdgcn_raw_buffer_load_b128(XGr, (((step & 1) * H + colf) * 16 + 4 * qq) * 4, 0, 16));
#pragma unroll
            for (int i = 0; i < 4; ++i) img[t16_pos(4 * qq + i, colf, XS16)] = f[i];
        }
        __syncthreads();
    };
    f32x4 hr, acc;
    f32x2 rb[FS_WIDE16H_PD];
    gemm16h_pre<FS_WIDE16H_PD>(W, (int)(PL.win * 4), PL.kg_in, tile, c, rb);
    gemm16h<XS16, FS_WIDE16H_PD, FS_WIDE16H_XB, false>(X, W, (int)(PL.win * 4), PL.kg_in, tile, c, hr, rb);
    for (int jb = 0; jb < a.nb; ++jb) {  // ResidualBlock (resnet.py:37-50), eval BN folded
        const float *VB = V + PL.v_blocks + (int64_t)4 * H * jb;
        const float e0 = VB[col], e1 = VB[H + col], e2 = VB[2 * H + col], e3 = VB[3 * H + col];
        const int w0 = (int)((PL.blocks + jb * PL.block_stride) * 4), w1 = w0 + (int)(PL.block_stride * 2);
        f32x4 v;
        gemm16h_pre<FS_WIDE16H_PD>(W, w0, PL.kg_h, tile, c, rb);
#pragma unroll
        for (int i = 0; i < 4; ++i) Y[pos[i]] = v[i] = FS_EPI(hr[i], e0, e1);
        hand_off(2 * jb, Y, v);
        gemm16h<XS16, FS_WIDE16H_PD, FS_WIDE16H_XB, false>(Y, W, w0, PL.kg_h, tile, c, acc, rb);
        gemm16h_pre<FS_WIDE16H_PD>(W, w1, PL.kg_h, tile, c, rb);
#pragma unroll
        for (int i = 0; i < 4; ++i) X[pos[i]] = v[i] = FS_EPI(acc[i], e2, e3);
        hand_off(2 * jb + 1, X, v);
        gemm16h<XS16, FS_WIDE16H_PD, FS_WIDE16H_XB, true>(X, W, w1, PL.kg_h, tile, c, hr, rb);  // h += Lin1(t)
    }
    const float sh = V[col];
#pragma unroll
    for (int i = 0; i < 4; ++i) w.XB[(rowt + 4 * q + i) * XS + col] = hr[i] + sh;
}

// Final layer + conditional spline of one feature unit (a transform feature, or a pair of
// them for K <= 16) per wave, for one 64-row block; (density) also the unconditional
// spline of the same-index identity feature(s).  WPB waves per workgroup share the
// block's final-layer input staged in LDS.  Log-dets go to LDC / LDU per feature; the
// next start / output launch adds them in the fused kernel's order (wide_fold).
template <int H, int K, int MODE, int WPB, int RB = kRows>
__global__ void __launch_bounds__(64 * WPB) wide_final_kernel(WideArgs w) {
    // RB = 32: 32-row blocks, half the MFMA chain per wave for batches that leave most of the
    // chip idle (or, K > 16, at two workgroups per CU); each chain's spline runs in both lane
    // halves, the lower one stores
    static_assert(RB == kRows || RB == 32, "64- or 32-row final blocks");
    constexpr int XS = (H < 2 * kMaxN ? 2 * kMaxN : H) + 4;
    constexpr int RM = RB - 1;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float *X = (float *)smem;
    const FlowArgs &a = w.a;
    const int N = a.N, D = 2 * N;
    const PackLayout PL = pack_layout(N, H, a.nb, a.K);
    const int lane = threadIdx.x & RM;
    const bool store = RB == kRows || (threadIdx.x & 32) == 0;
    const int u = __builtin_amdgcn_readfirstlane((int)blockIdx.y * WPB + (int)(threadIdx.x >> 6));
    const int64_t row0 = (int64_t)blockIdx.x * RB;
    const float *Xg = w.XB + row0 * XS;
    for (int e = threadIdx.x; e < RB * (H / 4); e += blockDim.x) {
        const int rr = e / (H / 4), q = e - rr * (H / 4);
        *(f32x4 *)(X + rr * XS + 4 * q) = *(const f32x4 *)(Xg + rr * XS + 4 * q);
    }
    __syncthreads();
    constexpr int UPF = K <= 16 ? 2 : 1;  // features per unit
    if (u * UPF >= N) return;
    float *CO = w.CO + row0 * D;
    const int cs = D, off = w.off;
    const float *P = a.packed + (int64_t)w.layer * PL.stride;
    const float *V = P + PL.vec;
    const __amdgpu_buffer_rsrc_t W =
        __builtin_amdgcn_make_buffer_rsrc((void *)P, (short)0, (int)(PL.stride * 4), 0x00020000);
    bool nan_any = false;
    Prof pf;
    float *lc = w.LDC + (row0 + lane) * N;
    if constexpr (K <= 16) {
        constexpr bool INV = MODE != MODE_DENSITY;
        constexpr int TS = INV ? 1 : 0;
        const int pp = u, ja = 2 * pp, jb = 2 * pp + 1;
        const bool hb = jb < N;
        const float *ba = V + PL.v_bf + 96 * ja;
        const float *bb = hb ? V + PL.v_bf + 96 * jb : ba + 16;
        f32x16 tS[2][1], tO[2][1];
        if constexpr (RB == kRows) {
            final_tile_pair<XS, kWideFPD>(X, W, (int)(PL.wf * 4), PL.kg_h, 2 * pp + TS, ba + 32 * TS, bb + 32 * TS, tS);
            final_tile_pair<XS, kWideFPD>(X, W, (int)(PL.wf * 4), PL.kg_h, 2 * pp + 1 - TS, ba + 32 * (1 - TS),
                                          bb + 32 * (1 - TS), tO);
        } else {
            final_tile_pair32<XS, kWideFPD>(X, W, (int)(PL.wf * 4), PL.kg_h, 2 * pp + TS, ba + 32 * TS, bb + 32 * TS,
                                            tS);
            final_tile_pair32<XS, kWideFPD>(X, W, (int)(PL.wf * 4), PL.kg_h, 2 * pp + 1 - TS, ba + 32 * (1 - TS),
                                            bb + 32 * (1 - TS), tO);
        }
        const float la = spline_from_tiles<XS, H, K, INV, RM>(tS, tO, 0, X, W,
                                                              (int)((PL.wd + (int64_t)ja * H * (K + 1)) * 4),
                                                              V + PL.v_bd + ja * (K + 1), CO, cs, (2 * ja + 1 + off) % D,
                                                              a, nan_any, pf);
        if (store) lc[ja] = la;
        if (hb) {
            const float lb = spline_from_tiles<XS, H, K, INV, RM>(tS, tO, 16, X, W,
                                                                  (int)((PL.wd + (int64_t)jb * H * (K + 1)) * 4),
                                                                  V + PL.v_bd + jb * (K + 1), CO, cs,
                                                                  (2 * jb + 1 + off) % D, a, nan_any, pf);
            if (store) lc[jb] = lb;
        }
    } else if constexpr (RB == kRows) {
        const int j = u;
        lc[j] = cond_spline<XS, H, K, MODE != MODE_DENSITY, kWideFPD>(
            X, W, (int)(PL.wf * 4), PL.kg_h, V + PL.v_bf + 96 * j, (int)((PL.wd + (int64_t)j * H * (K + 1)) * 4),
            V + PL.v_bd + j * (K + 1), CO, cs, (2 * j + 1 + off) % D, j, a, nan_any, pf);
    } else {  // K > 16 on 32-row blocks: cond_spline's tiles and spline, split as for the pairs
        constexpr bool INV = MODE != MODE_DENSITY;
        constexpr int TS = INV ? 1 : 0;
        const int j = u;
        const float *bf = V + PL.v_bf + 96 * j;
        f32x16 tS[2][1], tO[2][1];
        final_tile32<XS, kWideFPD>(X, W, (int)(PL.wf * 4), PL.kg_h, 2 * j + TS, bf + 32 * TS, tS);
        final_tile32<XS, kWideFPD>(X, W, (int)(PL.wf * 4), PL.kg_h, 2 * j + 1 - TS, bf + 32 * (1 - TS), tO);
        const float l = spline_from_tiles<XS, H, K, INV, RM>(tS, tO, 0, X, W,
                                                             (int)((PL.wd + (int64_t)j * H * (K + 1)) * 4),
                                                             V + PL.v_bd + j * (K + 1), CO, cs, (2 * j + 1 + off) % D,
                                                             a, nan_any, pf);
        if (store) lc[j] = l;
    }
    if (MODE == MODE_DENSITY && store) {
        float *lu = w.LDU + (row0 + lane) * N;
        for (int f = u * UPF; f < (u + 1) * UPF && f < N; ++f)
            lu[f] = uncond_at<K, false>(P + PL.unc, CO + lane * cs, (2 * f + off) % D, a, nan_any, f);
    }
    if (nan_any && store && row0 + lane < a.nrows && a.err) atomicOr(a.err, 1);
}

// The final phase on 16-row blocks (K <= 16, small batches): the feature pair's two tiles
// for 16 chains on v_mfma_f32_16x16x4_f32 fed the 32x32x2 k order (the 16-row trunk's
// trick: the same exact chain, bit-identical), a quarter of the 64-row blocks' MFMA chain
// per wave; the tiles go through LDS to one lane per (chain, feature), so the pair's two
// splines run side by side instead of one after the other.
// acc[c]: columns 16 c + 4 q + i of the pair tile (c = 0: feature a, 1: feature b) for the
// lane's chain r, bias preset (the bias add rides on the MFMAs, as in final_tile_pair).
template <int XS, int PD>
__device__ __forceinline__ void final_pair16(const float *__restrict__ X, __amdgpu_buffer_rsrc_t W, int sec, int kg,
                                             int tile, const float *__restrict__ ba, const float *__restrict__ bb,
                                             f32x4 (&acc)[2]) {
    const int lane = threadIdx.x & 63, q = lane >> 4, r = lane & 15, qo = q & 1, qh = q >> 1;
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[c][i] = (c == 0 ? ba : bb)[4 * q + i];
    const float *xr = X + r * XS + 4 * qo + qh;
    // lane (q, r) of half c takes the 32-row fragment's lane 32 qo + 16 c + r, elements qh, 2 + qh
    const int vb = (32 * qo + r) * 16;
    const int fb = sec + tile * kg * 1024;
    f32x4 rw[PD][2];
    float rx[PD][2];
#pragma unroll
    for (int s = 0; s < PD; ++s)
        if (s < kg) {
#pragma unroll
            for (int c = 0; c < 2; ++c) rw[s][c] = ldb_frag(W, vb + 256 * c, fb + s * 1024);
            rx[s][0] = xr[8 * s];
            rx[s][1] = xr[8 * s + 2];
        }
    for (int g0 = 0; g0 < kg; g0 += PD) {
#pragma unroll
        for (int s = 0; s < PD; ++s) {
            const int g = g0 + s;
            if (g < kg) {
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const float e0 = qh ? rw[s][c][1] : rw[s][c][0], e1 = qh ? rw[s][c][3] : rw[s][c][2];
                    acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(e0, rx[s][0], acc[c], 0, 0, 0);
                    acc[c] = __builtin_amdgcn_mfma_f32_16x16x4f32(e1, rx[s][1], acc[c], 0, 0, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
                const int gn = g + PD;
                if (gn < kg) {
#pragma unroll
                    for (int c = 0; c < 2; ++c) rw[s][c] = ldb_frag(W, vb + 256 * c, fb + gn * 1024);
                    rx[s][0] = xr[8 * gn];
                    rx[s][1] = xr[8 * gn + 2];
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
    }
}

template <int H, int K, int MODE, int WPB>
__global__ void __launch_bounds__(64 * WPB) wide_final16_kernel(WideArgs w) {
    static_assert(K <= 16, "16-row final blocks: feature pairs only");
    constexpr int XS = (H < 2 * kMaxN ? 2 * kMaxN : H) + 4;
    constexpr bool INV = MODE != MODE_DENSITY;
    constexpr int TS = INV ? 1 : 0;
    __shared__ __attribute__((aligned(16))) float X[16 * XS];
    __shared__ float T[WPB][2][16][33];  // per wave: the two tiles, chain-major (33: no bank conflicts)
    const FlowArgs &a = w.a;
    const int N = a.N, D = 2 * N;
    const PackLayout PL = pack_layout(N, H, a.nb, a.K);
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, q = lane >> 4, r = lane & 15;
    const int u = __builtin_amdgcn_readfirstlane((int)blockIdx.y * WPB + wv);
    const int64_t row0 = (int64_t)blockIdx.x * 16;
    const float *Xg = w.XB + row0 * XS;
    for (int e = threadIdx.x; e < 16 * (H / 4); e += blockDim.x) {
        const int rr = e / (H / 4), qq = e - rr * (H / 4);
        *(f32x4 *)(X + rr * XS + 4 * qq) = *(const f32x4 *)(Xg + rr * XS + 4 * qq);
    }
    __syncthreads();
    if (2 * u >= N) return;
    float *CO = w.CO + row0 * D;
    const int cs = D, off = w.off;
    const float *P = a.packed + (int64_t)w.layer * PL.stride;
    const float *V = P + PL.vec;
    const __amdgpu_buffer_rsrc_t W =
        __builtin_amdgcn_make_buffer_rsrc((void *)P, (short)0, (int)(PL.stride * 4), 0x00020000);
    const int pp = u, ja = 2 * pp, jb = 2 * pp + 1;
    const bool hb = jb < N;
    const float *ba = V + PL.v_bf + 96 * ja;
    const float *bb = hb ? V + PL.v_bf + 96 * jb : ba + 16;
    f32x4 tS[2], tO[2];
    final_pair16<XS, kWideFPD>(X, W, (int)(PL.wf * 4), PL.kg_h, 2 * pp + TS, ba + 32 * TS, bb + 32 * TS, tS);
    final_pair16<XS, kWideFPD>(X, W, (int)(PL.wf * 4), PL.kg_h, 2 * pp + 1 - TS, ba + 32 * (1 - TS),
                               bb + 32 * (1 - TS), tO);
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            T[wv][0][r][16 * c + 4 * q + i] = tS[c][i];
            T[wv][1][r][16 * c + 4 * q + i] = tO[c][i];
        }
    wave_lds_sync();  // this wave's tiles are in LDS
    // lane (f, chain): the spline of feature ja + f of chain lane & 15 (lanes 32-63 repeat
    // lanes 0-31 without storing)
    const int ch = lane & 15, f = (lane >> 4) & 1;
    const bool store = lane < 32;
    const int j = f ? jb : ja;
    bool nan_any = false;
    Prof pf;
    if (!f || hb) {
        float uS[K], uO[K];
#pragma unroll
        for (int k = 0; k < K; ++k) {
            uS[k] = T[wv][0][ch][16 * f + k];
            uO[k] = T[wv][1][ch][16 * f + k];
        }
        const float l = spline_from_logits<H, K, INV>(uS, uO, X + ch * XS, W,
                                                      (int)((PL.wd + (int64_t)j * H * (K + 1)) * 4),
                                                      V + PL.v_bd + j * (K + 1), CO + ch * cs, (2 * j + 1 + off) % D,
                                                      store, a, nan_any, pf);
        if (store) w.LDC[(row0 + ch) * N + j] = l;
        if (MODE == MODE_DENSITY && store) {
            const float lu = uncond_at<K, false>(P + PL.unc, CO + ch * cs, (2 * j + off) % D, a, nan_any, j);
            w.LDU[(row0 + ch) * N + j] = lu;
        }
    }
    if (nan_any && store && row0 + ch < a.nrows && a.err) atomicOr(a.err, 1);
}

template <int K, int MODE>
__global__ void __launch_bounds__(kThreads) wide_output_kernel(WideArgs w) {
    const FlowArgs &a = w.a;
    const int N = a.N, D = 2 * N;
    const int64_t row0 = (int64_t)blockIdx.x * kRows;
    const float *CO = w.CO + row0 * D;
    const int off = w.off;
    {
        const int vw = threadIdx.x >> 6;
        const int64_t row = row0 + (threadIdx.x & 63);
        float ld = w.LDW[row * kWaves + vw];
        if (MODE != MODE_DENSITY) {  // the last layer's unconditional log-dets (wide_start_s_kernel)
            const float *lu = (w.layer & 1) ? w.LDU2 : w.LDU;
            float su = 0.f;
            for (int f = vw; f < N; f += kWaves) su += lu[row * N + f];
            ld += su;
        }
        w.LDW[row * kWaves + vw] = wide_fold<K, MODE>(w, row, vw, ld);
    }
    __syncthreads();
    if (threadIdx.x < kRows) {
        const int lane = threadIdx.x;
        float tot = 0.f;
#pragma unroll
        for (int v = 0; v < kWaves; ++v) tot += w.LDW[(row0 + lane) * kWaves + v];
        float outv = tot;
        if (MODE == MODE_DENSITY && a.add_base) {
            bool inb = true;
            for (int i = 0; i < D; ++i) {
                const float z = CO[lane * D + i];
                inb = inb && (z >= a.negB) && (z <= a.B);
            }
            outv = tot + (inb ? a.base_lp : -INFINITY);
        }
        if (MODE == MODE_PROPOSE && a.add_base) outv = a.base_lp - tot;
        if (row0 + lane < a.nrows && a.scalar_out) a.scalar_out[row0 + lane] = outv;
    }
    for (int e = threadIdx.x; e < kRows * D; e += blockDim.x) {
        const int rr = e / D, i = e - rr * D;
        const int64_t gr = row0 + rr;
        if (gr >= a.nrows) continue;
        const float v = CO[rr * D + (i + off) % D];
        if (a.out) a.out[gr * D + i] = v;
        if (MODE == MODE_PROPOSE) {
            const float cfg = v + a.B;
            if (a.config) a.config[gr * D + i] = cfg;
            if (a.centered) a.centered[gr * D + i] = (float)((double)cfg - a.half_width);
        }
    }
}

// ---------------------------------------------------------------------------
// Packing kernels
// ---------------------------------------------------------------------------
// Every packing kernel covers all layers (blockIdx.y, raw / packed strides sl / dl) and,
// for the residual blocks, all blocks (blockIdx.z, strides sz / dz) in one launch.
// kind 0: plain linear W[nout][kin] (ResidualNet; lane values in kResPos order);  kind 1: final
// layer widths / heights (2 tiles per feature)
__global__ void pack_linear_kernel(float *__restrict__ dst, const float *__restrict__ src, int kin, int kg,
                                   int ntiles, int nout, int kind, int K, float wh_scale, int64_t sl, int64_t dl,
                                   int64_t sz, int64_t dz) {
    src += blockIdx.y * sl + blockIdx.z * sz;
    dst += blockIdx.y * dl + blockIdx.z * dz;
    const int64_t total = (int64_t)ntiles * kg * 256;
    const int P = 3 * K + 1;
    for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int pos = idx & 3;
        // kind 0 (ResidualNet): positions 0..3 hold j = 0, 2, 1, 3 (kResPos)
        const int j = kind == 0 ? (pos == 1 ? 2 : pos == 2 ? 1 : pos) : pos;
        const int lane = (idx >> 2) & 63;
        const int64_t tg = idx >> 8;
        const int g = (int)(tg % kg);
        const int tile = (int)(tg / kg);
        const int k = 8 * g + 4 * (lane >> 5) + j;
        const int c = lane & 31;
        int64_t row = -1;
        float sc = 1.f;
        if (kind == 0) {
            const int col = 32 * tile + c;
            row = col < nout ? col : -1;
        } else if (kind == 1) {
            const int feat = tile / 2, t = tile % 2;
            if (c < K) row = (int64_t)feat * P + t * K + c;
            sc = wh_scale;  // / sqrt(H) (coupling.py:340-342) and * log2(e) folded in
        } else {  // K <= 16: one tile per feature pair, feature 2p in columns 0..15, 2p+1 in 16..31
            const int pair = tile / 2, t = tile % 2, feat = 2 * pair + (c >> 4), cc = c & 15;
            if (feat < nout && cc < K) row = (int64_t)feat * P + t * K + cc;
            sc = wh_scale;
        }
        dst[idx] = (row >= 0 && k < kin) ? src[row * kin + k] * sc : 0.f;
    }
}

// derivative rows d_0..d_K of every feature (final-layer rows 2K..3K, unscaled) as
// [N][H/4][K+1][4]: cond_spline's per-lane gathers
__global__ void pack_deriv_kernel(float *__restrict__ dst, const float *__restrict__ src, int N, int H, int K,
                                  int64_t sl, int64_t dl) {
    src += blockIdx.y * sl;
    dst += blockIdx.y * dl;
    const int K1 = K + 1, P = 3 * K + 1;
    const int64_t total = (int64_t)N * H * K1;
    for (int64_t idx = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; idx < total;
         idx += (int64_t)gridDim.x * blockDim.x) {
        const int i = idx & 3;
        const int64_t t = idx >> 2;
        const int b = (int)(t % K1);
        const int64_t fq = t / K1;
        const int q = (int)(fq % (H / 4));
        const int feat = (int)(fq / (H / 4));
        dst[idx] = src[((int64_t)feat * P + 2 * K + b) * H + 4 * q + i];
    }
}

#pragma clang fp contract(off)
// vectors: biases, folded eval BatchNorm (alpha = w / sqrt(var + eps), beta = b - mean*alpha),
// final-layer biases in packed column order, unconditional-spline knots.
__global__ void pack_vec_kernel(float *__restrict__ dst, const float *__restrict__ src, int N, int H, int nb,
                                int K, double tail_bound, int64_t sl, int64_t dl) {
    src += blockIdx.y * sl;
    dst += blockIdx.y * dl;
    const RawLayout R = raw_layout(N, H, nb, K);
    const PackLayout PL = pack_layout(N, H, nb, K);
    float *V = dst + PL.vec;
    const int P = 3 * K + 1;
    const int tid = blockIdx.x * blockDim.x + threadIdx.x;
    const int nthr = gridDim.x * blockDim.x;
    // ResidualBlocks with the biases re-associated (the kernel's residual stream hr
    // omits b_in and the blocks' b1; S_jb = b_in + sum_{j<jb} b1_j is carried here):
    //   relu(BN0(h)) = relu(a0*hr + (c0 + a0*S_jb))        -> {a0, c0'}
    //   relu(BN1(Lin0 + b0)) = relu(a1*acc + (c1 + a1*b0))  -> {a1, c1'}
    //   final input h = hr + S_nb                           -> s_h = V[0:H)
    // with eval BN a = w / sqrt(var + eps), c = b - mean * a.
    const float eps = 1e-3f;
    for (int c = tid; c < H; c += nthr) {
        double S = src[R.bin + c];
        for (int jb = 0; jb < nb; ++jb) {
            const float *B = src + R.blocks + (int64_t)jb * R.block_stride;
            float *VB = V + PL.v_blocks + (int64_t)4 * H * jb;
            {
                const float w = B[c], b = B[H + c], m = B[2 * H + c], v = B[3 * H + c];
                const float al = (1.f / sqrtf(v + eps)) * w;
                VB[c] = al;
                VB[H + c] = (float)((double)(b - m * al) + (double)al * S);
            }
            {
                const float *B1 = B + RawLayout::bn1(H);
                const float w = B1[c], b = B1[H + c], m = B1[2 * H + c], v = B1[3 * H + c];
                const float al = (1.f / sqrtf(v + eps)) * w;
                VB[2 * H + c] = al;
                VB[3 * H + c] = (float)((double)(b - m * al) + (double)al * B[RawLayout::b0(H) + c]);
            }
            S += B[RawLayout::b1(H) + c];
        }
        V[c] = (float)S;
    }
    for (int i = tid; i < N * 96; i += nthr) {
        const int feat = i / 96, t = (i % 96) / 32, c = i % 32;
        // widths, heights: / sqrt(H) and * log2(e) folded in (the kernel's softmax uses exp2)
        const float sc = t < 2 ? (float)(1.4426950408889634 / sqrt((double)H)) : 1.f;
        V[PL.v_bf + i] = (c < K) ? (t < 2 ? src[R.bf + (int64_t)feat * P + t * K + c] * sc
                                         : src[R.bf + (int64_t)feat * P + t * K + c]) : 0.f;
    }
    for (int i = tid; i < PL.ntt * 32; i += nthr) V[PL.v_bt + i] = (i < N) ? src[R.bf + (int64_t)i * P + 3 * K] : 0.f;
    // derivative biases d_0..d_K per feature (cond_spline's gathers)
    for (int i = tid; i < N * (K + 1); i += nthr) V[PL.v_bd + i] = src[R.bf + (int64_t)(i / (K + 1)) * P + 2 * K + i % (K + 1)];
    // unconditional knots (PiecewiseRationalQuadraticCDF, coupling.py:227-259): batch independent
    const float B = (float)tail_bound, negB = (float)(-tail_bound);
    const int K1 = K + 1;
    for (int f = tid; f < N; f += nthr) {
        float *T = dst + PL.unc + (int64_t)f * 3 * K1;
        // batch independent, so computed in double and rounded once (the conditional
        // knots' rationale, knots_from_logits in flow_device.h)
        for (int which = 0; which < 2; ++which) {
            const float *u = src + (which == 0 ? R.uw : R.uh) + (int64_t)f * K;
            double m = u[0];
            for (int k = 1; k < K; ++k) m = fmax(m, (double)u[k]);
            double s = 0.0;
            for (int k = 0; k < K; ++k) s += exp((double)u[k] - m);
            const double mn = which == 0 ? kMinWd : kMinHd;
            const double sc = (1.0 - mn * (double)K) / s;
            double cum = 0.0;
            float *kn = T + which * K1;
            kn[0] = negB;
            for (int k = 0; k < K - 1; ++k) {
                cum += mn + sc * exp((double)u[k] - m);
                kn[k + 1] = (float)(2.0 * tail_bound * cum - tail_bound);
            }
            kn[K] = B;
        }
        const float *ud = src + R.ud + (int64_t)f * K1;
        for (int k = 0; k < K1; ++k) {  // min_derivative + softplus (threshold 20), rounded once
            const double x = ud[k];
            T[2 * K1 + k] = (float)(1e-3 + (x > 20.0 ? x : log1p(exp(x))));
        }
    }
}
#pragma clang fp contract(on)

// ---------------------------------------------------------------------------
// host-side launchers
// ---------------------------------------------------------------------------
template <int H, int K, int MODE>
static hipError_t launch_pass_t(const FlowArgs &a, int N, hipStream_t st) {
    auto kfn = flow_pass_kernel<H, K, MODE>;
    static std::atomic<unsigned long long> attr_set{0};  // per instantiation, bit d = device d
    if (hipError_t e = fs_set_max_lds_once((const void *)kfn, attr_set); e != hipSuccess) return e;
    const int64_t blocks = (a.nrows + kRows - 1) / kRows;
    hipLaunchKernelGGL(kfn, dim3((unsigned)blocks), dim3(kThreads), lds_layout(N, H).total, st, a);
    return hipGetLastError();
}

template <int MODE>
static hipError_t launch_pass_mode(const FlowArgs &a, int N, int H, int K, hipStream_t st) {
#define FS_CASE(HH, KK) \
    if (H == HH && K == KK) return launch_pass_t<HH, KK, MODE>(a, N, st);
    FS_FLOW_INSTANCES
#undef FS_CASE
    return hipErrorInvalidValue;
}

// ---------------------------------------------------------------------------
// wide path: host side
// ---------------------------------------------------------------------------
// Largest batch that takes the wide path (FS_WIDE_ROWS, or fs_set_wide_rows(); 0 disables
// it).  Above it the fused kernel has enough 64-row workgroups to occupy the chip.
static std::atomic<int64_t> g_wide_rows{-1};
static int64_t wide_rows_limit() {
    int64_t lim = g_wide_rows.load(std::memory_order_relaxed);
    if (lim < 0) {
        const char *e = getenv("FS_WIDE_ROWS");
        lim = e ? atoll(e) : 12288;
        if (lim < 0) lim = 0;
        int64_t expect = -1;
        g_wide_rows.compare_exchange_strong(expect, lim);
        lim = g_wide_rows.load(std::memory_order_relaxed);
    }
    return lim;
}

// Internal workspace of the wide path, one per (device, stream), allocated once at the
// size of the largest supported shape (never freed or moved: a captured graph may hold
// its address).  nullptr when it would have to be allocated during stream capture.
static void *wide_workspace(size_t bytes, hipStream_t st) {
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, std::pair<void *, size_t>> ws;
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) return nullptr;
    std::lock_guard<std::mutex> g(mu);
    auto &e = ws[{dev, st}];
    if (e.first && e.second >= bytes) return e.first;
    if (e.first) return nullptr;  // a larger shape than the first one sized for: fused kernel
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(st, &cs) != hipSuccess || cs != hipStreamCaptureStatusNone) return nullptr;
    void *p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    e = {p, bytes};
    return p;
}

constexpr int64_t kWideMaxRows = 65536;  // the workspace never grows beyond this many rows

// compute units of the current device (cached per device)
static int device_cus() {
    static std::atomic<int> cus[64];
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
    int v = cus[dev].load(std::memory_order_relaxed);
    if (v <= 0) {
        if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || v <= 0) v = 256;
        cus[dev].store(v, std::memory_order_relaxed);
    }
    return v;
}

// the trunk on 16-row tiles with the layer's start merged in and each 32-column tile split
// over two waves (wide_trunk16s_kernel<..., true>, 3, the default), the same with one wave per
// tile (2), on 16-row tiles after a separate start launch (1) or on 32-row ones (0);
// FS_WIDE_TRUNK16, fs_set_wide_trunk16.  Bit-identical in every setting.
static std::atomic<int> g_trunk16{-1};
static std::atomic<unsigned> g_gspin{kGSpinMax};
static int wide_trunk16() {
    int v = g_trunk16.load(std::memory_order_relaxed);
    if (v < 0) {
        const char *e = getenv("FS_WIDE_TRUNK16");
        int expect = -1;
        g_trunk16.compare_exchange_strong(expect, (e && e[0] >= '0' && e[0] <= '5') ? e[0] - '0' : 5);
        v = g_trunk16.load(std::memory_order_relaxed);
    }
    return v;
}

// the final phase on 16- or 32-row blocks for small batches (2, default), 32-row at most (1),
// or 64-row blocks (0): FS_WIDE_FINAL32, fs_set_wide_final32; bit-identical in every setting
static std::atomic<int> g_final32{-1};
static int wide_final32() {
    int v = g_final32.load(std::memory_order_relaxed);
    if (v < 0) {
        const char *e = getenv("FS_WIDE_FINAL32");
        int expect = -1;
        g_final32.compare_exchange_strong(expect, (e && (e[0] == '0' || e[0] == '1')) ? e[0] - '0' : 2);
        v = g_final32.load(std::memory_order_relaxed);
    }
    return v;
}

static size_t wide_bytes(int64_t R, int N, int H) {
    const int64_t XS = flow_xw(H) + 4;
    return (size_t)(rup(R * 2 * N * 4, 256) + 2 * rup(R * XS * 4, 256) + rup(R * kWaves * 4, 256) +
                    3 * rup(R * N * 4, 256) + rup(R * 2 * H * 4, 256) + rup((R / 16) * 2 * 4, 256));
}

struct WideLaunch {
    const void *func;
    dim3 grid, block;
    unsigned lds;
    WideArgs w;
};

// Replaying a pass: ~67 launches per A1 layer, each a few microseconds of GPU work, so
// launch overhead would dominate.  Outside stream capture the sequence is instantiated
// once as a HIP graph per (shape, image, workspace) and replayed; only the input and
// output launches see the call's own pointers and Philox keys, so they are the only
// nodes updated per call.  Inside a caller's capture the launches go straight into it.
struct WideGraph {
    std::vector<char> key;
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
    hipGraphNode_t first = nullptr, last = nullptr;
};

static std::vector<char> wide_key(const WideArgs &w, const void *kfn0, int H, int K, int mode, int variant) {
    WideArgs k = w;
    FlowArgs &a = k.a;  // the call-specific fields only the input / output launches read
    a.in = nullptr;
    a.out = a.scalar_out = a.config = a.centered = nullptr;
    a.seed = a.counter = 0;
    a.row_offset = a.rows_per_counter = 0;
    a.half_width = 0.0;
    a.add_base = 0;
    k.off = k.layer = k.jb = 0;
    std::vector<char> key(sizeof(WideArgs) + sizeof(void *) + 4 * sizeof(int));
    char *p = key.data();
    memset(p, 0, key.size());
    memcpy(p, &k, sizeof(WideArgs));
    memcpy(p + sizeof(WideArgs), &kfn0, sizeof(void *));
    const int hk[4] = {H, K, mode, variant};
    memcpy(p + sizeof(WideArgs) + sizeof(void *), hk, sizeof(hk));
    return key;
}

static hipError_t wide_run(const std::vector<WideLaunch> &seq, std::vector<char> key, hipStream_t st) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipError_t e = hipStreamIsCapturing(st, &cs); e != hipSuccess) return e;
    if (cs != hipStreamCaptureStatusNone) {
        for (const WideLaunch &l : seq) {
            WideArgs w = l.w;
            void *args[] = {&w};
            if (hipError_t e = hipLaunchKernel(l.func, l.grid, l.block, args, l.lds, st); e != hipSuccess) return e;
        }
        return hipSuccess;
    }
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, std::vector<WideGraph>> cache;  // most recent last
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev); e != hipSuccess) return e;
    std::lock_guard<std::mutex> g(mu);
    std::vector<WideGraph> &lst = cache[{dev, st}];
    int hit = -1;
    for (int i = 0; i < (int)lst.size(); ++i)
        if (lst[i].key == key) hit = i;
    auto params = [](const WideLaunch &l, WideArgs *w, void **args) {
        *w = l.w;
        args[0] = w;
        hipKernelNodeParams p;
        memset(&p, 0, sizeof(p));
        p.func = (void *)l.func;
        p.gridDim = l.grid;
        p.blockDim = l.block;
        p.sharedMemBytes = l.lds;
        p.kernelParams = args;
        p.extra = nullptr;
        return p;
    };
    if (hit < 0) {
        WideGraph wg;
        wg.key = std::move(key);
        if (hipError_t e = hipGraphCreate(&wg.graph, 0); e != hipSuccess) return e;
        hipGraphNode_t prev = nullptr;
        for (size_t i = 0; i < seq.size(); ++i) {
            WideArgs w;
            void *args[1];
            hipKernelNodeParams p = params(seq[i], &w, args);
            hipGraphNode_t node;
            hipError_t e = hipGraphAddKernelNode(&node, wg.graph, prev ? &prev : nullptr, prev ? 1 : 0, &p);
            if (e != hipSuccess) {
                (void)hipGraphDestroy(wg.graph);
                return e;
            }
            if (i == 0) wg.first = node;
            prev = node;
        }
        wg.last = prev;
        if (hipError_t e = hipGraphInstantiate(&wg.exec, wg.graph, nullptr, nullptr, 0); e != hipSuccess) {
            (void)hipGraphDestroy(wg.graph);
            return e;
        }
        if (lst.size() >= 16) {  // evict the least recently used (after the stream's work drains)
            (void)hipStreamSynchronize(st);
            (void)hipGraphExecDestroy(lst.front().exec);
            (void)hipGraphDestroy(lst.front().graph);
            lst.erase(lst.begin());
        }
        lst.push_back(std::move(wg));
    } else {
        WideGraph wg = std::move(lst[hit]);
        lst.erase(lst.begin() + hit);
        lst.push_back(std::move(wg));
        // this call's pointers / Philox keys: the input and output launches
        WideArgs w0, w1;
        void *a0[1], *a1[1];
        hipKernelNodeParams p0 = params(seq.front(), &w0, a0);
        hipKernelNodeParams p1 = params(seq.back(), &w1, a1);
        if (hipError_t e = hipGraphExecKernelNodeSetParams(lst.back().exec, lst.back().first, &p0); e != hipSuccess)
            return e;
        if (hipError_t e = hipGraphExecKernelNodeSetParams(lst.back().exec, lst.back().last, &p1); e != hipSuccess)
            return e;
    }
    return hipGraphLaunch(lst.back().exec, st);
}

template <int H, int K, int MODE>
static hipError_t wide_pass_t(const FlowArgs &a, int N, hipStream_t st, bool &used) {
    used = false;
    const int64_t R = rup(a.nrows, kRows);
    // one allocation per (device, stream), sized for at least 16384 rows at the widest
    // supported shape (~60 MB) or the current limit if larger
    const int64_t lim = wide_rows_limit() < 16384 ? 16384 : wide_rows_limit();
    const size_t cap = wide_bytes(rup(lim, kRows), kMaxN, 256);
    if (wide_bytes(R, N, H) > cap) return hipSuccess;
    char *p = (char *)wide_workspace(cap, st);
    if (!p) return hipSuccess;
    constexpr int XS = (H < 2 * kMaxN ? 2 * kMaxN : H) + 4;
    const int D = 2 * N;
    WideArgs w;
    memset(&w, 0, sizeof(w));
    w.a = a;
    w.R = R;
    w.CO = (float *)p;
    p += rup(R * D * 4, 256);
    w.XA = (float *)p;
    p += rup(R * XS * 4, 256);
    w.XB = (float *)p;
    p += rup(R * XS * 4, 256);
    w.LDW = (float *)p;
    p += rup(R * kWaves * 4, 256);
    w.LDC = (float *)p;
    p += rup(R * N * 4, 256);
    w.LDU = (float *)p;
    p += rup(R * N * 4, 256);
    w.LDU2 = (float *)p;
    p += rup(R * N * 4, 256);
    w.XG = (float *)p;  // the column-split trunk's hand-off slices and counters
    p += rup(R * 2 * H * 4, 256);
    w.CNT = (unsigned *)p;
    w.T = (int)(R / 16);
    w.spin = g_gspin.load(std::memory_order_relaxed);
    w.pending = 0;
    const unsigned nblk = (unsigned)(R / kRows);
#ifndef FS_WIDE_WPW
#define FS_WIDE_WPW 4
#endif
#ifndef FS_FINAL32_CUS
#define FS_FINAL32_CUS 1  // K > 16: 32-row final blocks while the grid is at most this many per CU
#endif
    constexpr int WPW = FS_WIDE_WPW;  // feature units (waves) per final-phase workgroup
    const int units = K <= 16 ? (N + 1) / 2 : N;
    const unsigned fin_lds = (unsigned)(kRows * XS * 4);
    {
        auto kf = wide_final_kernel<H, K, MODE, WPW>;
        static std::atomic<unsigned long long> attr_set{0};
        if (hipError_t e = fs_set_max_lds_once((const void *)kf, attr_set); e != hipSuccess) return e;
    }
    // 16-row trunk tiles while they fit the chip in one round (4096 rows on 256 CUs): past
    // that the 32-row tiles' higher arithmetic intensity wins (8192 rows: 9.0 vs 11.6 ms per
    // A1 N=16 pass, profiles/r04/)
    // 5 (default): the column-split trunk (4) for the A1 trunk (H = 256, 64 GEMMs per layer) on
    // batches of at most FS_GSPLIT_AUTO_WG / FS_GSPLIT tiles, else two waves per column tile (3).
    // 4 forces it wherever the tiles x FS_GSPLIT fit half the chip.
    // The column-split trunk reports a hand-off that gave up waiting only through err
    // (|= 4, its output is then wrong): without an err word to report it in, never take it.
    int trunk16 = R / 16 <= device_cus() ? wide_trunk16() : 0;
    const bool gfit = gsplit_ok<H>() && a.nb > 0 && a.err && (R / 16) * FS_GSPLIT <= device_cus() / 2;
    if (trunk16 == 5) trunk16 = (gfit && H >= 256 && (R / 16) * FS_GSPLIT <= FS_GSPLIT_AUTO_WG) ? 4 : 3;
    if (trunk16 == 4 && !gfit) trunk16 = 3;
    // 16- or 32-row final-phase blocks (feature pairs) while the grid fits the chip in a round;
    // K > 16 (one feature per wave): 32-row blocks on the same rule (at two workgroups per CU,
    // A1 N=16 4096 rows, no faster than 64-row blocks; 1024 rows ~2 % faster:
    // profiles/r05/r05y_final32_k32.log)
    const int fgy = (units + WPW - 1) / WPW, fsel = wide_final32();
    const int frows = K <= 16 ? ((fsel >= 2 && (R / 16) * fgy <= device_cus()) ? 16
                                 : (fsel >= 1 && (R / 32) * fgy <= device_cus()) ? 32 : kRows)
                              : ((fsel >= 1 && (R / 32) * fgy <= FS_FINAL32_CUS * device_cus()) ? 32 : kRows);
    const void *final_fn = (const void *)wide_final_kernel<H, K, MODE, WPW>;
    if (frows == 32) final_fn = (const void *)wide_final_kernel<H, K, MODE, WPW, 32>;
    if constexpr (K <= 16) {
        if (frows == 16) final_fn = (const void *)wide_final16_kernel<H, K, MODE, WPW>;
    }
    std::vector<WideLaunch> seq;
    seq.reserve(4 + (size_t)a.L * 3);
    auto add = [&](const void *f, dim3 g, dim3 b, unsigned lds) { seq.push_back({f, g, b, lds, w}); };
    add((const void *)wide_input_kernel<MODE>, dim3(nblk), dim3(256), 0);
    for (int s = 0; s < a.L; ++s) {
        w.layer = (MODE == MODE_DENSITY) ? a.L - 1 - s : s;
        if (MODE != MODE_DENSITY) w.off = (w.off + N) % D;
        w.pending = s > 0;
        if (trunk16 == 4) {
            if constexpr (gsplit_ok<H>())
                add((const void *)wide_trunk16g_kernel<H, K, MODE, FS_GSPLIT>,
                    dim3(FS_GSPLIT_XCD ? (unsigned)((R / 16 + 7) / 8) * 8 * FS_GSPLIT : (unsigned)(R / 16) * FS_GSPLIT),
                    dim3(64 * (2 * (H / 32) / FS_GSPLIT)), 0);
        } else if (trunk16 == 3)
            add((const void *)wide_trunk16s_kernel<H, K, MODE, true>, dim3((unsigned)(R / 16)),
                dim3(64 * trunk16s_waves<H, true>()), 0);
        else if (trunk16 == 2)
            add((const void *)wide_trunk16s_kernel<H, K, MODE>, dim3((unsigned)(R / 16)), dim3(64 * trunk16s_waves<H>()),
                0);
        else if (MODE == MODE_DENSITY)
            add((const void *)wide_start_kernel<H, K, MODE>, dim3(nblk), dim3(kThreads), 0);
        else
            add((const void *)wide_start_s_kernel<H, K, MODE>, dim3(nblk, kWaves), dim3(kThreads), 0);
        if (trunk16 == 1)
            add((const void *)wide_trunk16_kernel<H>, dim3((unsigned)(R / 16)), dim3(64 * (H / 32)), 0);
        else if (trunk16 == 0)
            add((const void *)wide_trunk_kernel<H>, dim3((unsigned)(R / 32)), dim3(64 * (H / 32)), 0);
        if (frows == 16)
            add(final_fn, dim3((unsigned)(R / 16), fgy), dim3(64 * WPW), 0);
        else if (frows == 32)
            add(final_fn, dim3((unsigned)(R / 32), fgy), dim3(64 * WPW), fin_lds / 2);
        else
            add(final_fn, dim3(nblk, fgy), dim3(64 * WPW), fin_lds);
        if (MODE == MODE_DENSITY) w.off = (w.off + N) % D;
    }
    w.pending = 1;
    add((const void *)wide_output_kernel<K, MODE>, dim3(nblk), dim3(kThreads), 0);
    w.off = w.layer = w.jb = w.pending = 0;
    hipError_t e = wide_run(seq, wide_key(w, seq.front().func, H, K, MODE, trunk16 | (frows << 4)), st);
    if (e == hipSuccess) used = true;
    return e;
}

template <int MODE>
static hipError_t wide_pass_mode(const FlowArgs &a, int N, int H, int K, hipStream_t st, bool &used) {
    used = false;
#define FS_CASE(HH, KK) \
    if (H == HH && K == KK) return wide_pass_t<HH, KK, MODE>(a, N, st, used);
    FS_FLOW_INSTANCES
#undef FS_CASE
    return hipSuccess;
}

}  // namespace fs

using namespace fs;

int32_t fs_set_wide_trunk16_impl(int32_t on) {
    const int32_t prev = wide_trunk16();
    if (on >= 0) g_trunk16.store(on > 5 ? 5 : on, std::memory_order_relaxed);
    return prev;
}

int64_t fs_set_wide_handoff_spins_impl(int64_t spins) {
    const int64_t prev = g_gspin.load(std::memory_order_relaxed);
    if (spins >= 0) g_gspin.store(spins > 0xffffffffll ? 0xffffffffu : (unsigned)spins, std::memory_order_relaxed);
    return prev;
}

int32_t fs_set_wide_final32_impl(int32_t on) {
    const int32_t prev = wide_final32();
    if (on >= 0) g_final32.store(on > 2 ? 2 : on, std::memory_order_relaxed);
    return prev;
}

int64_t fs_set_wide_rows_impl(int64_t rows) {
    const int64_t prev = wide_rows_limit();
    g_wide_rows.store(rows < 0 ? 0 : (rows > kWideMaxRows ? kWideMaxRows : rows), std::memory_order_relaxed);
    return prev;
}

#ifdef FS_PROF
extern "C" int fs_prof_read(unsigned long long *out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_prof), sizeof(unsigned long long) * 16) != hipSuccess) return 1;
    if (reset) {
        unsigned long long z[16] = {0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof(z)) != hipSuccess) return 1;
    }
    return 0;
}
#endif

bool fs_flow_supported(const fs_flow_dims *d, char *why, size_t n) {
    if (!d) return false;
    if (d->precision < 0 || d->precision > 2) {
        snprintf(why, n, "precision %d: 0 (f32 MFMA), 1 (bf16x6 split) or 2 (bf16x3 split)", d->precision);
        return false;
    }
    if (d->precision != 0 && !fs_flow_split_supported(d, why, n)) return false;
    bool ok_hk = d->precision != 0;
#define FS_CASE(HH, KK) ok_hk |= (d->H == HH && d->K == KK);
    FS_FLOW_INSTANCES
#undef FS_CASE
    if (!ok_hk) {
        snprintf(why, n, "unsupported (H=%d, K=%d): instantiated (H, K) pairs are listed in FS_FLOW_INSTANCES "
                 "(flow_kernels.hip)", d->H, d->K);
        return false;
    }
    if (d->N < 1 || d->N > kMaxN || d->L < 1 || d->nb < 0 || d->K < 1 || d->K > kMaxK || !(d->tail_bound > 0)) {
        snprintf(why, n, "invalid dims N=%d L=%d nb=%d K=%d B=%g (N<=%d, K<=%d)", d->N, d->L, d->nb, d->K,
                 d->tail_bound, kMaxN, kMaxK);
        return false;
    }
    if (2 * d->N > flow_xw(d->H)) {
        snprintf(why, n, "2N=%d input features exceed the activation tile width %d (H=%d)", 2 * d->N,
                 flow_xw(d->H), d->H);
        return false;
    }
    if (lds_layout(d->N, d->H).total > 163840) {
        snprintf(why, n, "LDS budget exceeded for N=%d H=%d", d->N, d->H);
        return false;
    }
    return true;
}

int64_t fs_flow_raw_floats_impl(const fs_flow_dims *d) {
    return raw_layout(d->N, d->H, d->nb, d->K).stride * d->L;
}

int64_t fs_flow_packed_bytes_impl(const fs_flow_dims *d) {
    if (d->precision != 0) return fs_flow_split_packed_bytes(d);
    return pack_layout(d->N, d->H, d->nb, d->K).stride * d->L * 4;
}

// The raw parameter image gathered from the layers' own tensors in one launch: chunk c of
// tab [n][3] = (source address, destination offset, length <= 8192 floats), one workgroup
// per chunk (the host builds the table once per set of tensor addresses).
__global__ void __launch_bounds__(256) gather_chunks_kernel(const int64_t *__restrict__ tab, float *__restrict__ dst) {
    const int64_t *t = tab + 3 * (int64_t)blockIdx.x;
    const float *src = (const float *)(uintptr_t)t[0];
    float *d = dst + t[1];
    const int64_t len = t[2];
    for (int64_t i = threadIdx.x; i < len; i += blockDim.x) d[i] = src[i];
}

hipError_t fs_gather_chunks_impl(const int64_t *tab, int64_t n, float *dst, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    if (n > 0x7fffffff) return hipErrorInvalidValue;
    hipLaunchKernelGGL(gather_chunks_kernel, dim3((unsigned)n), dim3(256), 0, st, tab, dst);
    return hipGetLastError();
}

hipError_t fs_flow_pack_vec(float *dst, const float *raw_layer, const fs_flow_dims *d, hipStream_t st) {
    hipLaunchKernelGGL(pack_vec_kernel, dim3(16), dim3(256), 0, st, dst, raw_layer, d->N, d->H, d->nb, d->K,
                       d->tail_bound, (int64_t)0, (int64_t)0);
    return hipGetLastError();
}

hipError_t fs_flow_pack_impl(const fs_flow_dims *d, const float *raw, float *packed, hipStream_t st) {
    if (d->precision != 0) return fs_flow_split_pack(d, raw, packed, st);
    const int N = d->N, H = d->H, nb = d->nb, K = d->K;
    const RawLayout R = raw_layout(N, H, nb, K);
    const PackLayout PL = pack_layout(N, H, nb, K);
    hipError_t e = hipMemsetAsync(packed, 0, (size_t)PL.stride * d->L * 4, st);
    if (e != hipSuccess) return e;
    // one launch per kind of matrix for all layers (and blocks): 6 launches, not ~8 per layer
    const unsigned NL = (unsigned)d->L;
    const int64_t sl = R.stride, dl = PL.stride;
    auto lin = [&](float *o, const float *w, int kin, int kg, int ntiles, int nout, int kind, unsigned nz, int64_t sz,
                   int64_t dz) {
        int64_t tot = (int64_t)ntiles * kg * 256;
        int blocks = (int)((tot + 255) / 256);
        if (blocks > 1024) blocks = 1024;
        hipLaunchKernelGGL(pack_linear_kernel, dim3(blocks, NL, nz), dim3(256), 0, st, o, w, kin, kg, ntiles, nout,
                           kind, K, (float)(1.4426950408889634 / sqrt((double)H)), sl, dl, sz, dz);
    };
    lin(packed + PL.win, raw + R.win, 2 * N, PL.kg_in, H / 32, H, 0, 1, 0, 0);
    if (nb > 0) {
        lin(packed + PL.blocks, raw + R.blocks + RawLayout::w0(H), H, PL.kg_h, H / 32, H, 0, (unsigned)nb,
            R.block_stride, PL.block_stride);
        lin(packed + PL.blocks + PL.block_stride / 2, raw + R.blocks + RawLayout::w1(H), H, PL.kg_h, H / 32, H, 0,
            (unsigned)nb, R.block_stride, PL.block_stride);
    }
    if (K <= 16)
        lin(packed + PL.wf, raw + R.wf, H, PL.kg_h, 2 * ((N + 1) / 2), N, 2, 1, 0, 0);  // feature pairs
    else
        lin(packed + PL.wf, raw + R.wf, H, PL.kg_h, 2 * N, 0, 1, 1, 0, 0);
    {
        const int64_t tot = (int64_t)N * H * (K + 1);
        int blocks = (int)((tot + 255) / 256);
        if (blocks > 1024) blocks = 1024;
        hipLaunchKernelGGL(pack_deriv_kernel, dim3(blocks, NL), dim3(256), 0, st, packed + PL.wd, raw + R.wf, N, H, K,
                           sl, dl);
    }
    hipLaunchKernelGGL(pack_vec_kernel, dim3(16, NL), dim3(256), 0, st, packed, raw, N, H, nb, K, d->tail_bound, sl,
                       dl);
    return hipGetLastError();
}

static void fill_args(FlowArgs &a, const fs_flow_dims *d, const void *packed, int64_t B) {
    memset(&a, 0, sizeof(a));
    a.packed = (const float *)packed;
    a.nrows = B;
    a.N = d->N;
    a.L = d->L;
    a.nb = d->nb;
    a.K = d->K;
    const double tb = d->tail_bound;
    a.B = (float)tb;
    a.twoB = (float)(2.0 * tb);
    a.negB = (float)(-tb);
    a.Bd = tb;
    a.twoBd = 2.0 * tb;
    a.scale_pf = (float)(M_PI / tb);
    a.sqrtH = (float)sqrt((double)d->H);
    // UniformParticle.log_prob: -D * torch.log(torch.tensor(2*B)) in float32
    const float lg = logf((float)(2.0 * tb));
    a.base_lp = (float)(-2 * d->N) * lg;
}

hipError_t fs_flow_pass_impl(const fs_flow_dims *d, const void *packed, int mode, const float *in, int64_t B,
                             float *out, float *scalar, int add_base, float *config, float *centered,
                             uint64_t seed, uint64_t counter, int64_t row_offset, double half_width,
                             int32_t *err, hipStream_t st, int64_t rows_per_counter) {
    if (B <= 0) return hipSuccess;
    FlowArgs a;
    fill_args(a, d, packed, B);
    a.in = in;
    a.out = out;
    a.scalar_out = scalar;
    a.add_base = add_base;
    a.config = config;
    a.centered = centered;
    a.seed = seed;
    a.counter = counter;
    a.row_offset = row_offset;
    a.rows_per_counter = rows_per_counter;
    a.half_width = half_width;
    a.err = err;
    if (d->precision != 0) return fs_flow_split_pass(a, mode, d->precision, d->N, d->H, d->K, st);
    if (B <= wide_rows_limit() && (B + kRows - 1) / kRows < 2 * 256) {
        // small batch: the wide path (bit-identical results), when its workspace is available
        bool used = false;
        hipError_t e = mode == MODE_DENSITY  ? wide_pass_mode<MODE_DENSITY>(a, d->N, d->H, d->K, st, used)
                       : mode == MODE_SAMPLE ? wide_pass_mode<MODE_SAMPLE>(a, d->N, d->H, d->K, st, used)
                                             : wide_pass_mode<MODE_PROPOSE>(a, d->N, d->H, d->K, st, used);
        if (e != hipSuccess || used) return e;
    }
    if (mode == MODE_DENSITY) return launch_pass_mode<MODE_DENSITY>(a, d->N, d->H, d->K, st);
    if (mode == MODE_SAMPLE) return launch_pass_mode<MODE_SAMPLE>(a, d->N, d->H, d->K, st);
    return launch_pass_mode<MODE_PROPOSE>(a, d->N, d->H, d->K, st);
}
