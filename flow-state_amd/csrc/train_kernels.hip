// Conditioner pieces of the Algorithm-2 training step (SURVEY §8(f) row 4,
// hybrid_NF_MCMC/main_algorithm_2.py:314-331) on the A2 shapes: batch 256, H = 128.
//
// gemm_f32_kernel: C = A . B (+ bias[n]) (+ R), exact f32 (v_mfma_f32_32x32x2_f32), A and B
// strided so that one kernel serves nn.Linear's forward (X W^T), its input gradient (dY W)
// and its weight gradient (dY^T X).  hipBLASLt runs a 256 x 128 x 128 product as one or two
// 128 x 256 macro tiles on one or two CUs (19 us); here every 32 x 32 output tile is one
// workgroup whose SPLIT waves share the reduction dimension and add their partial tiles in a
// fixed order (deterministic), so the same product spreads over 32 workgroups.
// The optional rowsum_a output (= sum_k A[m][k], written by the workgroups of the first
// column tile) is nn.Linear's bias gradient when A = dY^T.
//
// bn_relu_train_*: BatchNorm1d in train mode followed by ReLU (resnet.py:35-51, the
// block's batch_norm_layers[i] then the activation), forward and backward.  A workgroup
// owns 4 feature columns (64 row groups) over the whole batch, so the batch statistics are workgroup
// reductions in a fixed order: two-pass mean / biased variance, running statistics
// updated as torch does (momentum, unbiased variance), num_batches_tracked += 1.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

#include <atomic>

#include "fs_internal.h"

// Defaults from A/B builds of the A2 training step (tools/gpu_gemm_ab.sh, batch 256,
// profiles/r02/train/gemm_split_ab.log): 8 waves per tile, one k-block of loads in flight
// per wave: 113 steps/s against 106 for (4, 4, 2) and 109-112 for the other mixes.
// These GEMMs are latency-bound (2 to 4 k-blocks per wave): more waves each walking
// fewer k-blocks shorten the dependent chain more than deeper prefetch does.
#ifndef FS_GEMM_PF
#define FS_GEMM_PF 1  // k-blocks of operand loads in flight per wave
#endif
#ifndef FS_GEMM_SPLIT
#define FS_GEMM_SPLIT 8  // waves sharing one 32 x 32 tile's reduction (short K)
#endif
#ifndef FS_GEMM_SPLIT_MID
#define FS_GEMM_SPLIT_MID 8  // ... for 256 <= K <= 512 (the weight gradients at batch 256)
#endif
#ifndef FS_GEMM_SPLIT_LONG
#define FS_GEMM_SPLIT_LONG 16  // ... for K > 512
#endif

namespace fs {

typedef float t4 __attribute__((ext_vector_type(4)));
typedef float t16 __attribute__((ext_vector_type(16)));


// lane (r = lane & 31, h = lane >> 5) supplies A[m0 + r][kb + 4h + j] and B[kb + 4h + j][n0 + r]
// for MFMA step j = 0..3 of the 8-wide k-block kb (A and B use the same k order).
template <bool CONTIG>
__device__ __forceinline__ t4 load4(const float *p, int64_t stride, int64_t k0, int64_t K, bool ok) {
    t4 v = {0.f, 0.f, 0.f, 0.f};
    if (!ok) return v;  // no address outside the operand is formed (an empty operand may be NULL)
    if (CONTIG && k0 + 3 < K) {
        v = *(const t4 *)(p + k0);
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (k0 + j < K) v[j] = p[(k0 + j) * stride];
    }
    return v;
}

// BatchNorm running statistics, torch's momentum form (1 - m) r + m v, rounded per
// operation: no contraction into an FMA (which hipcc otherwise chooses per call site), so
// the in-launch and the deferred update agree bit for bit
__device__ __forceinline__ float running_update(float r, float v, float m) {
#pragma clang fp contract(off)
    const float a = (1.f - m) * r;
    const float b = m * v;
    return a + b;
}
__device__ __forceinline__ float unbiased(float var, int64_t rows) {
#pragma clang fp contract(off)
    const float p = var * (float)rows;
    return p / (float)(rows - 1);
}

// One step of Chan's pairwise update of a column's (n, mean, M2) by a tile of nb rows with
// statistics v = (tile mean, tile M2), rounded per operation (no contraction into FMAs, which
// the compiler would otherwise choose per call site and per constant), so that every
// BatchNorm-in-load prologue (generic, lean, the full-batch fast path) agrees bit for bit.
__device__ __forceinline__ void chan_update(float &n, float &mean, float &m2, float v_mean, float v_m2, float nb) {
#pragma clang fp contract(off)
    const float nn = n + nb, d = v_mean - mean;
    mean = mean + d * (nb / nn);
    m2 = m2 + v_m2 + d * d * (n * nb / nn);
    n = nn;
}

template <int SPLIT>
struct GemmLds {
    t16 part[SPLIT > 1 ? SPLIT - 1 : 1][64];
    float rs_part[SPLIT][64];
};

constexpr int kBnMaxK = 256;  // BatchNorm-in-load: widest A (the conditioner's hidden width)
constexpr int kBnStTiles = 8;  // producer tile statistics loaded per round (batch 256 = one round)
// k-blocks in flight per wave in the forward products (the A2 shapes: K = 128 over 8 waves
// = 2 k-blocks each, so all of a wave's operand loads go out before the prologue)
#ifndef FS_GEMM_BN_PF
#define FS_GEMM_BN_PF 2
#endif
constexpr int kBnPF = FS_GEMM_BN_PF;

// A operand with BatchNorm + ReLU applied on load (bn_relu_train_fwd's arithmetic).
struct BnLoad {
    const float *mu, *is, *gm, *bt;  // LDS, per k
    float *a_out;                    // nullable: u written back, [M][K] row-major
    int64_t lda;
    // the workgroups of column tile `by` of `nt` write u's 32-wide k slices ks with
    // ks % nt == by, so the write-back is spread over every column tile
    int64_t by, nt;
};

struct NoPrologue {
    __device__ void operator()() const {}
};

// One 32 x 32 output tile (bx, by) of g by the workgroup's SPLIT waves.  pro() runs after
// the first PF k-blocks of operand loads are issued and before they are used (the
// BatchNorm-in-load statistics prologue, whose own loads then share their round trip).
template <int SPLIT, bool AK, bool BK, bool BNA = false, int PF = FS_GEMM_PF, class Pro = NoPrologue>
__device__ __forceinline__ void gemm_tile(const GemmArgs &g, int64_t bx, int64_t by, GemmLds<SPLIT> &L,
                                          const BnLoad *bnl = nullptr, Pro pro = {}) {
    auto &part = L.part;
    auto &rs_part = L.rs_part;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int64_t m0 = bx * 32, n0 = by * 32;
    const bool aok = m0 + r < g.M, bok = n0 + r < g.N;
    const float *Ap = aok ? g.A + (m0 + r) * g.sam : g.A;
    const float *Bp = bok ? g.B + (n0 + r) * g.sbn : g.B;
    const bool rows = g.rowsum_a != nullptr && by == 0;
    t16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    float rs = 0.f;
    // PF k-blocks of loads in flight per wave (the operands come from L2 / the last
    // kernel's output, so the loop is latency-bound without them)
    const int64_t step = 8 * SPLIT;
    const int64_t kb0 = 8 * w;
    t4 a[PF], b[PF];
    // BNA: u = relu(gamma (x - mean) invstd + beta) of the loaded A elements (k < K only)
    auto bn = [&](t4 v, int64_t k0, bool ok) {
        if constexpr (BNA) {
            if (!ok) return v;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int64_t k = k0 + j;
                if (k < g.K) {
                    const float o = bnl->gm[k] * ((v[j] - bnl->mu[k]) * bnl->is[k]) + bnl->bt[k];
                    v[j] = o > 0.f ? o : 0.f;
                }
            }
            // k0 is a multiple of 4: the four elements sit in one 32-wide k slice
            if (bnl->a_out && (k0 >> 5) % bnl->nt == bnl->by) {
                float *dst = bnl->a_out + (m0 + r) * bnl->lda + k0;
                if (AK && k0 + 3 < g.K) {
                    *(t4 *)dst = v;  // 16-byte aligned: the host checks a_out and lda
                } else {
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        if (k0 + j < g.K) dst[j] = v[j];
                }
            }
        }
        return v;
    };
#pragma unroll
    for (int s = 0; s < PF; ++s) {
        const int64_t k = kb0 + s * step;
        a[s] = load4<AK>(Ap, g.sak, k + 4 * h, g.K, aok && k < g.K);
        b[s] = load4<BK>(Bp, g.sbk, k + 4 * h, g.K, bok && k < g.K);
    }
    // the epilogue's bias and residual operands (wave 0 writes the tile) loaded with the
    // first operands, so that their round trip is not left for after the reduction
    const int64_t col = n0 + r;
    float ep_bias = 0.f, ep_r[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) ep_r[i] = 0.f;
    if (SPLIT == 1 || w == 0) {
        ep_bias = (g.bias && bok) ? g.bias[col] : 0.f;
        if (g.R) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int64_t row = m0 + 8 * (i >> 2) + 4 * h + (i & 3);
                if (row < g.M && bok) ep_r[i] = g.R[row * g.ldr + col];
            }
        }
    }
    pro();
    if constexpr (BNA) {
#pragma unroll
        for (int s = 0; s < PF; ++s) {
            const int64_t k = kb0 + s * step;
            a[s] = bn(a[s], k + 4 * h, aok && k < g.K);
        }
    }
    for (int64_t kb = kb0; kb < g.K; kb += PF * step) {
#pragma unroll
        for (int s = 0; s < PF; ++s) {
            const int64_t k = kb + s * step;
            if (k < g.K) {  // wave-uniform
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s][j], b[s][j], acc, 0, 0, 0);
                if (rows) rs += ((a[s][0] + a[s][1]) + a[s][2]) + a[s][3];
                const int64_t kn = k + PF * step;
                a[s] = bn(load4<AK>(Ap, g.sak, kn + 4 * h, g.K, aok && kn < g.K), kn + 4 * h, aok && kn < g.K);
                b[s] = load4<BK>(Bp, g.sbk, kn + 4 * h, g.K, bok && kn < g.K);
            }
        }
    }
    if (SPLIT > 1) {
        if (w > 0) part[w - 1][lane] = acc;
        if (rows) rs_part[w][lane] = rs;
        __syncthreads();
        if (w > 0) return;
#pragma unroll 1
        for (int p = 0; p < SPLIT - 1; ++p) acc += part[p][lane];
        if (rows) {
#pragma unroll
            for (int p = 1; p < SPLIT; ++p) rs += rs_part[p][lane];
        }
    }
    if (rows) {  // the two k-halves of row m0 + r live in lanes r and r + 32
        rs += __shfl_xor(rs, 32);
        if (h == 0 && aok) g.rowsum_a[m0 + r] = rs;
    }
    const float bias = ep_bias;
    float sv = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int64_t row = m0 + 8 * (i >> 2) + 4 * h + (i & 3);
        float v = acc[i] + bias;
        if (row < g.M && bok) {
            if (g.R) v = v + ep_r[i];
            g.C[row * g.ldc + col] = v;
        }
        acc[i] = v;
        if (row < g.M) sv += v;
    }
    if (g.stats) {  // this tile's column mean and sum of squared deviations (the consumer's BatchNorm)
        const int64_t nr = g.M - m0 < 32 ? g.M - m0 : 32;
        const float mean = (sv + __shfl_xor(sv, 32)) / (float)nr;
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int64_t row = m0 + 8 * (i >> 2) + 4 * h + (i & 3);
            const float d = acc[i] - mean;
            if (row < g.M) q += d * d;
        }
        q += __shfl_xor(q, 32);
        if (h == 0 && bok) {
            g.stats[(bx * g.N + col) * 2] = mean;
            g.stats[(bx * g.N + col) * 2 + 1] = q;
        }
    }
}

template <int SPLIT, bool AK, bool BK>
__global__ __launch_bounds__(64 * SPLIT) void gemm_f32_kernel(GemmArgs g) {
    __shared__ GemmLds<SPLIT> L;
    gemm_tile<SPLIT, AK, BK>(g, blockIdx.x, blockIdx.y, L);
}

// The BatchNorm of a BatchNorm-in-load product: every workgroup combines the producer's
// tile statistics of all K columns (Chan's pairwise update, tiles in order; biased
// variance) into LDS; the problem's lead workgroup writes mean / invstd (/ var) and updates
// the running statistics.  Thread k owns column k (the host guarantees blockDim.x >= K) and
// loads its kBnStTiles (mean, M2) pairs of a round at once, straight into registers: one
// round trip per round and a single barrier, where staging the statistics through LDS
// cost two more barriers (profiles/r03/).
struct BnLds {
    float mu[kBnMaxK], is[kBnMaxK], gm[kBnMaxK], bt[kBnMaxK];
};

template <int NT>
__device__ __forceinline__ void bn_prologue(const GemmArgs &g, const BnIn &bn, bool lead, BnLds &S) {
    const int k = threadIdx.x;
    typedef float f2 __attribute__((ext_vector_type(2)));
    // gamma / beta loads issued with the statistics' (one round trip for all)
    const float gk = k < g.K ? bn.gamma[k] : 0.f, bk = k < g.K ? bn.beta[k] : 0.f;
    float n = 0.f, mean = 0.f, m2 = 0.f;
    if (k < g.K) {
        for (int64_t t0 = 0; t0 < bn.tiles; t0 += kBnStTiles) {
            const int nt = (int)(bn.tiles - t0 < kBnStTiles ? bn.tiles - t0 : kBnStTiles);
            const f2 *src = (const f2 *)bn.stats + t0 * g.K + k;  // [tile][K] pairs, 8-byte aligned
            f2 v[kBnStTiles];
#pragma unroll
            for (int t = 0; t < kBnStTiles; ++t) v[t] = t < nt ? src[t * g.K] : f2{0.f, 0.f};
#pragma unroll
            for (int t = 0; t < kBnStTiles; ++t) {  // Chan's pairwise update, tiles in order
                if (t < nt) {
                    const int64_t row0 = 32 * (t0 + t);
                    chan_update(n, mean, m2, v[t][0], v[t][1], (float)(bn.rows - row0 < 32 ? bn.rows - row0 : 32));
                }
            }
        }
    }
    if (k < g.K) {
        const float var = m2 / (float)bn.rows;
        const float invstd = 1.f / sqrtf(var + bn.eps);
        S.mu[k] = mean;
        S.is[k] = invstd;
        S.gm[k] = gk;
        S.bt[k] = bk;
        if (lead) {
            if (bn.mean_out) bn.mean_out[k] = mean;
            if (bn.invstd_out) bn.invstd_out[k] = invstd;
            if (bn.var_out) bn.var_out[k] = var;
            if (bn.running_mean) {
                bn.running_mean[k] = running_update(bn.running_mean[k], mean, bn.momentum);
                bn.running_var[k] = running_update(bn.running_var[k], unbiased(var, bn.rows), bn.momentum);
            }
        }
    }
    if (lead && threadIdx.x == 0 && bn.num_batches) *bn.num_batches += 1;
    __syncthreads();
}

// nn.Linear of relu(BatchNorm1d_train(x)): bn_prologue, then the tile with the BatchNorm +
// ReLU applied to A on load.
template <int SPLIT, bool AK, bool BK>
__global__ __launch_bounds__(64 * SPLIT) void gemm_bn_f32_kernel(GemmArgs g, BnIn bn) {
    __shared__ GemmLds<SPLIT> L;
    __shared__ BnLds S;
    const BnLoad bl{S.mu, S.is, S.gm, S.bt, bn.a_out, g.sam, blockIdx.y, gridDim.y};
    gemm_tile<SPLIT, AK, BK, true, kBnPF>(g, blockIdx.x, blockIdx.y, L, &bl,
                                         [&] { bn_prologue<64 * SPLIT>(g, bn, blockIdx.x == 0 && blockIdx.y == 0, S); });
}

// Two independent forward products in one launch (the training step's two passes: the
// density pass's Linear and the sampling pass's, of other layers): workgroups [0, t0) take
// the tiles of g0 (column-major over its mt0 row tiles), the rest those of g1; each problem
// with or without its BatchNorm-in-load (bit b of bnmask), each tile exactly as the
// single-problem kernels compute it.  A and B contiguous along k.
template <int SPLIT>
__global__ __launch_bounds__(64 * SPLIT) void gemm_ex2_kernel(GemmArgs g0, BnIn b0, GemmArgs g1, BnIn b1, unsigned t0,
                                                             unsigned mt0, unsigned mt1, int bnmask) {
    __shared__ GemmLds<SPLIT> L;
    __shared__ BnLds S;
    const bool second = blockIdx.x >= t0;
    const unsigned b = second ? blockIdx.x - t0 : blockIdx.x;
    const unsigned mt = second ? mt1 : mt0;
    const GemmArgs &g = second ? g1 : g0;
    const BnIn &bn = second ? b1 : b0;
    const unsigned bx = b % mt, by = b / mt;
    if (bnmask & (second ? 2 : 1)) {
        const BnLoad bl{S.mu, S.is, S.gm, S.bt, bn.a_out, g.sam, by, (g.N + 31) / 32};
        gemm_tile<SPLIT, true, true, true, kBnPF>(g, bx, by, L, &bl, [&] { bn_prologue<64 * SPLIT>(g, bn, bx == 0 && by == 0, S); });
    } else {
        gemm_tile<SPLIT, true, true, false, kBnPF>(g, bx, by, L);
    }
}

// ---------------------------------------------------------------------------
// Lean forward products.  nn.Linear's forward at the training shapes (A = x row-major
// [M][K], B = W row-major [N][K], K a multiple of 64 up to 256, N a multiple of 32) is
// every product of gemm_ex2_kernel / gemm_bn_f32_kernel and the contiguous ones of
// gemm_f32_kernel.  Those generic kernels carry 64-bit strided addressing, bounds tests per
// element and, for two problems per launch, more kernel arguments than SGPRs (spilled to
// VGPR lanes): 5.5 k instructions for gemm_ex2_kernel, a few thousand executed per wave
// around its 8 MFMAs.  gemm_lin_kernel computes the same tile with the same k order,
// partial-sum order, BatchNorm-in-load and epilogue arithmetic (bit-identical results,
// tests/test_gpu_train_fused.py), with 32-bit buffer offsets (rows past M read as zero
// through the buffer descriptor's range) and each problem's arguments read only by the
// workgroups that compute it.
struct LinP {
    const float *A, *W, *bias, *R;
    float *C, *stats;
    int M, N, ldr, ldc;
};
struct LinBn {
    const float *st, *gamma, *beta;
    float *mean_out, *invstd_out, *var_out, *a_out, *rm, *rv;
    int64_t *nbt;
    float eps, momentum;
    int tiles, on;
};
struct Lin2 {
    LinP p[2];
    LinBn b[2];
    unsigned t0, mt0, mt1;
};
struct LinLds {
    t16 part[7][64];
    BnLds S;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t lin_rsrc(const float *p, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)p, (short)0, bytes, 0x00020000);
}
__device__ __forceinline__ t4 lin_ld(__amdgpu_buffer_rsrc_t r, int off) {
    return __builtin_bit_cast(t4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

typedef float f2s __attribute__((ext_vector_type(2)));
// the first round of producer tile statistics (column k = thread k), loaded before the GEMM
// operands so that waiting for them does not wait for the operands (in-order vmcnt)
template <int K>
__device__ __forceinline__ void lin_bn_first(const LinBn &bn, f2s (&v)[kBnStTiles], float &gk, float &bk) {
    const int k = threadIdx.x;
    if (k < K) {
        const int nt = bn.tiles < kBnStTiles ? bn.tiles : kBnStTiles;
        const f2s *src = (const f2s *)bn.st + k;
#pragma unroll
        for (int t = 0; t < kBnStTiles; ++t) v[t] = t < nt ? src[t * K] : f2s{0.f, 0.f};
        gk = bn.gamma[k];
        bk = bn.beta[k];
    }
}

// bn_prologue's arithmetic (column k = thread k, Chan's update over the producer's tiles
// in order, biased variance, invstd; the lead workgroup's outputs and running statistics);
// v0 / gk / bk: lin_bn_first's loads
template <int K, bool FULL>
__device__ __forceinline__ void lin_bn_prologue(const LinBn &bn, int rows, bool lead, BnLds &S,
                                                const f2s (&v0)[kBnStTiles], float gk, float bk) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    const int k = threadIdx.x;
    if (k < K) {
        float n = 0.f, mean = 0.f, m2 = 0.f;
        if constexpr (FULL) {
            // the full training batch (256 rows, one round of 8 full tiles): the same update
            // with the tile sizes known, so its divisions fold to constants.  Bit-identical:
            // nb / nn and n nb / nn are correctly rounded quotients either way (the run-time
            // form below is the IEEE division) and chan_update rounds per operation.  0.45 us
            // per launch in a dependent chain (tools/probes/block_fuse: 9.45 -> 8.55 us per
            // block; tools/train_lin_chain.py 5.70 -> 5.28 us; profiles/r06/).
#pragma unroll
            for (int t = 0; t < kBnStTiles; ++t) chan_update(n, mean, m2, v0[t][0], v0[t][1], 32.f);
        } else {
            for (int t0 = 0; t0 < bn.tiles; t0 += kBnStTiles) {
                const int nt = bn.tiles - t0 < kBnStTiles ? bn.tiles - t0 : kBnStTiles;
                const f2 *src = (const f2 *)bn.st + t0 * K + k;
                f2 v[kBnStTiles];
#pragma unroll
                for (int t = 0; t < kBnStTiles; ++t) v[t] = t0 == 0 ? v0[t] : (t < nt ? src[t * K] : f2{0.f, 0.f});
#pragma unroll
                for (int t = 0; t < kBnStTiles; ++t) {
                    if (t < nt) {
                        const int row0 = 32 * (t0 + t);
                        chan_update(n, mean, m2, v[t][0], v[t][1], (float)(rows - row0 < 32 ? rows - row0 : 32));
                    }
                }
            }
        }
        const float var = m2 / (float)rows;
        const float invstd = 1.f / sqrtf(var + bn.eps);
        S.mu[k] = mean;
        S.is[k] = invstd;
        S.gm[k] = gk;
        S.bt[k] = bk;
        if (lead) {
            if (bn.mean_out) bn.mean_out[k] = mean;
            if (bn.invstd_out) bn.invstd_out[k] = invstd;
            if (bn.var_out) bn.var_out[k] = var;
            if (bn.rm) {
                bn.rm[k] = running_update(bn.rm[k], mean, bn.momentum);
                bn.rv[k] = running_update(bn.rv[k], unbiased(var, rows), bn.momentum);
            }
        }
    }
    if (lead && threadIdx.x == 0 && bn.nbt) *bn.nbt += 1;
    __syncthreads();
}

// FULL (the full training batch, bn.tiles == kBnStTiles and M == 32 kBnStTiles, uniform per
// problem): the producer statistics as unconditional buffer loads and the combine's fast
// path; the same loads and arithmetic, so the same bits (tools/probes/block_fuse's tile
// form: 4.3 us per BatchNorm-in-load product in a dependent chain).
template <int K, bool FULL>
__device__ __forceinline__ void lin_bn_first_t(const LinBn &bn, f2s (&v)[kBnStTiles], float &gk, float &bk) {
    if constexpr (FULL) {
        const int k = threadIdx.x;
        if (k < K) {
            const __amdgpu_buffer_rsrc_t Sr =
                __builtin_amdgcn_make_buffer_rsrc((void *)bn.st, (short)0, kBnStTiles * K * 8, 0x00020000);
#pragma unroll
            for (int t = 0; t < kBnStTiles; ++t)
                v[t] = __builtin_bit_cast(f2s, __builtin_amdgcn_raw_buffer_load_b64(Sr, (t * K + k) * 8, 0, 0));
            gk = bn.gamma[k];
            bk = bn.beta[k];
        }
    } else {
        lin_bn_first<K>(bn, v, gk, bk);
    }
}

// One 32 x 32 tile (bx, by) of P by 8 waves: wave w reduces the k-blocks 8w + 64s
template <int KBW, bool FULL = false>
__device__ __forceinline__ void lin_tile(const LinP &P, const LinBn &bn, unsigned bx, unsigned by, LinLds &L) {
    constexpr int K = 64 * KBW;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int M = P.M;
    const int m = (int)bx * 32 + r, col = (int)by * 32 + r;
    const bool aok = m < M;
    const __amdgpu_buffer_rsrc_t Ar = lin_rsrc(P.A, M * K * 4), Wr = lin_rsrc(P.W, P.N * K * 4);
    const int kq = 8 * w + 4 * h;  // this lane's first k in each k-block
    f2s st0[kBnStTiles];
    float gk = 0.f, bk = 0.f;
    if (bn.on) lin_bn_first_t<K, FULL>(bn, st0, gk, bk);
    t4 a[KBW], b[KBW];
#pragma unroll
    for (int s = 0; s < KBW; ++s) {
        a[s] = lin_ld(Ar, (m * K + kq + 64 * s) * 4);
        b[s] = lin_ld(Wr, (col * K + kq + 64 * s) * 4);
    }
    float ep_bias = 0.f, ep_r[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) ep_r[i] = 0.f;
    if (w == 0) {
        // buffer loads, the bias last: rows past M read zero, no per-row branch, and no load
        // waits for another's result register (the bias's once fed an address computation)
        if (P.R) {
            const __amdgpu_buffer_rsrc_t Rr = lin_rsrc(P.R, M * P.ldr * 4);
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int row = (int)bx * 32 + 8 * (i >> 2) + 4 * h + (i & 3);
                ep_r[i] = __builtin_bit_cast(
                    float, __builtin_amdgcn_raw_buffer_load_b32(Rr, (row < M ? row * P.ldr + col : M * P.ldr) * 4, 0, 0));
            }
        }
        if (P.bias)
            ep_bias = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(lin_rsrc(P.bias, P.N * 4), col * 4, 0, 0));
    }
    if (bn.on) {
        lin_bn_prologue<K, FULL>(bn, M, bx == 0 && by == 0, L.S, st0, gk, bk);
        const int nt = P.N / 32;
#pragma unroll
        for (int s = 0; s < KBW; ++s) {
            const int k0 = kq + 64 * s;
            if (aok) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int k = k0 + j;
                    const float o = L.S.gm[k] * ((a[s][j] - L.S.mu[k]) * L.S.is[k]) + L.S.bt[k];
                    a[s][j] = o > 0.f ? o : 0.f;
                }
                if (bn.a_out && (k0 >> 5) % nt == (int)by) *(t4 *)(bn.a_out + m * K + k0) = a[s];
            }
        }
    }
    t16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
#pragma unroll
    for (int s = 0; s < KBW; ++s)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s][j], b[s][j], acc, 0, 0, 0);
    if (w > 0) L.part[w - 1][lane] = acc;
    __syncthreads();
    if (w > 0) return;
#pragma unroll 1
    for (int p = 0; p < 7; ++p) acc += L.part[p][lane];
    const float bias = ep_bias;
    float sv = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int row = (int)bx * 32 + 8 * (i >> 2) + 4 * h + (i & 3);
        float v = acc[i] + bias;
        if (row < M) {
            if (P.R) v = v + ep_r[i];
            P.C[row * P.ldc + col] = v;
        }
        acc[i] = v;
        if (row < M) sv += v;
    }
    if (P.stats) {
        const int nr = M - (int)bx * 32 < 32 ? M - (int)bx * 32 : 32;
        const float mean = (sv + __shfl_xor(sv, 32)) / (float)nr;
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int row = (int)bx * 32 + 8 * (i >> 2) + 4 * h + (i & 3);
            const float d = acc[i] - mean;
            if (row < M) q += d * d;
        }
        q += __shfl_xor(q, 32);
        if (h == 0) {
            P.stats[((int)bx * P.N + col) * 2] = mean;
            P.stats[((int)bx * P.N + col) * 2 + 1] = q;
        }
    }
}

static bool lin_full(const LinP &P, const LinBn &bn) {
    return bn.tiles == kBnStTiles && P.M == 32 * kBnStTiles;
}

// workgroups [0, t0) compute problem 0 (column-major over its mt0 row tiles), the rest
// problem 1; the branch is uniform, so each workgroup reads only its own problem's arguments
// FULL: every BatchNorm-in-load problem of the launch is a full training batch (lin_full;
// the host picks the kernel), so the generic kernel keeps its register budget (74 VGPRs, three
// workgroups per CU for the final Linear's 1472-workgroup launch) and the hidden layers'
// BatchNorm-in-load products take the full-batch form
template <int KBW, bool FULL>
__global__ __launch_bounds__(512) void gemm_lin_kernel(Lin2 a) {
    __shared__ LinLds L;
    const unsigned b = blockIdx.x;
    if (b < a.t0) {
        lin_tile<KBW, FULL>(a.p[0], a.b[0], b % a.mt0, b / a.mt0, L);
    } else {
        const unsigned c = b - a.t0;
        lin_tile<KBW, FULL>(a.p[1], a.b[1], c % a.mt1, c / a.mt1, L);
    }
}

// Lean general products: any of the strided layouts gemm_tile takes (A[m][k] at
// A[m sam + k sak], B[k][n] at B[k sbk + n sbn]; AK / BK: contiguous along k), with the
// row sum, at 8 waves per tile: nn.Linear's backward pair (the input gradient dY W and the
// weight / bias gradient dY^T X), the final Linear's backward group (split-K input
// gradient, weight gradient, the unconditional spline's row sum) and the single products
// outside the forward layout.  gemm_tile's k order (wave w: k-blocks 8w + 64s ascending),
// partial-sum order, row sum and epilogue, so the results are bit-identical to it, with
// 32-bit buffer offsets: the descriptors' byte ranges are the operands' extents and a lane
// loads only quads below K, so nothing past an operand (or a split-K chunk) is read and
// no per-element test is needed.  Loads run kLingPF k-blocks ahead of the MFMAs.
struct LinG {
    const float *A, *B, *bias, *R;
    float *C, *stats, *rowsum;
    int M, N, K, sam, sak, sbk, sbn, ldr, ldc, abytes, bbytes;
    int pstats;  // (fs_linear_f32_pair_bn, producer) per-tile BatchNorm-backward sums of C
    int ach, astr;  // A = the ordered sum of ach split-K partials astr floats apart (ach = 1: A itself)
    float *aout;    // (ach > 1, row-major A) the summed A written out by the first column tile
};
// A BatchNorm1d (train) + ReLU backward folded into the backward pairs on either side of it
// (fs_linear_f32_pair_bn): the producer pair's input gradient is the BatchNorm output's
// gradient gu; its epilogue writes per 32-row tile the column sums of dz = gu (u > 0) and
// dz xhat; the consumer pair loads dy = BatchNorm-input gradient on the fly from gu, u, y
// and the combined sums (bn_relu_train_bwd_kernel's formula), so dy is never written and
// the BatchNorm backward launch disappears.  Workgroup 0 of the consumer writes dgamma,
// dbeta.
// (struct BnFold: fs_internal.h)
constexpr int kFoldMaxH = 256;
struct LinGLds {
    t16 part[7][64];
    float rs_part[8][64];
};
struct LinGFLds : LinGLds {  // gemm_ling_fold_kernel: + the folded BatchNorm's column terms
    float mdb[kFoldMaxH], mdg[kFoldMaxH], mu[kFoldMaxH], is[kFoldMaxH], sc[kFoldMaxH];
};
constexpr int kLingPF = 4;

template <bool CONTIG>
__device__ __forceinline__ t4 ling_ld(__amdgpu_buffer_rsrc_t r, int base, int stride) {
    if (CONTIG) return lin_ld(r, base * 4);
    t4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        v[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, (base + j * stride) * 4, 0, 0));
    return v;
}

// the BatchNorm-input gradient of one element (bn_relu_train_bwd_kernel's dx, no dx_add)
__device__ __forceinline__ float fold_dx(float g, float u, float y, const LinGFLds &L, int c) {
    const float dz = u > 0.f ? g : 0.f;
    const float xh = (y - L.mu[c]) * L.is[c];
    return (dz - L.mdb[c] - xh * L.mdg[c]) * L.sc[c];
}

// V = 1: A is dy [B][H] (k = column), V = 2: A is dy^T (m = column); a quad of A from gu, u, y
// (loaded into the ring raw, turned into dy right before its MFMAs)
constexpr int kSkMax = 3;  // split-K partials an operand may be summed from on load
template <bool RSK>
struct FoldQ {
    t4 g, u, y, r;          // r: the residual gradient (dx_add), zero without one
    t4 rz[RSK ? kSkMax - 1 : 1];  // (RSK) its split-K partials 1.. (r: partial 0)
};

// a quad of a row-major (V = 1) or transposed operand
template <int V>
__device__ __forceinline__ t4 quad_ld(__amdgpu_buffer_rsrc_t R, int base, int stride) {
    if (V == 1) return lin_ld(R, base * 4);
    t4 v;
#pragma unroll
    for (int j = 0; j < 4; ++j)
        v[j] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(R, (base + j * stride) * 4, 0, 0));
    return v;
}

// RSK: dx_add is the ordered sum of nch split-K partials rstr floats apart (the reduction
// splitk_reduce_kernel would have written, summed here on load instead)
template <int V, bool RSK>
__device__ __forceinline__ FoldQ<RSK> fold_raw(__amdgpu_buffer_rsrc_t Gr, __amdgpu_buffer_rsrc_t Ur,
                                               __amdgpu_buffer_rsrc_t Yr, __amdgpu_buffer_rsrc_t Rr, bool add,
                                               int base, int stride, int nch = 1, int rstr = 0) {
    FoldQ<RSK> q;
    const t4 zero = {0.f, 0.f, 0.f, 0.f};
    q.g = quad_ld<V>(Gr, base, stride);
    q.u = quad_ld<V>(Ur, base, stride);
    q.y = quad_ld<V>(Yr, base, stride);
    q.r = add ? quad_ld<V>(Rr, base, stride) : zero;
    if constexpr (RSK) {
#pragma unroll
        for (int z = 1; z < kSkMax; ++z) q.rz[z - 1] = z < nch ? quad_ld<V>(Rr, base + z * rstr, stride) : zero;
    }
    return q;
}

// dy of a quad (+ the residual gradient when the BatchNorm backward had one: dx_add)
template <int V, bool RSK>
__device__ __forceinline__ t4 fold_apply(const FoldQ<RSK> &q, int c, const LinGFLds &L, bool add, int nch = 1) {
    t4 r = q.r;
    if constexpr (RSK) {  // splitk_reduce_kernel's order: partials 0, 1, ..., then + 0 (no bias)
#pragma unroll
        for (int z = 1; z < kSkMax; ++z)
            if (z < nch) r = r + q.rz[z - 1];
        r = r + 0.f;
    }
    t4 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const float d = fold_dx(q.g[j], q.u[j], q.y[j], L, V == 1 ? c + j : c);
        o[j] = add ? d + r[j] : d;
    }
    return o;
}

// V: (fold consumer) A loaded as dy, 1 row-major, 2 transposed; PS: (fold producer) the
// epilogue's tile sums; both only in gemm_ling_fold_kernel (LDS = LinGFLds).  SK: (V = 0) A is
// the ordered sum of P.ach split-K partials, (V != 0) so is the residual gradient dx_add
// (F.add_ch partials): the reduction is done on load, in splitk_reduce_kernel's order
template <bool AK, bool BK, int V = 0, bool PS = false, class LDS = LinGLds, bool SK = false>
__device__ __forceinline__ void ling_tile(const LinG &P, unsigned bx, unsigned by, LDS &L, const BnFold &F,
                                          const BnFold &Fo) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int M = P.M, N = P.N, K = P.K;
    const int m = (int)bx * 32 + r, col = (int)by * 32 + r;
    const bool rows = P.rowsum != nullptr && by == 0;
    // rows past M / columns past N: an offset past the operand, read as zero
    const int am = m < M ? m * P.sam : P.abytes / 4, bn = col < N ? col * P.sbn : P.bbytes / 4;
    const __amdgpu_buffer_rsrc_t Ar = lin_rsrc(P.A, P.abytes), Br = lin_rsrc(P.B, P.bbytes);
    __amdgpu_buffer_rsrc_t Gr = Ar, Ur = Ar, Yr = Ar, Rr = Ar;
    const bool fadd = V != 0 && F.dx_add != nullptr;
    // (V = 1) this row tile's dy written out by the first column tile's workgroup
    float *const aout = (V == 1 && by == 0 && F.a_out && m < M) ? F.a_out : nullptr;
    // (SK, V = 0) this row tile's summed A written out by the first column tile's workgroup
    float *const skout = (SK && V == 0 && AK && by == 0 && P.aout && m < M) ? P.aout : nullptr;
    if constexpr (V != 0) {
        Gr = lin_rsrc(F.gu, P.abytes);
        Ur = lin_rsrc(F.u, P.abytes);
        Yr = lin_rsrc(F.y, P.abytes);
        if (fadd) Rr = lin_rsrc(F.dx_add, P.abytes + (SK ? (F.add_ch - 1) * F.add_str * 4 : 0));
    }
    const int mc = m < M ? m : 0;  // (V = 2) the column of A's row m
    const t4 zero = {0.f, 0.f, 0.f, 0.f};
    constexpr bool ASK = SK && V == 0, RSK = SK && V != 0;
    t4 a[kLingPF], b[kLingPF];
    t4 az[ASK ? kLingPF : 1][ASK ? kSkMax - 1 : 1];  // (ASK) A's partials 1.. (a: partial 0)
    FoldQ<RSK> q[V != 0 ? kLingPF : 1];
    const int kb0 = 8 * w;
    const int ach = ASK ? P.ach : 1, rch = RSK ? F.add_ch : 1, rstr = RSK ? F.add_str : 0;
#pragma unroll
    for (int s = 0; s < kLingPF; ++s) {
        const int k = kb0 + 64 * s + 4 * h;
        if constexpr (V != 0) {
            if (k < K) q[s] = fold_raw<V, RSK>(Gr, Ur, Yr, Rr, fadd, am + k * P.sak, P.sak, rch, rstr);
        } else {
            a[s] = k < K ? ling_ld<AK>(Ar, am + k * P.sak, P.sak) : zero;
            if constexpr (ASK) {
#pragma unroll
                for (int z = 1; z < kSkMax; ++z)
                    az[s][z - 1] = (k < K && z < ach) ? ling_ld<AK>(Ar, am + k * P.sak + z * P.astr, P.sak) : zero;
            }
        }
        b[s] = k < K ? ling_ld<BK>(Br, bn + k * P.sbk, P.sbk) : zero;
    }
    if constexpr (V != 0) {  // the folded BatchNorm's column sums (their loads under the ring's)
        for (int t = threadIdx.x; t < F.H; t += blockDim.x) {
            float db = 0.f, dg = 0.f;
            for (int i0 = 0; i0 < F.tiles; i0 += 8) {  // 8 tiles' loads in flight, added in order
                float pd[8], px[8];
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (i0 + j < F.tiles) {
                        pd[j] = F.part[((int64_t)(i0 + j) * F.H + t) * 2];
                        px[j] = F.part[((int64_t)(i0 + j) * F.H + t) * 2 + 1];
                    }
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    if (i0 + j < F.tiles) {
                        db += pd[j];
                        dg += px[j];
                    }
            }
            const float is = F.invstd[t];
            L.mdb[t] = db / (float)F.B;
            L.mdg[t] = dg / (float)F.B;
            L.mu[t] = F.mean[t];
            L.is[t] = is;
            L.sc[t] = is * F.gamma[t];
            if (blockIdx.x == 0) {
                if (F.dgamma) F.dgamma[t] = dg;
                if (F.dbeta) F.dbeta[t] = db;
            }
        }
        __syncthreads();
    }
    float ep_bias = 0.f, ep_r[16], ps_u[16], ps_y[16], ps_mu = 0.f, ps_is = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) ep_r[i] = ps_u[i] = ps_y[i] = 0.f;
    if (w == 0 && col < N) {
        ep_bias = P.bias ? P.bias[col] : 0.f;
        if (P.R) {
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int row = (int)bx * 32 + 8 * (i >> 2) + 4 * h + (i & 3);
                if (row < M) ep_r[i] = P.R[row * P.ldr + col];
            }
        }
        if (PS) {  // the folded BatchNorm's u, y at this lane's outputs (issued early)
            ps_mu = Fo.mean[col];
            ps_is = Fo.invstd[col];
#pragma unroll
            for (int i = 0; i < 16; ++i) {  // rows past M read row M - 1 (excluded from the sums)
                int row = (int)bx * 32 + 8 * (i >> 2) + 4 * h + (i & 3);
                row = row < M ? row : M - 1;
                ps_u[i] = Fo.u[row * P.ldc + col];
                ps_y[i] = Fo.y[row * P.ldc + col];
            }
        }
    }
    t16 acc;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] = 0.f;
    float rs = 0.f;
    for (int kb = kb0; kb < K; kb += 64 * kLingPF) {
#pragma unroll
        for (int s = 0; s < kLingPF; ++s) {
            const int k = kb + 64 * s;
            if (k < K) {  // wave-uniform
                if constexpr (V != 0) {
                    a[s] = fold_apply<V, RSK>(q[s], V == 1 ? k + 4 * h : mc, L, fadd, rch);
                    if (aout) *(t4 *)(aout + am + k + 4 * h) = a[s];
                }
                if constexpr (ASK) {  // splitk_reduce_kernel's order: partials 0, 1, ..., then + 0
#pragma unroll
                    for (int z = 1; z < kSkMax; ++z)
                        if (z < ach) a[s] = a[s] + az[s][z - 1];
                    a[s] = a[s] + 0.f;
                    if (skout) *(t4 *)(skout + am + k + 4 * h) = a[s];
                }
#pragma unroll
                for (int j = 0; j < 4; ++j)
                    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a[s][j], b[s][j], acc, 0, 0, 0);
                if (rows) rs += ((a[s][0] + a[s][1]) + a[s][2]) + a[s][3];
                const int kn = k + 64 * kLingPF + 4 * h;
                if constexpr (V != 0) {
                    if (kn < K) q[s] = fold_raw<V, RSK>(Gr, Ur, Yr, Rr, fadd, am + kn * P.sak, P.sak, rch, rstr);
                } else {
                    a[s] = kn < K ? ling_ld<AK>(Ar, am + kn * P.sak, P.sak) : zero;
                    if constexpr (ASK) {
#pragma unroll
                        for (int z = 1; z < kSkMax; ++z)
                            az[s][z - 1] =
                                (kn < K && z < ach) ? ling_ld<AK>(Ar, am + kn * P.sak + z * P.astr, P.sak) : zero;
                    }
                }
                b[s] = kn < K ? ling_ld<BK>(Br, bn + kn * P.sbk, P.sbk) : zero;
            }
        }
    }
    if (w > 0) L.part[w - 1][lane] = acc;
    if (rows) L.rs_part[w][lane] = rs;
    __syncthreads();
    if (w > 0) return;
#pragma unroll 1
    for (int p = 0; p < 7; ++p) acc += L.part[p][lane];
    if (rows) {
#pragma unroll
        for (int p = 1; p < 8; ++p) rs += L.rs_part[p][lane];
        rs += __shfl_xor(rs, 32);
        if (h == 0 && m < M) P.rowsum[m] = rs;
    }
    const bool bok = col < N;
    const float bias = ep_bias;
    float sv = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int row = (int)bx * 32 + 8 * (i >> 2) + 4 * h + (i & 3);
        float v = acc[i] + bias;
        if (row < M && bok) {
            if (P.R) v = v + ep_r[i];
            P.C[row * P.ldc + col] = v;
        }
        acc[i] = v;
        if (row < M) sv += v;
    }
    if (P.stats) {
        const int nr = M - (int)bx * 32 < 32 ? M - (int)bx * 32 : 32;
        const float mean = (sv + __shfl_xor(sv, 32)) / (float)nr;
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int row = (int)bx * 32 + 8 * (i >> 2) + 4 * h + (i & 3);
            const float d = acc[i] - mean;
            if (row < M) q += d * d;
        }
        q += __shfl_xor(q, 32);
        if (h == 0 && bok) {
            P.stats[((int)bx * N + col) * 2] = mean;
            P.stats[((int)bx * N + col) * 2 + 1] = q;
        }
    }
    if (PS) {  // this tile's column sums of dz and dz xhat for the folded BatchNorm
        float pd = 0.f, pdx = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int row = (int)bx * 32 + 8 * (i >> 2) + 4 * h + (i & 3);
            const float dz = ps_u[i] > 0.f ? acc[i] : 0.f;
            const float xh = (ps_y[i] - ps_mu) * ps_is;
            if (row < M) {
                pd += dz;
                pdx += dz * xh;
            }
        }
        pd += __shfl_xor(pd, 32);
        pdx += __shfl_xor(pdx, 32);
        if (h == 0 && bok) {
            Fo.part[((int)bx * N + col) * 2] = pd;
            Fo.part[((int)bx * N + col) * 2 + 1] = pdx;
        }
    }
}

// Up to kLingMax products in one launch, each whole or split along K into S chunks (chunk z
// a partial tile by the same arithmetic over its k range, written to part + z M N and added
// in chunk order by splitk_reduce_kernel after the launch).  Workgroups [begin_i,
// begin_{i+1}) compute problem i; its layout (AK, BK) picks one of four tile bodies by a
// uniform branch.
constexpr int kLingMax = 4;
struct LinGProb {
    LinG g;
    float *part;
    int kchunk;
    unsigned S, mt, nt, begin;
    int ak, bk, vmode;  // vmode: (fs_linear_f32_pair_bn, consumer) 1 A = dy, 2 A = dy^T
};
struct LinGrp {
    LinGProb p[kLingMax];
    int n;
    BnFold fold, fold_out;  // (gemm_ling_fold_kernel) the BatchNorm dy is loaded from / tile sums go to
};

__global__ __launch_bounds__(512) void gemm_ling_kernel(LinGrp ga) {
    __shared__ LinGLds L;
    int i = 0;
#pragma unroll
    for (int t = 1; t < kLingMax; ++t)
        if (t < ga.n && blockIdx.x >= ga.p[t].begin) i = t;
    const LinGProb &Q = ga.p[i];
    unsigned b = blockIdx.x - Q.begin;
    const unsigned per = Q.mt * Q.nt, z = b / per;
    b -= z * per;
    const unsigned bx = b % Q.mt, by = b / Q.mt;
    LinG c = Q.g;
    if (Q.S > 1) {  // chunk z of the reduction: its own partial tile, nothing else
        c.pstats = 0;
        const int k0 = (int)z * Q.kchunk;
        c.A = Q.g.A + k0 * Q.g.sak;
        c.B = Q.g.B + k0 * Q.g.sbk;
        c.abytes = Q.g.abytes - k0 * Q.g.sak * 4;
        c.bbytes = Q.g.bbytes - k0 * Q.g.sbk * 4;
        c.K = Q.g.K - k0 < Q.kchunk ? Q.g.K - k0 : Q.kchunk;
        c.bias = nullptr;
        c.R = nullptr;
        c.rowsum = nullptr;
        c.stats = nullptr;
        c.C = Q.part + (int64_t)z * Q.g.M * Q.g.N;
        c.ldc = Q.g.N;
    }
    if (Q.ak) {
        if (Q.bk)
            ling_tile<true, true>(c, bx, by, L, ga.fold, ga.fold);
        else
            ling_tile<true, false>(c, bx, by, L, ga.fold, ga.fold);
    } else {
        if (Q.bk)
            ling_tile<false, true>(c, bx, by, L, ga.fold, ga.fold);
        else
            ling_tile<false, false>(c, bx, by, L, ga.fold, ga.fold);
    }
}

// nn.Linear's backward pair around a folded BatchNorm (fs_linear_f32_pair_bn): the producer's
// (vmode 0) input gradient with the tile sums in its epilogue (pstats) and its weight
// gradient, or the consumer's two products with dy loaded on the fly (vmode 1, 2)
__global__ __launch_bounds__(512) void gemm_ling_fold_kernel(LinGrp ga) {
    __shared__ LinGFLds L;
    const int i = (ga.n > 1 && blockIdx.x >= ga.p[1].begin) ? 1 : 0;
    const LinGProb &Q = ga.p[i];
    const unsigned b = blockIdx.x - Q.begin, bx = b % Q.mt, by = b / Q.mt;
    const BnFold &Fi = ga.fold, &Fo = ga.fold_out;
    if (Q.vmode == 1) {
        if (Q.g.pstats)
            ling_tile<true, false, 1, true, LinGFLds>(Q.g, bx, by, L, Fi, Fo);
        else
            ling_tile<true, false, 1, false, LinGFLds>(Q.g, bx, by, L, Fi, Fo);
    } else if (Q.vmode == 2) {
        ling_tile<false, false, 2, false, LinGFLds>(Q.g, bx, by, L, Fi, Fo);
    } else if (Q.g.pstats) {
        ling_tile<true, false, 0, true, LinGFLds>(Q.g, bx, by, L, Fi, Fo);
    } else {
        ling_tile<false, false, 0, false, LinGFLds>(Q.g, bx, by, L, Fi, Fo);
    }
}

// The same with split-K operands summed on load (fs_linear_f32_pair_bn_sk): the consumer's
// dx_add (fold.add_ch partials) or the producer's A (ach partials).  A kernel of its own, so
// that the extra partials' registers do not weigh on gemm_ling_fold_kernel.
__global__ __launch_bounds__(512) void gemm_ling_fold_sk_kernel(LinGrp ga) {
    __shared__ LinGFLds L;
    const int i = (ga.n > 1 && blockIdx.x >= ga.p[1].begin) ? 1 : 0;
    const LinGProb &Q = ga.p[i];
    const unsigned b = blockIdx.x - Q.begin, bx = b % Q.mt, by = b / Q.mt;
    const BnFold &Fi = ga.fold, &Fo = ga.fold_out;
    if (Q.vmode == 1) {
        if (Q.g.pstats)
            ling_tile<true, false, 1, true, LinGFLds, true>(Q.g, bx, by, L, Fi, Fo);
        else
            ling_tile<true, false, 1, false, LinGFLds, true>(Q.g, bx, by, L, Fi, Fo);
    } else if (Q.vmode == 2) {
        ling_tile<false, false, 2, false, LinGFLds, true>(Q.g, bx, by, L, Fi, Fo);
    } else if (Q.g.pstats) {
        ling_tile<true, false, 0, true, LinGFLds, true>(Q.g, bx, by, L, Fi, Fo);
    } else {
        ling_tile<false, false, 0, false, LinGFLds, true>(Q.g, bx, by, L, Fi, Fo);
    }
}

// Deferred BatchNorm running statistics: for each of nbn BatchNorms of width H (flat
// running buffers rm / rv [nbn][H], counters nbt [nbn]) the momentum updates of `passes`
// passes in pass order, from stats [passes][nbn][2][H] (batch mean, biased variance;
// rows of the pass), exactly as the in-launch update computes them; nbt += passes.
// Nothing is written when the skip word (nullable) is set.
__global__ void __launch_bounds__(256) bn_running_update_kernel(int nbn, int H, float *rm, float *rv, int64_t *nbt,
                                                                const float *stats, int passes, int64_t rows0,
                                                                int64_t rows1, float m, const int32_t *skip) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)nbn * H || (skip && *skip != 0)) return;
    const int64_t bnx = i / H, h = i - bnx * H;
    float a = rm[i], v = rv[i];
    for (int p = 0; p < passes; ++p) {
        const int64_t rows = p == 0 ? rows0 : rows1;
        const float *s = stats + (((int64_t)p * nbn + bnx) * 2) * H;
        a = running_update(a, s[h], m);
        v = running_update(v, unbiased(s[H + h], rows), m);
    }
    rm[i] = a;
    rv[i] = v;
    if (h == 0) nbt[bnx] += passes;
}

// Two independent products in one launch (nn.Linear's backward: input gradient and weight
// gradient): workgroups [0, t0) take the tiles of g0 (column-major over its mt0 row
// tiles), the rest those of g1.  Each tile is computed exactly as gemm_f32_kernel does.
template <int SPLIT, bool A0K, bool B0K, bool A1K, bool B1K>
__global__ __launch_bounds__(64 * SPLIT) void gemm2_f32_kernel(GemmArgs g0, GemmArgs g1, unsigned t0, unsigned mt0,
                                                              unsigned mt1) {
    __shared__ GemmLds<SPLIT> L;
    const unsigned b = blockIdx.x;
    if (b < t0)
        gemm_tile<SPLIT, A0K, B0K>(g0, b % mt0, b / mt0, L);
    else
        gemm_tile<SPLIT, A1K, B1K>(g1, (b - t0) % mt1, (b - t0) / mt1, L);
}

// ---------------------------------------------------------------------------
// BatchNorm1d (train) + ReLU.  Workgroup = kBnCols columns x kBnRg row groups.
// 4 columns x 64 row groups (32 workgroups at H = 128, 4 register-cached rows per thread):
// A/B builds of the A2 step (profiles/r02/train/bn_tiling_ab.log) gave 122-124 steps/s
// against 113 for 16 x 16 (8 workgroups, 16 rows per thread) at batch 256
#ifndef FS_BN_COLS
#define FS_BN_COLS 4
#endif
#ifndef FS_BN_RG
#define FS_BN_RG 64
#endif
constexpr int kBnCols = FS_BN_COLS, kBnRg = FS_BN_RG;
constexpr int kBnR = (256 + kBnRg - 1) / kBnRg;  // register-cached rows per thread (batch <= 256)

__device__ __forceinline__ float wg_colsum(float v, float (*red)[kBnCols], int c, int rg) {
    red[rg][c] = v;
    __syncthreads();
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < kBnRg; ++q) s += red[q][c];
    __syncthreads();
    return s;
}

// R > 0: every thread holds its R rows (rows rg + q kBnRg) in registers, so each column is
// read once and all of a thread's loads are in flight together; R = 0: any batch, re-read
template <int R>
__global__ __launch_bounds__(kBnCols *kBnRg) void bn_relu_train_fwd_kernel(
    int64_t B, int H, const float *__restrict__ x, const float *__restrict__ gamma, const float *__restrict__ beta,
    float *running_mean, float *running_var, int64_t *num_batches, float momentum, float eps, float *__restrict__ y,
    float *__restrict__ mean_out, float *__restrict__ invstd_out) {
    __shared__ float red[kBnRg][kBnCols];
    const int c = threadIdx.x % kBnCols, rg = threadIdx.x / kBnCols;
    const int col = blockIdx.x * kBnCols + c;
    const bool ok = col < H;
    const float *xc = x + (ok ? col : 0);
    float v[R > 0 ? R : 1];
    float s = 0.f;
    if (R > 0) {
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const int64_t i = rg + (int64_t)q * kBnRg;
            v[q] = (ok && i < B) ? xc[i * H] : 0.f;
        }
#pragma unroll
        for (int q = 0; q < R; ++q) s += v[q];
    } else if (ok) {
        for (int64_t i = rg; i < B; i += kBnRg) s += xc[i * H];
    }
    const float mean = wg_colsum(s, red, c, rg) / (float)B;
    float sq = 0.f;
    if (R > 0) {
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const float d = v[q] - mean;
            if (rg + (int64_t)q * kBnRg < B) sq += d * d;
        }
    } else if (ok) {
        for (int64_t i = rg; i < B; i += kBnRg) {
            const float d = xc[i * H] - mean;
            sq += d * d;
        }
    }
    const float var = wg_colsum(sq, red, c, rg) / (float)B;
    const float invstd = 1.f / sqrtf(var + eps);
    if (!ok) return;
    const float gm = gamma[col], bt = beta[col];
    if (R > 0) {
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const int64_t i = rg + (int64_t)q * kBnRg;
            if (i < B) {
                const float o = gm * ((v[q] - mean) * invstd) + bt;
                y[i * H + col] = o > 0.f ? o : 0.f;
            }
        }
    } else {
        for (int64_t i = rg; i < B; i += kBnRg) {
            const float o = gm * ((xc[i * H] - mean) * invstd) + bt;
            y[i * H + col] = o > 0.f ? o : 0.f;
        }
    }
    if (rg == 0) {
        mean_out[col] = mean;
        invstd_out[col] = invstd;
        if (running_mean) {
            running_mean[col] = running_update(running_mean[col], mean, momentum);
            running_var[col] = running_update(running_var[col], unbiased(var, B), momentum);
        }
        if (num_batches && col == 0) *num_batches += 1;
    }
}

// dz = dy * (y > 0); dbeta = sum dz; dgamma = sum dz xhat;
// dx = gamma invstd (dz - dbeta / B - xhat dgamma / B)   (torch's batch_norm_backward_elemt)
template <int R>
__global__ __launch_bounds__(kBnCols *kBnRg) void bn_relu_train_bwd_kernel(
    int64_t B, int H, const float *__restrict__ x, const float *__restrict__ y, const float *__restrict__ dy,
    const float *__restrict__ gamma, const float *__restrict__ mean, const float *__restrict__ invstd,
    float *__restrict__ dx, const float *__restrict__ dx_add, float *__restrict__ dgamma, float *__restrict__ dbeta) {
    __shared__ float red[kBnRg][kBnCols];
    const int c = threadIdx.x % kBnCols, rg = threadIdx.x / kBnCols;
    const int col = blockIdx.x * kBnCols + c;
    const bool ok = col < H;
    const int64_t o = ok ? col : 0;
    const float mu = mean[o], is = invstd[o];
    float dzv[R > 0 ? R : 1], xhv[R > 0 ? R : 1];
    float sd = 0.f, sdx = 0.f;
    if (R > 0) {
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const int64_t i = rg + (int64_t)q * kBnRg;
            const bool in = ok && i < B;
            const float yv = in ? y[i * H + o] : 0.f, g = in ? dy[i * H + o] : 0.f, xv = in ? x[i * H + o] : mu;
            dzv[q] = yv > 0.f ? g : 0.f;
            xhv[q] = (xv - mu) * is;
        }
#pragma unroll
        for (int q = 0; q < R; ++q) {
            sd += dzv[q];
            sdx += dzv[q] * xhv[q];
        }
    } else if (ok) {
        for (int64_t i = rg; i < B; i += kBnRg) {
            const float dz = y[i * H + o] > 0.f ? dy[i * H + o] : 0.f;
            sd += dz;
            sdx += dz * ((x[i * H + o] - mu) * is);
        }
    }
    const float db = wg_colsum(sd, red, c, rg);
    const float dg = wg_colsum(sdx, red, c, rg);
    if (!ok) return;
    const float gm = gamma[col];
    const float mdb = db / (float)B, mdg = dg / (float)B;
    if (R > 0) {
#pragma unroll
        for (int q = 0; q < R; ++q) {
            const int64_t i = rg + (int64_t)q * kBnRg;
            if (i < B) dx[i * H + col] = (dzv[q] - mdb - xhv[q] * mdg) * (is * gm) + (dx_add ? dx_add[i * H + col] : 0.f);
        }
    } else {
        for (int64_t i = rg; i < B; i += kBnRg) {
            const float dz = y[i * H + col] > 0.f ? dy[i * H + col] : 0.f;
            const float xh = (x[i * H + col] - mu) * is;
            dx[i * H + col] = (dz - mdb - xh * mdg) * (is * gm) + (dx_add ? dx_add[i * H + col] : 0.f);
        }
    }
    if (rg == 0) {
        if (dgamma) dgamma[col] = dg;
        if (dbeta) dbeta[col] = db;
    }
}


// Long-reduction products with few output tiles (the input gradient of the 2944-wide final
// layer: 256 x 128 over K = 2944, 32 tiles): the reduction is cut into S chunks, each a
// grid slice computing its partial tile exactly as gemm_f32_kernel does over its k range,
// then one launch adds the S partials in chunk order (+ bias, + R).  Deterministic.
template <int SPLIT, bool AK, bool BK>
__global__ __launch_bounds__(64 * SPLIT) void gemm_splitk_kernel(GemmArgs g, float *part, int64_t kchunk) {
    __shared__ GemmLds<SPLIT> L;
    const int64_t z = blockIdx.z, k0 = z * kchunk;
    GemmArgs c = g;
    c.A = g.A + k0 * g.sak;
    c.B = g.B + k0 * g.sbk;
    c.K = (g.K - k0 < kchunk ? g.K - k0 : kchunk);
    c.bias = nullptr;
    c.R = nullptr;
    c.rowsum_a = nullptr;
    c.stats = nullptr;
    c.C = part + z * g.M * g.N;
    c.ldc = g.N;
    gemm_tile<SPLIT, AK, BK>(c, blockIdx.x, blockIdx.y, L);
}

__global__ void __launch_bounds__(256) splitk_reduce_kernel(GemmArgs g, const float *part, int S) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= g.M * g.N) return;
    const int64_t m = i / g.N, n = i - m * g.N;
    float v = part[i];
    for (int z = 1; z < S; ++z) v += part[z * g.M * g.N + i];
    v = v + (g.bias ? g.bias[n] : 0.f);
    if (g.R) v = v + g.R[m * g.ldr + n];
    g.C[m * g.ldc + n] = v;
}

// Up to kGroupMax independent products in one launch, each plain or split-K (partial tiles
// into its workspace slice, added by splitk_reduce_kernel after the launch): the backward
// of a coupling layer's final Linear (input gradient over K = n (3K+1), weight + bias
// gradient) together with the unconditional spline parameters' row sum.  Each tile is
// computed exactly as gemm_f32_kernel / gemm_splitk_kernel compute it alone.
constexpr int kGroupMax = 4;
struct GroupProblem {
    GemmArgs g;
    float *part;  // split-K partial tiles (S > 1)
    int64_t kchunk;
    unsigned S, mt, nt, begin;
    int ak, bk;
};
struct GroupArgs {
    GroupProblem p[kGroupMax];
    int n;
};

template <int SPLIT>
__global__ __launch_bounds__(64 * SPLIT) void gemm_group_kernel(GroupArgs ga) {
    __shared__ GemmLds<SPLIT> L;
    int i = 0;
    while (i + 1 < ga.n && blockIdx.x >= ga.p[i + 1].begin) ++i;
    const GroupProblem &P = ga.p[i];
    unsigned b = blockIdx.x - P.begin;
    const unsigned per = P.mt * P.nt, z = b / per;
    b -= z * per;
    const unsigned bx = b % P.mt, by = b / P.mt;
    GemmArgs c = P.g;
    if (P.S > 1) {
        const int64_t k0 = (int64_t)z * P.kchunk;
        c.A = P.g.A + k0 * P.g.sak;
        c.B = P.g.B + k0 * P.g.sbk;
        c.K = (P.g.K - k0 < P.kchunk ? P.g.K - k0 : P.kchunk);
        c.bias = nullptr;
        c.R = nullptr;
        c.rowsum_a = nullptr;
        c.stats = nullptr;
        c.C = P.part + (int64_t)z * P.g.M * P.g.N;
        c.ldc = P.g.N;
    }
    if (P.ak) {
        if (P.bk)
            gemm_tile<SPLIT, true, true>(c, bx, by, L);
        else
            gemm_tile<SPLIT, true, false>(c, bx, by, L);
    } else {
        if (P.bk)
            gemm_tile<SPLIT, false, true>(c, bx, by, L);
        else
            gemm_tile<SPLIT, false, false>(c, bx, by, L);
    }
}

}  // namespace fs

using namespace fs;

static bool lean_gemm();
static bool ling_ok(const GemmArgs &g);
static hipError_t ling_group(const GemmArgs *gs, int n, float *const *part, const int *S, const int64_t *kchunk,
                             hipStream_t st, bool keep0 = false);

static int gemm_split(const GemmArgs &g) {
    return g.K > 8 * 4 * 16 ? FS_GEMM_SPLIT_LONG : g.K >= 256 ? FS_GEMM_SPLIT_MID : FS_GEMM_SPLIT;
}

hipError_t fs_linear_f32_impl(const fs::GemmArgs &g, hipStream_t st);

// Split-K plan of a product: chunks S and the partial-tile floats it needs (0 = not used):
// long reductions (K >= 2048) over at most 128 output tiles, no row sum / statistics.
static int64_t splitk_plan(const GemmArgs &g, int &S, int64_t &kchunk) {
    const int64_t tiles = ((g.M + 31) / 32) * ((g.N + 31) / 32);
    if (!(g.K >= 2048 && g.M > 0 && g.N > 0 && tiles <= 128 && !g.rowsum_a && !g.stats)) return 0;
    S = (int)(g.K / 256);
    if (S > 16) S = 16;
    kchunk = ((g.K + S - 1) / S + 7) / 8 * 8;
    S = (int)((g.K + kchunk - 1) / kchunk);
    return (int64_t)S * g.M * g.N;
}

int64_t fs_linear_f32_splitk_floats_impl(const GemmArgs &g) {
    int S = 0;
    int64_t kc = 0;
    return splitk_plan(g, S, kc);
}

hipError_t fs_linear_f32_splitk_impl(const GemmArgs &g, float *part, int64_t part_floats, hipStream_t st) {
    int S = 0;
    int64_t kchunk = 0;
    const int64_t need = splitk_plan(g, S, kchunk);
    if (need == 0 || !part || part_floats < need) return fs_linear_f32_impl(g, st);
    if (lean_gemm() && ling_ok(g)) return ling_group(&g, 1, &part, &S, &kchunk, st);
    const bool ak = g.sak == 1 && ((uintptr_t)g.A & 15) == 0 && g.sam % 4 == 0 && kchunk % 4 == 0;
    const bool bk = g.sbk == 1 && ((uintptr_t)g.B & 15) == 0 && g.sbn % 4 == 0 && kchunk % 4 == 0;
    const dim3 grid((unsigned)((g.M + 31) / 32), (unsigned)((g.N + 31) / 32), (unsigned)S);
#define FS_SK(A, B)                                                                                                  \
    if (ak == A && bk == B)                                                                                          \
        hipLaunchKernelGGL((gemm_splitk_kernel<FS_GEMM_SPLIT, A, B>), grid, dim3(64 * FS_GEMM_SPLIT), 0, st, g, part, \
                           kchunk);
    FS_SK(true, true) FS_SK(true, false) FS_SK(false, true) FS_SK(false, false)
#undef FS_SK
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    const int64_t n = g.M * g.N;
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, g,
                       (const float *)part, S);
    return hipGetLastError();
}

// A group launch (gemm_group_kernel) of n <= kGroupMax products: those with a split-K plan
// whose partials fit the workspace take it, the others run whole; every product must take
// FS_GEMM_SPLIT waves per tile (K <= 512 or split).  hipErrorNotSupported: run them one
// by one (the caller's fallback).
hipError_t fs_linear_f32_group_impl(const GemmArgs *gs, int n, float *ws, int64_t ws_floats, hipStream_t st) {
    if (n < 0 || n > kGroupMax) return hipErrorInvalidValue;
    if (lean_gemm()) {  // the same split-K plans on the lean kernel
        GemmArgs lg[kGroupMax];
        float *part[kGroupMax];
        int S[kGroupMax];
        int64_t kc[kGroupMax];
        int m = 0;
        int64_t used = 0;
        bool ok = true;
        for (int i = 0; i < n && ok; ++i) {
            const GemmArgs &g = gs[i];
            if (g.M <= 0 || (g.N <= 0 && !g.rowsum_a)) continue;
            ok = ling_ok(g);
            int s = 0;
            int64_t kchunk = 0;
            const int64_t need = splitk_plan(g, s, kchunk);
            lg[m] = g;
            if (need > 0 && ws && ws_floats - used >= need) {
                part[m] = ws + used;
                used += need;
                S[m] = s;
                kc[m] = kchunk;
            } else {
                part[m] = nullptr;
                S[m] = 1;
                kc[m] = g.K;
            }
            ++m;
        }
        if (ok) return m ? ling_group(lg, m, part, S, kc, st) : hipSuccess;
    }
    GroupArgs ga{};
    unsigned wg = 0;
    int64_t used = 0;
    for (int i = 0; i < n; ++i) {
        const GemmArgs &g = gs[i];
        if (g.M <= 0 || (g.N <= 0 && !g.rowsum_a)) continue;  // nothing to compute
        GroupProblem &P = ga.p[ga.n];
        P.g = g;
        P.part = nullptr;
        P.S = 1;
        P.kchunk = g.K;
        int S = 0;
        int64_t kchunk = 0;
        const int64_t need = splitk_plan(g, S, kchunk);
        if (need > 0 && ws && ws_floats - used >= need) {
            P.part = ws + used;
            used += need;
            P.S = (unsigned)S;
            P.kchunk = kchunk;
        } else if (gemm_split(g) != FS_GEMM_SPLIT) {
            return hipErrorNotSupported;
        }
        P.ak = g.sak == 1 && ((uintptr_t)g.A & 15) == 0 && g.sam % 4 == 0 && (P.S == 1 || P.kchunk % 4 == 0);
        P.bk = g.sbk == 1 && ((uintptr_t)g.B & 15) == 0 && g.sbn % 4 == 0 && (P.S == 1 || P.kchunk % 4 == 0);
        P.mt = (unsigned)((g.M + 31) / 32);
        P.nt = (unsigned)(g.N > 0 ? (g.N + 31) / 32 : 1);
        P.begin = wg;
        wg += P.mt * P.nt * P.S;
        ++ga.n;
    }
    if (ga.n == 0) return hipSuccess;
    hipLaunchKernelGGL(gemm_group_kernel<FS_GEMM_SPLIT>, dim3(wg), dim3(64 * FS_GEMM_SPLIT), 0, st, ga);
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    for (int i = 0; i < ga.n; ++i) {
        const GroupProblem &P = ga.p[i];
        if (P.S <= 1) continue;
        const int64_t m = P.g.M * P.g.N;
        hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, P.g,
                           (const float *)P.part, (int)P.S);
        if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    }
    return hipSuccess;
}

// gemm_lin_kernel takes a product: nn.Linear's forward layout, K = 64, 128, 192 or 256, N a
// multiple of 32, 16-byte aligned operands, no row sum, 32-bit offsets
static bool lin_ok(const GemmArgs &g, const BnIn *bn) {
    // element counts whose byte offsets (x 4, computed in 32-bit int) stay below 2^31
    const int64_t lim = (int64_t)1 << 29;
    return g.M > 0 && g.N > 0 && g.K > 0 && g.K % 64 == 0 && g.K <= 256 && g.N % 32 == 0 && g.sak == 1 &&
           g.sam == g.K && g.sbk == 1 && g.sbn == g.K && ((uintptr_t)g.A & 15) == 0 && ((uintptr_t)g.B & 15) == 0 &&
           !g.rowsum_a && g.M * g.K < lim && g.N * g.K < lim && g.M * g.ldc < lim && (!g.R || g.M * g.ldr < lim / 2) &&
           g.M <= 32LL * 65535 && (!bn || (bn->rows == g.M && (!bn->a_out || ((uintptr_t)bn->a_out & 15) == 0)));
}

static void lin_fill(LinP &p, LinBn &b, const GemmArgs &g, const BnIn *bn) {
    p = LinP{g.A, g.B, g.bias, g.R, g.C, g.stats, (int)g.M, (int)g.N, (int)g.ldr, (int)g.ldc};
    b = LinBn{};
    if (bn)
        b = LinBn{bn->stats, bn->gamma, bn->beta, bn->mean_out, bn->invstd_out, bn->var_out, bn->a_out,
                  bn->running_mean, bn->running_var, bn->num_batches, bn->eps, bn->momentum, (int)bn->tiles, 1};
}

// the lean kernels (default) or the generic ones (FS_LEAN_GEMM=0, fs_set_lean_gemm)
static std::atomic<int> g_lean{-1};
static bool lean_gemm() {
    int v = g_lean.load(std::memory_order_relaxed);
    if (v < 0) {
        const char *e = getenv("FS_LEAN_GEMM");
        int expect = -1;
        g_lean.compare_exchange_strong(expect, (e && e[0] == '0') ? 0 : 1);
        v = g_lean.load(std::memory_order_relaxed);
    }
    return v != 0;
}

int32_t fs_set_lean_gemm_impl(int32_t on) {
    const int32_t prev = lean_gemm() ? 1 : 0;
    if (on >= 0) g_lean.store(on ? 1 : 0, std::memory_order_relaxed);
    return prev;
}

static bool ak_of(const GemmArgs &g) { return g.sak == 1 && ((uintptr_t)g.A & 15) == 0 && g.sam % 4 == 0; }
static bool bk_of(const GemmArgs &g) { return g.sbk == 1 && ((uintptr_t)g.B & 15) == 0 && g.sbn % 4 == 0; }

// byte extent of a strided operand: the element past the last one addressed, (rows - 1)
// strides along one dimension plus (depth - 1) along the other
static int64_t extent_bytes(int64_t n0, int64_t s0, int64_t n1, int64_t s1) {
    if (n0 <= 0 || n1 <= 0) return 0;
    return ((n0 - 1) * s0 + (n1 - 1) * s1 + 1) * 4;
}

// gemm_ling_kernel takes a product: K a multiple of 4 (a lane's quad of k is wholly inside
// or wholly past the reduction), non-negative strides, 32-bit offsets
static bool ling_ok(const GemmArgs &g) {
    const int64_t lim = (int64_t)1 << 30;
    if (g.M <= 0 || g.K <= 0 || g.K % 4 != 0 || (g.N <= 0 && !g.rowsum_a) || g.N < 0) return false;
    if (g.sam < 0 || g.sak < 0 || g.sbk < 0 || g.sbn < 0 || g.M > 32LL * 65535 || g.N > 32LL * 65535) return false;
    const int64_t ab = extent_bytes(g.M, g.sam, g.K, g.sak), bb = extent_bytes(g.K, g.sbk, g.N, g.sbn);
    const int64_t el = lim / 2;  // element counts: byte offsets (x 4, 32-bit int) below 2^31
    return ab < lim && bb < lim && g.M * g.ldc < el && (!g.R || g.M * g.ldr < el) && g.K < lim / 4 &&
           g.M * g.sam < el && g.K * g.sak < el && g.K * g.sbk < el && g.N * g.sbn < el && g.M * g.N < el;
}

static LinG ling_fill(const GemmArgs &g) {
    return LinG{g.A, g.B, g.bias, g.R, g.C, g.stats, g.rowsum_a, (int)g.M, (int)g.N, (int)g.K, (int)g.sam, (int)g.sak,
                (int)g.sbk, (int)g.sbn, (int)g.ldr, (int)g.ldc, (int)extent_bytes(g.M, g.sam, g.K, g.sak),
                (int)extent_bytes(g.K, g.sbk, g.N, g.sbn), 0, 1, 0, nullptr};
}

// n products (all ling_ok) in one gemm_ling_kernel launch; part[i] / S[i] / kchunk[i]: the
// split-K plan of product i (S = 1: whole), then one splitk_reduce_kernel per split product
static hipError_t ling_group(const GemmArgs *gs, int n, float *const *part, const int *S, const int64_t *kchunk,
                             hipStream_t st, bool keep0) {
    if (n <= 0 || n > kLingMax) return hipErrorInvalidValue;
    LinGrp ga{};
    unsigned wg = 0;
    for (int i = 0; i < n; ++i) {
        const GemmArgs &g = gs[i];
        LinGProb &Q = ga.p[ga.n++];
        Q.g = ling_fill(g);
        Q.S = (unsigned)S[i];
        Q.part = part[i];
        Q.kchunk = (int)kchunk[i];
        // split chunks: contiguous loads need chunk starts on 16-byte boundaries
        Q.ak = ak_of(g) && (Q.S == 1 || Q.kchunk % 4 == 0);
        Q.bk = bk_of(g) && (Q.S == 1 || Q.kchunk % 4 == 0);
        Q.mt = (unsigned)((g.M + 31) / 32);
        Q.nt = (unsigned)(g.N > 0 ? (g.N + 31) / 32 : 1);
        Q.begin = wg;
        wg += Q.mt * Q.nt * Q.S;
    }
    hipLaunchKernelGGL(gemm_ling_kernel, dim3(wg), dim3(512), 0, st, ga);
    if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    for (int i = 0; i < n; ++i) {
        if (S[i] <= 1 || (i == 0 && keep0)) continue;  // keep0: product 0's partials left for its consumers
        const GemmArgs &g = gs[i];
        const int64_t m = g.M * g.N;
        hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, st, g,
                           (const float *)part[i], S[i]);
        if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    }
    return hipSuccess;
}

// fs_linear_f32_group with product 0's split-K partials left unreduced: at most max_ch chunks
// (whole multiples of 8 along K) at ws + z M N, summed on load by their consumers (the
// backward pairs' ach / add_ch, or fs_splitk_sum); ch_out = the chunk count.
// hipErrorNotSupported: product 0 has no split-K plan (or a bias / residual / padded C), or
// some product does not take the lean kernel.
hipError_t fs_linear_f32_group_partial_impl(const GemmArgs *gs, int n, float *ws, int64_t ws_floats, int max_ch,
                                            int *ch_out, hipStream_t st) {
    *ch_out = 1;
    if (n < 1 || n > kLingMax || max_ch < 2 || max_ch > kSkMax || !lean_gemm()) return hipErrorNotSupported;
    const GemmArgs &g0 = gs[0];
    int s0 = 0;
    int64_t kc0 = 0;
    if (splitk_plan(g0, s0, kc0) == 0 || g0.bias || g0.R || g0.ldc != g0.N) return hipErrorNotSupported;
    GemmArgs lg[kLingMax];
    float *part[kLingMax];
    int S[kLingMax];
    int64_t kc[kLingMax];
    int64_t used = 0;
    for (int i = 0; i < n; ++i) {
        const GemmArgs &g = gs[i];
        if (!ling_ok(g) || g.M <= 0 || (g.N <= 0 && !g.rowsum_a)) return hipErrorNotSupported;
        int s = 0;
        int64_t kchunk = 0;
        int64_t need = splitk_plan(g, s, kchunk);
        if (i == 0) {
            kchunk = ((g.K + max_ch - 1) / max_ch + 7) / 8 * 8;
            s = (int)((g.K + kchunk - 1) / kchunk);
            need = (int64_t)s * g.M * g.N;
        }
        lg[i] = g;
        if (need > 0 && ws && ws_floats - used >= need) {
            part[i] = ws + used;
            used += need;
            S[i] = s;
            kc[i] = kchunk;
        } else if (i == 0) {
            return hipErrorNotSupported;
        } else {
            part[i] = nullptr;
            S[i] = 1;
            kc[i] = g.K;
        }
    }
    const hipError_t e = ling_group(lg, n, part, S, kc, st, true);
    if (e == hipSuccess) *ch_out = S[0];
    return e;
}

// out [n] = the ordered sum of ch partials stride floats apart (splitk_reduce_kernel's)
hipError_t fs_splitk_sum_impl(const float *part, int ch, int64_t stride, int64_t n, float *out, hipStream_t st) {
    if (n <= 0) return hipSuccess;
    if (ch < 1 || stride != n) return hipErrorInvalidValue;
    const GemmArgs g{1, n, 0, nullptr, 0, 0, nullptr, 0, 0, nullptr, nullptr, 0, out, n, nullptr};
    hipLaunchKernelGGL(splitk_reduce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, g, part, ch);
    return hipGetLastError();
}

// nn.Linear's backward pair around folded BatchNorms + ReLU (struct BnFold): fout, the
// BatchNorm this Linear applies to its input, whose output gradient gu is g0's output (its
// epilogue writes the tile sums); fin, the BatchNorm that consumes this Linear's output, whose
// input gradient dy is both products' A, loaded on the fly (A = fin->gu as the layout: g0
// row-major, g1 its transpose; + fin->dx_add; fin->a_out gets dy from g0's first column
// tile), workgroup 0 writing that BatchNorm's dgamma / dbeta
hipError_t fs_linear_f32_pair_bn_impl(const GemmArgs &g0, const GemmArgs &g1, const BnFold *fin, const BnFold *fout,
                                      hipStream_t st, int a_ch, int64_t a_str) {
    auto fold_ok = [](const BnFold &f) {
        return f.H > 0 && f.H <= kFoldMaxH && f.B > 0 && f.tiles == (f.B + 31) / 32 && f.gu && f.u && f.y && f.mean &&
               f.invstd && f.part && f.add_ch >= 1 && f.add_ch <= kSkMax &&
               (f.add_ch == 1 || (f.dx_add && f.add_str >= (int64_t)f.B * f.H &&
                                  (int64_t)f.B * f.H * 4 + (int64_t)(f.add_ch - 1) * f.add_str * 4 < INT32_MAX));
    };
    if (a_ch < 1 || a_ch > kSkMax || (a_ch > 1 && (fin || !fout || a_str < g0.M * g0.K ||
                                                   g0.M * g0.K * 4 + (a_ch - 1) * a_str * 4 >= INT32_MAX)))
        return hipErrorInvalidValue;
    if (!lean_gemm() || !ling_ok(g0) || !ling_ok(g1) || (!fin && !fout) || (fin && !fold_ok(*fin)) ||
        (fout && !fold_ok(*fout)))
        return hipErrorInvalidValue;
    LinGrp ga{};
    if (fin) ga.fold = *fin;
    if (fout) ga.fold_out = *fout;
    unsigned wg = 0;
    const GemmArgs *gs[2] = {&g0, &g1};
    for (int i = 0; i < 2; ++i) {
        const GemmArgs &g = *gs[i];
        LinGProb &Q = ga.p[ga.n++];
        Q.g = ling_fill(g);
        Q.S = 1;
        Q.part = nullptr;
        Q.kchunk = (int)g.K;
        Q.ak = ak_of(g);
        Q.bk = bk_of(g);
        Q.mt = (unsigned)((g.M + 31) / 32);
        Q.nt = (unsigned)(g.N > 0 ? (g.N + 31) / 32 : 1);
        Q.begin = wg;
        wg += Q.mt * Q.nt;
    }
    if (ga.p[0].bk || ga.p[1].bk || ga.p[1].ak) return hipErrorInvalidValue;
    if (a_ch > 1) {  // (producer) A of both products = the ordered sum of a_ch split-K partials
        if (g0.A != g1.A) return hipErrorInvalidValue;
        for (int i = 0; i < 2; ++i) {
            ga.p[i].g.ach = a_ch;
            ga.p[i].g.astr = (int)a_str;
            ga.p[i].g.abytes += (a_ch - 1) * (int)a_str * 4;  // the descriptor spans every partial
        }
        ga.p[0].g.aout = fout->a_out;  // nullable: the reduced A for its other readers
    }
    if (fout) {  // g0's output is the BatchNorm output's gradient gu [B][H]
        const BnFold &f = *fout;
        if (g0.M != f.B || g0.N != f.H || g0.ldc != f.H || g0.C != f.gu || !ga.p[0].ak) return hipErrorInvalidValue;
        ga.p[0].g.pstats = 1;
    }
    if (fin) {  // A of both products is dy (g0 row-major, g1 transposed), f.gu its layout
        const BnFold &f = *fin;
        if (!f.gamma || g0.A != f.gu || g1.A != f.gu || g0.M != f.B || g0.K != f.H || g0.sam != f.H || g0.sak != 1 ||
            !ga.p[0].ak || g1.M != f.H || g1.K != f.B || g1.sam != 1 || g1.sak != f.H)
            return hipErrorInvalidValue;
        ga.p[0].vmode = 1;
        ga.p[1].vmode = 2;
    }
    if (a_ch > 1 || (fin && fin->add_ch > 1))
        hipLaunchKernelGGL(gemm_ling_fold_sk_kernel, dim3(wg), dim3(512), 0, st, ga);
    else
        hipLaunchKernelGGL(gemm_ling_fold_kernel, dim3(wg), dim3(512), 0, st, ga);
    return hipGetLastError();
}

// one or two whole products (g1 nullable; both ling_ok) in one launch
static hipError_t ling_launch(const GemmArgs &g0, const GemmArgs *g1, hipStream_t st) {
    GemmArgs gs[2] = {g0, g1 ? *g1 : g0};
    float *part[2] = {nullptr, nullptr};
    const int S[2] = {1, 1};
    const int64_t kc[2] = {g0.K, g1 ? g1->K : g0.K};
    return ling_group(gs, g1 ? 2 : 1, part, S, kc, st);
}

// one or two products (g1 nullable) in one gemm_lin_kernel launch; both lin_ok, one K
static hipError_t lin_launch(const GemmArgs &g0, const BnIn *b0, const GemmArgs *g1, const BnIn *b1, hipStream_t st) {
    Lin2 a{};
    lin_fill(a.p[0], a.b[0], g0, b0);
    a.mt0 = (unsigned)((g0.M + 31) / 32);
    a.t0 = a.mt0 * (unsigned)(g0.N / 32);
    unsigned t1 = 0;
    if (g1) {
        lin_fill(a.p[1], a.b[1], *g1, b1);
        a.mt1 = (unsigned)((g1->M + 31) / 32);
        t1 = a.mt1 * (unsigned)(g1->N / 32);
    } else {
        a.mt1 = 1;
    }
    const dim3 grid(a.t0 + t1), block(512);
    // the full-batch kernel when some problem has a BatchNorm-in-load and every one that has
    // is a full training batch
    const bool any_bn = a.b[0].on || (g1 && a.b[1].on);
    const bool full = any_bn && (!a.b[0].on || lin_full(a.p[0], a.b[0])) && (!g1 || !a.b[1].on || lin_full(a.p[1], a.b[1]));
#define FS_LIN_K(KB)                                                                               \
    if (full)                                                                                      \
        hipLaunchKernelGGL((gemm_lin_kernel<KB, true>), grid, block, 0, st, a);                    \
    else                                                                                           \
        hipLaunchKernelGGL((gemm_lin_kernel<KB, false>), grid, block, 0, st, a);
    switch (g0.K) {
        case 64: FS_LIN_K(1) break;
        case 128: FS_LIN_K(2) break;
        case 192: FS_LIN_K(3) break;
        case 256: FS_LIN_K(4) break;
        default: return hipErrorInvalidValue;
    }
#undef FS_LIN_K
    return hipGetLastError();
}

hipError_t fs_linear_f32_impl(const fs::GemmArgs &g, hipStream_t st) {
    if (g.M <= 0 || (g.N <= 0 && !g.rowsum_a)) return hipSuccess;
    if (lean_gemm()) {
        if (lin_ok(g, nullptr)) return lin_launch(g, nullptr, nullptr, nullptr, st);
        if (ling_ok(g)) return ling_launch(g, nullptr, st);
    }
    // one column tile even when N = 0, so that rowsum_a is still written
    const dim3 grid((unsigned)((g.M + 31) / 32), (unsigned)(g.N > 0 ? (g.N + 31) / 32 : 1));
    const bool ak = g.sak == 1 && ((uintptr_t)g.A & 15) == 0 && g.sam % 4 == 0;
    const bool bk = g.sbk == 1 && ((uintptr_t)g.B & 15) == 0 && g.sbn % 4 == 0;
    // enough waves per tile that each walks at most ~16 k-blocks
    const int split = gemm_split(g);
#define FS_G(S, A, B)                                                                           \
    if (split == S && ak == A && bk == B) {                                                     \
        hipLaunchKernelGGL((gemm_f32_kernel<S, A, B>), grid, dim3(64 * S), 0, st, g);           \
        return hipGetLastError();                                                               \
    }
    FS_G(FS_GEMM_SPLIT, true, true) FS_G(FS_GEMM_SPLIT, true, false) FS_G(FS_GEMM_SPLIT, false, true)
    FS_G(FS_GEMM_SPLIT, false, false)
    FS_G(FS_GEMM_SPLIT_MID, true, true) FS_G(FS_GEMM_SPLIT_MID, true, false) FS_G(FS_GEMM_SPLIT_MID, false, true)
    FS_G(FS_GEMM_SPLIT_MID, false, false)
    FS_G(FS_GEMM_SPLIT_LONG, true, true) FS_G(FS_GEMM_SPLIT_LONG, true, false) FS_G(FS_GEMM_SPLIT_LONG, false, true)
    FS_G(FS_GEMM_SPLIT_LONG, false, false)
#undef FS_G
    return hipErrorInvalidValue;
}

hipError_t fs_linear_f32_pair_impl(const fs::GemmArgs &g0, const fs::GemmArgs &g1, hipStream_t st) {
    const bool a0 = g0.sak == 1 && ((uintptr_t)g0.A & 15) == 0 && g0.sam % 4 == 0;
    const bool b0 = g0.sbk == 1 && ((uintptr_t)g0.B & 15) == 0 && g0.sbn % 4 == 0;
    const bool a1 = g1.sak == 1 && ((uintptr_t)g1.A & 15) == 0 && g1.sam % 4 == 0;
    const bool b1 = g1.sbk == 1 && ((uintptr_t)g1.B & 15) == 0 && g1.sbn % 4 == 0;
    const bool live0 = g0.M > 0 && g0.N > 0, live1 = g1.M > 0 && g1.N > 0;
    if (lean_gemm() && live0 && live1 && ling_ok(g0) && ling_ok(g1) && a0 && !b0 && !a1 && !b1)
        return ling_launch(g0, &g1, st);
    // the instantiated pair: nn.Linear's input gradient (dY W) and weight gradient (dY^T X)
    if (live0 && live1 && gemm_split(g0) == FS_GEMM_SPLIT && gemm_split(g1) == FS_GEMM_SPLIT && a0 && !b0 && !a1 &&
        !b1) {
        const unsigned mt0 = (unsigned)((g0.M + 31) / 32), mt1 = (unsigned)((g1.M + 31) / 32);
        const unsigned t0 = mt0 * (unsigned)((g0.N + 31) / 32), t1 = mt1 * (unsigned)((g1.N + 31) / 32);
        hipLaunchKernelGGL((gemm2_f32_kernel<FS_GEMM_SPLIT, true, false, false, false>), dim3(t0 + t1),
                           dim3(64 * FS_GEMM_SPLIT), 0, st, g0, g1, t0, mt0, mt1);
        return hipGetLastError();
    }
    if (hipError_t e = fs_linear_f32_impl(g0, st); e != hipSuccess) return e;
    return fs_linear_f32_impl(g1, st);
}

// u's write-back stores 4 floats at once where A is contiguous along k
static bool bn_out_ok(const GemmArgs &g, const BnIn *bn) {
    return !bn || !bn->a_out || (((uintptr_t)bn->a_out & 15) == 0 && g.sam % 4 == 0);
}

hipError_t fs_linear_bn_f32_impl(const fs::GemmArgs &g, const fs::BnIn *bn, hipStream_t st) {
    if (!bn) return fs_linear_f32_impl(g, st);
    if (g.M <= 0 || g.N <= 0) return hipSuccess;
    if (lean_gemm() && lin_ok(g, bn)) return lin_launch(g, bn, nullptr, nullptr, st);
    const bool ak = g.sak == 1 && ((uintptr_t)g.A & 15) == 0 && g.sam % 4 == 0;
    const bool bk = g.sbk == 1 && ((uintptr_t)g.B & 15) == 0 && g.sbn % 4 == 0;
    if (g.K > kBnMaxK || g.rowsum_a || !bn_out_ok(g, bn)) return hipErrorInvalidValue;
    const dim3 grid((unsigned)((g.M + 31) / 32), (unsigned)((g.N + 31) / 32));
    const int split = gemm_split(g);
    if (64 * split < g.K) return hipErrorInvalidValue;  // one thread per column in the statistics prologue
#define FS_GB(S, A, B)                                                                                     \
    if (split == S && ak == A && bk == B) {                                                                \
        hipLaunchKernelGGL((gemm_bn_f32_kernel<S, A, B>), grid, dim3(64 * S), 0, st, g, *bn);             \
        return hipGetLastError();                                                                          \
    }
    FS_GB(FS_GEMM_SPLIT, true, true) FS_GB(FS_GEMM_SPLIT, true, false) FS_GB(FS_GEMM_SPLIT, false, true)
    FS_GB(FS_GEMM_SPLIT, false, false)
#undef FS_GB
    return hipErrorInvalidValue;
}

static bool ex2_operand_ok(const GemmArgs &g, const BnIn *bn) {
    const bool ak = g.sak == 1 && ((uintptr_t)g.A & 15) == 0 && g.sam % 4 == 0;
    const bool bk = g.sbk == 1 && ((uintptr_t)g.B & 15) == 0 && g.sbn % 4 == 0;
    return ak && bk && g.M > 0 && g.N > 0 && !g.rowsum_a && bn_out_ok(g, bn) &&
           (!bn || (g.K <= kBnMaxK && 64 * gemm_split(g) >= g.K));
}

bool fs_linear_ex2_ok(const GemmArgs &g0, const BnIn *b0, const GemmArgs &g1, const BnIn *b1) {
    return ex2_operand_ok(g0, b0) && ex2_operand_ok(g1, b1) && gemm_split(g0) == FS_GEMM_SPLIT &&
           gemm_split(g1) == FS_GEMM_SPLIT;
}

hipError_t fs_linear_ex2_impl(const GemmArgs &g0, const BnIn *b0, const GemmArgs &g1, const BnIn *b1, hipStream_t st) {
    if (!fs_linear_ex2_ok(g0, b0, g1, b1)) return hipErrorInvalidValue;
    if (lean_gemm() && lin_ok(g0, b0) && lin_ok(g1, b1) && g0.K == g1.K) return lin_launch(g0, b0, &g1, b1, st);
    const unsigned mt0 = (unsigned)((g0.M + 31) / 32), mt1 = (unsigned)((g1.M + 31) / 32);
    const unsigned t0 = mt0 * (unsigned)((g0.N + 31) / 32), t1 = mt1 * (unsigned)((g1.N + 31) / 32);
    const BnIn none{};
    hipLaunchKernelGGL(gemm_ex2_kernel<FS_GEMM_SPLIT>, dim3(t0 + t1), dim3(64 * FS_GEMM_SPLIT), 0, st, g0,
                       b0 ? *b0 : none, g1, b1 ? *b1 : none, t0, mt0, mt1, (b0 ? 1 : 0) | (b1 ? 2 : 0));
    return hipGetLastError();
}

hipError_t fs_bn_running_update_impl(int nbn, int H, float *rm, float *rv, int64_t *nbt, const float *stats,
                                     int passes, int64_t rows0, int64_t rows1, float momentum, const int32_t *skip,
                                     hipStream_t st) {
    if (nbn <= 0 || H <= 0 || passes <= 0) return hipSuccess;
    const int64_t n = (int64_t)nbn * H;
    hipLaunchKernelGGL(bn_running_update_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, nbn, H, rm, rv,
                       nbt, stats, passes, rows0, rows1, momentum, skip);
    return hipGetLastError();
}

hipError_t fs_bn_relu_train_fwd_impl(int64_t B, int H, const float *x, const float *gamma, const float *beta,
                                     float *rm, float *rv, int64_t *nbt, float momentum, float eps, float *y,
                                     float *mean, float *invstd, hipStream_t st) {
    if (B <= 0 || H <= 0) return hipSuccess;
    const dim3 grid((unsigned)((H + kBnCols - 1) / kBnCols)), block(kBnCols * kBnRg);
    if (B <= kBnR * kBnRg)
        hipLaunchKernelGGL(bn_relu_train_fwd_kernel<kBnR>, grid, block, 0, st, B, H, x, gamma, beta, rm, rv, nbt,
                           momentum, eps, y, mean, invstd);
    else
        hipLaunchKernelGGL(bn_relu_train_fwd_kernel<0>, grid, block, 0, st, B, H, x, gamma, beta, rm, rv, nbt,
                           momentum, eps, y, mean, invstd);
    return hipGetLastError();
}

hipError_t fs_bn_relu_train_bwd_impl(int64_t B, int H, const float *x, const float *y, const float *dy,
                                     const float *gamma, const float *mean, const float *invstd, float *dx,
                                     const float *dx_add, float *dgamma, float *dbeta, hipStream_t st) {
    if (B <= 0 || H <= 0) return hipSuccess;
    const dim3 grid((unsigned)((H + kBnCols - 1) / kBnCols)), block(kBnCols * kBnRg);
    if (B <= kBnR * kBnRg)
        hipLaunchKernelGGL(bn_relu_train_bwd_kernel<kBnR>, grid, block, 0, st, B, H, x, y, dy, gamma, mean, invstd, dx,
                           dx_add, dgamma, dbeta);
    else
        hipLaunchKernelGGL(bn_relu_train_bwd_kernel<0>, grid, block, 0, st, B, H, x, y, dy, gamma, mean, invstd, dx,
                           dx_add, dgamma, dbeta);
    return hipGetLastError();
}
