// A/B probe for VERDICT r05 item 2: does an in-launch hand-off beat the launch boundary
// between the two Linears of a training-mode ResidualBlock (resnet.py:37-50) at the A2
// training shapes (batch 256, H = 128)?
//
// (a) launches: the product's form, two BatchNorm-in-load products per block, each its own
//     launch of 32 workgroups (one 32 x 32 output tile each, 8 waves sharing the k range, as
//     train_kernels.hip's gemm_lin_kernel): u = Lin0(relu(BN0(t))) with u's per-tile
//     statistics, then out = Lin1(relu(BN1(u))) + t with out's statistics.
// (b) fused: the same two tiles per workgroup in ONE launch.  Lin1's BatchNorm needs every
//     row tile's statistics of all 128 columns of u and its tile needs u's four column tiles
//     of its rows, so the hand-off is an all-to-all among the 32 workgroups: u and its
//     statistics stored write-through (`sc1` 16-byte / 8-byte stores), every storing wave's
//     `s_waitcnt vmcnt(0)`, a workgroup barrier, one lane's agent-scope atomic add on one
//     counter, lane 0 polls it with `sc1` loads, a barrier, then `sc1` loads of u and the
//     statistics (the guide's first valid hand-off form, MI355X_MICROARCH.md "Workgroup
//     dispatch ... inter-workgroup visibility").  The last workgroup out resets the counters
//     for the next replay.
// Both variants run as HIP graphs of `chain` blocks (the A2 forward's 46 blocks per pass),
// replayed; the outputs of (a) and (b) are compared bit for bit.
//
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -munsafe-fp-atomics block_fuse.hip -o block_fuse
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

typedef float t4 __attribute__((ext_vector_type(4)));
typedef float t16 __attribute__((ext_vector_type(16)));
typedef float f2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

constexpr int M = 256, K = 128, NC = 128;  // rows, input width, output width
constexpr int MT = M / 32, NT = NC / 32;    // 8 x 4 output tiles
constexpr int TILES = MT * NT;
constexpr int KBW = K / 64;  // k-blocks per wave (8 waves x 8-wide k-blocks)
constexpr int SC1 = 16;      // buffer-instruction cache policy: sc1 (as flow_kernels.hip's hand-offs)

struct Lin {
    const float *A, *W, *bias, *R, *st;  // st: producer tile statistics of A [MT][K][2]
    const float *gamma, *beta;
    float *C, *stats, *a_out;
    int rows, tiles;  // (GENERIC prologue) the batch and its statistics tiles, at run time
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void *p, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void *)p, (short)0, bytes, 0x00020000);
}

struct Lds {
    t16 part[7][64];
    float mu[K], is[K], gm[K], bt[K];
};

// One 32 x 32 tile of relu(BN(A)) W^T + bias (+ R), BatchNorm statistics combined from the
// producer's tiles (Chan's update, tiles in order), this tile's (mean, M2) written.  SC: the
// A / statistics loads and the C / statistics stores through sc1 (the fused variant's
// hand-off).  Returns with every wave alive (no early return).
template <bool SC_IN, bool SC_OUT, bool GENERIC = false>
__device__ __forceinline__ void tile(const Lin &P, int bx, int by, Lds &L) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = lane & 31, h = lane >> 5;
    const int m = bx * 32 + r, col = by * 32 + r;
    const auto Ar = rsrc(P.A, M * K * 4), Wr = rsrc(P.W, NC * K * 4), Sr = rsrc(P.st, MT * K * 8);
    const int kq = 8 * w + 4 * h;
    const int k = threadIdx.x;
    f2 st[MT];
    float gk = 0.f, bk = 0.f;
    if (k < K) {
#pragma unroll
        for (int t = 0; t < MT; ++t)
            st[t] = __builtin_bit_cast(f2, __builtin_amdgcn_raw_buffer_load_b64(Sr, (t * K + k) * 8, 0, SC_IN ? SC1 : 0));
        gk = P.gamma[k];
        bk = P.beta[k];
    }
    t4 a[KBW], b[KBW];
#pragma unroll
    for (int s = 0; s < KBW; ++s) {
        a[s] = __builtin_bit_cast(t4, __builtin_amdgcn_raw_buffer_load_b128(Ar, (m * K + kq + 64 * s) * 4, 0, SC_IN ? SC1 : 0));
        b[s] = __builtin_bit_cast(t4, __builtin_amdgcn_raw_buffer_load_b128(Wr, (col * K + kq + 64 * s) * 4, 0, 0));
    }
    float ep_r[16], ep_bias = 0.f;
    if (w == 0) {
        const auto Rr = rsrc(P.R, M * NC * 4);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int row = bx * 32 + 8 * (i >> 2) + 4 * h + (i & 3);
            ep_r[i] = P.R ? __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(Rr, (row * NC + col) * 4, 0, 0)) : 0.f;
        }
        ep_bias = P.bias[col];
    }
    if (k < K) {
        float n = 0.f, mean = 0.f, m2 = 0.f;
        if (GENERIC) {  // train_kernels.hip lin_bn_prologue's form: batch and tiles at run time
            const int rows = P.rows;
#pragma unroll
            for (int t = 0; t < MT; ++t) {
                if (t < P.tiles) {
                    const int row0 = 32 * t;
                    const float nb = (float)(rows - row0 < 32 ? rows - row0 : 32);
                    const float nn = n + nb, d = st[t][0] - mean;
                    mean = mean + d * (nb / nn);
                    m2 = m2 + st[t][1] + d * d * (n * nb / nn);
                    n = nn;
                }
            }
            L.is[k] = 1.f / sqrtf(m2 / (float)rows + 1e-5f);
        } else {
#pragma unroll
            for (int t = 0; t < MT; ++t) {
                const float nb = 32.f, nn = n + nb, d = st[t][0] - mean;
                mean = mean + d * (nb / nn);
                m2 = m2 + st[t][1] + d * d * (n * nb / nn);
                n = nn;
            }
            L.is[k] = 1.f / sqrtf(m2 / (float)M + 1e-5f);
        }
        L.mu[k] = mean;
        L.gm[k] = gk;
        L.bt[k] = bk;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < KBW; ++s) {
        const int k0 = kq + 64 * s;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int kk = k0 + j;
            const float o = L.gm[kk] * ((a[s][j] - L.mu[kk]) * L.is[kk]) + L.bt[kk];
            a[s][j] = o > 0.f ? o : 0.f;
        }
        if (P.a_out && (k0 >> 5) % NT == by) *(t4 *)(P.a_out + m * K + k0) = a[s];
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
    if (w == 0) {
#pragma unroll 1
        for (int p = 0; p < 7; ++p) acc += L.part[p][lane];
        float sv = 0.f;
        const auto Cr = rsrc(P.C, M * NC * 4);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int row = bx * 32 + 8 * (i >> 2) + 4 * h + (i & 3);
            const float v = acc[i] + ep_bias + ep_r[i];
            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), Cr, (row * NC + col) * 4, 0,
                                                  SC_OUT ? SC1 : 0);
            acc[i] = v;
            sv += v;
        }
        const float mean = (sv + __shfl_xor(sv, 32)) / 32.f;
        float q = 0.f;
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float d = acc[i] - mean;
            q += d * d;
        }
        q += __shfl_xor(q, 32);
        if (h == 0)
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, f2{mean, q}), rsrc(P.stats, MT * NC * 8),
                                                  ((bx * NC + col) * 8), 0, SC_OUT ? SC1 : 0);
    }
}

template <bool GENERIC>
__global__ __launch_bounds__(512) void lin_kernel(Lin P) {
    __shared__ Lds L;
    tile<false, false, GENERIC>(P, (int)blockIdx.x % MT, (int)blockIdx.x / MT, L);
}

// cnt[0]: arrivals after Lin0, cnt[1]: workgroups done (the last one resets both)
__global__ __launch_bounds__(512) void block_fused_kernel(Lin P0, Lin P1, unsigned *cnt, int *err) {
    __shared__ Lds L;
    __shared__ int dead;
    const int bx = (int)blockIdx.x % MT, by = (int)blockIdx.x / MT;
    tile<false, true>(P0, bx, by, L);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        dead = 0;
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        unsigned spins = 0;
        while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)TILES) {
            __builtin_amdgcn_s_sleep(1);
            if (++spins > (1u << 20)) {
                dead = 1;
                atomicOr(err, 1);
                break;
            }
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");  // (compiler only)
    __syncthreads();
    tile<true, false>(P1, bx, by, L);
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned done = __hip_atomic_fetch_add(cnt + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (done == TILES - 1) {  // last out: every workgroup has passed its poll
            __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(cnt + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

static float frand(uint64_t &s) {
    s = s * 6364136223846793005ull + 1442695040888963407ull;
    return (float)((s >> 40) & 0xffffff) / 16777216.f * 2.f - 1.f;
}

int main(int argc, char **argv) {
    const int chain = argc > 1 ? atoi(argv[1]) : 46;
    const int reps = argc > 2 ? atoi(argv[2]) : 50;
    uint64_t seed = 1;
    // per block: W0, b0, W1, b1, gamma0/beta0, gamma1/beta1 (shared across the chain: timing)
    std::vector<float> h(NC * K);
    auto upload = [&](float scale, size_t n, float add = 0.f) {
        std::vector<float> v(n);
        for (auto &x : v) x = add + scale * frand(seed);
        float *d;
        CK(hipMalloc(&d, n * 4));
        CK(hipMemcpy(d, v.data(), n * 4, hipMemcpyHostToDevice));
        return d;
    };
    float *W0 = upload(0.1f, NC * K), *W1 = upload(0.1f, NC * K), *b0 = upload(0.1f, NC), *b1 = upload(0.1f, NC);
    float *g0 = upload(0.2f, K, 1.f), *be0 = upload(0.1f, K), *g1 = upload(0.2f, K, 1.f), *be1 = upload(0.1f, K);
    // activations: t_i (block inputs) and u_i, their statistics, a_out buffers, per variant
    auto alloc = [](size_t n) {
        float *d;
        CK(hipMalloc(&d, n * 4));
        CK(hipMemset(d, 0, n * 4));
        return d;
    };
    struct Bufs {
        std::vector<float *> t, st, u, su, a0, a1;
    } V[3];
    float *t0 = upload(1.f, M * K);
    // the first block's input statistics (exact enough: computed on the host per tile)
    std::vector<float> ht(M * K), hst(MT * K * 2);
    CK(hipMemcpy(ht.data(), t0, M * K * 4, hipMemcpyDeviceToHost));
    for (int t = 0; t < MT; ++t)
        for (int k = 0; k < K; ++k) {
            float s = 0.f;
            for (int i = 0; i < 32; ++i) s += ht[(t * 32 + i) * K + k];
            const float mean = s / 32.f;
            float q = 0.f;
            for (int i = 0; i < 32; ++i) q += (ht[(t * 32 + i) * K + k] - mean) * (ht[(t * 32 + i) * K + k] - mean);
            hst[(t * K + k) * 2] = mean;
            hst[(t * K + k) * 2 + 1] = q;
        }
    float *st0 = alloc(MT * K * 2);
    CK(hipMemcpy(st0, hst.data(), hst.size() * 4, hipMemcpyHostToDevice));
    for (int v = 0; v < 3; ++v) {
        V[v].t.push_back(t0);
        V[v].st.push_back(st0);
        for (int i = 0; i < chain; ++i) {
            V[v].u.push_back(alloc(M * NC));
            V[v].su.push_back(alloc(MT * NC * 2));
            V[v].t.push_back(alloc(M * NC));
            V[v].st.push_back(alloc(MT * NC * 2));
            V[v].a0.push_back(alloc(M * K));
            V[v].a1.push_back(alloc(M * K));
        }
    }
    unsigned *cnt;
    int *err;
    CK(hipMalloc(&cnt, 64));
    CK(hipMemset(cnt, 0, 64));
    CK(hipMalloc(&err, 4));
    CK(hipMemset(err, 0, 4));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipGraphExec_t ex[3];
    for (int v = 0; v < 3; ++v) {
        hipGraph_t g;
        CK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
        for (int i = 0; i < chain; ++i) {
            Lin P0{V[v].t[i], W0, b0, nullptr, V[v].st[i], g0, be0, V[v].u[i], V[v].su[i], V[v].a0[i], M, MT};
            Lin P1{V[v].u[i], W1, b1, V[v].t[i], V[v].su[i], g1, be1, V[v].t[i + 1], V[v].st[i + 1], V[v].a1[i], M, MT};
            if (v == 0) {
                hipLaunchKernelGGL(lin_kernel<false>, dim3(TILES), dim3(512), 0, s, P0);
                hipLaunchKernelGGL(lin_kernel<false>, dim3(TILES), dim3(512), 0, s, P1);
            } else if (v == 2) {
                hipLaunchKernelGGL(lin_kernel<true>, dim3(TILES), dim3(512), 0, s, P0);
                hipLaunchKernelGGL(lin_kernel<true>, dim3(TILES), dim3(512), 0, s, P1);
            } else {
                hipLaunchKernelGGL(block_fused_kernel, dim3(TILES), dim3(512), 0, s, P0, P1, cnt, err);
            }
        }
        CK(hipStreamEndCapture(s, &g));
        CK(hipGraphInstantiate(&ex[v], g, nullptr, nullptr, 0));
    }
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    float best[3] = {1e30f, 1e30f, 1e30f};
    const char *names[3] = {"launches (2 per block)", "fused (1 launch, in-launch hand-off)",
                            "launches, run-time prologue (2 per block)"};
    for (int round = 0; round < 3; ++round)
        for (int v = 0; v < 3; ++v) {
            CK(hipGraphLaunch(ex[v], s));
            CK(hipStreamSynchronize(s));
            CK(hipEventRecord(e0, s));
            for (int r = 0; r < reps; ++r) CK(hipGraphLaunch(ex[v], s));
            CK(hipEventRecord(e1, s));
            CK(hipStreamSynchronize(s));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const float us = ms * 1e3f / reps / chain;
            if (us < best[v]) best[v] = us;
            printf("round %d %s: %.2f us per block (%d blocks per graph, %d replays)\n", round, names[v], us, chain,
                   reps);
        }
    int herr = 0;
    CK(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    std::vector<float> o0(M * NC), o1(M * NC);
    size_t ndiff = 0, ndiff_generic = 0;
    for (int i = 1; i <= chain; ++i) {
        CK(hipMemcpy(o0.data(), V[0].t[i], M * NC * 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(o1.data(), V[1].t[i], M * NC * 4, hipMemcpyDeviceToHost));
        ndiff += memcmp(o0.data(), o1.data(), M * NC * 4) != 0;
        CK(hipMemcpy(o1.data(), V[2].t[i], M * NC * 4, hipMemcpyDeviceToHost));
        ndiff_generic += memcmp(o0.data(), o1.data(), M * NC * 4) != 0;
    }
    bool finite = true;
    for (float x : o0) finite &= std::isfinite(x);
    printf("{\"probe\": \"block_fuse\", \"shape\": \"A2 ResidualBlock forward, batch %d, H %d\", \"chain\": %d, "
           "\"us_per_block_launches\": %.3f, \"us_per_block_fused\": %.3f, \"fused_over_launches\": %.3f, "
           "\"us_per_block_launches_runtime_prologue\": %.3f, "
           "\"blocks_differing\": %zu, \"blocks_differing_runtime_prologue\": %zu, \"handoff_timeouts\": %d, "
           "\"finite\": %s}\n",
           M, K, chain, best[0], best[1], best[1] / best[0], best[2], ndiff, ndiff_generic, herr,
           finite ? "true" : "false");
    return (ndiff || ndiff_generic || herr || !finite) ? 1 : 0;
}
