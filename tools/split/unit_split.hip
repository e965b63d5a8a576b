// Unit harness for the split-bf16 building blocks of flow_split_kernels.hip
// (sgemm + split_epilogue round trip through the LDS planes, and the final-layer
// path preset_bias + sgemm + lanes_to_chains + tile_row), against f64 on the host.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I../../flow-state_amd/csrc unit_split.hip -o unit_split
#define FS_SPLIT_NO_HOST
#include "../../flow-state_amd/csrc/flow_split_kernels.hip"

#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>

using namespace fs;

template <int H, int P>
__global__ void __launch_bounds__(kThreads, 1) unit_kernel(const float *X, const float *Wp, const float *Wf,
                                                           const float *bias, const float *zeros, float *out_x0,
                                                           float *out_hidden, float *out_final) {
    using WK = SplitWork<H>;
    constexpr int CTW = WK::CTW, RTW = WK::RTW, RD = FS_SPLIT_RD;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const SplitLds LL = split_lds(H / 2 < 64 ? H / 2 : 64, H, P);
    const int plane = LL.plane, xsb = LL.xsb;
    char *XP = smem;
    const int tid = threadIdx.x, wid = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int kst = H / 16;
    // X -> planes (pairs of columns per word)
    for (int c2 = wid; c2 < H / 2; c2 += kWaves) {
        uint32_t o[P];
        split2<P>(X[lane * H + 2 * c2], X[lane * H + 2 * c2 + 1], o);
#pragma unroll
        for (int p = 0; p < P; ++p) *(uint32_t *)(XP + p * plane + lane * xsb + 4 * c2) = o[p];
    }
    __syncthreads();
    for (int c = wid; c < H; c += kWaves) {
        float s = 0.f;
        for (int p = P - 1; p >= 0; --p) s += __builtin_bit_cast(float, (uint32_t)(*(const uint16_t *)(XP + p * plane + lane * xsb + 2 * c)) << 16);
        out_x0[lane * H + c] = s;
    }
    __syncthreads();
    const __amdgpu_buffer_rsrc_t W = __builtin_amdgcn_make_buffer_rsrc((void *)Wp, (short)0, (int)(H / 32 * kst * P * 1024), 0x00020000);
    const bool active = wid < WK::NUNITS;
    const int tile0 = WK::tile0(wid), rt0 = WK::rt0(wid);
    f32x16 acc[CTW][RTW];
    SRing<P, CTW, RD> R;
    if (active) {
        sring_prologue<P, CTW, RD>(R, W, 0, kst, tile0);
        sgemm<P, CTW, RTW, RD, false>(XP, plane, xsb, W, 0, kst, tile0, rt0, R, acc);
    }
    __syncthreads();
    EpiVec<CTW> ev;
    load_epi<CTW>(ev, nullptr, zeros, tile0);
    if (active) split_epilogue<P, H, CTW, RTW, false>(XP, plane, xsb, tile0, rt0, ev, acc);
    __syncthreads();
    for (int c = wid; c < H; c += kWaves) {
        float s = 0.f;
        for (int p = P - 1; p >= 0; --p) s += __builtin_bit_cast(float, (uint32_t)(*(const uint16_t *)(XP + p * plane + lane * xsb + 2 * c)) << 16);
        out_hidden[lane * H + c] = s;
    }
    __syncthreads();
    if (wid == 0) {
        const __amdgpu_buffer_rsrc_t WF = __builtin_amdgcn_make_buffer_rsrc((void *)Wf, (short)0, (int)(kst * P * 1024), 0x00020000);
        SRing<P, 1, RD> R2;
        f32x16 a2[1][2];
        sring_prologue<P, 1, RD>(R2, WF, 0, kst, 0);
        preset_bias(a2, bias);
        sgemm<P, 1, 2, RD, true>(XP, plane, xsb, WF, 0, kst, 0, 0, R2, a2);
        lanes_to_chains(a2[0][0], a2[0][1]);
#pragma unroll
        for (int m = 0; m < 32; ++m) out_final[lane * 32 + m] = tile_row(a2[0][0], a2[0][1], m);
    }
}

static double sum_planes_ref(float v, int P) {  // what P RNE-bf16 planes of v sum to
    double s = 0;
    for (int p = 0; p < P; ++p) {
        uint32_t u;
        memcpy(&u, &v, 4);
        const uint32_t b = (u + 0x7FFFu + ((u >> 16) & 1u)) & 0xffff0000u;
        float bf;
        memcpy(&bf, &b, 4);
        s += bf;
        v -= bf;
    }
    return s;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

template <int H, int P>
static int run(unsigned seed) {
    const int kst = H / 16;
    srand(seed);
    auto rnd = [] { return (float)rand() / RAND_MAX * 2.f - 1.f; };
    std::vector<float> X(64 * H), Wm(H * H), Wf(32 * H), bias(32), zeros(H, 0.f);
    for (auto &v : X) v = rnd();
    for (auto &v : Wm) v = rnd() * 0.2f;
    for (auto &v : Wf) v = rnd() * 0.2f;
    for (auto &v : bias) v = rnd();
    float *dX, *dW, *dWf, *dWp, *dWfp, *db, *dz, *dx0, *dh, *dfo;
    CK(hipMalloc(&dX, X.size() * 4));
    CK(hipMalloc(&dW, Wm.size() * 4));
    CK(hipMalloc(&dWf, Wf.size() * 4));
    const size_t wpb = (size_t)H / 32 * kst * P * 1024, wfb = (size_t)kst * P * 1024;
    CK(hipMalloc(&dWp, wpb));
    CK(hipMalloc(&dWfp, wfb));
    CK(hipMalloc(&db, 32 * 4));
    CK(hipMalloc(&dz, H * 4));
    CK(hipMalloc(&dx0, 64 * H * 4));
    CK(hipMalloc(&dh, 64 * H * 4));
    CK(hipMalloc(&dfo, 64 * 32 * 4));
    CK(hipMemcpy(dX, X.data(), X.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dW, Wm.data(), Wm.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dWf, Wf.data(), Wf.size() * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(db, bias.data(), 32 * 4, hipMemcpyHostToDevice));
    CK(hipMemcpy(dz, zeros.data(), H * 4, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(pack_split_linear_kernel, dim3(64), dim3(256), 0, 0, (uint16_t *)dWp, dW, H, kst, H / 32, H, 0, 0, 1.f, P, 1, 1);
    hipLaunchKernelGGL(pack_split_linear_kernel, dim3(64), dim3(256), 0, 0, (uint16_t *)dWfp, dWf, H, kst, 1, 32, 0, 0, 1.f, P, 1, 1);
    const int lds = split_lds(H / 2 < 64 ? H / 2 : 64, H, P).total;
    CK(hipFuncSetAttribute((const void *)unit_kernel<H, P>, hipFuncAttributeMaxDynamicSharedMemorySize, 163840));
    hipLaunchKernelGGL((unit_kernel<H, P>), dim3(1), dim3(kThreads), lds, 0, dX, dWp, dWfp, db, dz, dx0, dh, dfo);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    std::vector<float> x0(64 * H), hid(64 * H), fo(64 * 32);
    CK(hipMemcpy(x0.data(), dx0, x0.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(hid.data(), dh, hid.size() * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(fo.data(), dfo, fo.size() * 4, hipMemcpyDeviceToHost));
    double e0 = 0, e1 = 0, e2 = 0;
    int bad1c = -1, bad1f = -1;
    for (int c = 0; c < 64; ++c)
        for (int f = 0; f < H; ++f) {
            e0 = fmax(e0, fabs(x0[c * H + f] - sum_planes_ref(X[c * H + f], P)));
            double s = 0, a = 0;
            for (int k = 0; k < H; ++k) {
                s += (double)Wm[f * H + k] * X[c * H + k];
                a += fabs((double)Wm[f * H + k] * X[c * H + k]);
            }
            const double e = fabs(hid[c * H + f] - s) / a;
            if (e > e1) { e1 = e; bad1c = c; bad1f = f; }
        }
    int bad2c = -1, bad2m = -1;
    for (int c = 0; c < 64; ++c)
        for (int m = 0; m < 32; ++m) {
            double s = bias[m], a = fabs(bias[m]);
            for (int k = 0; k < H; ++k) {
                s += (double)Wf[m * H + k] * hid[c * H + k];
                a += fabs((double)Wf[m * H + k] * hid[c * H + k]);
            }
            const double e = fabs(fo[c * 32 + m] - s) / a;
            if (e > e2) { e2 = e; bad2c = c; bad2m = m; }
        }
    printf("H=%d P=%d: x planes err %.3e | hidden GEMM rel %.3e (chain %d feat %d) | final rel %.3e (chain %d row %d)\n",
           H, P, e0, e1, bad1c, bad1f, e2, bad2c, bad2m);
    if (e2 > 1e-5) {
        printf("  final, chain %d: ", bad2c);
        for (int m = 0; m < 32; ++m) {
            double s = bias[m];
            for (int k = 0; k < H; ++k) s += (double)Wf[m * H + k] * hid[bad2c * H + k];
            printf("%d:%.2e ", m, fo[bad2c * 32 + m] - s);
        }
        printf("\n");
        int nbad[64] = {0};
        for (int c = 0; c < 64; ++c)
            for (int m = 0; m < 32; ++m) {
                double s = bias[m], a = fabs(bias[m]);
                for (int k = 0; k < H; ++k) { s += (double)Wf[m * H + k] * hid[c * H + k]; a += fabs((double)Wf[m * H + k] * hid[c * H + k]); }
                if (fabs(fo[c * 32 + m] - s) / a > 1e-5) nbad[c]++;
            }
        printf("  bad rows per chain: ");
        for (int c = 0; c < 64; ++c) printf("%d ", nbad[c]);
        printf("\n");
    }
    return 0;
}

int main() {
    run<32, 3>(1);
    run<32, 2>(1);
    run<64, 3>(2);
    run<128, 3>(3);
    run<256, 3>(4);
    run<256, 2>(4);
    return 0;
}
