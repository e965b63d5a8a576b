// Are v_mfma_f32_32x32x2_f32 and v_mfma_f32_16x16x4_f32 the same fmaf chain?  For random
// operands (wide exponent range, so every rounding shows), a 32 x 32 tile over one 8-wide
// k-group is computed (a) as the flow kernels do: 4 x 32x32x2, MFMA j taking k = j (lanes
// 0-31) and k = 4 + j (lanes 32-63); (b) as four 16 x 16 quadrants, each 2 x 16x16x4 with
// the k-slots (0, 4, 1, 5) then (2, 6, 3, 7); (c) on the CPU as fmaf chains in candidate
// orders.  Prints how many of the 1024 outputs differ bitwise between (a) and (b), and
// between each and the CPU orders.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));

__global__ void k32(const float *A, const float *B, const float *C0, float *C) {
    const int lane = threadIdx.x, r = lane & 31, h = lane >> 5;
    f16v acc;
    for (int i = 0; i < 16; ++i) acc[i] = C0[(8 * (i >> 2) + 4 * h + (i & 3)) * 32 + r];
    for (int j = 0; j < 4; ++j)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(A[r * 8 + 4 * h + j], B[(4 * h + j) * 32 + r], acc, 0, 0, 0);
    for (int i = 0; i < 16; ++i) C[(8 * (i >> 2) + 4 * h + (i & 3)) * 32 + r] = acc[i];
}

__global__ void k16(const float *A, const float *B, const float *C0, float *C) {
    const int lane = threadIdx.x, r = lane & 15, q = lane >> 4;
    const int slot0[4] = {0, 4, 1, 5}, slot1[4] = {2, 6, 3, 7};
    for (int qr = 0; qr < 2; ++qr)
        for (int qc = 0; qc < 2; ++qc) {
            f4 acc;
            // 16x16 accumulator: lane (q, r) holds rows 4q + i, column r
            for (int i = 0; i < 4; ++i) acc[i] = C0[(16 * qr + 4 * q + i) * 32 + 16 * qc + r];
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[(16 * qr + r) * 8 + slot0[q]], B[slot0[q] * 32 + 16 * qc + r],
                                                       acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(A[(16 * qr + r) * 8 + slot1[q]], B[slot1[q] * 32 + 16 * qc + r],
                                                       acc, 0, 0, 0);
            for (int i = 0; i < 4; ++i) C[(16 * qr + 4 * q + i) * 32 + 16 * qc + r] = acc[i];
        }
}

static float rnd(unsigned &s) {
    s = s * 1664525u + 1013904223u;
    const float m = (float)((s >> 8) & 0xffff) / 65536.f - 0.5f;
    s = s * 1664525u + 1013904223u;
    return ldexpf(m, (int)((s >> 24) % 24) - 12);
}

int main() {
    const int nA = 32 * 8, nB = 8 * 32, nC = 32 * 32;
    float hA[nA], hB[nB], hC0[nC], c32[nC], c16[nC];
    unsigned s = 12345;
    for (float &v : hA) v = rnd(s);
    for (float &v : hB) v = rnd(s);
    for (float &v : hC0) v = rnd(s);
    float *A, *B, *C0, *C;
    hipMalloc(&A, sizeof hA);
    hipMalloc(&B, sizeof hB);
    hipMalloc(&C0, sizeof hC0);
    hipMalloc(&C, sizeof c32);
    hipMemcpy(A, hA, sizeof hA, hipMemcpyHostToDevice);
    hipMemcpy(B, hB, sizeof hB, hipMemcpyHostToDevice);
    hipMemcpy(C0, hC0, sizeof hC0, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k32, dim3(1), dim3(64), 0, 0, A, B, C0, C);
    hipMemcpy(c32, C, sizeof c32, hipMemcpyDeviceToHost);
    hipLaunchKernelGGL(k16, dim3(1), dim3(64), 0, 0, A, B, C0, C);
    hipMemcpy(c16, C, sizeof c16, hipMemcpyDeviceToHost);
    // CPU fmaf chains: order "pairs" = 0,4,1,5,2,6,3,7 ; "seq" = 0..7
    const int ord_pairs[8] = {0, 4, 1, 5, 2, 6, 3, 7}, ord_seq[8] = {0, 1, 2, 3, 4, 5, 6, 7};
    const int ord_pairs_rev[8] = {4, 0, 5, 1, 6, 2, 7, 3};
    int d_ab = 0, d_a_pairs = 0, d_b_pairs = 0, d_a_seq = 0, d_a_rev = 0;
    for (int m = 0; m < 32; ++m)
        for (int n = 0; n < 32; ++n) {
            float vp = hC0[m * 32 + n], vs = vp, vr = vp;
            for (int t = 0; t < 8; ++t) {
                vp = fmaf(hA[m * 8 + ord_pairs[t]], hB[ord_pairs[t] * 32 + n], vp);
                vs = fmaf(hA[m * 8 + ord_seq[t]], hB[ord_seq[t] * 32 + n], vs);
                vr = fmaf(hA[m * 8 + ord_pairs_rev[t]], hB[ord_pairs_rev[t] * 32 + n], vr);
            }
            const float a = c32[m * 32 + n], b = c16[m * 32 + n];
            d_ab += memcmp(&a, &b, 4) != 0;
            d_a_pairs += memcmp(&a, &vp, 4) != 0;
            d_b_pairs += memcmp(&b, &vp, 4) != 0;
            d_a_seq += memcmp(&a, &vs, 4) != 0;
            d_a_rev += memcmp(&a, &vr, 4) != 0;
        }
    printf("{\"outputs\": 1024, \"diff_32x32x2_vs_16x16x4\": %d, \"diff_32_vs_cpu_pairs\": %d, "
           "\"diff_16_vs_cpu_pairs\": %d, \"diff_32_vs_cpu_seq\": %d, \"diff_32_vs_cpu_pairs_hfirst1\": %d}\n",
           d_ab, d_a_pairs, d_b_pairs, d_a_seq, d_a_rev);
    return 0;
}
