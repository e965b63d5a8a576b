// Adam for the Algorithm-2 training step (main_algorithm_2.py:310,326,440,451:
// torch.optim.Adam(model.parameters(), lr, weight_decay), L2 weight decay added to the
// gradient) over the flat parameter / gradient / moment buffers of GraphedTrainStep, in
// one pass: p, g, m, v read once, p, m, v written once (28 bytes per parameter).  torch's
// capturable multi-tensor Adam takes ~16 launches for the same update, and the step's
// "skip on a non-finite loss" rule (main_algorithm_2.py:324-326) cost a snapshot and a
// select of every buffer around it; here the kernel reads the loss and writes nothing when
// it is NaN / inf, or when the caller's skip word is set.
//
// The per-element arithmetic is torch's capturable _multi_tensor_adam (torch/optim/adam.py)
// op by op in float32: g' = g + wd p; m = lerp(m, g', 1 - beta1); v = v beta2 + (1 - beta2)
// g' g'; step_size = 1 / ((beta1^t - 1) / lr); d = (sqrt(v) / sqrt(1 - beta2^t) + eps) /
// step_size; p = p + m / d, with t the incremented step count (a float tensor, as torch
// keeps it).  The step count itself is bumped by a second one-thread launch after the
// update (every workgroup of the first reads the old value).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#include "fs_internal.h"

namespace fs {

struct AdamScalars {
    float lr, beta1, beta2, one_m_beta1, one_m_beta2, eps, wd;
};

__device__ __forceinline__ bool loss_finite(const float *loss) {
    const float l = *loss;
    return !(isnan(l) || isinf(l));
}

// The step writes nothing when the loss is not finite or the caller's skip word is set (a
// graphed epoch's sticky NaN flag: no update after a failed step).
__device__ __forceinline__ bool skip_step(const float *loss, const int32_t *skip) {
    return (loss && !loss_finite(loss)) || (skip && *skip != 0);
}

__device__ __forceinline__ void adam_elem(float &p, float g, float &m, float &v, float wd, float w1, float b2,
                                          float w2, float bc2s, float eps, float step_size) {
    const float gd = g + wd * p;
    // torch's lerp: weight < 0.5 -> self + weight (end - self)
    m = w1 < 0.5f ? m + w1 * (gd - m) : gd - (gd - m) * (1.f - w1);
    v = v * b2;
    v = v + w2 * gd * gd;
    float d = sqrtf(v);
    d = d / bc2s;
    d = d + eps;
    d = d / step_size;
    p = p + m / d;
}

__global__ void __launch_bounds__(256) adam_kernel(float *__restrict__ p, const float *__restrict__ g,
                                                   float *__restrict__ m, float *__restrict__ v, int64_t n,
                                                   const float *__restrict__ step, const float *__restrict__ loss,
                                                   const int32_t *__restrict__ skip, AdamScalars s) {
    if (skip_step(loss, skip)) return;
    const float t = *step + 1.f;
    float bc1 = powf(s.beta1, t), bc2 = powf(s.beta2, t);
    bc1 = bc1 - 1.f;
    bc2 = bc2 - 1.f;
    bc2 = -bc2;
    bc1 = bc1 / s.lr;
    const float step_size = 1.f / bc1;
    const float bc2s = sqrtf(bc2);
    const int64_t n4 = n / 4;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    typedef float f4 __attribute__((ext_vector_type(4)));
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
        f4 pv = ((f4 *)p)[i], mv = ((f4 *)m)[i], vv = ((f4 *)v)[i];
        const f4 gv = ((const f4 *)g)[i];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            float pj = pv[j], mj = mv[j], vj = vv[j];
            adam_elem(pj, gv[j], mj, vj, s.wd, s.one_m_beta1, s.beta2, s.one_m_beta2, bc2s, s.eps, step_size);
            pv[j] = pj;
            mv[j] = mj;
            vv[j] = vj;
        }
        ((f4 *)p)[i] = pv;
        ((f4 *)m)[i] = mv;
        ((f4 *)v)[i] = vv;
    }
    for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        adam_elem(p[i], g[i], m[i], v[i], s.wd, s.one_m_beta1, s.beta2, s.one_m_beta2, bc2s, s.eps, step_size);
}

__global__ void adam_count_kernel(float *step, const float *loss, const int32_t *skip) {
    if (skip_step(loss, skip)) return;
    *step = *step + 1.f;
}

// The Algorithm-2 loss head (main_algorithm_2.py:316-318 with ALPHA = 1; core.py
// forward_kld / reverse_kld): loss = -mean(log_q) + 0 * (mean(E) + mean(lq_rev)), the
// three means, the negation, the zero-weighted reverse term (NaN / inf when it is, so the
// skip rule sees it) and the adds in one workgroup instead of seven launches; nan_out (a
// torch bool) = the sticky spline-NaN word is set.  Each mean is an ordered tree sum: the
// value agrees with torch's reduction within float32 rounding, not bit for bit.
__device__ __forceinline__ float block_sum256(const float *__restrict__ x, int64_t n, float *red) {
    const int t = threadIdx.x;
    float a = 0.f;
    for (int64_t i = t; i < n; i += 256) a += x[i];
    red[t] = a;
    __syncthreads();
#pragma unroll
    for (int w = 128; w > 0; w >>= 1) {
        if (t < w) red[t] = red[t] + red[t + w];
        __syncthreads();
    }
    const float r = red[0];
    __syncthreads();
    return r;
}

__global__ void __launch_bounds__(256) kld_loss_kernel(const float *__restrict__ log_q, int64_t B,
                                                       const float *__restrict__ E, const float *__restrict__ lq_rev,
                                                       int64_t R, const int32_t *__restrict__ nan_word,
                                                       float *__restrict__ loss, uint8_t *__restrict__ nan_out) {
    __shared__ float red[256];
    const float sq = block_sum256(log_q, B, red);
    float energy = 0.f;
    if (E) {
        const float se = block_sum256(E, R, red);
        const float sl = block_sum256(lq_rev, R, red);
        energy = se * (1.f / (float)R) + sl * (1.f / (float)R);  // torch's MeanOps: sum x (1 / n)
    }
    if (threadIdx.x == 0) {
        const float sample = -(sq * (1.f / (float)B));
        loss[0] = sample + 0.f * energy;
        if (nan_out) nan_out[0] = (nan_word && nan_word[0] != 0) ? 1 : 0;
    }
}

// d loss / d log_q = -g x (1 / B) per row (torch's NegBackward then MeanBackward)
__global__ void __launch_bounds__(256) kld_loss_bwd_kernel(const float *__restrict__ g, int64_t B,
                                                           float *__restrict__ out) {
    const float v = (-g[0]) * (1.f / (float)B);  // torch divides by a scalar as a product with its reciprocal
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < B; i += (int64_t)gridDim.x * 256) out[i] = v;
}

}  // namespace fs

using namespace fs;

hipError_t fs_adam_step_impl(float *p, const float *g, float *m, float *v, int64_t n, float *step, const float *loss,
                             const int32_t *skip, double lr, double beta1, double beta2, double eps, double weight_decay, hipStream_t st) {
    if (n < 0) return hipErrorInvalidValue;
    // 16-byte aligned buffers (the flat torch buffers are): the vector loop reads 4 at a time
    if ((((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v) & 15) != 0) return hipErrorInvalidValue;
    // scalars as torch hands them to its float32 kernels (python floats cast once)
    const AdamScalars s{(float)lr, (float)beta1, (float)beta2, (float)(1.0 - beta1), (float)(1.0 - beta2),
                        (float)eps, (float)weight_decay};
    if (n > 0) {
        int64_t blocks = (n / 4 + 255) / 256;
        if (blocks > 4096) blocks = 4096;  // grid-stride beyond ~16 workgroups per CU
        if (blocks < 1) blocks = 1;
        hipLaunchKernelGGL(adam_kernel, dim3((unsigned)blocks), dim3(256), 0, st, p, g, m, v, n, (const float *)step,
                           loss, skip, s);
        if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(adam_count_kernel, dim3(1), dim3(1), 0, st, step, loss, skip);
    return hipGetLastError();
}

hipError_t fs_kld_loss_impl(const float *log_q, int64_t B, const float *E, const float *lq_rev, int64_t R,
                            const int32_t *nan_word, float *loss, uint8_t *nan_out, hipStream_t st) {
    hipLaunchKernelGGL(kld_loss_kernel, dim3(1), dim3(256), 0, st, log_q, B, E, lq_rev, R, nan_word, loss, nan_out);
    return hipGetLastError();
}

hipError_t fs_kld_loss_bwd_impl(const float *g, int64_t B, float *grad_log_q, hipStream_t st) {
    const int64_t blocks = B / 256 + 1 < 64 ? B / 256 + 1 : 64;
    hipLaunchKernelGGL(kld_loss_bwd_kernel, dim3((unsigned)blocks), dim3(256), 0, st, g, B, grad_log_q);
    return hipGetLastError();
}
