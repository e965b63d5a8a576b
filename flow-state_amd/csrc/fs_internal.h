// Internal declarations shared by the HIP translation units of libflowstate.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <stdio.h>
#include <string.h>

#include "../../include/flowstate.h"

bool fs_flow_supported(const fs_flow_dims *d, char *why, size_t n);
int64_t fs_flow_raw_floats_impl(const fs_flow_dims *d);
int64_t fs_flow_packed_bytes_impl(const fs_flow_dims *d);
hipError_t fs_flow_pack_impl(const fs_flow_dims *d, const float *raw, float *packed, hipStream_t st);
// mode: 0 density (Coupling.forward stack, layers L-1..0), 1 sample (Coupling.inverse stack,
// layers 0..L-1, base draws supplied), 2 propose (sample with in-kernel base draws + box coords)
hipError_t fs_flow_pass_impl(const fs_flow_dims *d, const void *packed, int mode, const float *in, int64_t B,
                             float *out, float *scalar, int add_base, float *config, float *centered,
                             uint64_t seed, uint64_t counter, int64_t row_offset, double half_width,
                             int32_t *err, hipStream_t st, int64_t rows_per_counter = 0);

// split-bf16 flow image and pass (flow_split_kernels.hip; fs_flow_dims.precision 1 or 2)
namespace fs { struct FlowArgs; }
bool fs_flow_split_supported(const fs_flow_dims *d, char *why, size_t n);
int64_t fs_flow_split_packed_bytes(const fs_flow_dims *d);
hipError_t fs_flow_split_pack(const fs_flow_dims *d, const float *raw, float *packed, hipStream_t st);
hipError_t fs_flow_split_pass(const fs::FlowArgs &a, int mode, int precision, int N, int H, int K, hipStream_t st);
// pack_vec_kernel of the f32 image (biases, folded BatchNorm, unconditional knots), launched
// with dst shifted so that its vector section lands where the caller's image keeps it
hipError_t fs_gather_chunks_impl(const int64_t *tab, int64_t n, float *dst, hipStream_t st);
hipError_t fs_flow_pack_vec(float *dst, const float *raw_layer, const fs_flow_dims *d, hipStream_t st);

hipError_t fs_energy_impl(const fs_phys *p, const void *pos, int pos_is_f32, int64_t C, int N, double *E,
                          double *W, uint8_t *overlap, uint64_t *nbr, hipStream_t st,
                          const uint8_t *chain_is_f32 = nullptr);
hipError_t fs_mh_accept_impl(const fs_phys *p, int64_t C, int N, double *E_old, double *W_old, double *nll_old,
                             const double *E_new, const double *W_new, const float *log_q_new, uint64_t *pcg,
                             double *state, uint8_t *state_is_f32, const float *config, uint8_t *accept,
                             int64_t *attempts, int64_t *accepted, unsigned long long *n_accept, int flags,
                             hipStream_t st, const float *log_q_old = nullptr, const double *E_cur = nullptr,
                             const double *W_cur = nullptr);
hipError_t fs_min_image_impl(const fs_phys *p, const void *a, int64_t sa, const void *b, int f32, int64_t n,
                            double *delta, double *r, hipStream_t st);
hipError_t fs_particle_energy_impl(const fs_phys *p, const void *pos, int f32, int64_t C, int N, const int32_t *part,
                                   double *E, double *W, hipStream_t st);
hipError_t fs_metropolis_judge_impl(double beta, int64_t C, int64_t M, const double *E_ref, const double *E_new,
                                   uint64_t *pcg, uint8_t *accept, int64_t *n_accept, hipStream_t st);
hipError_t fs_adjust_displacement_impl(int64_t C, double *max_disp, const int64_t *attempts, const int64_t *accepted,
                                       int64_t *prev, double target, hipStream_t st);
hipError_t fs_classify_wells_impl(const void *pos, int f32, int64_t M, int N, double half_box, double r0,
                                  uint8_t *cls, uint8_t *state, double *avg_x, hipStream_t st);
hipError_t fs_pair_hist_impl(const void *pos, int f32, int64_t M, int N, double bound, const double *edges, int nb,
                             int32_t *counts, hipStream_t st);
hipError_t fs_rdf_mean_impl(const int32_t *counts, int64_t M, int nb, const double *denom, double *g, hipStream_t st);
hipError_t fs_rqs_forward_impl(int64_t M, int K, int inverse, const float *x, const float *uw, const float *uh,
                               const float *ud, float B, float *out, float *lad, int32_t *nan_flag, hipStream_t st);
hipError_t fs_rqs_backward_impl(int64_t M, int K, int inverse, const float *x, const float *uw, const float *uh,
                                const float *ud, float B, const float *g_out, const float *g_lad, float *gx,
                                float *guw, float *guh, float *gud, hipStream_t st);
int64_t fs_set_wide_rows_impl(int64_t rows);
int32_t fs_set_wide_trunk16_impl(int32_t on);
int32_t fs_set_wide_final32_impl(int32_t on);
int64_t fs_set_wide_handoff_spins_impl(int64_t spins);
int32_t fs_set_coupling_waves_impl(int32_t on);
int32_t fs_set_lean_gemm_impl(int32_t on);
hipError_t fs_target_energy_impl(const float *x, int64_t B, int N, double bound, double temperature, int num_wells,
                                 double v0a, double v0b, double r0, double k, float *E, float *gx, hipStream_t st);
hipError_t fs_center_impl(const double *state, int64_t n, double hw, float *out, hipStream_t st);
hipError_t fs_local_moves_impl(const fs_phys *p, int64_t C, int N, double *state, const uint8_t *is_f32,
                               double *E, double *W, uint64_t *pcg, uint64_t *pcg_buf, double *max_disp,
                               int64_t *attempts, int64_t *accepted, int64_t *prev, int64_t n_moves, int64_t step0,
                               int adjust_every, double target, int sample_every, double *samples_xy,
                               double *samples_ew, uint8_t *accept_log, unsigned long long *n_accept,
                               hipStream_t st, const uint8_t *gate = nullptr);
hipError_t fs_chains_copy_if_impl(const uint8_t *gate, int64_t C, int N, const fs_local_chains *src,
                                  const fs_local_chains *dst, hipStream_t st);

void fs_set_error(const char *fmt, ...);

// Raise a kernel's dynamic-LDS limit to the full 160 KiB once per device: the
// attribute belongs to the current device, and the library runs on whichever device
// the caller made current (flowstate._lib.on_device).  `done` is one bit per device.
inline hipError_t fs_set_max_lds_once(const void *kfn, std::atomic<unsigned long long> &done) {
    int dev = 0;
    if (hipError_t e = hipGetDevice(&dev); e != hipSuccess) return e;
    const unsigned long long bit = dev < 64 ? 1ull << dev : 0ull;
    if (bit && (done.load(std::memory_order_acquire) & bit)) return hipSuccess;
    hipError_t e = hipFuncSetAttribute(kfn, hipFuncAttributeMaxDynamicSharedMemorySize, 163840);
    if (e == hipSuccess && bit) done.fetch_or(bit, std::memory_order_release);
    return e;
}

// training conditioner pieces (train_kernels.hip): C = A . B (+ bias) (+ R), A[m][k] at
// A[m sam + k sak], B[k][n] at B[k sbk + n sbn]; rowsum_a (nullable) = sum_k A[m][k]
namespace fs {
struct GemmArgs {
    int64_t M, N, K;
    const float *A;
    int64_t sam, sak;
    const float *B;
    int64_t sbk, sbn;
    const float *bias;
    const float *R;
    int64_t ldr;
    float *C;
    int64_t ldc;
    float *rowsum_a;
    float *stats = nullptr;  // [ceil(M/32)][N][2] per 32-row tile: column mean, sum of squared deviations
};
// BatchNorm1d (train) + ReLU applied to the A operand as it is loaded (A = the raw
// pre-BatchNorm activations x [rows][K], row-major): batch statistics combined from the
// producer's per-tile column statistics (Chan's formula, tiles in order), u = relu(gamma
// (x - mean) invstd + beta).  Workgroup (0, 0) writes mean / invstd and updates the
// running statistics; the workgroups of column tile 0 write u (a_out, nullable).
struct BnIn {
    const float *stats;  // [tiles][K][2] from the producer's epilogue
    int64_t tiles, rows;
    const float *gamma, *beta;
    float eps, momentum;
    float *running_mean, *running_var;
    int64_t *num_batches;
    float *mean_out, *invstd_out;
    float *a_out;
    float *var_out;  // nullable: the biased batch variance [K] (deferred running-statistics updates)
};
// a BatchNorm1d (train) + ReLU backward folded into the backward pairs around it
// (fs_linear_f32_pair_bn; train_kernels.hip)
struct BnFold {
    const float *gu, *u, *y, *mean, *invstd, *gamma;
    float *part, *dgamma, *dbeta;
    const float *dx_add;  // (consumer) the residual gradient added to dy, nullable
    float *a_out;         // (consumer) dy written out by the input gradient's first column tile, nullable
    int B, H, tiles;
    int add_ch = 1, add_str = 0;  // (consumer) dx_add = the ordered sum of add_ch split-K partials add_str floats apart
};
}  // namespace fs
hipError_t fs_linear_f32_impl(const fs::GemmArgs &g, hipStream_t st);
hipError_t fs_linear_f32_pair_impl(const fs::GemmArgs &g0, const fs::GemmArgs &g1, hipStream_t st);
hipError_t fs_linear_f32_pair_bn_impl(const fs::GemmArgs &g0, const fs::GemmArgs &g1, const fs::BnFold *fin,
                                      const fs::BnFold *fout, hipStream_t st, int a_ch = 1, int64_t a_str = 0);
hipError_t fs_linear_f32_group_partial_impl(const fs::GemmArgs *gs, int n, float *ws, int64_t ws_floats, int max_ch,
                                            int *ch_out, hipStream_t st);
hipError_t fs_splitk_sum_impl(const float *part, int ch, int64_t stride, int64_t n, float *out, hipStream_t st);
hipError_t fs_linear_bn_f32_impl(const fs::GemmArgs &g, const fs::BnIn *bn, hipStream_t st);
bool fs_linear_ex2_ok(const fs::GemmArgs &g0, const fs::BnIn *b0, const fs::GemmArgs &g1, const fs::BnIn *b1);
hipError_t fs_linear_ex2_impl(const fs::GemmArgs &g0, const fs::BnIn *b0, const fs::GemmArgs &g1, const fs::BnIn *b1,
                              hipStream_t st);
hipError_t fs_bn_running_update_impl(int nbn, int H, float *rm, float *rv, int64_t *nbt, const float *stats,
                                     int passes, int64_t rows0, int64_t rows1, float momentum, const int32_t *skip,
                                     hipStream_t st);
int64_t fs_linear_f32_splitk_floats_impl(const fs::GemmArgs &g);
hipError_t fs_linear_f32_splitk_impl(const fs::GemmArgs &g, float *part, int64_t part_floats, hipStream_t st);
hipError_t fs_adam_step_impl(float *p, const float *g, float *m, float *v, int64_t n, float *step, const float *loss,
                             const int32_t *skip, double lr, double beta1, double beta2, double eps, double weight_decay, hipStream_t st);
hipError_t fs_kld_loss_impl(const float *log_q, int64_t B, const float *E, const float *lq_rev, int64_t R,
                            const int32_t *nan_word, float *loss, uint8_t *nan_out, hipStream_t st);
hipError_t fs_kld_loss_bwd_impl(const float *g, int64_t B, float *grad_log_q, hipStream_t st);
hipError_t fs_linear_f32_group_impl(const fs::GemmArgs *gs, int n, float *ws, int64_t ws_floats, hipStream_t st);
hipError_t fs_bn_relu_train_fwd_impl(int64_t B, int H, const float *x, const float *gamma, const float *beta,
                                     float *rm, float *rv, int64_t *nbt, float momentum, float eps, float *y,
                                     float *mean, float *invstd, hipStream_t st);
hipError_t fs_bn_relu_train_bwd_impl(int64_t B, int H, const float *x, const float *y, const float *dy,
                                     const float *gamma, const float *mean, const float *invstd, float *dx,
                                     const float *dx_add, float *dgamma, float *dbeta, hipStream_t st);
hipError_t fs_coupling_density_fwd_impl(const fs_coupling *cp, const float *x, const float *params, const float *uw,
                                        const float *uh, const float *ud, const float *lq_in, float *out, float *lq_out,
                                        hipStream_t st);
hipError_t fs_coupling_features_fwd_impl(const fs_coupling *cp, const float *x, float *t, hipStream_t st);
hipError_t fs_coupling_pair_pre_impl(const fs_coupling *sp, const float *z, const float *uw, const float *uh,
                                     const float *ud, float *t, float *out, float *lad_u, int32_t *nan_flag,
                                     const fs_coupling *dp, const float *x, float *td, hipStream_t st);
hipError_t fs_coupling_pair_step_impl(const fs_coupling *sp, const float *params, const float *lad_u,
                                      const float *lq_in, float *out, float *lq_out, int32_t *nan_flag,
                                      const fs_coupling *sp2, const float *uw2, const float *uh2, const float *ud2,
                                      float *t2, float *out2, float *lad_u2, const fs_coupling *dp, const float *x,
                                      const float *params_d, const float *uw, const float *uh, const float *ud,
                                      const float *lq_in_d, float *out_d, float *lq_out_d, const fs_coupling *dp2,
                                      float *t_d2, hipStream_t st);
hipError_t fs_coupling_bwd_step_impl(const fs_coupling *fp, const float *xf, const float *g_t, float *gxf,
                                     const float *gx_add, const fs_coupling *cp, const float *x, const float *params,
                                     const float *uw, const float *uh, const float *ud, const float *g_lq, float *gx,
                                     float *g_params, float *g_u, hipStream_t st);
hipError_t fs_coupling_pair_post_impl(const fs_coupling *sp, const float *params, const float *lad_u,
                                      const float *lq_in, float *out, float *lq_out, int32_t *nan_flag,
                                      const fs_coupling *dp, const float *x, const float *params_d, const float *uw,
                                      const float *uh, const float *ud, const float *lq_in_d, float *out_d,
                                      float *lq_out_d, hipStream_t st);
hipError_t fs_coupling_density_bwd_impl(const fs_coupling *cp, const float *x, const float *params, const float *uw,
                                        const float *uh, const float *ud, const float *g_out, const float *g_lq,
                                        float *gx, float *g_params, float *g_u, hipStream_t st);
hipError_t fs_coupling_sample_pre_impl(const fs_coupling *cp, const float *z, const float *uw, const float *uh,
                                       const float *ud, float *t, float *out, float *lad_u, int32_t *nan_flag,
                                       hipStream_t st);
hipError_t fs_coupling_sample_post_impl(const fs_coupling *cp, const float *params, const float *lad_u,
                                        const float *lq_in, float *out, float *lq_out, int32_t *nan_flag,
                                        hipStream_t st);
hipError_t fs_coupling_features_bwd_impl(const fs_coupling *cp, const float *x, const float *g_t, float *gx,
                                         const float *gx_add, hipStream_t st);
