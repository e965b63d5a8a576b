// extern "C" boundary of libflowstate (include/flowstate.h): argument checks,
// dispatch to the HIP launchers, thread-local error strings.  No exception
// crosses the ABI; no call synchronises the device.
#include <stdarg.h>

#include "fs_internal.h"
#include "flow_layout.h"

hipError_t fs_pcg64_seed_impl(const uint64_t *seeds, int64_t C, uint64_t *state, hipStream_t st);
hipError_t fs_pcg64_random_impl(uint64_t *state, int64_t C, double *out, hipStream_t st);
hipError_t fs_hist2d_impl(const double *pos, int64_t C, int N, double shift, const double *edges, int nb,
                          int64_t *hist, hipStream_t st);
hipError_t fs_well_stats_impl(const double *pos, const uint8_t *is_f32, int64_t C, int N, double half_box, double r0,
                              int64_t *counts, hipStream_t st);

static thread_local char g_err[512] = "";

void fs_set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

static int hip_rc(hipError_t e, const char *where) {
    if (e == hipSuccess) return FS_OK;
    fs_set_error("%s: %s", where, hipGetErrorString(e));
    return (int)e > 0 ? (int)e : 1;
}

#define REQUIRE(cond, ...)              \
    do {                                \
        if (!(cond)) {                  \
            fs_set_error(__VA_ARGS__);  \
            return FS_EINVAL;           \
        }                               \
    } while (0)

static int check_dims(const fs_flow_dims *d) {
    char why[256];
    REQUIRE(d != nullptr, "dims is NULL");
    if (!fs_flow_supported(d, why, sizeof(why))) {
        fs_set_error("%s", why);
        return FS_EUNSUPPORTED;
    }
    return FS_OK;
}

extern "C" {

const char *fs_last_error(void) { return g_err; }

int fs_version(void) { return 10000; }

int64_t fs_flow_raw_floats(const fs_flow_dims *d) {
    if (check_dims(d) != FS_OK) return -1;
    return fs_flow_raw_floats_impl(d);
}

int fs_gather_chunks(const int64_t *tab, int64_t n, float *dst, void *stream) {
    REQUIRE(n >= 0 && (n == 0 || (tab && dst)), "fs_gather_chunks: invalid arguments");
    return hip_rc(fs_gather_chunks_impl(tab, n, dst, (hipStream_t)stream), "fs_gather_chunks");
}

int64_t fs_flow_packed_bytes(const fs_flow_dims *d) {
    if (check_dims(d) != FS_OK) return -1;
    return fs_flow_packed_bytes_impl(d);
}

int fs_flow_pack(const fs_flow_dims *d, const float *raw, void *packed, void *stream) {
    int rc = check_dims(d);
    if (rc) return rc;
    REQUIRE(raw && packed, "fs_flow_pack: NULL buffer");
    REQUIRE(((uintptr_t)packed & 15) == 0, "fs_flow_pack: packed must be 16-byte aligned");
    return hip_rc(fs_flow_pack_impl(d, raw, (float *)packed, (hipStream_t)stream), "fs_flow_pack");
}

int fs_flow_log_prob(const fs_flow_dims *d, const void *packed, const float *x, int64_t B, float *log_q,
                     float *z_out, int32_t *err, void *stream) {
    int rc = check_dims(d);
    if (rc) return rc;
    REQUIRE(B == 0 || (packed && x && log_q && B > 0), "fs_flow_log_prob: invalid arguments");
    return hip_rc(fs_flow_pass_impl(d, packed, 0, x, B, z_out, log_q, 1, nullptr, nullptr, 0, 0, 0, 0.0, err,
                                    (hipStream_t)stream),
                  "fs_flow_log_prob");
}

int fs_flow_inverse(const fs_flow_dims *d, const void *packed, const float *x, int64_t B, float *z_out,
                    float *log_det, int32_t *err, void *stream) {
    int rc = check_dims(d);
    if (rc) return rc;
    REQUIRE(B == 0 || (packed && x && (z_out || log_det) && B > 0), "fs_flow_inverse: invalid arguments");
    return hip_rc(fs_flow_pass_impl(d, packed, 0, x, B, z_out, log_det, 0, nullptr, nullptr, 0, 0, 0, 0.0, err,
                                    (hipStream_t)stream),
                  "fs_flow_inverse");
}

int fs_flow_forward(const fs_flow_dims *d, const void *packed, const float *z, int64_t B, float *x_out,
                    float *log_det, int32_t *err, void *stream) {
    int rc = check_dims(d);
    if (rc) return rc;
    REQUIRE(B == 0 || (packed && z && (x_out || log_det) && B > 0), "fs_flow_forward: invalid arguments");
    return hip_rc(fs_flow_pass_impl(d, packed, 1, z, B, x_out, log_det, 0, nullptr, nullptr, 0, 0, 0, 0.0, err,
                                    (hipStream_t)stream),
                  "fs_flow_forward");
}

int fs_flow_propose(const fs_flow_dims *d, const void *packed, int64_t B, uint64_t seed, uint64_t counter,
                    int64_t row_offset, double half_width, float *config, float *centered, float *x_out,
                    int32_t *err, void *stream) {
    int rc = check_dims(d);
    if (rc) return rc;
    REQUIRE(B >= 0 && (B == 0 || (packed && (config || centered || x_out))), "fs_flow_propose: invalid arguments");
    return hip_rc(fs_flow_pass_impl(d, packed, 2, nullptr, B, x_out, nullptr, 0, config, centered, seed, counter,
                                    row_offset, half_width, err, (hipStream_t)stream),
                  "fs_flow_propose");
}

int fs_flow_propose_lq(const fs_flow_dims *d, const void *packed, int64_t B, uint64_t seed, uint64_t counter,
                       int64_t row_offset, double half_width, float *config, float *centered, float *x_out,
                       float *log_q, int32_t *err, void *stream) {
    int rc = check_dims(d);
    if (rc) return rc;
    REQUIRE(B >= 0 && (B == 0 || (packed && log_q)), "fs_flow_propose_lq: invalid arguments");
    return hip_rc(fs_flow_pass_impl(d, packed, 2, nullptr, B, x_out, log_q, 1, config, centered, seed, counter,
                                    row_offset, half_width, err, (hipStream_t)stream),
                  "fs_flow_propose_lq");
}

int fs_energy_lj_dw(const fs_phys *p, const void *pos, int pos_is_f32, int64_t C, int32_t N, double *E, double *W,
                    uint8_t *overlap, uint64_t *nbr, void *stream) {
    REQUIRE(p && C >= 0 && (C == 0 || (pos && E)), "fs_energy_lj_dw: invalid arguments");
    REQUIRE(N >= 1 && N <= fs::kMaxN, "fs_energy_lj_dw: N=%d outside [1, %d]", N, fs::kMaxN);
    REQUIRE(p->Lx > 0 && p->Ly > 0, "fs_energy_lj_dw: box must be positive");
    return hip_rc(fs_energy_impl(p, pos, pos_is_f32, C, N, E, W, overlap, nbr, (hipStream_t)stream),
                  "fs_energy_lj_dw");
}

int fs_energy_state(const fs_phys *p, const double *state, const uint8_t *state_is_f32, int64_t C, int32_t N,
                    double *E, double *W, void *stream) {
    REQUIRE(p && C >= 0 && (C == 0 || (state && state_is_f32 && E && W)), "fs_energy_state: invalid arguments");
    REQUIRE(N >= 1 && N <= fs::kMaxN, "fs_energy_state: N=%d outside [1, %d]", N, fs::kMaxN);
    REQUIRE(p->Lx > 0 && p->Ly > 0, "fs_energy_state: box must be positive");
    return hip_rc(fs_energy_impl(p, state, 0, C, N, E, W, nullptr, nullptr, (hipStream_t)stream, state_is_f32),
                  "fs_energy_state");
}

int fs_pcg64_seed(const uint64_t *seeds, int64_t C, uint64_t *state, void *stream) {
    REQUIRE(C >= 0 && (C == 0 || (seeds && state)), "fs_pcg64_seed: invalid arguments");
    return hip_rc(fs_pcg64_seed_impl(seeds, C, state, (hipStream_t)stream), "fs_pcg64_seed");
}

int fs_pcg64_random(uint64_t *state, int64_t C, double *out, void *stream) {
    REQUIRE(C >= 0 && (C == 0 || (state && out)), "fs_pcg64_random: invalid arguments");
    return hip_rc(fs_pcg64_random_impl(state, C, out, (hipStream_t)stream), "fs_pcg64_random");
}

int fs_mh_accept(const fs_phys *p, int64_t C, int32_t N, double *E_old, double *W_old, double *nll_old,
                 const double *E_new, const double *W_new, const float *log_q_new, uint64_t *pcg, double *state,
                 uint8_t *state_is_f32, const float *config, uint8_t *accept, int64_t *attempts, int64_t *accepted,
                 unsigned long long *n_accept, int flags, void *stream) {
    REQUIRE(p && C >= 0 && (C == 0 || (E_old && nll_old && E_new && log_q_new && pcg && accept)),
            "fs_mh_accept: invalid arguments");
    REQUIRE(N >= 1 && N <= fs::kMaxN, "fs_mh_accept: N=%d outside [1, %d]", N, fs::kMaxN);
    REQUIRE((state == nullptr) == (config == nullptr), "fs_mh_accept: state and config go together");
    return hip_rc(fs_mh_accept_impl(p, C, N, E_old, W_old, nll_old, E_new, W_new, log_q_new, pcg, state,
                                    state_is_f32, config, accept, attempts, accepted, n_accept, flags,
                                    (hipStream_t)stream),
                  "fs_mh_accept");
}

int fs_min_image(const fs_phys *p, const void *pos1, int64_t stride1, const void *pos2, int pos_is_f32, int64_t n,
                 double *delta, double *r, void *stream) {
    REQUIRE(p && n >= 0 && (n == 0 || (pos1 && pos2)) && (stride1 == 0 || stride1 == 1), "fs_min_image: invalid arguments");
    REQUIRE(p->Lx > 0 && p->Ly > 0, "fs_min_image: box lengths must be positive");
    return hip_rc(fs_min_image_impl(p, pos1, stride1, pos2, pos_is_f32, n, delta, r, (hipStream_t)stream),
                  "fs_min_image");
}

int fs_particle_energy(const fs_phys *p, const void *pos, int pos_is_f32, int64_t C, int32_t N,
                       const int32_t *particle, double *E, double *W, void *stream) {
    REQUIRE(p && C >= 0 && (C == 0 || (pos && particle && E && W)), "fs_particle_energy: invalid arguments");
    REQUIRE(N >= 2 && N <= fs::kMaxN, "fs_particle_energy: N=%d outside [2, %d]", N, fs::kMaxN);
    return hip_rc(fs_particle_energy_impl(p, pos, pos_is_f32, C, N, particle, E, W, (hipStream_t)stream),
                  "fs_particle_energy");
}

int fs_metropolis_judge(double beta, int64_t C, int64_t M, const double *E_ref, const double *E_new, uint64_t *pcg,
                        uint8_t *accept, int64_t *n_accept, void *stream) {
    REQUIRE(C >= 0 && M >= 0 && (C == 0 || (E_ref && pcg && (M == 0 || E_new))), "fs_metropolis_judge: invalid arguments");
    REQUIRE(beta == beta, "fs_metropolis_judge: beta is NaN");
    return hip_rc(fs_metropolis_judge_impl(beta, C, M, E_ref, E_new, pcg, accept, n_accept, (hipStream_t)stream),
                  "fs_metropolis_judge");
}

int64_t fs_nf_mh_step_ws_bytes(const fs_flow_dims *d, int64_t C) {
    if (check_dims(d) != FS_OK || C < 0) return -1;
    const int64_t D = 2 * d->N;
    // config f32 [C][D] | centered f32 [C][D] + centered_old f32 [C][D] | log_q f32 [C] +
    // log_q_old f32 [C] | E_new f64 [C] | W_new f64 [C] | E_cur f64 [C] | W_cur f64 [C]
    return fs::rup(C * D * 4, 256) + fs::rup(2 * C * D * 4, 256) + fs::rup(2 * C * 4, 256) + fs::rup(C * 8, 256) * 4;
}

int fs_nf_mh_step(const fs_flow_dims *d, const void *packed, const fs_phys *p, int64_t C, uint64_t seed,
                  uint64_t step, int64_t chain_offset, double *E_old, double *W_old, double *nll_old, uint64_t *pcg, double *state,
                  uint8_t *state_is_f32, uint8_t *accept, int64_t *attempts, int64_t *accepted,
                  unsigned long long *n_accept, int32_t *err, int flags, void *ws, void *stream) {
    int rc = check_dims(d);
    if (rc) return rc;
    REQUIRE(p && C >= 0 && (C == 0 || (packed && E_old && nll_old && pcg && accept && ws)), "fs_nf_mh_step: invalid arguments");
    REQUIRE(((uintptr_t)ws & 255) == 0, "fs_nf_mh_step: workspace must be 256-byte aligned");
    if (C == 0) return FS_OK;
    const int64_t D = 2 * d->N;
    char *w = (char *)ws;
    float *config = (float *)w;
    w += fs::rup(C * D * 4, 256);
    float *centered = (float *)w;  // [C][D], then centered_old [C][D] right behind it
    float *centered_old = centered + C * D;
    w += fs::rup(2 * C * D * 4, 256);
    float *log_q = (float *)w;  // [C], then log_q_old [C]
    float *log_q_old = log_q + C;
    w += fs::rup(2 * C * 4, 256);
    double *E_new = (double *)w;
    w += fs::rup(C * 8, 256);
    double *W_new = (double *)w;
    w += fs::rup(C * 8, 256);
    double *E_cur = (double *)w;
    w += fs::rup(C * 8, 256);
    double *W_cur = (double *)w;
    hipStream_t st = (hipStream_t)stream;
    const double half_width = p->Lx / 2.0;  // MonteCarlo.half_width (monte_carlo.py:66)
    const bool hybrid = (flags & FS_MH_HYBRID) != 0;
    const bool single = (flags & FS_MH_SINGLE_PASS) != 0;
    REQUIRE(!hybrid || state, "fs_nf_mh_step: FS_MH_HYBRID needs the state");
    hipError_t e = fs_flow_pass_impl(d, packed, 2, nullptr, C, nullptr, single ? log_q : nullptr, single ? 1 : 0,
                                     config, centered, seed, step, chain_offset, half_width, err, st);
    if (e != hipSuccess) return hip_rc(e, "fs_nf_mh_step/propose");
    if (hybrid) {  // the state moved since nll_old / E_old were exact: re-derive both
        e = fs_center_impl(state, C * D, half_width, centered_old, st);
        if (e != hipSuccess) return hip_rc(e, "fs_nf_mh_step/center");
    }
    // log q of the proposals and (hybrid) of the current states: one density launch over
    // C or 2C rows (the rows are independent, so a small C gets twice the workgroups);
    // with FS_MH_SINGLE_PASS the proposals' log q came from the propose launch
    if (!single)
        e = fs_flow_pass_impl(d, packed, 0, centered, hybrid ? 2 * C : C, nullptr, log_q, 1, nullptr, nullptr, 0, 0,
                              0, 0.0, err, st);
    else if (hybrid)
        e = fs_flow_pass_impl(d, packed, 0, centered_old, C, nullptr, log_q_old, 1, nullptr, nullptr, 0, 0, 0, 0.0,
                              err, st);
    if (e != hipSuccess) return hip_rc(e, "fs_nf_mh_step/log_prob");
    e = fs_energy_impl(p, config, 1, C, d->N, E_new, W_new, nullptr, nullptr, st);
    if (e != hipSuccess) return hip_rc(e, "fs_nf_mh_step/energy");
    if (hybrid) {
        e = fs_energy_impl(p, state, 0, C, d->N, E_cur, W_cur, nullptr, nullptr, st, state_is_f32);
        if (e != hipSuccess) return hip_rc(e, "fs_nf_mh_step/energy_old");
    }
    e = fs_mh_accept_impl(p, C, d->N, E_old, W_old, nll_old, E_new, W_new, log_q, pcg, state, state_is_f32,
                          state ? config : nullptr, accept, attempts, accepted, n_accept, flags, st,
                          hybrid ? log_q_old : nullptr, hybrid ? E_cur : nullptr, hybrid ? W_cur : nullptr);
    return hip_rc(e, "fs_nf_mh_step/accept");
}

int64_t fs_nf_mh_steps_ws_bytes(const fs_flow_dims *d, int64_t C, int64_t S) {
    if (check_dims(d) != FS_OK || C < 0 || S < 1) return -1;
    const int64_t D = 2 * d->N, R = C * S;
    // config f32 [S C][D] | centered f32 [S C][D] | log_q f32 [S C] | E_new f64 [S C] | W_new f64 [S C]
    return fs::rup(R * D * 4, 256) * 2 + fs::rup(R * 4, 256) + fs::rup(R * 8, 256) * 2;
}

namespace {
// sections of an S-step proposal bank (the fs_nf_mh_steps workspace): rows s*C + c hold
// step step0+s of chain c
struct Bank {
    float *config, *centered, *log_q;
    double *E_new, *W_new;
};
Bank bank_sections(void *ws, int64_t R, int64_t D) {
    char *w = (char *)ws;
    Bank b;
    b.config = (float *)w;
    w += fs::rup(R * D * 4, 256);
    b.centered = (float *)w;
    w += fs::rup(R * D * 4, 256);
    b.log_q = (float *)w;
    w += fs::rup(R * 4, 256);
    b.E_new = (double *)w;
    w += fs::rup(R * 8, 256);
    b.W_new = (double *)w;
    return b;
}

// the proposals of steps step0 .. step0+S-1 do not depend on the chain states: one launch
// of S*C rows per pass (the same Philox draws as S single steps), then their energies
int fill_bank(const fs_flow_dims *d, const void *packed, const fs_phys *p, int64_t C, int64_t S, uint64_t seed,
              uint64_t step0, int64_t chain_offset, int32_t *err, const Bank &b, hipStream_t st, const char *who) {
    const int64_t R = C * S;
    const double half_width = p->Lx / 2.0;  // MonteCarlo.half_width (monte_carlo.py:66)
    hipError_t e = fs_flow_pass_impl(d, packed, 2, nullptr, R, nullptr, nullptr, 0, b.config, b.centered, seed,
                                     step0, chain_offset, half_width, err, st, C);
    if (e != hipSuccess) return hip_rc(e, who);
    e = fs_flow_pass_impl(d, packed, 0, b.centered, R, nullptr, b.log_q, 1, nullptr, nullptr, 0, 0, 0, 0.0, err, st);
    if (e != hipSuccess) return hip_rc(e, who);
    e = fs_energy_impl(p, b.config, 1, R, d->N, b.E_new, b.W_new, nullptr, nullptr, st);
    return hip_rc(e, who);
}
}  // namespace

int fs_nf_mh_steps(const fs_flow_dims *d, const void *packed, const fs_phys *p, int64_t C, int64_t S, uint64_t seed,
                   uint64_t step0, int64_t chain_offset, double *E_old, double *W_old, double *nll_old, uint64_t *pcg,
                   double *state, uint8_t *state_is_f32, uint8_t *accept, int64_t *attempts, int64_t *accepted,
                   unsigned long long *n_accept, int32_t *err, int flags, void *ws, void *stream) {
    int rc = check_dims(d);
    if (rc) return rc;
    REQUIRE(p && C >= 0 && S >= 1 && (C == 0 || (packed && E_old && nll_old && pcg && accept && ws)),
            "fs_nf_mh_steps: invalid arguments");
    REQUIRE(!(flags & FS_MH_HYBRID), "fs_nf_mh_steps: FS_MH_HYBRID needs one step at a time (fs_nf_mh_step)");
    REQUIRE(!(flags & FS_MH_SINGLE_PASS), "fs_nf_mh_steps: FS_MH_SINGLE_PASS is a flag of fs_nf_mh_step");
    REQUIRE(((uintptr_t)ws & 255) == 0, "fs_nf_mh_steps: workspace must be 256-byte aligned");
    if (C == 0) return FS_OK;
    const int64_t D = 2 * d->N;
    const Bank b = bank_sections(ws, C * S, D);
    hipStream_t st = (hipStream_t)stream;
    rc = fill_bank(d, packed, p, C, S, seed, step0, chain_offset, err, b, st, "fs_nf_mh_steps/bank");
    if (rc) return rc;
    for (int64_t s = 0; s < S; ++s) {
        hipError_t e = fs_mh_accept_impl(p, C, d->N, E_old, W_old, nll_old, b.E_new + s * C, b.W_new + s * C,
                                         b.log_q + s * C, pcg, state, state_is_f32,
                                         state ? b.config + s * C * D : nullptr, accept, attempts, accepted, n_accept,
                                         flags, st);
        if (e != hipSuccess) return hip_rc(e, "fs_nf_mh_steps/accept");
    }
    return FS_OK;
}

int fs_nf_mh_bank(const fs_flow_dims *d, const void *packed, const fs_phys *p, int64_t C, int64_t S, uint64_t seed,
                  uint64_t step0, int64_t chain_offset, int32_t *err, void *bank, void *stream) {
    int rc = check_dims(d);
    if (rc) return rc;
    REQUIRE(p && C >= 0 && S >= 1 && (C == 0 || (packed && bank)), "fs_nf_mh_bank: invalid arguments");
    REQUIRE(((uintptr_t)bank & 255) == 0, "fs_nf_mh_bank: bank must be 256-byte aligned");
    if (C == 0) return FS_OK;
    return fill_bank(d, packed, p, C, S, seed, step0, chain_offset, err, bank_sections(bank, C * S, 2 * d->N),
                     (hipStream_t)stream, "fs_nf_mh_bank");
}

int64_t fs_nf_mh_banked_ws_bytes(const fs_flow_dims *d, int64_t C) {
    if (check_dims(d) != FS_OK || C < 0) return -1;
    // centered_old f32 [C][D] | log_q_old f32 [C] | E_cur f64 [C] | W_cur f64 [C]
    return fs::rup(C * 2 * d->N * 4, 256) + fs::rup(C * 4, 256) + fs::rup(C * 8, 256) * 2;
}

int fs_nf_mh_step_banked(const fs_flow_dims *d, const void *packed, const fs_phys *p, int64_t C, int64_t S, int64_t s,
                         const void *bank, double *E_old, double *W_old, double *nll_old, uint64_t *pcg, double *state,
                         uint8_t *state_is_f32, uint8_t *accept, int64_t *attempts, int64_t *accepted,
                         unsigned long long *n_accept, int32_t *err, int flags, void *hws, void *stream) {
    int rc = check_dims(d);
    if (rc) return rc;
    const bool hybrid = (flags & FS_MH_HYBRID) != 0;
    REQUIRE(p && C >= 0 && S >= 1 && s >= 0 && s < S &&
                (C == 0 || (packed && bank && E_old && nll_old && pcg && accept && (!hybrid || (state && hws)))),
            "fs_nf_mh_step_banked: invalid arguments");
    REQUIRE(((uintptr_t)bank & 255) == 0 && ((uintptr_t)hws & 255) == 0,
            "fs_nf_mh_step_banked: bank and workspace must be 256-byte aligned");
    if (C == 0) return FS_OK;
    const int64_t D = 2 * d->N;
    const Bank b = bank_sections(const_cast<void *>(bank), C * S, D);
    hipStream_t st = (hipStream_t)stream;
    float *centered_old = nullptr, *log_q_old = nullptr;
    double *E_cur = nullptr, *W_cur = nullptr;
    if (hybrid) {  // monte_carlo.py:251-261 (old NLL of the moved state) and :299-301 (its energy)
        char *w = (char *)hws;
        centered_old = (float *)w;
        w += fs::rup(C * D * 4, 256);
        log_q_old = (float *)w;
        w += fs::rup(C * 4, 256);
        E_cur = (double *)w;
        w += fs::rup(C * 8, 256);
        W_cur = (double *)w;
        hipError_t e = fs_center_impl(state, C * D, p->Lx / 2.0, centered_old, st);
        if (e != hipSuccess) return hip_rc(e, "fs_nf_mh_step_banked/center");
        e = fs_flow_pass_impl(d, packed, 0, centered_old, C, nullptr, log_q_old, 1, nullptr, nullptr, 0, 0, 0, 0.0,
                              err, st);
        if (e != hipSuccess) return hip_rc(e, "fs_nf_mh_step_banked/log_prob_old");
        e = fs_energy_impl(p, state, 0, C, d->N, E_cur, W_cur, nullptr, nullptr, st, state_is_f32);
        if (e != hipSuccess) return hip_rc(e, "fs_nf_mh_step_banked/energy_old");
    }
    hipError_t e = fs_mh_accept_impl(p, C, d->N, E_old, W_old, nll_old, b.E_new + s * C, b.W_new + s * C,
                                     b.log_q + s * C, pcg, state, state_is_f32, state ? b.config + s * C * D : nullptr,
                                     accept, attempts, accepted, n_accept, flags, st, log_q_old, E_cur, W_cur);
    return hip_rc(e, "fs_nf_mh_step_banked/accept");
}

int fs_local_moves(const fs_phys *p, int64_t C, int32_t N, double *state, const uint8_t *state_is_f32, double *E,
                   double *W, uint64_t *pcg, uint64_t *pcg_buf, double *max_disp, int64_t *attempts,
                   int64_t *accepted, int64_t *prev_counts, int64_t n_moves, int64_t step0, int32_t adjust_every,
                   double target_acceptance, int32_t sample_every, double *samples_xy, double *samples_ew,
                   uint8_t *accept_log, unsigned long long *n_accept, void *stream) {
    REQUIRE(p && C >= 0 && n_moves >= 0 && step0 >= 0 &&
                (C == 0 || (state && E && pcg && pcg_buf && max_disp && attempts && accepted)),
            "fs_local_moves: invalid arguments");
    REQUIRE(N >= 1 && N <= fs::kMaxN, "fs_local_moves: N=%d outside [1, %d]", N, fs::kMaxN);
    REQUIRE(adjust_every <= 0 || (prev_counts && target_acceptance > 0.0),
            "fs_local_moves: adjust_every needs prev_counts and target_acceptance > 0");
    REQUIRE(fs_local_samples_per_chain(step0, n_moves, sample_every) == 0 || samples_xy || samples_ew,
            "fs_local_moves: sample_every needs a sample buffer");
    return hip_rc(fs_local_moves_impl(p, C, N, state, state_is_f32, E, W, pcg, pcg_buf, max_disp, attempts, accepted,
                                      prev_counts, n_moves, step0, adjust_every, target_acceptance, sample_every,
                                      samples_xy, samples_ew, accept_log, n_accept, (hipStream_t)stream),
                  "fs_local_moves");
}

int fs_local_moves_if(const uint8_t *gate, const fs_phys *p, int64_t C, int32_t N, double *state,
                      const uint8_t *state_is_f32, double *E, double *W, uint64_t *pcg, uint64_t *pcg_buf,
                      double *max_disp, int64_t *attempts, int64_t *accepted, int64_t *prev_counts,
                      int64_t n_moves, int64_t step0, int32_t adjust_every, double target_acceptance,
                      int32_t sample_every, double *samples_xy, double *samples_ew, uint8_t *accept_log,
                      unsigned long long *n_accept, void *stream) {
    REQUIRE(gate, "fs_local_moves_if: gate is required");
    REQUIRE(p && C >= 0 && n_moves >= 0 && step0 >= 0 &&
                (C == 0 || (state && E && pcg && pcg_buf && max_disp && attempts && accepted)),
            "fs_local_moves_if: invalid arguments");
    REQUIRE(N >= 1 && N <= fs::kMaxN, "fs_local_moves_if: N=%d outside [1, %d]", N, fs::kMaxN);
    REQUIRE(adjust_every <= 0 || (prev_counts && target_acceptance > 0.0),
            "fs_local_moves_if: adjust_every needs prev_counts and target_acceptance > 0");
    REQUIRE(fs_local_samples_per_chain(step0, n_moves, sample_every) == 0 || samples_xy || samples_ew,
            "fs_local_moves_if: sample_every needs a sample buffer");
    return hip_rc(fs_local_moves_impl(p, C, N, state, state_is_f32, E, W, pcg, pcg_buf, max_disp, attempts, accepted,
                                      prev_counts, n_moves, step0, adjust_every, target_acceptance, sample_every,
                                      samples_xy, samples_ew, accept_log, n_accept, (hipStream_t)stream, gate),
                  "fs_local_moves_if");
}

int fs_chains_copy_if(const uint8_t *gate, int64_t C, int32_t N, const fs_local_chains *src,
                      const fs_local_chains *dst, void *stream) {
    REQUIRE(gate && src && dst && C >= 0, "fs_chains_copy_if: invalid arguments");
    REQUIRE(N >= 1 && N <= fs::kMaxN, "fs_chains_copy_if: N=%d outside [1, %d]", N, fs::kMaxN);
    REQUIRE(C == 0 || (src->state && dst->state && src->E && dst->E && src->pcg && dst->pcg && src->pcg_buf &&
                       dst->pcg_buf && src->max_disp && dst->max_disp && src->attempts && dst->attempts &&
                       src->accepted && dst->accepted),
            "fs_chains_copy_if: missing arrays");
    REQUIRE(!src->state_is_f32 == !dst->state_is_f32 && !src->W == !dst->W &&
                !src->prev_counts == !dst->prev_counts,
            "fs_chains_copy_if: src and dst must have the same optional arrays");
    return hip_rc(fs_chains_copy_if_impl(gate, C, N, src, dst, (hipStream_t)stream), "fs_chains_copy_if");
}

int fs_adjust_displacement(int64_t C, double *max_disp, const int64_t *attempts, const int64_t *accepted,
                           int64_t *prev_counts, double target_acceptance, void *stream) {
    REQUIRE(C >= 0 && target_acceptance > 0.0 && (C == 0 || (max_disp && attempts && accepted && prev_counts)),
            "fs_adjust_displacement: invalid arguments");
    return hip_rc(fs_adjust_displacement_impl(C, max_disp, attempts, accepted, prev_counts, target_acceptance,
                                              (hipStream_t)stream),
                  "fs_adjust_displacement");
}

int fs_hist2d(const double *pos, int64_t C, int32_t N, double shift, const double *edges, int32_t nbins,
              int64_t *hist, void *stream) {
    REQUIRE(edges && hist && C >= 0 && N >= 1 && nbins >= 1 && (C == 0 || pos), "fs_hist2d: invalid arguments");
    return hip_rc(fs_hist2d_impl(pos, C, N, shift, edges, nbins, hist, (hipStream_t)stream), "fs_hist2d");
}

int fs_well_stats(const double *pos, const uint8_t *state_is_f32, int64_t C, int32_t N, double half_box, double r0,
                  int64_t *counts, void *stream) {
    REQUIRE(C >= 0 && N >= 1 && half_box > 0 && (C == 0 || (pos && counts)), "fs_well_stats: invalid arguments");
    return hip_rc(fs_well_stats_impl(pos, state_is_f32, C, N, half_box, r0, counts, (hipStream_t)stream),
                  "fs_well_stats");
}

int fs_rqs_forward(int64_t M, int32_t K, int32_t inverse, const float *x, const float *uw, const float *uh,
                   const float *ud, double tail_bound, float *out, float *lad, int32_t *nan_flag, void *stream) {
    REQUIRE(M >= 0 && tail_bound > 0 && (M == 0 || (x && uw && uh && ud && out && lad)), "fs_rqs_forward: invalid arguments");
    REQUIRE(K == 5 || K == 8 || K == 15 || K == 32, "fs_rqs_forward: K=%d not instantiated (5, 8, 15, 32)", K);
    return hip_rc(fs_rqs_forward_impl(M, K, inverse, x, uw, uh, ud, (float)tail_bound, out, lad, nan_flag,
                                      (hipStream_t)stream),
                  "fs_rqs_forward");
}

int fs_rqs_backward(int64_t M, int32_t K, int32_t inverse, const float *x, const float *uw, const float *uh,
                    const float *ud, double tail_bound, const float *g_out, const float *g_lad, float *gx,
                    float *guw, float *guh, float *gud, void *stream) {
    REQUIRE(M >= 0 && tail_bound > 0 && (M == 0 || (x && uw && uh && ud && gx && guw && guh && gud)),
            "fs_rqs_backward: invalid arguments");
    REQUIRE(K == 5 || K == 8 || K == 15 || K == 32, "fs_rqs_backward: K=%d not instantiated (5, 8, 15, 32)", K);
    return hip_rc(fs_rqs_backward_impl(M, K, inverse, x, uw, uh, ud, (float)tail_bound, g_out, g_lad, gx, guw, guh,
                                       gud, (hipStream_t)stream),
                  "fs_rqs_backward");
}

int64_t fs_set_wide_rows(int64_t rows) { return fs_set_wide_rows_impl(rows); }
int32_t fs_set_wide_trunk16(int32_t on) { return fs_set_wide_trunk16_impl(on); }
int32_t fs_set_wide_final32(int32_t on) { return fs_set_wide_final32_impl(on); }
int64_t fs_set_wide_handoff_spins(int64_t spins) { return fs_set_wide_handoff_spins_impl(spins); }
int32_t fs_set_coupling_waves(int32_t on) { return fs_set_coupling_waves_impl(on); }
int32_t fs_set_lean_gemm(int32_t on) { return fs_set_lean_gemm_impl(on); }

int fs_adam_step(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n, float *step,
                 const float *loss, const int32_t *skip, double lr, double beta1, double beta2, double eps,
                 double weight_decay, void *stream) {
    REQUIRE(n >= 0 && step && (n == 0 || (param && grad && exp_avg && exp_avg_sq)) && lr > 0.0 && beta1 >= 0.0 &&
                beta1 < 1.0 && beta2 >= 0.0 && beta2 < 1.0 && eps >= 0.0 && weight_decay >= 0.0,
            "fs_adam_step: invalid arguments");
    REQUIRE((((uintptr_t)param | (uintptr_t)grad | (uintptr_t)exp_avg | (uintptr_t)exp_avg_sq) & 15) == 0,
            "fs_adam_step: buffers must be 16-byte aligned");
    return hip_rc(fs_adam_step_impl(param, grad, exp_avg, exp_avg_sq, n, step, loss, skip, lr, beta1, beta2, eps,
                                    weight_decay, (hipStream_t)stream),
                  "fs_adam_step");
}

int fs_kld_loss(const float *log_q, int64_t B, const float *energy, const float *lq_rev, int64_t R,
                const int32_t *nan_word, float *loss, uint8_t *nan_out, void *stream) {
    REQUIRE(B >= 1 && log_q && loss && (!energy || (R >= 1 && lq_rev)), "fs_kld_loss: invalid arguments");
    return hip_rc(fs_kld_loss_impl(log_q, B, energy, lq_rev, R, nan_word, loss, nan_out, (hipStream_t)stream),
                  "fs_kld_loss");
}

int fs_kld_loss_backward(const float *grad_loss, int64_t B, float *grad_log_q, void *stream) {
    REQUIRE(B >= 1 && grad_loss && grad_log_q, "fs_kld_loss_backward: invalid arguments");
    return hip_rc(fs_kld_loss_bwd_impl(grad_loss, B, grad_log_q, (hipStream_t)stream), "fs_kld_loss_backward");
}

int fs_target_energy(const float *x, int64_t B, int32_t N, double bound, double temperature, int32_t num_wells,
                     double V0_0, double V0_1, double r0, double k, float *E, float *grad_x, void *stream) {
    REQUIRE(B >= 0 && N >= 1 && N <= 1024 && bound > 0.0 && temperature > 0.0 && num_wells >= 0 && num_wells <= 2 &&
                (B == 0 || (x && E)),
            "fs_target_energy: invalid arguments");
    return hip_rc(fs_target_energy_impl(x, B, N, bound, temperature, num_wells, V0_0, V0_1, r0, k, E, grad_x,
                                        (hipStream_t)stream),
                  "fs_target_energy");
}

int fs_classify_wells(const void *pos, int pos_is_f32, int64_t M, int32_t N, double half_box, double r0,
                      uint8_t *cls, uint8_t *state, double *avg_x, void *stream) {
    REQUIRE(M >= 0 && N >= 1 && half_box > 0.0 && (M == 0 || pos), "fs_classify_wells: invalid arguments");
    return hip_rc(fs_classify_wells_impl(pos, pos_is_f32, M, N, half_box, r0, cls, state, avg_x, (hipStream_t)stream),
                  "fs_classify_wells");
}

int fs_pair_hist(const void *pos, int pos_is_f32, int64_t M, int32_t N, double bound, const double *edges,
                 int32_t nbins, int32_t *counts, void *stream) {
    REQUIRE(edges && M >= 0 && N >= 1 && bound > 0.0 && (M == 0 || (pos && counts)), "fs_pair_hist: invalid arguments");
    REQUIRE(N <= 256 && nbins >= 1 && nbins <= 128, "fs_pair_hist: N <= 256 and 1 <= nbins <= 128 (got %d, %d)", N,
            nbins);
    return hip_rc(fs_pair_hist_impl(pos, pos_is_f32, M, N, bound, edges, nbins, counts, (hipStream_t)stream),
                  "fs_pair_hist");
}

int fs_rdf_mean(const int32_t *counts, int64_t M, int32_t nbins, const double *denom, double *g_r, void *stream) {
    REQUIRE(counts && denom && g_r && M >= 1 && nbins >= 1, "fs_rdf_mean: invalid arguments");
    return hip_rc(fs_rdf_mean_impl(counts, M, nbins, denom, g_r, (hipStream_t)stream), "fs_rdf_mean");
}

}  // extern "C"

int fs_linear_f32(int64_t M, int64_t N, int64_t K, const float *A, int64_t sam, int64_t sak, const float *B,
                  int64_t sbk, int64_t sbn, const float *bias, const float *R, int64_t ldr, float *C, int64_t ldc,
                  float *rowsum_a, void *stream) {
    REQUIRE(M >= 0 && N >= 0 && K >= 0 && (M == 0 || N == 0 || (C && (K == 0 || (A && B)))) && ldc >= N && (!R || ldr >= N),
            "fs_linear_f32: invalid arguments");
    REQUIRE(M <= 32LL * 65535 && N <= 32LL * 65535, "fs_linear_f32: M, N at most %lld", 32LL * 65535);
    fs::GemmArgs g{M, N, K, A, sam, sak, B, sbk, sbn, bias, R, ldr, C, ldc, rowsum_a};
    return hip_rc(fs_linear_f32_impl(g, (hipStream_t)stream), "fs_linear_f32");
}

int fs_linear_f32_pair(const fs_gemm_f32 *g0, const fs_gemm_f32 *g1, void *stream) {
    REQUIRE(g0 && g1, "fs_linear_f32_pair: NULL descriptor");
    fs::GemmArgs a[2];
    const fs_gemm_f32 *gs[2] = {g0, g1};
    for (int i = 0; i < 2; ++i) {
        const fs_gemm_f32 &g = *gs[i];
        REQUIRE(g.M >= 0 && g.N >= 0 && g.K >= 0 && (g.M == 0 || g.N == 0 || (g.C && (g.K == 0 || (g.A && g.B)))) &&
                    g.ldc >= g.N && (!g.R || g.ldr >= g.N),
                "fs_linear_f32_pair: invalid arguments (product %d)", i);
        REQUIRE(g.M <= 32LL * 65535 && g.N <= 32LL * 65535, "fs_linear_f32_pair: M, N at most %lld", 32LL * 65535);
        a[i] = fs::GemmArgs{g.M, g.N, g.K, g.A, g.sam, g.sak, g.B, g.sbk, g.sbn, g.bias, g.R, g.ldr, g.C, g.ldc,
                            g.rowsum_a};
    }
    return hip_rc(fs_linear_f32_pair_impl(a[0], a[1], (hipStream_t)stream), "fs_linear_f32_pair");
}

int fs_linear_f32_pair_bn(const fs_gemm_f32 *g0, const fs_gemm_f32 *g1, const fs_bn_fold *fin,
                          const fs_bn_fold *fout, void *stream) {
    return fs_linear_f32_pair_bn_sk(g0, g1, fin, fout, 1, 0, 1, 0, stream);
}

int fs_linear_f32_pair_bn_sk(const fs_gemm_f32 *g0, const fs_gemm_f32 *g1, const fs_bn_fold *fin,
                             const fs_bn_fold *fout, int32_t a_chunks, int64_t a_stride, int32_t add_chunks,
                             int64_t add_stride, void *stream) {
    REQUIRE(g0 && g1 && (fin || fout), "fs_linear_f32_pair_bn: NULL descriptor");
    REQUIRE(a_chunks >= 1 && a_chunks <= 3 && add_chunks >= 1 && add_chunks <= 3 && (add_chunks == 1 || fin) &&
                (a_chunks == 1 || a_stride > 0) && (add_chunks == 1 || add_stride > 0),
            "fs_linear_f32_pair_bn: invalid split-K operands (a_chunks=%d, add_chunks=%d)", a_chunks, add_chunks);
    const fs_bn_fold *fs_[2] = {fin, fout};
    fs::BnFold bf[2];
    for (int i = 0; i < 2; ++i) {
        const fs_bn_fold *f = fs_[i];
        if (!f) continue;
        REQUIRE(f->B >= 2 && f->B <= 32LL * 65535 && f->H >= 1 && f->H <= 256 && f->gu && f->u && f->y && f->mean &&
                    f->invstd && f->part && (i == 1 || f->gamma),
                "fs_linear_f32_pair_bn: invalid %s fold (B=%lld, H=%d)", i ? "output" : "input", (long long)f->B, f->H);
        bf[i] = fs::BnFold{f->gu, f->u, f->y, f->mean, f->invstd, f->gamma, f->part, f->dgamma, f->dbeta,
                           f->dx_add, f->a_out, (int)f->B, (int)f->H, (int)((f->B + 31) / 32)};
    }
    if (fin && add_chunks > 1) {
        REQUIRE(fin->dx_add && add_stride < INT32_MAX, "fs_linear_f32_pair_bn: add_chunks needs dx_add");
        bf[0].add_ch = add_chunks;
        bf[0].add_str = (int)add_stride;
    }
    fs::GemmArgs a[2];
    const fs_gemm_f32 *gs[2] = {g0, g1};
    for (int i = 0; i < 2; ++i) {
        const fs_gemm_f32 &g = *gs[i];
        REQUIRE(g.M > 0 && g.N > 0 && g.K > 0 && g.A && g.B && g.C && g.ldc >= g.N && !g.R,
                "fs_linear_f32_pair_bn: invalid arguments (product %d)", i);
        a[i] = fs::GemmArgs{g.M, g.N, g.K, g.A, g.sam, g.sak, g.B, g.sbk, g.sbn, g.bias, g.R, g.ldr, g.C, g.ldc,
                            g.rowsum_a};
    }
    return hip_rc(fs_linear_f32_pair_bn_impl(a[0], a[1], fin ? &bf[0] : nullptr, fout ? &bf[1] : nullptr,
                                             (hipStream_t)stream, a_chunks, a_stride),
                  "fs_linear_f32_pair_bn");
}

static bool bn_in_ok(const fs_gemm_f32 &g, const fs_bn_in *bn) {
    return bn->stats && bn->gamma && bn->beta && bn->rows >= 2 && bn->tiles == (bn->rows + 31) / 32 &&
           bn->rows == g.M && g.K <= 256 && bn->eps > 0.f && (!bn->running_mean) == (!bn->running_var);
}

static fs::BnIn bn_in_args(const fs_bn_in *bn) {
    return fs::BnIn{bn->stats,        bn->tiles,      bn->rows,         bn->gamma,     bn->beta,
                    bn->eps,          bn->momentum,   bn->running_mean, bn->running_var, bn->num_batches,
                    bn->mean_out,     bn->invstd_out, bn->a_out,        bn->var_out};
}

int fs_linear_f32_ex(const fs_gemm_f32 *d, const fs_bn_in *bn, float *stats_out, void *stream) {
    REQUIRE(d, "fs_linear_f32_ex: NULL descriptor");
    const fs_gemm_f32 &g = *d;
    REQUIRE(g.M >= 0 && g.N >= 0 && g.K >= 0 && (g.M == 0 || g.N == 0 || (g.C && (g.K == 0 || (g.A && g.B)))) &&
                g.ldc >= g.N && (!g.R || g.ldr >= g.N),
            "fs_linear_f32_ex: invalid arguments");
    REQUIRE(g.M <= 32LL * 65535 && g.N <= 32LL * 65535, "fs_linear_f32_ex: M, N at most %lld", 32LL * 65535);
    fs::GemmArgs a{g.M, g.N, g.K, g.A, g.sam, g.sak, g.B, g.sbk, g.sbn, g.bias, g.R, g.ldr, g.C, g.ldc, g.rowsum_a};
    a.stats = stats_out;
    if (!bn) return hip_rc(fs_linear_f32_impl(a, (hipStream_t)stream), "fs_linear_f32_ex");
    REQUIRE(bn_in_ok(g, bn), "fs_linear_f32_ex: invalid BatchNorm arguments");
    const fs::BnIn b = bn_in_args(bn);
    return hip_rc(fs_linear_bn_f32_impl(a, &b, (hipStream_t)stream), "fs_linear_f32_ex");
}

int fs_linear_f32_ex2(const fs_gemm_f32 *d0, const fs_bn_in *bn0, float *stats0, const fs_gemm_f32 *d1,
                      const fs_bn_in *bn1, float *stats1, void *stream) {
    REQUIRE(d0 && d1, "fs_linear_f32_ex2: NULL descriptor");
    const fs_gemm_f32 *d[2] = {d0, d1};
    const fs_bn_in *bn[2] = {bn0, bn1};
    float *so[2] = {stats0, stats1};
    fs::GemmArgs a[2];
    fs::BnIn b[2];
    for (int i = 0; i < 2; ++i) {
        const fs_gemm_f32 &g = *d[i];
        REQUIRE(g.M >= 0 && g.N >= 0 && g.K >= 0 && (g.M == 0 || g.N == 0 || (g.C && (g.K == 0 || (g.A && g.B)))) &&
                    g.ldc >= g.N && (!g.R || g.ldr >= g.N) && g.M <= 32LL * 65535 && g.N <= 32LL * 65535,
                "fs_linear_f32_ex2: invalid arguments (problem %d)", i);
        REQUIRE(!bn[i] || bn_in_ok(g, bn[i]), "fs_linear_f32_ex2: invalid BatchNorm arguments (problem %d)", i);
        a[i] = fs::GemmArgs{g.M, g.N, g.K, g.A, g.sam, g.sak, g.B, g.sbk, g.sbn, g.bias, g.R, g.ldr, g.C, g.ldc,
                            g.rowsum_a};
        a[i].stats = so[i];
        if (bn[i]) b[i] = bn_in_args(bn[i]);
    }
    if (fs_linear_ex2_ok(a[0], bn0 ? &b[0] : nullptr, a[1], bn1 ? &b[1] : nullptr))
        return hip_rc(fs_linear_ex2_impl(a[0], bn0 ? &b[0] : nullptr, a[1], bn1 ? &b[1] : nullptr, (hipStream_t)stream),
                      "fs_linear_f32_ex2");
    for (int i = 0; i < 2; ++i) {  // shapes the two-problem kernel does not take: one launch each
        const hipError_t e = bn[i] ? fs_linear_bn_f32_impl(a[i], &b[i], (hipStream_t)stream)
                                   : fs_linear_f32_impl(a[i], (hipStream_t)stream);
        if (int rc = hip_rc(e, "fs_linear_f32_ex2")) return rc;
    }
    return 0;
}

int fs_bn_running_update(int32_t nbn, int32_t H, float *running_mean, float *running_var, int64_t *num_batches,
                         const float *stats, int32_t passes, int64_t rows0, int64_t rows1, double momentum,
                         const int32_t *skip, void *stream) {
    REQUIRE(nbn >= 0 && H >= 0 && passes >= 1 && passes <= 2 && rows0 >= 2 && (passes < 2 || rows1 >= 2),
            "fs_bn_running_update: invalid arguments");
    REQUIRE(nbn == 0 || H == 0 || (running_mean && running_var && num_batches && stats),
            "fs_bn_running_update: NULL buffer");
    return hip_rc(fs_bn_running_update_impl(nbn, H, running_mean, running_var, num_batches, stats, passes, rows0,
                                            rows1, (float)momentum, skip, (hipStream_t)stream),
                  "fs_bn_running_update");
}

static bool gemm_desc_ok(const fs_gemm_f32 &g) {
    return g.M >= 0 && g.N >= 0 && g.K >= 0 && (g.M == 0 || g.N == 0 || (g.C && (g.K == 0 || (g.A && g.B)))) &&
           g.ldc >= g.N && (!g.R || g.ldr >= g.N) && g.M <= 32LL * 65535 && g.N <= 32LL * 65535;
}

int64_t fs_linear_f32_splitk_floats(const fs_gemm_f32 *d) {
    if (!d || !gemm_desc_ok(*d)) return -1;
    const fs_gemm_f32 &g = *d;
    fs::GemmArgs a{g.M, g.N, g.K, g.A, g.sam, g.sak, g.B, g.sbk, g.sbn, g.bias, g.R, g.ldr, g.C, g.ldc, g.rowsum_a};
    return fs_linear_f32_splitk_floats_impl(a);
}

int fs_linear_f32_splitk(const fs_gemm_f32 *d, float *workspace, int64_t workspace_floats, void *stream) {
    REQUIRE(d && gemm_desc_ok(*d), "fs_linear_f32_splitk: invalid arguments");
    const fs_gemm_f32 &g = *d;
    fs::GemmArgs a{g.M, g.N, g.K, g.A, g.sam, g.sak, g.B, g.sbk, g.sbn, g.bias, g.R, g.ldr, g.C, g.ldc, g.rowsum_a};
    return hip_rc(fs_linear_f32_splitk_impl(a, workspace, workspace_floats, (hipStream_t)stream),
                  "fs_linear_f32_splitk");
}

int fs_linear_f32_group(const fs_gemm_f32 *const *gs, int32_t n, float *workspace, int64_t workspace_floats,
                        void *stream) {
    REQUIRE(gs && n >= 0 && n <= 4, "fs_linear_f32_group: 0..4 products");
    fs::GemmArgs a[4];
    for (int i = 0; i < n; ++i) {
        REQUIRE(gs[i] && gemm_desc_ok(*gs[i]), "fs_linear_f32_group: invalid product %d", i);
        const fs_gemm_f32 &g = *gs[i];
        a[i] = fs::GemmArgs{g.M, g.N, g.K, g.A, g.sam, g.sak, g.B, g.sbk, g.sbn, g.bias, g.R, g.ldr, g.C, g.ldc,
                            g.rowsum_a};
    }
    hipError_t e = fs_linear_f32_group_impl(a, n, workspace, workspace_floats, (hipStream_t)stream);
    if (e == hipErrorNotSupported) {  // one by one
        int64_t off = 0;
        for (int i = 0; i < n; ++i) {
            const int64_t f = fs_linear_f32_splitk_floats_impl(a[i]);
            if (f > 0 && workspace && workspace_floats - off >= f) {
                e = fs_linear_f32_splitk_impl(a[i], workspace + off, f, (hipStream_t)stream);
                off += f;
            } else {
                e = fs_linear_f32_impl(a[i], (hipStream_t)stream);
            }
            if (e != hipSuccess) break;
        }
    }
    return hip_rc(e, "fs_linear_f32_group");
}

int fs_linear_f32_group_partial(const fs_gemm_f32 *const *gs, int32_t n, float *workspace, int64_t workspace_floats,
                                int32_t max_chunks, int32_t *chunks_out, void *stream) {
    REQUIRE(gs && n >= 1 && n <= 4 && chunks_out && max_chunks >= 2 && max_chunks <= 3,
            "fs_linear_f32_group_partial: invalid arguments");
    fs::GemmArgs a[4];
    for (int i = 0; i < n; ++i) {
        REQUIRE(gs[i] && gemm_desc_ok(*gs[i]), "fs_linear_f32_group_partial: invalid product %d", i);
        const fs_gemm_f32 &g = *gs[i];
        a[i] = fs::GemmArgs{g.M, g.N, g.K, g.A, g.sam, g.sak, g.B, g.sbk, g.sbn, g.bias, g.R, g.ldr, g.C, g.ldc,
                            g.rowsum_a};
    }
    int ch = 1;
    hipError_t e = fs_linear_f32_group_partial_impl(a, n, workspace, workspace_floats, max_chunks, &ch,
                                                    (hipStream_t)stream);
    if (e == hipErrorNotSupported) {  // the ordinary group: product 0 reduced into its C
        *chunks_out = 1;
        return fs_linear_f32_group(gs, n, workspace, workspace_floats, stream);
    }
    *chunks_out = ch;
    return hip_rc(e, "fs_linear_f32_group_partial");
}

int fs_splitk_sum(const float *part, int32_t chunks, int64_t stride, int64_t n, float *out, void *stream) {
    REQUIRE(n >= 0 && (n == 0 || (part && out && chunks >= 1 && stride == n)), "fs_splitk_sum: invalid arguments");
    return hip_rc(fs_splitk_sum_impl(part, chunks, stride, n, out, (hipStream_t)stream), "fs_splitk_sum");
}

int fs_bn_relu_train_fwd(int64_t Bn, int32_t H, const float *x, const float *gamma, const float *beta,
                         float *running_mean, float *running_var, int64_t *num_batches, double momentum, double eps,
                         float *y, float *mean, float *invstd, void *stream) {
    REQUIRE(Bn >= 2 && H >= 1 && x && gamma && beta && y && mean && invstd && eps > 0.0,
            "fs_bn_relu_train_fwd: invalid arguments");
    REQUIRE((running_mean == nullptr) == (running_var == nullptr), "fs_bn_relu_train_fwd: running stats go together");
    return hip_rc(fs_bn_relu_train_fwd_impl(Bn, H, x, gamma, beta, running_mean, running_var, num_batches,
                                            (float)momentum, (float)eps, y, mean, invstd, (hipStream_t)stream),
                  "fs_bn_relu_train_fwd");
}

int fs_bn_relu_train_bwd(int64_t Bn, int32_t H, const float *x, const float *y, const float *dy, const float *gamma,
                         const float *mean, const float *invstd, float *dx, const float *dx_add, float *dgamma,
                         float *dbeta, void *stream) {
    REQUIRE(Bn >= 2 && H >= 1 && x && y && dy && gamma && mean && invstd && dx,
            "fs_bn_relu_train_bwd: invalid arguments");
    return hip_rc(fs_bn_relu_train_bwd_impl(Bn, H, x, y, dy, gamma, mean, invstd, dx, dx_add, dgamma, dbeta,
                                            (hipStream_t)stream),
                  "fs_bn_relu_train_bwd");
}

static int check_coupling(const fs_coupling *c, const char *what) {
    REQUIRE(c && c->rows >= 0 && c->D >= 2 && c->D % 2 == 0 && c->hidden >= 1 && c->tail_bound > 0.0,
            "%s: invalid coupling description", what);
    REQUIRE(c->K == 5 || c->K == 8 || c->K == 15 || c->K == 32, "%s: K=%d not instantiated (5, 8, 15, 32)", what,
            c->K);
    REQUIRE(c->rows == 0 || (c->identity_features && c->transform_features), "%s: feature indices are NULL", what);
    return FS_OK;
}

int fs_coupling_features_fwd(const fs_coupling *c, const float *x, float *t, void *stream) {
    int rc = check_coupling(c, "fs_coupling_features_fwd");
    if (rc) return rc;
    REQUIRE(c->rows == 0 || (x && t), "fs_coupling_features_fwd: invalid arguments");
    return hip_rc(fs_coupling_features_fwd_impl(c, x, t, (hipStream_t)stream), "fs_coupling_features_fwd");
}

int fs_coupling_density_fwd(const fs_coupling *c, const float *x, const float *params, const float *uw,
                            const float *uh, const float *ud, const float *lq_in, float *out, float *lq_out,
                            void *stream) {
    int rc = check_coupling(c, "fs_coupling_density_fwd");
    if (rc) return rc;
    REQUIRE(c->rows == 0 || (x && params && uw && uh && ud && out && lq_out),
            "fs_coupling_density_fwd: invalid arguments");
    REQUIRE(x != out, "fs_coupling_density_fwd: out must not alias x");
    return hip_rc(fs_coupling_density_fwd_impl(c, x, params, uw, uh, ud, lq_in, out, lq_out, (hipStream_t)stream),
                  "fs_coupling_density_fwd");
}

int fs_coupling_density_bwd(const fs_coupling *c, const float *x, const float *params, const float *uw,
                            const float *uh, const float *ud, const float *g_out, const float *g_lq, float *gx,
                            float *g_params, float *g_u, void *stream) {
    int rc = check_coupling(c, "fs_coupling_density_bwd");
    if (rc) return rc;
    REQUIRE(c->rows == 0 || (x && params && uw && uh && ud && gx && g_params && g_u),
            "fs_coupling_density_bwd: invalid arguments");
    return hip_rc(fs_coupling_density_bwd_impl(c, x, params, uw, uh, ud, g_out, g_lq, gx, g_params, g_u,
                                               (hipStream_t)stream),
                  "fs_coupling_density_bwd");
}

int fs_coupling_features_bwd(const fs_coupling *c, const float *x, const float *g_t, float *gx, const float *gx_add,
                             void *stream) {
    int rc = check_coupling(c, "fs_coupling_features_bwd");
    if (rc) return rc;
    REQUIRE(c->rows == 0 || (x && g_t && gx), "fs_coupling_features_bwd: invalid arguments");
    return hip_rc(fs_coupling_features_bwd_impl(c, x, g_t, gx, gx_add, (hipStream_t)stream), "fs_coupling_features_bwd");
}

int fs_coupling_sample_pre(const fs_coupling *c, const float *z, const float *uw, const float *uh, const float *ud,
                           float *t, float *out, float *lad_u, int32_t *nan_flag, void *stream) {
    int rc = check_coupling(c, "fs_coupling_sample_pre");
    if (rc) return rc;
    REQUIRE(c->rows == 0 || (z && uw && uh && ud && t && out && lad_u), "fs_coupling_sample_pre: invalid arguments");
    REQUIRE(z != out, "fs_coupling_sample_pre: out must not alias z");
    return hip_rc(fs_coupling_sample_pre_impl(c, z, uw, uh, ud, t, out, lad_u, nan_flag, (hipStream_t)stream),
                  "fs_coupling_sample_pre");
}

int fs_coupling_sample_post(const fs_coupling *c, const float *params, const float *lad_u, const float *lq_in,
                            float *out, float *lq_out, int32_t *nan_flag, void *stream) {
    int rc = check_coupling(c, "fs_coupling_sample_post");
    if (rc) return rc;
    REQUIRE(c->rows == 0 || (params && lad_u && out && lq_out), "fs_coupling_sample_post: invalid arguments");
    return hip_rc(fs_coupling_sample_post_impl(c, params, lad_u, lq_in, out, lq_out, nan_flag, (hipStream_t)stream),
                  "fs_coupling_sample_post");
}

int fs_coupling_pair_pre(const fs_coupling *s, const float *z, const float *uw, const float *uh, const float *ud,
                         float *t, float *out, float *lad_u, int32_t *nan_flag, const fs_coupling *d, const float *x,
                         float *t_density, void *stream) {
    int rc = check_coupling(s, "fs_coupling_pair_pre");
    if (rc || (rc = check_coupling(d, "fs_coupling_pair_pre"))) return rc;
    REQUIRE(s->K == d->K && s->D == d->D, "fs_coupling_pair_pre: the two layers differ in K or D");
    REQUIRE(s->rows == 0 || (z && uw && uh && ud && t && out && lad_u), "fs_coupling_pair_pre: invalid arguments");
    REQUIRE(z != out, "fs_coupling_pair_pre: out must not alias z");
    REQUIRE(d->rows == 0 || (x && t_density), "fs_coupling_pair_pre: invalid density arguments");
    return hip_rc(fs_coupling_pair_pre_impl(s, z, uw, uh, ud, t, out, lad_u, nan_flag, d, x, t_density,
                                            (hipStream_t)stream),
                  "fs_coupling_pair_pre");
}

int fs_coupling_bwd_step(const fs_coupling *f, const float *x_f, const float *g_t, float *gx_f, const float *gx_add,
                         const fs_coupling *c, const float *x, const float *params, const float *uw, const float *uh,
                         const float *ud, const float *g_lq, float *gx, float *g_params, float *g_u, void *stream) {
    int rc = check_coupling(f, "fs_coupling_bwd_step");
    if (rc || (rc = check_coupling(c, "fs_coupling_bwd_step"))) return rc;
    REQUIRE(f->rows == c->rows && f->D == c->D && c->D <= 256, "fs_coupling_bwd_step: the layers differ in rows or D");
    REQUIRE(c->rows == 0 || (x_f && g_t && gx_f && x && params && uw && uh && ud && gx && g_params && g_u),
            "fs_coupling_bwd_step: invalid arguments");
    return hip_rc(fs_coupling_bwd_step_impl(f, x_f, g_t, gx_f, gx_add, c, x, params, uw, uh, ud, g_lq, gx, g_params,
                                            g_u, (hipStream_t)stream),
                  "fs_coupling_bwd_step");
}

int fs_coupling_pair_step(const fs_coupling *s, const float *params, const float *lad_u, const float *lq_in,
                          float *out, float *lq_out, int32_t *nan_flag, const fs_coupling *s_next, const float *uw_next,
                          const float *uh_next, const float *ud_next, float *t_next, float *out_next,
                          float *lad_u_next, const fs_coupling *d, const float *x, const float *params_d,
                          const float *uw, const float *uh, const float *ud, const float *lq_in_d, float *out_d,
                          float *lq_out_d, const fs_coupling *d_next, float *t_density_next, void *stream) {
    int rc = check_coupling(s, "fs_coupling_pair_step");
    if (rc || (rc = check_coupling(d, "fs_coupling_pair_step")) || (rc = check_coupling(s_next, "fs_coupling_pair_step")) ||
        (rc = check_coupling(d_next, "fs_coupling_pair_step")))
        return rc;
    REQUIRE(s->K == d->K && s->D == d->D && s_next->K == s->K && s_next->D == s->D && d_next->D == d->D &&
                s_next->rows == s->rows && d_next->rows == d->rows && s->D <= 256,
            "fs_coupling_pair_step: the layers differ in K, D or rows (D <= 256)");
    REQUIRE(s->rows == 0 || (params && lad_u && out && lq_out && uw_next && uh_next && ud_next && t_next && out_next &&
                             lad_u_next),
            "fs_coupling_pair_step: invalid sampling arguments");
    REQUIRE(d->rows == 0 || (x && params_d && uw && uh && ud && out_d && lq_out_d && t_density_next),
            "fs_coupling_pair_step: invalid density arguments");
    REQUIRE(x != out_d && out != out_next, "fs_coupling_pair_step: outputs must not alias inputs");
    return hip_rc(fs_coupling_pair_step_impl(s, params, lad_u, lq_in, out, lq_out, nan_flag, s_next, uw_next, uh_next,
                                             ud_next, t_next, out_next, lad_u_next, d, x, params_d, uw, uh, ud, lq_in_d,
                                             out_d, lq_out_d, d_next, t_density_next, (hipStream_t)stream),
                  "fs_coupling_pair_step");
}

int fs_coupling_pair_post(const fs_coupling *s, const float *params, const float *lad_u, const float *lq_in,
                          float *out, float *lq_out, int32_t *nan_flag, const fs_coupling *d, const float *x,
                          const float *params_d, const float *uw, const float *uh, const float *ud,
                          const float *lq_in_d, float *out_d, float *lq_out_d, void *stream) {
    int rc = check_coupling(s, "fs_coupling_pair_post");
    if (rc || (rc = check_coupling(d, "fs_coupling_pair_post"))) return rc;
    REQUIRE(s->K == d->K && s->D == d->D, "fs_coupling_pair_post: the two layers differ in K or D");
    REQUIRE(s->rows == 0 || (params && lad_u && out && lq_out), "fs_coupling_pair_post: invalid arguments");
    REQUIRE(d->rows == 0 || (x && params_d && uw && uh && ud && out_d && lq_out_d),
            "fs_coupling_pair_post: invalid density arguments");
    REQUIRE(x != out_d, "fs_coupling_pair_post: out must not alias x");
    return hip_rc(fs_coupling_pair_post_impl(s, params, lad_u, lq_in, out, lq_out, nan_flag, d, x, params_d, uw, uh,
                                             ud, lq_in_d, out_d, lq_out_d, (hipStream_t)stream),
                  "fs_coupling_pair_post");
}
