/*
 * flowstate.h — C ABI of the MI355X-native NF-proposed Metropolis–Hastings
 * hot path (libflowstate.so, built for gfx950).
 *
 * The reference (Inesalmansa/flow-state) is pure Python and has no FFI; the
 * boundary it exposes is the Python API that hybrid_NF_MCMC/main_algorithm_1.py
 * calls.  Each entry point below replaces one reference function (cited as
 * path:line in the reference tree); INTEGRATION.md shows the ctypes binding
 * the reference side would add, and flow-state_amd/flowstate/ is that binding
 * plus the drop-in NormalizingFlow / MonteCarlo classes.
 *
 * Conventions
 *   - every tensor argument is a DEVICE pointer owned by the caller;
 *   - `stream` is a hipStream_t passed as void* (no HIP types in the ABI);
 *   - calls are stream-ordered and never synchronise the device;
 *   - return 0 on success, <0 for an invalid argument, >0 for a HIP error
 *     code; fs_last_error() returns a thread-local message for the last
 *     failure of the calling thread.  No C++ exception crosses the ABI.
 */
#ifndef FLOWSTATE_H
#define FLOWSTATE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FS_OK 0
#define FS_EINVAL (-1)
#define FS_EUNSUPPORTED (-2)

/* Flow hyper-parameters.  Mirrors the CircularCoupledRationalQuadraticSpline
 * stack built by main_algorithm_1.py:280-284 (wrapper.py:103-119):
 * N particles (D = 2N), L layers, H hidden units, nb residual blocks,
 * K spline bins, tail_bound = HALF_BOX; precision selects the GEMM arithmetic
 * (the reference's is float32: precision 0). */
typedef struct {
    int32_t N;
    int32_t L;
    int32_t H;
    int32_t nb;
    int32_t K;
    int32_t precision;   /* conditioner GEMM arithmetic: 0 = f32 MFMA (exact f32 products, the
                          * default); 1 = bf16x6 (f32 operands as 3 bf16 planes, 6 plane
                          * products: f32-level error); 2 = bf16x3 (2 planes, 3 products:
                          * 16-bit operands).  1 and 2 use their own packed image. */
    double tail_bound;
} fs_flow_dims;

/* Physics of the 2D NVT LJ double-well system (main_algorithm_1.py:40-53,
 * energy_calculator.py:79-80, monte_carlo.py:66-67). */
typedef struct {
    double Lx, Ly;        /* SimulationBox.box_size_x / _y                 */
    double V0[2];         /* V0_list                                       */
    double r0, k;         /* well radius, steepness                        */
    int32_t num_wells;    /* 0, 1, 2                                       */
    int32_t reserved;
    double r_cut;         /* 2.5 (inclusive)                               */
    double r_core;        /* 0.5 hard core                                 */
    double beta;          /* 1 / temperature                               */
} fs_phys;

const char *fs_last_error(void);
int fs_version(void);

/* ------------------------------------------------------------------ */
/* Normalizing flow (NF/normflows)                                     */
/* ------------------------------------------------------------------ */

/* Number of floats of the canonical raw parameter buffer: for each layer
 * i = 0..L-1, in this order (all float32, row-major as in the state_dict):
 *   initial_layer.weight [H][2N], initial_layer.bias [H],
 *   for each block j: batch_norm_layers.0.{weight,bias,running_mean,running_var} [H] x4,
 *                     linear_layers.0.{weight [H][H], bias [H]},
 *                     batch_norm_layers.1.{weight,bias,running_mean,running_var} [H] x4,
 *                     linear_layers.1.{weight [H][H], bias [H]},
 *   final_layer.weight [N(3K+1)][H], final_layer.bias [N(3K+1)],
 *   unconditional_transform.unnormalized_{widths [N][K], heights [N][K],
 *                                         derivatives [N][K+1]}.
 * Keys are those of flows.{i}.prqct.transform_net.* (wrapper.py:168-185,
 * resnet.py:53-104) and flows.{i}.prqct.unconditional_transform.* (coupling.py:176-221). */
int64_t fs_flow_raw_floats(const fs_flow_dims *d);

/* Bytes of the packed (MFMA-fragment-ordered, BatchNorm-folded, unconditional
 * spline knots precomputed) parameter image. */
/* Gather float32 device buffers into one: tab [n][3] (device) holds per chunk the source
 * address, the destination offset (floats) and the length (<= 8192 floats); one launch.
 * The raw parameter image of fs_flow_pack from the layers' own tensors
 * (fs_flow_raw_floats). */
int fs_gather_chunks(const int64_t *tab, int64_t n, float *dst, void *stream);
int64_t fs_flow_packed_bytes(const fs_flow_dims *d);

/* Pack raw -> packed on the device.  Must be re-run after any weight update
 * (eval-mode BatchNorm statistics are folded here, resnet.py:37-50). */
int fs_flow_pack(const fs_flow_dims *d, const float *raw, void *packed, void *stream);

/* NormalizingFlow.log_prob (NF/normflows/core.py:198-214): layers L-1..0 in
 * the density direction (CircularCoupled...inverse = Coupling.forward,
 * wrapper.py:273-275, coupling.py:71-102) + UniformParticle.log_prob
 * (Energy/Uniform.py:50-74).  x, z_out: [B][2N] float32 (z_out nullable);
 * log_q: [B].  err (nullable, device int32): bit0 set on a NaN discriminant (|= 4: a
 * wide-path trunk hand-off timed out and the outputs are wrong; the pass can then be re-run
 * with err = NULL, which never takes the column-split trunk, fs_set_wide_trunk16). */
int fs_flow_log_prob(const fs_flow_dims *d, const void *packed, const float *x, int64_t B,
                     float *log_q, float *z_out, int32_t *err, void *stream);

/* NormalizingFlow.inverse_and_log_det without the base term (core.py:71-86). */
int fs_flow_inverse(const fs_flow_dims *d, const void *packed, const float *x, int64_t B,
                    float *z_out, float *log_det, int32_t *err, void *stream);

/* NormalizingFlow.forward_and_log_det / sample body (core.py:41-56, 178-196):
 * layers 0..L-1 in the sampling direction (CircularCoupled...forward =
 * Coupling.inverse, wrapper.py:269-271, coupling.py:104-134) from supplied
 * base draws z [B][2N] -> x [B][2N]; log_det nullable.  err bit0: NaN
 * discriminant (the reference raises ValueError, splines.py:176-183). */
int fs_flow_forward(const fs_flow_dims *d, const void *packed, const float *z, int64_t B,
                    float *x_out, float *log_det, int32_t *err, void *stream);

/* Proposal generation for the batched MH step (utils.py:422-450 +
 * main_algorithm_1.py:340-343): base draws z ~ U(-B, B) from a counter-based
 * generator keyed (seed, counter, row_offset + row), sampling pass, then
 *   config   = fl32(x + fl32(tail_bound))         box coordinates [B][N][2]
 *   centered = fl32((double)config - half_width)   the NF input of nf_big_move
 *                                                   (monte_carlo.py:251-258).
 * x_out (centered model-space sample) and centered are nullable. */
int fs_flow_propose(const fs_flow_dims *d, const void *packed, int64_t B, uint64_t seed,
                    uint64_t counter, int64_t row_offset, double half_width, float *config,
                    float *centered, float *x_out, int32_t *err, void *stream);

/* fs_flow_propose that also writes log_q [B] = log q(x') from the sampling pass itself
 * (log q0(z) minus the sampling direction's summed log|dx/dz|, NormalizingFlow.sample
 * with its log-dets kept, core.py:178-196): the single-pass value of FS_MH_SINGLE_PASS.
 * The reference instead evaluates log_prob on `centered` with a second pass. */
int fs_flow_propose_lq(const fs_flow_dims *d, const void *packed, int64_t B, uint64_t seed,
                       uint64_t counter, int64_t row_offset, double half_width, float *config,
                       float *centered, float *x_out, float *log_q, int32_t *err, void *stream);

/* ------------------------------------------------------------------ */
/* Physics (MCMC/)                                                     */
/* ------------------------------------------------------------------ */

/* EnergyCalculator.calculate_total_energy_virial (energy_calculator.py:121-203)
 * for C chains: pos [C][N][2], float32 (pos_is_f32=1) or float64.
 * E, W: [C] float64 (+inf on a hard-core overlap, the reference's early return);
 * overlap [C] u8 nullable; nbr nullable: [C][N] u64, bit j of word i set iff
 * i<j and r_ij <= r_cut (the neighbour mask of potential.py:11).  N <= 64. */
int fs_energy_lj_dw(const fs_phys *p, const void *pos, int pos_is_f32, int64_t C, int32_t N,
                    double *E, double *W, uint8_t *overlap, uint64_t *nbr, void *stream);

/* The same over chain states held as float64 with a per-chain reference dtype
 * (state_is_f32[c] = 1: a float32 state after an accepted big move, monte_carlo.py:296, whose
 * energy the reference computes in float32; EnergyCalculator.__init__,
 * energy_calculator.py:46): one launch, no host round trip to split the chains by dtype. */
int fs_energy_state(const fs_phys *p, const double *state, const uint8_t *state_is_f32, int64_t C, int32_t N,
                    double *E, double *W, void *stream);

/* SimulationBox.minimum_image / compute_distance / compute_distances
 * (simulation_box.py:31-65) for n pairs (pos1[i * stride1], pos2[i]) of [2] positions,
 * float32 (pos_is_f32=1) or float64 (both the same dtype, numpy's promotion done by the
 * caller; box lengths np.float64 as initialise_fcc makes them); stride1 = 0 broadcasts
 * one first position.  delta [n][2] = the wrapped displacement (np.round half-even; in
 * the positions' dtype, widened), r [n] = np.linalg.norm(delta) (float32 sdot / float64
 * ddot with a correctly rounded sqrt), each nullable. */
int fs_min_image(const fs_phys *p, const void *pos1, int64_t stride1, const void *pos2, int pos_is_f32, int64_t n,
                 double *delta, double *r, void *stream);

/* EnergyCalculator.calculate_particle_energy_virial (energy_calculator.py:48-108) for one
 * particle per chain: pos [C][N][2] (float32 or float64), particle [C] int32.  E, W [C]
 * float64: +inf both on any r < 0.5 to the other particles, else the np.sum (pairwise
 * order, np.delete-compacted others) of the LJ terms, E plus the particle's double-well
 * term. */
int fs_particle_energy(const fs_phys *p, const void *pos, int pos_is_f32, int64_t C, int32_t N,
                       const int32_t *particle, double *E, double *W, void *stream);

/* np.random.default_rng(seed) (SeedSequence + PCG64 init, monte_carlo.py:92-95)
 * for C seeds -> state [C][4] u64 = {state_hi, state_lo, inc_hi, inc_lo}. */
int fs_pcg64_seed(const uint64_t *seeds, int64_t C, uint64_t *state, void *stream);

/* C x Generator.random() draws, advancing each state once. */
int fs_pcg64_random(uint64_t *state, int64_t C, double *out, void *stream);

/* MonteCarlo.nf_big_move decision + update (monte_carlo.py:235-303), batched:
 *   ratio = exp(-beta*(E_new - E_old) - (nll_new - nll_old))   (reference sign;
 *           flags bit0 FS_MH_CORRECT_SIGN uses +(nll_new - nll_old))
 *   accept iff ratio >= 1 (no draw) or Generator.random() < ratio.
 * On accept: state[c] <- config[c] (float32 values, state_is_f32[c] <- 1),
 * E_old/W_old/nll_old <- new values, accepted[c]++.  attempts[c]++ always
 * (monte_carlo.py:240).  accept [C] u8 out; n_accept (nullable) += accepts
 * (wave ballot + popcount, one atomic per wave). */
#define FS_MH_CORRECT_SIGN 1
/* flags bit1 (fs_nf_mh_step): the state moved (local moves) since E_old / nll_old
 * were exact.  The step then does what nf_big_move does on every call: old NLL
 * from a density pass of the current state (monte_carlo.py:251-261; the ratio
 * still uses the running E_old, :243), and on reject the total energy recomputed
 * from the current state (:299-301). */
#define FS_MH_HYBRID 2
/* flags bit2 (fs_nf_mh_step only; opt-in, never the reference's semantics): take the
 * proposals' log q from the sampling pass itself, log q(x') = log q0(z) - sum of the
 * sampling direction's log|dx/dz| (core.py:178-196 run with its log-dets kept), instead
 * of the reference's second, density-direction pass over fl32(config - half_width)
 * (monte_carlo.py:251-262).  One flow pass per step instead of two; the value differs
 * from the reference's by the two passes' float32 noise and the box-coordinate
 * rounding of x' (bench.py `single_pass` reports the deviation and the decision flips). */
#define FS_MH_SINGLE_PASS 4
int fs_mh_accept(const fs_phys *p, int64_t C, int32_t N, double *E_old, double *W_old,
                 double *nll_old, const double *E_new, const double *W_new, const float *log_q_new,
                 uint64_t *pcg, double *state, uint8_t *state_is_f32, const float *config,
                 uint8_t *accept, int64_t *attempts, int64_t *accepted,
                 unsigned long long *n_accept, int flags, void *stream);

/* Energy-only Metropolis judgement of supplied proposals, no state change:
 * MonteCarlo.judge_normalizing_flow (monte_carlo.py:305-329; M = 1, E_ref = the
 * chain's total energy) and bulk_judge_normalizing_flow (:331-370; M proposals per
 * chain against one reference energy), both via metropolis_acceptance_particle_move
 * (:191-223): E_new <= E_ref accepts and an infinite E_new rejects without a draw;
 * otherwise accept iff Generator.random() < exp(-beta*(E_new - E_ref)).  Chain c's
 * proposals are judged in order m = 0..M-1 on its PCG64 stream pcg[c] (advanced).
 * E_ref [C], E_new [C][M] float64; accept [C][M] u8 and n_accept [C] (accepted
 * count per chain) out, each nullable. */
int fs_metropolis_judge(double beta, int64_t C, int64_t M, const double *E_ref, const double *E_new,
                        uint64_t *pcg, uint8_t *accept, int64_t *n_accept, void *stream);

/* Fused batched NF-MH step over C chains: fs_flow_propose -> fs_flow_log_prob
 * (density pass on `centered`) -> fs_energy_lj_dw (config, float32) ->
 * fs_mh_accept.  chain_offset: global index of chain 0 (proposal stream row), so a
 * chain's trajectory does not depend on how chains are sharded over GPUs.
 * ws: caller workspace of fs_nf_mh_step_ws_bytes() bytes (256-byte aligned):
 * config f32 [C][2N] | centered f32 [C][2N] directly followed by centered_old f32
 * [C][2N] | log_q f32 [C] directly followed by log_q_old f32 [C] | E_new f64 [C] |
 * W_new f64 [C] | E_cur f64 [C] | W_cur f64 [C] (the *_old / *_cur parts used with
 * FS_MH_HYBRID, whose two density passes run as one launch over 2C rows), each
 * section padded to 256 bytes. */
int64_t fs_nf_mh_step_ws_bytes(const fs_flow_dims *d, int64_t C);
int fs_nf_mh_step(const fs_flow_dims *d, const void *packed, const fs_phys *p, int64_t C,
                  uint64_t seed, uint64_t step, int64_t chain_offset, double *E_old, double *W_old, double *nll_old,
                  uint64_t *pcg, double *state, uint8_t *state_is_f32, uint8_t *accept,
                  int64_t *attempts, int64_t *accepted, unsigned long long *n_accept,
                  int32_t *err, int flags, void *ws, void *stream);

/* S consecutive fs_nf_mh_step calls (steps step0 .. step0+S-1) with the same results:
 * the proposals, their log q and energies do not depend on the chain states, so each
 * pass runs once over S*C rows (a small C then fills the chip), followed by the S
 * accept/update launches in order.  Not with FS_MH_HYBRID.  Workspace: config f32
 * [S C][2N] | centered f32 [S C][2N] | log_q f32 [S C] | E_new f64 [S C] | W_new f64 [S C],
 * 256-byte padded sections. */
int64_t fs_nf_mh_steps_ws_bytes(const fs_flow_dims *d, int64_t C, int64_t S);
int fs_nf_mh_steps(const fs_flow_dims *d, const void *packed, const fs_phys *p, int64_t C, int64_t S,
                   uint64_t seed, uint64_t step0, int64_t chain_offset, double *E_old, double *W_old, double *nll_old,
                   uint64_t *pcg, double *state, uint8_t *state_is_f32, uint8_t *accept,
                   int64_t *attempts, int64_t *accepted, unsigned long long *n_accept,
                   int32_t *err, int flags, void *ws, void *stream);

/* Proposal bank for steps interleaved with local moves (Algorithm 1's cycle,
 * main_algorithm_1.py:384-395, which pre-generates its proposals in batches,
 * :340-343 / utils.py:422-450).  fs_nf_mh_bank fills `bank` (the fs_nf_mh_steps
 * workspace layout, fs_nf_mh_steps_ws_bytes(d, C, S) bytes) with the proposals of steps
 * step0 .. step0+S-1, their log q and their energies: one launch of S*C rows per pass.
 * fs_nf_mh_step_banked then runs step step0+s (0 <= s < S) of that bank exactly as
 * fs_nf_mh_step would, FS_MH_HYBRID included: the hybrid's density pass over the current
 * states (C rows) and their energy are its only flow / energy work.  hws: caller
 * workspace of fs_nf_mh_banked_ws_bytes() bytes (256-byte aligned), used with
 * FS_MH_HYBRID: centered_old f32 [C][2N] | log_q_old f32 [C] | E_cur f64 [C] | W_cur f64 [C]. */
int fs_nf_mh_bank(const fs_flow_dims *d, const void *packed, const fs_phys *p, int64_t C, int64_t S,
                  uint64_t seed, uint64_t step0, int64_t chain_offset, int32_t *err, void *bank, void *stream);
int64_t fs_nf_mh_banked_ws_bytes(const fs_flow_dims *d, int64_t C);
int fs_nf_mh_step_banked(const fs_flow_dims *d, const void *packed, const fs_phys *p, int64_t C, int64_t S,
                         int64_t s, const void *bank, double *E_old, double *W_old, double *nll_old, uint64_t *pcg,
                         double *state, uint8_t *state_is_f32, uint8_t *accept, int64_t *attempts,
                         int64_t *accepted, unsigned long long *n_accept, int32_t *err, int flags, void *hws,
                         void *stream);

/* Largest batch (rows) the flow passes run on the wide path: phase-by-phase launches
 * spread over the whole chip instead of one 64-row workgroup carrying its rows through
 * every layer, bit-identical results (f32 image only).  Default 12288 or the
 * FS_WIDE_ROWS environment variable; 0 disables it; capped at 65536.  Returns the
 * previous limit.  Process-wide. */
int64_t fs_set_wide_rows(int64_t rows);

/* Kernel-variant switches for A/B measurements and bit-identity tests, process-wide; each
 * returns the previous value (a negative argument only reads it).  The results do not
 * depend on them.
 * fs_set_wide_trunk16: 5 (default, or FS_WIDE_TRUNK16) = by batch: 4 for the A1 trunk
 *   (H = 256) on at most 512 rows, else 3; 4 = each 16-row tile's columns split over four
 *   workgroups (CUs) that hand their epilogue slices to each other inside the launch (where
 *   the tiles x 4 fit half the chip, else 3; err |= 4 if a hand-off wait gave up); 3 = the
 *   wide path's ResidualNet on 16-row tiles (v_mfma_f32_16x16x4_f32, twice the workgroups)
 *   with each layer's start phase merged into the trunk launch and each 32-column tile split
 *   over two waves (one 16-column half each), 2 = the same with one wave per tile, 1 = 16-row
 *   tiles after a separate start launch, 0 = 32-row tiles.
 * fs_set_wide_final32: 2 (default, or FS_WIDE_FINAL32) = the wide path's final phase on
 *   16- or 32-row blocks when that grid fits the chip in one round (16-row blocks on
 *   v_mfma_f32_16x16x4_f32 for spline bins K <= 16 only; K > 16, one feature per wave:
 *   32-row blocks), 1 = 32-row blocks at most, 0 = always 64-row blocks.
 * fs_set_wide_handoff_spins: polls (an sc1 load and an s_sleep each) a column-split trunk
 *   workgroup makes before a hand-off wait gives up (err |= 4; default 2^20); 0 makes every
 *   wait give up at once, the hook the timeout tests use.  Returns the previous value; a
 *   negative argument only reads it.  The column-split trunk runs only when the pass has an
 *   err word to report a timeout in (err == NULL: trunk 3 instead).
 * fs_set_coupling_waves: 1 (default, or FS_COUPLING_WAVES) = the training step's coupling
 *   launches (fs_coupling_pair_step, fs_coupling_bwd_step) with each row's splines spread
 *   over two / four waves (one knot set per wave), 0 = one / two waves per row.
 * fs_set_lean_gemm: 1 (default, or FS_LEAN_GEMM) = the training products on the lean
 *   kernels (32-bit buffer offsets), 0 = the generic strided kernels. */
int32_t fs_set_wide_trunk16(int32_t on);
int32_t fs_set_wide_final32(int32_t on);
int64_t fs_set_wide_handoff_spins(int64_t spins);
int32_t fs_set_coupling_waves(int32_t on);
int32_t fs_set_lean_gemm(int32_t on);

/* ------------------------------------------------------------------ */
/* Training (Algorithm 2): the circular RQS element-wise, with backward */
/* ------------------------------------------------------------------ */

/* Algorithm 2's target energy, DoubleWellLJ._energy (NF/normflows/Energy/SimpleLJ.py:
 * 15-39, 63-128; used by NormalizingFlow.reverse_kld, core.py:105-142), for B sample rows
 * x [B][2N] float32 in the flow's centred frame: LJ over all pairs plus an extra particle
 * at the origin (each particle wrapped into [-bound, bound), no minimum image between
 * particles, linear core -80 (r - 0.82) + 30 for r <= 0.82), divided by temperature, plus
 * the double well (num_wells <= 2, centres (-+bound/2, 0), depths V0_0 / V0_1, r0, k) on
 * the raw coordinates.  E [B] float32; grad_x (nullable) [B][2N] = dE/dx. */
int fs_target_energy(const float *x, int64_t B, int32_t N, double bound, double temperature, int32_t num_wells,
                     double V0_0, double V0_1, double r0, double k, float *E, float *grad_x, void *stream);

/* One Adam step (torch.optim.Adam, L2 weight decay added to the gradient; the Algorithm-2
 * optimizer, main_algorithm_2.py:310,440) over n float32 parameters param [n] with their
 * gradient grad and moments exp_avg / exp_avg_sq [n], in torch's capturable multi-tensor
 * arithmetic; step [1] is the float32 step count (incremented).  loss (nullable) [1]: when
 * it is NaN or inf nothing is written (main_algorithm_2.py:324-326 skips the step); skip
 * (nullable) [1]: when non-zero nothing is written either (a graphed epoch's sticky
 * spline-NaN flag: no update after the step that raised, splines.py:176-183).  All
 * buffers 16-byte aligned. */
int fs_adam_step(float *param, const float *grad, float *exp_avg, float *exp_avg_sq, int64_t n, float *step,
                 const float *loss, const int32_t *skip, double lr, double beta1, double beta2, double eps,
                 double weight_decay, void *stream);

/* The Algorithm-2 loss with ALPHA = 1 (main_algorithm_2.py:316-318; NF/normflows/core.py
 * forward_kld / reverse_kld): loss [1] = -mean(log_q [B]) + 0 * (mean(energy [R]) +
 * mean(lq_rev [R])), NaN / inf when the reverse term is (the step's skip rule reads it);
 * energy / lq_rev nullable (then the loss is -mean(log_q)).  nan_out (nullable, one byte)
 * = nan_word [1] (nullable) is non-zero.  One launch; the means are ordered tree sums. */
int fs_kld_loss(const float *log_q, int64_t B, const float *energy, const float *lq_rev, int64_t R,
                const int32_t *nan_word, float *loss, uint8_t *nan_out, void *stream);

/* Its gradient: grad_log_q [B] = -grad_loss[0] / B. */
int fs_kld_loss_backward(const float *grad_loss, int64_t B, float *grad_log_q, void *stream);

/* unconstrained_rational_quadratic_spline, circular tails (NF/normflows/utils/
 * splines.py:16-222) for M independent elements: x [M], unnormalised widths /
 * heights uw, uh [M][K], derivatives ud [M][K+1] (row-major, contiguous).
 * inverse = 0: forward map, 1: inverse map.  out, lad [M]; nan_flag (nullable)
 * |= 1 when an inverse discriminant is NaN (splines.py:176-183).  K in {5, 8, 15, 32}. */
int fs_rqs_forward(int64_t M, int32_t K, int32_t inverse, const float *x, const float *uw, const float *uh,
                   const float *ud, double tail_bound, float *out, float *lad, int32_t *nan_flag, void *stream);

/* Gradients of sum(g_out * out + g_lad * lad) with respect to x, uw, uh, ud (g_out /
 * g_lad nullable = zero), recomputing the forward from the same inputs. */
int fs_rqs_backward(int64_t M, int32_t K, int32_t inverse, const float *x, const float *uw, const float *uh,
                    const float *ud, double tail_bound, const float *g_out, const float *g_lad, float *gx,
                    float *guw, float *guh, float *gud, void *stream);

/* Conditioner pieces of the training step (ResidualNet in train mode, NF/normflows/
 * nets/resnet.py:7-104; nn.Linear / nn.BatchNorm1d semantics).
 * fs_linear_f32: C[m][n] = sum_k A[m][k] B[k][n] (+ bias[n]) (+ R[m][n]) in f32, with
 * A[m][k] at A[m*sam + k*sak], B[k][n] at B[k*sbk + n*sbn], R (ld ldr) and C (ld ldc)
 * row-major; bias, R nullable.  rowsum_a (nullable) [M] = sum_k A[m][k] (the bias
 * gradient when A = dY^T).  nn.Linear forward: A = X, B = W^T; input gradient: A = dY,
 * B = W; weight gradient: A = dY^T, B = X (replaces torch.addmm / mm, at::linear). */
int fs_linear_f32(int64_t M, int64_t N, int64_t K, const float *A, int64_t sam, int64_t sak, const float *B,
                  int64_t sbk, int64_t sbn, const float *bias, const float *R, int64_t ldr, float *C, int64_t ldc,
                  float *rowsum_a, void *stream);

/* Two independent fs_linear_f32 products in one launch (nn.Linear's backward: the input
 * gradient dY W and the weight / bias gradients dY^T X, which torch's autograd runs as two
 * GEMMs), each with exactly fs_linear_f32's arithmetic and results.  The arguments of
 * each are those of fs_linear_f32, in this POD. */
typedef struct fs_gemm_f32 {
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
} fs_gemm_f32;
int fs_linear_f32_pair(const fs_gemm_f32 *g0, const fs_gemm_f32 *g1, void *stream);

/* nn.Linear's backward pair with the BatchNorm1d (train) + ReLU backwards around it folded
 * in (replaces the pair, fs_bn_relu_train_bwd sequence of a ResidualNet: resnet.py:37-51).
 * fout (nullable): the BatchNorm this Linear applies to its input.  g0's output must be that
 *   BatchNorm's output gradient gu = dL/du, u = relu(BN(y)), [B][H] contiguous
 *   (g0.C == fout->gu); its epilogue writes per 32-row tile the column sums of
 *   dz = gu (u > 0) and dz xhat into fout->part.
 * fin (nullable): the BatchNorm that consumes this Linear's output.  Its input gradient
 *   dy = gamma invstd (dz - sum dz / B - xhat sum(dz xhat) / B) (+ fin->dx_add, the residual
 *   gradient) is not materialised: g0 = dy W and g1 = dy^T X take A = fin->gu as its layout
 *   (g0: row-major, sam = H, sak = 1; g1: the transpose, sam = 1, sak = H) and load dy from
 *   gu, u, y and the tile sums; workgroup 0 writes dgamma and dbeta (nullable); fin->a_out
 *   (nullable) receives dy.
 * Lean kernels only (fs_set_lean_gemm(1)); H <= 256, B a multiple of 4, no residual output. */
typedef struct fs_bn_fold {
    const float *gu, *u, *y;            /* [B][H] */
    const float *mean, *invstd, *gamma; /* [H] */
    float *part;                        /* [ceil(B / 32)][H][2] */
    float *dgamma, *dbeta;              /* [H], nullable (fin) */
    const float *dx_add;                /* [B][H], nullable (fin) */
    float *a_out;                       /* [B][H], nullable (fin) */
    int64_t B;
    int32_t H;
} fs_bn_fold;
int fs_linear_f32_pair_bn(const fs_gemm_f32 *g0, const fs_gemm_f32 *g1, const fs_bn_fold *fin,
                          const fs_bn_fold *fout, void *stream);
/* The same with split-K operands left unreduced by fs_linear_f32_group_partial: a_chunks > 1
 * (fout only, no fin; at most 3): A of both products is the ordered sum of a_chunks partials a_stride
 * floats apart (g0->A == g1->A = partial 0); add_chunks > 1 (fin): fin->dx_add likewise.
 * Each sum is fs_splitk_sum's, taken on load: the values are those of the reduced operand.
 * With a_chunks > 1, fout->a_out (nullable) receives the reduced A ([B][K] of g0's layout),
 * written by g0's first column tile, for A's other readers. */
int fs_linear_f32_pair_bn_sk(const fs_gemm_f32 *g0, const fs_gemm_f32 *g1, const fs_bn_fold *fin,
                             const fs_bn_fold *fout, int32_t a_chunks, int64_t a_stride, int32_t add_chunks,
                             int64_t add_stride, void *stream);

/* fs_linear_f32 with the ResidualNet's BatchNorm plumbing fused in (resnet.py:35-51):
 * stats_out (nullable) [ceil(M/32)][N][2] receives each 32-row tile's column mean and sum
 * of squared deviations of C, the batch statistics of the BatchNorm that consumes C; bn
 * (nullable) makes A = relu(BatchNorm1d_train(x)) of the raw x the descriptor points at,
 * from the producer's tile statistics (Chan's combination, tiles in order, biased
 * variance, eps): bn->mean_out / invstd_out [K] written, running statistics updated with
 * momentum (unbiased variance) and num_batches += 1 once, u (a_out, nullable, x's layout)
 * written for the backward.  Replaces the separate BatchNorm + ReLU launch in front of a
 * Linear (fs_bn_relu_train_fwd).  With bn: K <= 256, A and B contiguous along k. */
typedef struct fs_bn_in {
    const float *stats;
    int64_t tiles, rows;
    const float *gamma, *beta;
    float eps, momentum;
    float *running_mean, *running_var;
    int64_t *num_batches;
    float *mean_out, *invstd_out;
    float *a_out;
    float *var_out; /* nullable: the biased batch variance [K] (for deferred running statistics) */
} fs_bn_in;
int fs_linear_f32_ex(const fs_gemm_f32 *g, const fs_bn_in *bn, float *stats_out, void *stream);

/* Two independent fs_linear_f32_ex products in one launch (the Algorithm-2 training step's
 * two passes, main_algorithm_2.py:446-447: reverse_kld's sampling pass and forward_kld's
 * density pass run layer by layer side by side, each launch carrying one Linear of each).
 * Each problem is computed exactly as fs_linear_f32_ex computes it alone; shapes the shared
 * kernel does not take (non-contiguous operands, long reductions) run as two launches. */
int fs_linear_f32_ex2(const fs_gemm_f32 *g0, const fs_bn_in *bn0, float *stats0, const fs_gemm_f32 *g1,
                      const fs_bn_in *bn1, float *stats1, void *stream);

/* BatchNorm running statistics applied after the fact (torch.nn.BatchNorm1d.forward's
 * momentum update, unbiased variance): nbn BatchNorms of width H whose running buffers are
 * flat [nbn][H] (num_batches [nbn]); stats [passes][nbn][2][H] = each pass's batch mean and
 * biased variance (fs_bn_in mean_out / var_out of launches that left running_mean NULL);
 * the passes' updates are applied in pass order (rows0 / rows1 = their batch sizes) and
 * num_batches += passes.  With passes = 2 this is the reference's order when pass 0 is
 * reverse_kld's sampling pass and pass 1 forward_kld's density pass.  skip (nullable) [1]:
 * when non-zero nothing is written (as fs_adam_step's). */
int fs_bn_running_update(int32_t nbn, int32_t H, float *running_mean, float *running_var, int64_t *num_batches,
                         const float *stats, int32_t passes, int64_t rows0, int64_t rows1, double momentum,
                         const int32_t *skip, void *stream);

/* Long reductions over few output tiles (K >= 2048, <= 128 tiles of 32 x 32, no rowsum:
 * the input gradient of the 2944-wide final layer, 256 x 128 over K = 2944): the reduction
 * runs as S chunks of the grid, each a partial tile by fs_linear_f32's arithmetic, then one
 * launch adds the partials in chunk order (+ bias, + R).  workspace: caller-owned, at least
 * fs_linear_f32_splitk_floats(g) floats (0 = this product does not take the split-K path;
 * with a smaller or NULL workspace the call is plain fs_linear_f32). */
int64_t fs_linear_f32_splitk_floats(const fs_gemm_f32 *g);
int fs_linear_f32_splitk(const fs_gemm_f32 *g, float *workspace, int64_t workspace_floats, void *stream);

/* Up to 4 independent fs_linear_f32 products in one launch (a coupling layer's final
 * Linear backward: input gradient, weight + bias gradient, and the unconditional spline
 * parameters' row sum).  Products with a split-K plan take it while the workspace
 * (sum of their fs_linear_f32_splitk_floats, in order) lasts, followed by their ordered
 * reductions; each product's values are those of fs_linear_f32 / fs_linear_f32_splitk. */
/* fs_linear_f32_group with product 0 (no bias / R, C dense) split into at most max_chunks
 * (2..3) K chunks whose partial products stay in the workspace, unreduced: partial z of its
 * C at workspace + z M N; chunks_out = their count, 1 when product 0 takes no split-K plan
 * (then C is written as fs_linear_f32_group writes it).  The consumer sums them on load
 * (fs_linear_f32_pair_bn_sk) or calls fs_splitk_sum.  Workspace: as fs_linear_f32_group's. */
int fs_linear_f32_group_partial(const fs_gemm_f32 *const *gs, int32_t n, float *workspace, int64_t workspace_floats,
                                int32_t max_chunks, int32_t *chunks_out, void *stream);
/* out [n] = part[0 .. n) + part[stride ..) + ... (chunks partials, in order; stride == n),
 * the reduction fs_linear_f32_group would have written. */
int fs_splitk_sum(const float *part, int32_t chunks, int64_t stride, int64_t n, float *out, void *stream);
int fs_linear_f32_group(const fs_gemm_f32 *const *gs, int32_t n, float *workspace, int64_t workspace_floats,
                        void *stream);

/* BatchNorm1d (training mode) followed by ReLU over x [Bn][H] (row-major):
 * batch mean / biased variance, y = relu(gamma (x - mean) invstd + beta),
 * running_mean / running_var updated with `momentum` (unbiased variance) and
 * *num_batches += 1 when non-NULL (torch.nn.BatchNorm1d.forward); mean, invstd [H]
 * saved for the backward.  Bn >= 2. */
int fs_bn_relu_train_fwd(int64_t Bn, int32_t H, const float *x, const float *gamma, const float *beta,
                         float *running_mean, float *running_var, int64_t *num_batches, double momentum, double eps,
                         float *y, float *mean, float *invstd, void *stream);

/* Gradients of the above: dx [Bn][H], dgamma, dbeta [H] (nullable) from dy = dL/dy and
 * the forward's x, y, mean, invstd. */
/* fs_bn_relu_train_bwd: dx = the input gradient (+ dx_add [Bn][H], nullable: the block
 * input's residual-branch gradient, resnet.py:51, added in the same launch instead of by
 * autograd); dgamma, dbeta nullable. */
int fs_bn_relu_train_bwd(int64_t Bn, int32_t H, const float *x, const float *y, const float *dy, const float *gamma,
                         const float *mean, const float *invstd, float *dx, const float *dx_add, float *dgamma,
                         float *dbeta, void *stream);

/* One circular-RQS coupling layer of the training path around its conditioner
 * (Coupling.forward / inverse, NF/normflows/flows/neural_spline/coupling.py:71-134;
 * periodic features nn.py:120-137; replaces the per-layer gather / cos / sin / cat /
 * spline / index_copy / roll / sum kernels of autograd over torch ops).  x, z, out
 * [rows][D] f32 row-major; identity_features / transform_features [D/2] int64 (the
 * layer's buffers); params [rows][D/2][3K+1] = the conditioner output; uw, uh [D/2][K],
 * ud [D/2][K+1] = the unconditional spline; t [rows][D] = [cos(s x_id), sin(s x_id)],
 * s = pi / tail_bound; hidden = the conditioner width (params / sqrt(hidden)). */
typedef struct fs_coupling {
    int64_t rows;
    int32_t D, K, hidden;
    const int64_t *identity_features, *transform_features;
    double tail_bound;
} fs_coupling;

/* Density direction, before the conditioner: t from x. */
int fs_coupling_features_fwd(const fs_coupling *c, const float *x, float *t, void *stream);
/* ... and after it: out = the half-rolled layer output, lq_out = lq_in (nullable = 0) +
 * the two splines' log-det sums. */
int fs_coupling_density_fwd(const fs_coupling *c, const float *x, const float *params, const float *uw,
                            const float *uh, const float *ud, const float *lq_in, float *out, float *lq_out,
                            void *stream);
/* Its adjoints from g_out [rows][D] and g_lq [rows] (nullable = 0): gx [rows][D] through
 * the splines, g_params [rows][D/2][3K+1], g_u [rows][(D/2)(3K+1)] = per-row adjoints
 * of uw [D/2][K], uh [D/2][K], ud [D/2][K+1], back to back in each row (their sum over rows
 * is the parameter gradient). */
int fs_coupling_density_bwd(const fs_coupling *c, const float *x, const float *params, const float *uw,
                            const float *uh, const float *ud, const float *g_out, const float *g_lq, float *gx,
                            float *g_params, float *g_u, void *stream);
/* Adjoint of t: gx [rows][D] (zero at the transform positions). */
/* fs_coupling_features_bwd: gx = the features' adjoint (identity positions, 0 elsewhere)
 * + gx_add [rows][D] (nullable: the splines' gradient of the same x, added in this launch
 * instead of by autograd). */
int fs_coupling_features_bwd(const fs_coupling *c, const float *x, const float *g_t, float *gx,
                             const float *gx_add, void *stream);
/* Sampling direction, forward only, in two launches around the conditioner:
 * pre: t, out (identity half through the inverse unconditional spline, transform half
 * copied), lad_u [rows]; post: the transform half through the inverse conditional spline
 * (in place in out), lq_out = lq_in - (lad_u + its log-det sum).  nan_flag (nullable)
 * |= 1 on a NaN discriminant (splines.py:176-183). */
int fs_coupling_sample_pre(const fs_coupling *c, const float *z, const float *uw, const float *uh, const float *ud,
                           float *t, float *out, float *lad_u, int32_t *nan_flag, void *stream);
int fs_coupling_sample_post(const fs_coupling *c, const float *params, const float *lad_u, const float *lq_in,
                            float *out, float *lq_out, int32_t *nan_flag, void *stream);
/* The training step's two passes side by side (see fs_linear_f32_ex2): one launch runs
 * fs_coupling_sample_pre on layer s and fs_coupling_features_fwd on layer d; the other
 * fs_coupling_sample_post on s and fs_coupling_density_fwd on d (same K and D), each row
 * exactly as the single-layer entry points compute it. */
int fs_coupling_pair_pre(const fs_coupling *s, const float *z, const float *uw, const float *uh, const float *ud,
                         float *t, float *out, float *lad_u, int32_t *nan_flag, const fs_coupling *d, const float *x,
                         float *t_density, void *stream);
int fs_coupling_pair_post(const fs_coupling *s, const float *params, const float *lad_u, const float *lq_in,
                          float *out, float *lq_out, int32_t *nan_flag, const fs_coupling *d, const float *x,
                          const float *params_d, const float *uw, const float *uh, const float *ud,
                          const float *lq_in_d, float *out_d, float *lq_out_d, void *stream);

/* fs_coupling_features_bwd of layer f (x_f, g_t, gx_add nullable -> gx_f, the input
 * gradient of layer f = the output gradient of layer c) and fs_coupling_density_bwd of layer
 * c on that gradient (g_out = gx_f) in one launch, each row exactly as the two launches
 * compute it.  D <= 256. */
int fs_coupling_bwd_step(const fs_coupling *f, const float *x_f, const float *g_t, float *gx_f, const float *gx_add,
                         const fs_coupling *c, const float *x, const float *params, const float *uw, const float *uh,
                         const float *ud, const float *g_lq, float *gx, float *g_params, float *g_u, void *stream);

/* fs_coupling_pair_post of layers (s, d) and fs_coupling_pair_pre of the next layers
 * (s_next, d_next: the sampling pass's next layer reads z = out, the density pass's next
 * features read x = out_d) in one launch, each row exactly as the two launches compute it.
 * D <= 256. */
int fs_coupling_pair_step(const fs_coupling *s, const float *params, const float *lad_u, const float *lq_in,
                          float *out, float *lq_out, int32_t *nan_flag, const fs_coupling *s_next, const float *uw_next,
                          const float *uh_next, const float *ud_next, float *t_next, float *out_next,
                          float *lad_u_next, const fs_coupling *d, const float *x, const float *params_d,
                          const float *uw, const float *uh, const float *ud, const float *lq_in_d, float *out_d,
                          float *lq_out_d, const fs_coupling *d_next, float *t_density_next, void *stream);

/* ------------------------------------------------------------------ */
/* Local moves (MCMC/monte_carlo.py)                                   */
/* ------------------------------------------------------------------ */

/* n_moves x MonteCarlo.particle_displacement per chain (monte_carlo.py:146-189)
 * with metropolis_acceptance_particle_move (:191-223), batched over C chains.
 * The moves are numbered step0+1 .. step0+n_moves (the driver's step counter,
 * main_algorithm_1.py:204-210); after a move whose number s satisfies
 *   s % adjust_every == 0   adjust_displacement (:375-403) runs (0: never),
 *   s % sample_every == 0   a sample() snapshot (:416-444) is written (0: never).
 * state [C][N][2] float64 (float32 values where state_is_f32[c], nullable = all
 * float64); E, W [C] running total energy / virial (update_total_energy_virial);
 * pcg [C][4] as fs_pcg64_seed, pcg_buf [C][2] = {has_uint32, uinteger}, the
 * 32-bit half numpy buffers for Generator.integers (start at {0,0});
 * max_disp [C]; attempts / accepted [C] = attempts_ / accepted_displacement
 * (shared with fs_mh_accept, monte_carlo.py:240, 296); prev_counts [C][2] =
 * previous_{attempts,accepted}_displacement (needed when adjust_every > 0).
 * samples_xy [C][S][N][2], samples_ew [C][S][2] = {total_energy, total_virial},
 * S = fs_local_samples_per_chain(step0, n_moves, sample_every), either nullable.
 * accept_log [C][n_moves] (nullable), n_accept (nullable) += accepted moves. */
int fs_local_moves(const fs_phys *p, int64_t C, int32_t N, double *state, const uint8_t *state_is_f32,
                   double *E, double *W, uint64_t *pcg, uint64_t *pcg_buf, double *max_disp,
                   int64_t *attempts, int64_t *accepted, int64_t *prev_counts, int64_t n_moves,
                   int64_t step0, int32_t adjust_every, double target_acceptance, int32_t sample_every,
                   double *samples_xy, double *samples_ew, uint8_t *accept_log,
                   unsigned long long *n_accept, void *stream);

/* fs_local_moves that does nothing unless *gate != 0 (gate: one device byte, read by
 * the kernel, so the decision needs no host round trip).  Not in the reference: the
 * Algorithm-1 testing phase (main_algorithm_1.py:375-424) runs each attempt's local
 * moves ahead of the previous big move on a second stream, on a copy of the chains that
 * assumes every chain rejects; when some chain accepted, this reruns them from the real
 * chains (flowstate.algorithm1._Speculator). */
int fs_local_moves_if(const uint8_t *gate, const fs_phys *p, int64_t C, int32_t N, double *state,
                      const uint8_t *state_is_f32, double *E, double *W, uint64_t *pcg, uint64_t *pcg_buf,
                      double *max_disp, int64_t *attempts, int64_t *accepted, int64_t *prev_counts,
                      int64_t n_moves, int64_t step0, int32_t adjust_every, double target_acceptance,
                      int32_t sample_every, double *samples_xy, double *samples_ew, uint8_t *accept_log,
                      unsigned long long *n_accept, void *stream);

/* The per-chain arrays fs_local_moves reads and writes (state [C][N][2], the rest [C],
 * pcg [C][4], pcg_buf / prev_counts [C][2]); state_is_f32, W and prev_counts nullable
 * (then skipped). */
typedef struct fs_local_chains {
    double *state;
    uint8_t *state_is_f32;
    double *E, *W;
    uint64_t *pcg, *pcg_buf;
    double *max_disp;
    int64_t *attempts, *accepted, *prev_counts;
} fs_local_chains;

/* dst := src, every array of every chain, when *gate != 0 (device byte); nothing
 * otherwise.  The fix-up step of the pipeline above. */
int fs_chains_copy_if(const uint8_t *gate, int64_t C, int32_t N, const fs_local_chains *src,
                      const fs_local_chains *dst, void *stream);

/* MonteCarlo.adjust_displacement (monte_carlo.py:375-403) for C chains, arrays
 * as in fs_local_moves. */
int fs_adjust_displacement(int64_t C, double *max_disp, const int64_t *attempts, const int64_t *accepted,
                           int64_t *prev_counts, double target_acceptance, void *stream);

/* Number of sample() snapshots moves step0+1 .. step0+n_moves produce. */
int64_t fs_local_samples_per_chain(int64_t step0, int64_t n_moves, int32_t sample_every);

/* ------------------------------------------------------------------ */
/* Analysis reductions (hybrid_NF_MCMC/utils.py)                       */
/* ------------------------------------------------------------------ */

/* np.histogram2d over centered coordinates with the given edges
 * (utils.py:488-495: edges = linspace(-B, B, nb+1) per axis, last bin
 * right-inclusive).  pos [C][N][2] float64 box coords minus `shift`;
 * hist [nb][nb] int64 accumulated (+=). */
int fs_hist2d(const double *pos, int64_t C, int32_t N, double shift, const double *edges,
              int32_t nbins, int64_t *hist, void *stream);

/* classify_particles / calculate_well_statistics (utils.py:61-141) over the
 * batched engine's live states: for each chain, all particles within 1.1*r0 of
 * the left well (A) or all within the right well (B), wells at (box/4, box/2)
 * and (3box/4, box/2) with box = 2*half_box on both axes (utils.py:105-110).
 * pos [C][N][2] float64 holds each chain's values; a chain with
 * state_is_f32[c] != 0 is classified in float32 arithmetic (its reference
 * dtype), others in float64; state_is_f32 may be NULL (all float64).
 * counts[c][0] += all_A, counts[c][1] += all_B, counts[c][2] += 1. */
int fs_well_stats(const double *pos, const uint8_t *state_is_f32, int64_t C, int32_t N, double half_box,
                  double r0, int64_t *counts, void *stream);

/* classify_particles (utils.py:104-141) + the per-configuration part of
 * calculate_well_statistics (utils.py:61-101) for M configurations
 * pos [M][N][2] (float32 if pos_is_f32, else float64; numpy's promotion of the
 * Python-float centres / radius into that dtype is reproduced):
 *   cls [M][N]  0 = 'A' (left well), 1 = 'B', 2 = 'Outside'      (nullable)
 *   state [M]   1 = all in A, 2 = all in B, 0 = neither           (nullable)
 *   avg_x [M]   np.mean(config[:, 0]) in the array dtype          (nullable) */
int fs_classify_wells(const void *pos, int pos_is_f32, int64_t M, int32_t N, double half_box, double r0,
                      uint8_t *cls, uint8_t *state, double *avg_x, void *stream);

/* Pair-distance histogram of calculate_pair_correlation (utils.py:546-556) per
 * configuration: minimum image with box 2*bound in the array dtype, all ordered
 * pairs, zero distances dropped, np.histogram over edges [nbins+1] (f64, right
 * edge inclusive).  counts [M][nbins] int32 (overwritten). */
int fs_pair_hist(const void *pos, int pos_is_f32, int64_t M, int32_t N, double bound, const double *edges,
                 int32_t nbins, int32_t *counts, void *stream);

/* g(r) = mean over the M configurations of counts[m][k] / denom[k]
 * (utils.py:558-566: per-configuration float64 ratio, pandas mean = numpy
 * pairwise sum / M).  g_r [nbins] f64. */
int fs_rdf_mean(const int32_t *counts, int64_t M, int32_t nbins, const double *denom, double *g_r, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* FLOWSTATE_H */
