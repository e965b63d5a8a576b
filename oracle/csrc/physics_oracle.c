/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Not part of the product.
 *
 * Plain-C restatement of the reference's NVT Lennard-Jones + double-well
 * energy, its numpy PCG64 / SeedSequence random stream and the
 * nf_big_move acceptance rule.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library, and only as the checker.
 *
 * Every function names the reference line it restates (paths relative to
 * the reference repository root).  The restatement keeps the reference's
 * evaluation ORDER, because numpy's results depend on it:
 *   - minimum image per pair, MCMC/simulation_box.py:31-46, with numpy's
 *     dtype promotion: a float32 state computes the difference in float32,
 *     the wrap in float64 (box_size_x is an np.float64, initialise.py:30)
 *     and stores the wrapped component back as float32;
 *   - |delta| = np.linalg.norm (simulation_box.py:53) = sqrt(BLAS dot):
 *     float32: fl32(fl32(t0*t0) + fl32(t1*t1));  float64: sqrt(fma(t1,t1,t0*t0))
 *     (OpenBLAS Haswell ddot; pinned against the reference in
 *     tests/test_oracle_golden.py);
 *   - per-row np.sum = numpy pairwise summation (8 accumulators for n>=8),
 *     rows accumulated into a Python float, energy_calculator.py:139-169;
 *   - the double-well sum over particles, potential.py:55-116, then .sum().
 * Transcendentals (pow, tanh, exp) come from glibc; numpy's SIMD versions can
 * differ in the last ulp, so energies are pinned to ~1e-15 relative, while
 * distances, overlap flags and cutoff (neighbour) masks are bit-exact.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off, fma() where the
 * reference's BLAS uses one).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

typedef unsigned __int128 u128;

/* ------------------------------------------------------------------ */
/* numpy pairwise summation (numpy/_core/src/umath/loops_utils.h)      */
/* ------------------------------------------------------------------ */
static double pairwise_sum(const double *a, long n)
{
    if (n < 8) {
        double res = 0.0;
        for (long i = 0; i < n; i++) res += a[i];
        return res;
    } else if (n <= 128) {
        double r[8];
        long i;
        for (int j = 0; j < 8; j++) r[j] = a[j];
        for (i = 8; i < n - (n % 8); i += 8)
            for (int j = 0; j < 8; j++) r[j] += a[i + j];
        double res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += a[i];
        return res;
    } else {
        long n2 = n / 2;
        n2 -= n2 % 8;
        return pairwise_sum(a, n2) + pairwise_sum(a + n2, n - n2);
    }
}

double oracle_pairwise_sum(const double *a, long n) { return pairwise_sum(a, n); }

/* ------------------------------------------------------------------ */
/* minimum-image distance, simulation_box.py:31-56                    */
/* ------------------------------------------------------------------ */
static double min_image_dist_f32(float ax, float ay, float bx, float by, double Lx, double Ly)
{
    float d0 = ax - bx, d1 = ay - by;              /* float32 array subtraction */
    double w0 = (double)d0 - Lx * rint((double)d0 / Lx);  /* np.float32 op np.float64 -> f64 */
    double w1 = (double)d1 - Ly * rint((double)d1 / Ly);
    float t0 = (float)w0, t1 = (float)w1;          /* stored back into the f32 array */
    float s0 = t0 * t0, s1 = t1 * t1;
    float s = s0 + s1;                             /* sdot: fl32 products, exact f64 add, fl32 */
    return (double)sqrtf(s);                       /* float32 norm stored in f64 array */
}

static double min_image_dist_f64(double ax, double ay, double bx, double by, double Lx, double Ly)
{
    double d0 = ax - bx, d1 = ay - by;
    double t0 = d0 - Lx * rint(d0 / Lx);
    double t1 = d1 - Ly * rint(d1 / Ly);
    return sqrt(fma(t1, t1, t0 * t0));             /* OpenBLAS ddot (FMA kernel) */
}

double oracle_min_image_dist(const void *pos, int dtype_f32, int i, int j, double Lx, double Ly)
{
    if (dtype_f32) {
        const float *p = (const float *)pos;
        return min_image_dist_f32(p[2 * i], p[2 * i + 1], p[2 * j], p[2 * j + 1], Lx, Ly);
    }
    const double *p = (const double *)pos;
    return min_image_dist_f64(p[2 * i], p[2 * i + 1], p[2 * j], p[2 * j + 1], Lx, Ly);
}

/* minimum_image (simulation_box.py:31-46): the wrapped displacement in the dtype */
void oracle_min_image(const void *a, const void *b, int dtype_f32, double Lx, double Ly, double delta[2])
{
    if (dtype_f32) {
        const float *p = (const float *)a, *q = (const float *)b;
        float d0 = p[0] - q[0], d1 = p[1] - q[1];
        delta[0] = (float)((double)d0 - Lx * rint((double)d0 / Lx));
        delta[1] = (float)((double)d1 - Ly * rint((double)d1 / Ly));
    } else {
        const double *p = (const double *)a, *q = (const double *)b;
        double d0 = p[0] - q[0], d1 = p[1] - q[1];
        delta[0] = d0 - Lx * rint(d0 / Lx);
        delta[1] = d1 - Ly * rint(d1 / Ly);
    }
}

/* ------------------------------------------------------------------ */
/* physics parameters                                                  */
/* ------------------------------------------------------------------ */
typedef struct {
    double Lx, Ly;       /* box, SimulationBox.box_size_x/_y                          */
    double V0[2];        /* V0_list                                                  */
    double r0, k;        /* well radius and steepness                                 */
    int num_wells;       /* 0, 1 or 2                                                */
    double r_cut;        /* 2.5   (energy_calculator.py:80)                          */
    double r_core;       /* 0.5   hard core (energy_calculator.py:150)               */
} oracle_phys;

/* lennard_jones_energy_virial, potential.py:3-29 (epsilon = sigma = 1, shift) */
static void lj_pair(double r, double r_cut, double e_cut, double *e, double *w)
{
    if (r <= r_cut) {
        double sr6 = pow(1.0 / r, 6.0);
        double sr12 = sr6 * sr6;
        *e = 4.0 * (sr12 - sr6) - e_cut;
        *w = 48.0 * (sr12 - 0.5 * sr6);
    } else {
        *e = 0.0;
        *w = 0.0;
    }
}

/* double_well_potential for one particle, potential.py:89-112 */
static double dw_particle(double x, double y, const oracle_phys *p)
{
    double V = 0.0;
    double cy = p->Ly / 2.0;
    for (int i = 0; i < p->num_wells && i < 2; i++) {
        double cx = (i == 0) ? p->Lx / 4.0 : 3.0 * p->Lx / 4.0;
        double dx = x - cx, dy = y - cy;
        dx -= p->Lx * rint(dx / p->Lx);
        dy -= p->Ly * rint(dy / p->Ly);
        double r = sqrt(dx * dx + dy * dy);
        double transition = 0.5 * (1.0 + tanh(p->k * (r - p->r0)));
        V += p->V0[i] * (1.0 - transition);
    }
    return V;
}

/*
 * EnergyCalculator.calculate_total_energy_virial, energy_calculator.py:121-203.
 * One chain: pos (N,2) row-major, float32 or float64.  Returns 1 when the hard
 * core was hit (E = W = +inf, the reference's early return at :150-153).
 * cutoff_bits (nullable): N*N bits, bit (i*N+j) set iff i<j, both rows were
 * evaluated and r_ij <= r_cut (the "neighbour" mask of potential.py:11).
 */
int oracle_total_energy(const void *pos, int dtype_f32, int N, const oracle_phys *p,
                        double *E, double *W, uint64_t *cutoff_bits)
{
    double e_row[4096], w_row[4096];
    double sr6c = pow(1.0 / p->r_cut, 6.0);
    double e_cut = 4.0 * (sr6c * sr6c - sr6c);
    double total_e = 0.0, total_w = 0.0;
    if (cutoff_bits) memset(cutoff_bits, 0, (size_t)((N * N + 63) / 64) * 8);
    for (int i = 0; i < N - 1; i++) {
        int n = N - 1 - i;
        int hit = 0;
        for (int t = 0; t < n; t++) {
            double r = oracle_min_image_dist(pos, dtype_f32, i, i + 1 + t, p->Lx, p->Ly);
            if (r < p->r_core) hit = 1;
            lj_pair(r, p->r_cut, e_cut, &e_row[t], &w_row[t]);
            if (cutoff_bits && r <= p->r_cut) {
                long bit = (long)i * N + (i + 1 + t);
                cutoff_bits[bit >> 6] |= (uint64_t)1 << (bit & 63);
            }
        }
        if (hit) {
            *E = INFINITY;
            *W = INFINITY;
            return 1;
        }
        total_e += pairwise_sum(e_row, n);
        total_w += pairwise_sum(w_row, n);
    }
    if (p->num_wells > 0) {
        double v[4096];
        for (int i = 0; i < N; i++) {
            double x, y;
            if (dtype_f32) {
                x = ((const float *)pos)[2 * i];
                y = ((const float *)pos)[2 * i + 1];
            } else {
                x = ((const double *)pos)[2 * i];
                y = ((const double *)pos)[2 * i + 1];
            }
            v[i] = dw_particle(x, y, p);
        }
        total_e += pairwise_sum(v, N);
    }
    *E = total_e;
    *W = total_w;
    return 0;
}

/* Batched convenience: C chains, contiguous (C, N, 2). */
void oracle_total_energy_batch(const void *pos, int dtype_f32, long C, int N, const oracle_phys *p,
                               double *E, double *W, uint8_t *overlap)
{
    size_t stride = (size_t)N * 2 * (dtype_f32 ? 4 : 8);
    for (long c = 0; c < C; c++) {
        int hit = oracle_total_energy((const char *)pos + stride * c, dtype_f32, N, p, &E[c], &W[c], 0);
        if (overlap) overlap[c] = (uint8_t)hit;
    }
}

/* ------------------------------------------------------------------ */
/* numpy SeedSequence (numpy/random/bit_generator.pyx) + PCG64         */
/* (numpy/random/src/pcg64/pcg64.h), the rng of monte_carlo.py:92-95  */
/* ------------------------------------------------------------------ */
#define SS_INIT_A 0x43b0d7e5u
#define SS_MULT_A 0x931e8875u
#define SS_INIT_B 0x8b51f9ddu
#define SS_MULT_B 0x58f38dedu
#define SS_MIX_L 0xca01f9ddu
#define SS_MIX_R 0x4973f715u

static uint32_t ss_hashmix(uint32_t v, uint32_t *hc)
{
    v ^= *hc;
    *hc *= SS_MULT_A;
    v *= *hc;
    v ^= v >> 16;
    return v;
}

static uint32_t ss_mix(uint32_t x, uint32_t y)
{
    uint32_t r = SS_MIX_L * x - SS_MIX_R * y;
    r ^= r >> 16;
    return r;
}

/* default_rng(seed) for a non-negative integer seed -> PCG64 {state, inc}.
 * out[0]=state_hi out[1]=state_lo out[2]=inc_hi out[3]=inc_lo */
void oracle_pcg64_seed(uint64_t seed, uint64_t out[4])
{
    uint32_t ent[2];
    int n_ent = 0;
    if (seed == 0) ent[n_ent++] = 0;
    while (seed) { ent[n_ent++] = (uint32_t)seed; seed >>= 32; }
    uint32_t pool[4];
    uint32_t hc = SS_INIT_A;
    for (int i = 0; i < 4; i++) pool[i] = ss_hashmix(i < n_ent ? ent[i] : 0u, &hc);
    for (int s = 0; s < 4; s++)
        for (int d = 0; d < 4; d++)
            if (s != d) pool[d] = ss_mix(pool[d], ss_hashmix(pool[s], &hc));
    /* entropy words beyond the pool size: none for seeds < 2^128 with pool 4 */
    uint32_t words[8];
    uint32_t hb = SS_INIT_B;
    for (int i = 0; i < 8; i++) {
        uint32_t v = pool[i & 3];
        v ^= hb;
        hb *= SS_MULT_B;
        v *= hb;
        v ^= v >> 16;
        words[i] = v;
    }
    uint64_t val[4];
    for (int i = 0; i < 4; i++) val[i] = (uint64_t)words[2 * i] | ((uint64_t)words[2 * i + 1] << 32);
    /* pcg64_set_seed: PCG_128BIT_CONSTANT(high, low); pcg_setseq_128_srandom_r */
    u128 initstate = ((u128)val[0] << 64) | val[1];
    u128 initseq = ((u128)val[2] << 64) | val[3];
    const u128 mult = ((u128)0x2360ED051FC65DA4ull << 64) | 0x4385DF649FCCF645ull;
    u128 inc = (initseq << 1) | 1u;
    u128 st = 0;
    st = st * mult + inc;
    st += initstate;
    st = st * mult + inc;
    out[0] = (uint64_t)(st >> 64);
    out[1] = (uint64_t)st;
    out[2] = (uint64_t)(inc >> 64);
    out[3] = (uint64_t)inc;
}

/* Generator.random(): step, XSL-RR output, (u64 >> 11) * 2^-53 */
double oracle_pcg64_next_double(uint64_t s[4])
{
    const u128 mult = ((u128)0x2360ED051FC65DA4ull << 64) | 0x4385DF649FCCF645ull;
    u128 st = ((u128)s[0] << 64) | s[1];
    u128 inc = ((u128)s[2] << 64) | s[3];
    st = st * mult + inc;
    s[0] = (uint64_t)(st >> 64);
    s[1] = (uint64_t)st;
    uint64_t hi = s[0], lo = s[1];
    uint64_t x = hi ^ lo;
    unsigned rot = (unsigned)(hi >> 58);
    uint64_t out = (x >> rot) | (x << ((64 - rot) & 63));
    return (double)(out >> 11) * (1.0 / 9007199254740992.0);
}

/*
 * nf_big_move acceptance, MCMC/monte_carlo.py:264-301 (reference sign):
 *   ratio = exp(-beta*(E_new-E_old) - (nll_new-nll_old));
 *   accept if ratio >= 1 without a draw, else draw u and accept iff u < ratio.
 * flags bit0: CORRECT_SIGN -> use +(nll_new-nll_old) (independence-sampler
 * detailed balance) instead of the reference's sign.
 * Batched over C chains; pcg is [C][4].  Writes accept[c] (0/1) and u[c]
 * (the draw, or -1.0 when none was taken).
 */
void oracle_mh_accept(long C, const double *E_old, const double *E_new, const double *nll_old,
                      const double *nll_new, double beta, uint64_t *pcg, int flags,
                      uint8_t *accept, double *u_out)
{
    for (long c = 0; c < C; c++) {
        double dE = E_new[c] - E_old[c];
        double dN = nll_new[c] - nll_old[c];
        double ratio_log = (flags & 1) ? (-beta * dE + dN) : (-beta * dE - dN);
        double ratio = exp(ratio_log);
        int acc;
        double u = -1.0;
        if (ratio >= 1.0) {
            acc = 1;
        } else {
            u = oracle_pcg64_next_double(&pcg[4 * c]);
            acc = u < ratio;
        }
        accept[c] = (uint8_t)acc;
        if (u_out) u_out[c] = u;
    }
}

/*
 * judge_normalizing_flow / bulk_judge_normalizing_flow (MCMC/monte_carlo.py:305-370)
 * through metropolis_acceptance_particle_move (:191-223): for chain c, proposals
 * m = 0..M-1 in order against E_ref[c]: new <= old -> accept (no draw); isinf(new)
 * -> reject (no draw); else Generator.random() < exp(-beta*(new - old)).
 * E_new is [C][M]; pcg [C][4] advanced; accept [C][M] (0/1).
 */
void oracle_metropolis_judge(long C, long M, const double *E_ref, const double *E_new, double beta,
                             uint64_t *pcg, uint8_t *accept)
{
    for (long c = 0; c < C; c++) {
        for (long m = 0; m < M; m++) {
            double en = E_new[c * M + m], eo = E_ref[c];
            int acc;
            if (en <= eo) {
                acc = 1;
            } else if (isinf(en)) {
                acc = 0;
            } else {
                double bf = exp(-beta * (en - eo));
                acc = oracle_pcg64_next_double(&pcg[4 * c]) < bf;
            }
            accept[c * M + m] = (uint8_t)acc;
        }
    }
}

/* ------------------------------------------------------------------ */
/* Local moves: MonteCarlo.particle_displacement (monte_carlo.py:146-189),  */
/* metropolis_acceptance_particle_move (:191-223), adjust_displacement     */
/* (:375-403), EnergyCalculator.calculate_particle_energy_virial           */
/* (energy_calculator.py:48-108).  RNG state per chain: u64[6] =           */
/* {state_hi, state_lo, inc_hi, inc_lo, has_uint32, uinteger} (numpy       */
/* PCG64 keeps a 32-bit half buffered for next_uint32).                    */
/* ------------------------------------------------------------------ */
static uint64_t pcg_next64(uint64_t s[6])
{
    const u128 mult = ((u128)0x2360ED051FC65DA4ull << 64) | 0x4385DF649FCCF645ull;
    u128 st = ((u128)s[0] << 64) | s[1];
    u128 inc = ((u128)s[2] << 64) | s[3];
    st = st * mult + inc;
    s[0] = (uint64_t)(st >> 64);
    s[1] = (uint64_t)st;
    uint64_t x = s[0] ^ s[1];
    unsigned rot = (unsigned)(s[0] >> 58);
    return (x >> rot) | (x << ((64 - rot) & 63));
}

static double pcg_double(uint64_t s[6]) { return (double)(pcg_next64(s) >> 11) * (1.0 / 9007199254740992.0); }

static uint32_t pcg_next32(uint64_t s[6])  /* pcg64_next32 */
{
    if (s[4]) {
        s[4] = 0;
        return (uint32_t)s[5];
    }
    uint64_t v = pcg_next64(s);
    s[4] = 1;
    s[5] = v >> 32;
    return (uint32_t)(v & 0xffffffffu);
}

/* Generator.integers(n) for 1 <= n <= 2^32: random_bounded_uint64_fill ->
 * buffered_bounded_lemire_uint32 (numpy/random/src/distributions) */
static int64_t pcg_integers(uint64_t s[6], uint64_t n)
{
    uint32_t rng = (uint32_t)(n - 1);
    if (rng == 0) return 0;
    if (rng == 0xFFFFFFFFu) return pcg_next32(s);
    uint32_t rng_excl = rng + 1;
    uint64_t m = (uint64_t)pcg_next32(s) * rng_excl;
    uint32_t leftover = (uint32_t)m;
    if (leftover < rng_excl) {
        uint32_t threshold = (UINT32_MAX - rng) % rng_excl;
        while (leftover < threshold) {
            m = (uint64_t)pcg_next32(s) * rng_excl;
            leftover = (uint32_t)m;
        }
    }
    return (int64_t)(m >> 32);
}

int64_t oracle_pcg64_integers(uint64_t s[6], uint64_t n) { return pcg_integers(s, n); }
double oracle_pcg64_double6(uint64_t s[6]) { return pcg_double(s); }

/* numpy floor remainder (npy_divmod): fmod, sign-adjusted toward the divisor */
static double np_remainder(double a, double b)
{
    double mod = fmod(a, b);
    if (mod != 0.0) {
        if ((b < 0) != (mod < 0)) mod += b;
    } else {
        mod = copysign(0.0, b);
    }
    return mod;
}

/* calculate_particle_energy_virial for particle p; positions as doubles holding
 * the reference dtype's values.  Returns 1 on the hard core (E = W = inf). */
static int particle_energy(const double *xy, int f32, int N, int p, const oracle_phys *ph, double *E, double *W)
{
    double e_row[4096], w_row[4096];
    double sr6c = pow(1.0 / ph->r_cut, 6.0);
    double e_cut = 4.0 * (sr6c * sr6c - sr6c);
    int n = 0, hit = 0;
    for (int j = 0; j < N; j++) {
        if (j == p) continue;
        double r = f32 ? min_image_dist_f32((float)xy[2 * p], (float)xy[2 * p + 1], (float)xy[2 * j],
                                            (float)xy[2 * j + 1], ph->Lx, ph->Ly)
                       : min_image_dist_f64(xy[2 * p], xy[2 * p + 1], xy[2 * j], xy[2 * j + 1], ph->Lx, ph->Ly);
        if (r < ph->r_core) hit = 1;
        lj_pair(r, ph->r_cut, e_cut, &e_row[n], &w_row[n]);
        n++;
    }
    if (hit) {
        *E = INFINITY;
        *W = INFINITY;
        return 1;
    }
    double e = pairwise_sum(e_row, n), w = pairwise_sum(w_row, n);
    if (ph->num_wells > 0) e += dw_particle(xy[2 * p], xy[2 * p + 1], ph);
    *E = e;
    *W = w;
    return 0;
}

/* One chain, n_moves local moves.  xy: (N,2) as doubles (float32 values when
 * f32); E/W: running totals; counters: attempts/accepted; every adjust_every
 * moves (0 = never) adjust_displacement with prev_* bookkeeping.
 * accept_log (nullable): per-move 0/1. */
int oracle_particle_energy(const double *xy, int f32, int N, int p, const oracle_phys *ph, double *E, double *W)
{
    return particle_energy(xy, f32, N, p, ph, E, W);
}

void oracle_local_moves(double *xy, int f32, int N, const oracle_phys *ph, double beta, uint64_t s[6],
                        double *max_disp, double target_acc, double *E, double *W, int64_t *attempts,
                        int64_t *accepted, int64_t *prev_att, int64_t *prev_acc, int n_moves, int adjust_every,
                        int adjust_phase, int8_t *accept_log)
{
    for (int t = 0; t < n_moves; t++) {
        *attempts += 1;
        int p = (int)pcg_integers(s, (uint64_t)N);
        double eno, viro, enn, virn;
        particle_energy(xy, f32, N, p, ph, &eno, &viro);
        double u0 = pcg_double(s), u1 = pcg_double(s);
        double d0 = (u0 - 0.5) * *max_disp, d1 = (u1 - 0.5) * *max_disp;
        double ox = xy[2 * p], oy = xy[2 * p + 1];
        double nx, ny;
        if (f32) {
            float fx = (float)(ox + d0), fy = (float)(oy + d1);            /* f32 row += f64 array */
            nx = (double)(float)np_remainder((double)fx, ph->Lx);         /* f32 % f64 -> f64 -> f32 */
            ny = (double)(float)np_remainder((double)fy, ph->Ly);
        } else {
            nx = np_remainder(ox + d0, ph->Lx);
            ny = np_remainder(oy + d1, ph->Ly);
        }
        xy[2 * p] = nx;
        xy[2 * p + 1] = ny;
        particle_energy(xy, f32, N, p, ph, &enn, &virn);
        double dE = enn - eno, dW = virn - viro;
        int acc;
        if (enn <= eno) acc = 1;
        else if (isinf(enn)) acc = 0;
        else acc = pcg_double(s) < exp(-beta * (enn - eno));
        if (acc) {
            *accepted += 1;
            *E += dE;
            *W += dW;
        } else {
            xy[2 * p] = ox;
            xy[2 * p + 1] = oy;
        }
        if (accept_log) accept_log[t] = (int8_t)acc;
        if (adjust_every > 0 && (t + 1 + adjust_phase) % adjust_every == 0) {
            if (*attempts > *prev_att) {
                int64_t da = *attempts - *prev_att, dc = *accepted - *prev_acc;
                double frac = da > 0 ? (double)dc / (double)da : 0.0;
                double factor = frac / target_acc;
                double nm = *max_disp * factor;
                double ratio = nm / *max_disp;
                if (ratio > 1.5) nm = *max_disp * 1.5;
                else if (ratio < 0.5) nm = *max_disp * 0.5;
                *max_disp = nm;
                *prev_att = *attempts;
                *prev_acc = *accepted;
            }
        }
    }
}
