"""ORACLE (test infrastructure only): ctypes wrapper of csrc/physics_oracle.c.

Restates MCMC/energy_calculator.py:121-203, MCMC/potential.py:3-29,55-116,
MCMC/simulation_box.py:31-65 and MCMC/monte_carlo.py:264-301 (see the C file
header for the evaluation-order details).
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "libphysics_oracle.so")
_lib = None


class Phys(ctypes.Structure):
    """Physics constants (main_algorithm_1.py:40-53, energy_calculator.py:79-80)."""

    _fields_ = [
        ("Lx", ctypes.c_double),
        ("Ly", ctypes.c_double),
        ("V0", ctypes.c_double * 2),
        ("r0", ctypes.c_double),
        ("k", ctypes.c_double),
        ("num_wells", ctypes.c_int),
        ("r_cut", ctypes.c_double),
        ("r_core", ctypes.c_double),
    ]


def make_phys(N, rho=0.03, aspect=1.0, V0=(-10.0, -10.5), r0=1.2, k=15.0, num_wells=2):
    """Box from initialise_fcc (initialise.py:27-31): L = sqrt(N/rho)."""
    area = N / rho
    Lx = float(np.sqrt(area * aspect))
    Ly = float(np.sqrt(area / aspect))
    p = Phys()
    p.Lx, p.Ly = Lx, Ly
    p.V0[0], p.V0[1] = V0
    p.r0, p.k, p.num_wells = r0, k, num_wells
    p.r_cut, p.r_core = 2.5, 0.5
    return p


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        L.oracle_total_energy.restype = ctypes.c_int
        L.oracle_total_energy.argtypes = [
            ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(Phys),
            ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double), ctypes.c_void_p]
        L.oracle_total_energy_batch.restype = None
        L.oracle_total_energy_batch.argtypes = [
            ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_int, ctypes.POINTER(Phys),
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_min_image_dist.restype = ctypes.c_double
        L.oracle_min_image_dist.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                            ctypes.c_int, ctypes.c_double, ctypes.c_double]
        L.oracle_pcg64_seed.restype = None
        L.oracle_pcg64_seed.argtypes = [ctypes.c_uint64, ctypes.c_void_p]
        L.oracle_pcg64_next_double.restype = ctypes.c_double
        L.oracle_pcg64_next_double.argtypes = [ctypes.c_void_p]
        L.oracle_mh_accept.restype = None
        L.oracle_mh_accept.argtypes = [
            ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_double, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_min_image.restype = None
        L.oracle_min_image.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_double,
                                       ctypes.c_double, ctypes.c_void_p]
        L.oracle_particle_energy.restype = ctypes.c_int
        L.oracle_particle_energy.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                             ctypes.POINTER(Phys), ctypes.POINTER(ctypes.c_double),
                                             ctypes.POINTER(ctypes.c_double)]
        L.oracle_metropolis_judge.restype = None
        L.oracle_metropolis_judge.argtypes = [ctypes.c_long, ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p]
        L.oracle_local_moves.restype = None
        L.oracle_local_moves.argtypes = [
            ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(Phys), ctypes.c_double,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_double, ctypes.c_void_p, ctypes.c_void_p,
            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
            ctypes.c_int, ctypes.c_void_p]
        L.oracle_pcg64_double6.restype = ctypes.c_double
        L.oracle_pcg64_double6.argtypes = [ctypes.c_void_p]
        L.oracle_pcg64_integers.restype = ctypes.c_int64
        L.oracle_pcg64_integers.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        L.oracle_pairwise_sum.restype = ctypes.c_double
        L.oracle_pairwise_sum.argtypes = [ctypes.c_void_p, ctypes.c_long]
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def total_energy(pos, phys, with_cutoff=False):
    """One chain, pos (N,2) float32/float64 -> (E, W, overlap[, cutoff bool (N,N)])."""
    pos = np.ascontiguousarray(pos)
    assert pos.dtype in (np.float32, np.float64) and pos.ndim == 2 and pos.shape[1] == 2
    N = pos.shape[0]
    E = ctypes.c_double()
    W = ctypes.c_double()
    bits = np.zeros((N * N + 63) // 64, dtype=np.uint64) if with_cutoff else None
    hit = lib().oracle_total_energy(_ptr(pos), int(pos.dtype == np.float32), N, ctypes.byref(phys),
                                    ctypes.byref(E), ctypes.byref(W),
                                    _ptr(bits) if with_cutoff else None)
    if with_cutoff:
        flat = np.unpackbits(bits.view(np.uint8), bitorder="little")[: N * N].astype(bool)
        return E.value, W.value, bool(hit), flat.reshape(N, N)
    return E.value, W.value, bool(hit)


def total_energy_batch(pos, phys):
    """pos (C,N,2) -> E (C,) f64, W (C,) f64, overlap (C,) u8."""
    pos = np.ascontiguousarray(pos)
    C, N, _ = pos.shape
    E = np.empty(C, np.float64)
    W = np.empty(C, np.float64)
    ov = np.empty(C, np.uint8)
    lib().oracle_total_energy_batch(_ptr(pos), int(pos.dtype == np.float32), C, N,
                                    ctypes.byref(phys), _ptr(E), _ptr(W), _ptr(ov))
    return E, W, ov


def total_energy_pairloop(pos, phys):
    """calculate_total_energy_virial exactly as the reference runs it on the CPU
    (energy_calculator.py:121-203): for each row i a Python loop over the pairs j > i
    (SimulationBox.compute_distances, simulation_box.py:31-65: per-pair minimum_image
    with np.round and np.linalg.norm), the hard-core early return (:150-153),
    lennard_jones_energy_virial on the row (potential.py:3-29) summed into Python
    floats, then the double well over all particles (potential.py:55-116).  Numpy
    scalar code, one chain per call: the timed CPU baseline of bench.py (the C
    restatement above is the parity checker)."""
    pos = np.asarray(pos)
    # the box sizes are numpy float64 in the reference (np.sqrt in initialise_fcc), so a
    # float32 state's wrap runs in float64 (numpy 2 promotion)
    Lx, Ly = np.float64(phys.Lx), np.float64(phys.Ly)
    N = pos.shape[0]
    rc = phys.r_cut
    e_cut = 4.0 * ((1.0 / rc) ** 6 * (1.0 / rc) ** 6 - (1.0 / rc) ** 6)
    E = 0.0
    W = 0.0
    for i in range(N - 1):
        others = pos[i + 1:]
        r = np.zeros(len(others))
        for j, q in enumerate(others):
            d = pos[i] - q
            d[0] -= Lx * np.round(d[0] / Lx)
            d[1] -= Ly * np.round(d[1] / Ly)
            r[j] = np.linalg.norm(d)
        if np.any(r < phys.r_core):
            return float("inf"), float("inf")
        e = np.zeros_like(r)
        w = np.zeros_like(r)
        m = r <= rc
        sr6 = (1.0 / r[m]) ** 6
        sr12 = sr6 * sr6
        e[m] = 4.0 * (sr12 - sr6)
        w[m] = 48.0 * (sr12 - 0.5 * sr6)
        e[m] -= e_cut
        E += np.sum(e)
        W += np.sum(w)
    if phys.num_wells > 0:
        x, y = pos[:, 0], pos[:, 1]
        centres = [[Lx / 4, Ly / 2]] + ([[3 * Lx / 4, Ly / 2]] if phys.num_wells == 2 else [])
        V = np.zeros_like(x, dtype=np.float64)
        for i, c in enumerate(np.array(centres)):
            dx = x - c[0]
            dy = y - c[1]
            dx -= Lx * np.round(dx / Lx)
            dy -= Ly * np.round(dy / Ly)
            rr = np.sqrt(dx ** 2 + dy ** 2)
            V += phys.V0[i] * (1 - 0.5 * (1 + np.tanh(phys.k * (rr - phys.r0))))
        E += V.sum()
    return E, W


def min_image_dist(pos, i, j, phys):
    pos = np.ascontiguousarray(pos)
    return lib().oracle_min_image_dist(_ptr(pos), int(pos.dtype == np.float32), i, j,
                                       phys.Lx, phys.Ly)


def pcg64_seed(seed):
    """default_rng(seed) state as u64[4] = state_hi, state_lo, inc_hi, inc_lo."""
    out = np.zeros(4, np.uint64)
    lib().oracle_pcg64_seed(int(seed), _ptr(out))
    return out


def pcg64_seed_many(seeds):
    return np.stack([pcg64_seed(s) for s in seeds]) if len(seeds) else np.zeros((0, 4), np.uint64)


def pcg64_next_double(state):
    """Advance state (u64[4], modified in place) and return Generator.random()."""
    assert state.dtype == np.uint64 and state.flags.c_contiguous
    return lib().oracle_pcg64_next_double(_ptr(state))


def mh_accept(E_old, E_new, nll_old, nll_new, pcg, beta=1.0, correct_sign=False):
    """Batched reference acceptance (monte_carlo.py:264-301); pcg (C,4) u64 advanced in place."""
    E_old = np.ascontiguousarray(E_old, np.float64)
    E_new = np.ascontiguousarray(E_new, np.float64)
    nll_old = np.ascontiguousarray(nll_old, np.float64)
    nll_new = np.ascontiguousarray(nll_new, np.float64)
    assert pcg.dtype == np.uint64 and pcg.flags.c_contiguous
    C = E_old.shape[0]
    acc = np.empty(C, np.uint8)
    u = np.empty(C, np.float64)
    lib().oracle_mh_accept(C, _ptr(E_old), _ptr(E_new), _ptr(nll_old), _ptr(nll_new), beta,
                           _ptr(pcg), int(bool(correct_sign)), _ptr(acc), _ptr(u))
    return acc, u


def min_image(a, b, phys):
    """SimulationBox.minimum_image (simulation_box.py:31-46) of two (2,) positions of one dtype."""
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    assert a.dtype == b.dtype and a.dtype in (np.float32, np.float64)
    d = np.empty(2, np.float64)
    lib().oracle_min_image(_ptr(a), _ptr(b), int(a.dtype == np.float32), phys.Lx, phys.Ly, _ptr(d))
    return d.astype(a.dtype)


def particle_energy(pos, p, phys):
    """EnergyCalculator.calculate_particle_energy_virial (energy_calculator.py:48-108)."""
    pos = np.ascontiguousarray(pos)
    xy = np.ascontiguousarray(pos, np.float64)
    E = ctypes.c_double()
    W = ctypes.c_double()
    lib().oracle_particle_energy(_ptr(xy), int(pos.dtype == np.float32), pos.shape[0], int(p), ctypes.byref(phys),
                                 ctypes.byref(E), ctypes.byref(W))
    return E.value, W.value


def metropolis_judge(E_ref, E_new, pcg, beta=1.0):
    """judge / bulk_judge_normalizing_flow decisions (monte_carlo.py:191-223, 305-370):
    E_ref (C,), E_new (C, M); pcg (C, 4) u64 advanced in place; returns accept (C, M) u8."""
    E_ref = np.ascontiguousarray(E_ref, np.float64).reshape(-1)
    E_new = np.ascontiguousarray(E_new, np.float64).reshape(len(E_ref), -1)
    assert pcg.dtype == np.uint64 and pcg.flags.c_contiguous and pcg.shape == (len(E_ref), 4)
    acc = np.empty(E_new.shape, np.uint8)
    lib().oracle_metropolis_judge(E_new.shape[0], E_new.shape[1], _ptr(E_ref), _ptr(E_new), beta, _ptr(pcg),
                                  _ptr(acc))
    return acc


class LocalChain:
    """One chain's local-move state, as MonteCarlo holds it (monte_carlo.py:60-95):
    particles (float64, or float32 after an accepted big move), the running
    total energy / virial, max_displacement, the attempt/accept counters and
    their adjust_displacement snapshots, and the numpy PCG64 state including the
    buffered 32-bit half (u64[6])."""

    def __init__(self, particles, seed, phys, E=None, W=None, max_disp=0.65, target=0.5, beta=1.0):
        self.xy = np.array(particles, np.float64)
        self.f32 = np.asarray(particles).dtype == np.float32
        self.phys, self.beta, self.target = phys, beta, target
        self.pcg = np.zeros(6, np.uint64)
        self.pcg[:4] = pcg64_seed(seed)
        if E is None:
            E, W, _ = total_energy(np.asarray(particles), phys)
        self.E = np.array([E], np.float64)
        self.W = np.array([W], np.float64)
        self.max_disp = np.array([max_disp], np.float64)
        self.cnt = np.zeros(4, np.int64)   # attempts, accepted, prev_attempts, prev_accepted

    @property
    def particles(self):
        return self.xy.astype(np.float32) if self.f32 else self.xy.copy()

    def local_moves(self, n, adjust_every=0, phase=0):
        """n particle_displacement calls (monte_carlo.py:146-189), with
        adjust_displacement (:375-403) after every adjust_every-th; returns the
        per-move accept flags."""
        log = np.zeros(n, np.int8)
        c = self.cnt
        lib().oracle_local_moves(_ptr(self.xy), int(self.f32), self.xy.shape[0], ctypes.byref(self.phys),
                                 self.beta, _ptr(self.pcg), _ptr(self.max_disp), self.target, _ptr(self.E),
                                 _ptr(self.W), _ptr(c[0:]), _ptr(c[1:]), _ptr(c[2:]), _ptr(c[3:]), n,
                                 adjust_every, phase, _ptr(log))
        return log

    def big_move(self, cfg, nll_old, nll_new, correct_sign=False):
        """nf_big_move (monte_carlo.py:235-301) given both NLLs: the attempt counts
        as a displacement attempt (:240); on reject the total energy is recomputed
        from the current particles (:299-301), replacing the running sum."""
        self.cnt[0] += 1
        cfg = np.asarray(cfg, np.float32)
        En, Wn, _ = total_energy(cfg, self.phys)
        pcg4 = self.pcg[None, :4].copy()   # random() never touches the 32-bit buffer
        acc, _ = mh_accept(self.E, np.array([En]), np.array([nll_old]), np.array([nll_new]), pcg4,
                           self.beta, correct_sign)
        self.pcg[:4] = pcg4[0]
        if acc[0]:
            self.xy = cfg.astype(np.float64)
            self.f32 = True
            self.cnt[1] += 1
            self.E[0], self.W[0] = En, Wn
        else:
            self.E[0], self.W[0], _ = total_energy(self.particles, self.phys)
        return bool(acc[0])


class NumpyLocalChain:
    """One MonteCarlo chain's local moves in the reference's own per-call numpy form: the
    timed CPU baseline of bench.py's Algorithm-1 regime (LocalChain, the C restatement, is
    the parity checker; tests/test_oracle_local.py shows the two bit-identical).

    particle_displacement (monte_carlo.py:146-189): rng.integers(N); the particle's energy
    before and after by calculate_particle_energy_virial (energy_calculator.py:48-119):
    np.delete of the particle, compute_distances as a Python loop of minimum_image (np.round)
    + np.linalg.norm per pair (simulation_box.py:31-65), the r < 0.5 hard core, the masked
    lennard_jones_energy_virial (potential.py:3-29) summed by np.sum, plus the particle's
    double_well_potential (potential.py:55-116); displacement (rng.random(2) - 0.5) *
    max_displacement on a copy, apply_pbc by %; the Metropolis rule (:191-223); on accept
    the running totals += the differences.  The generator is numpy's own
    np.random.default_rng(seed) (monte_carlo.py:92-95).  nf_big_move given both NLLs
    (:235-301) and sample() (:416-444) as the reference runs them."""

    def __init__(self, particles, seed, phys, max_disp=0.65, beta=1.0, target=0.5):
        self.particles = np.array(particles, np.float64)
        self.target, self.prev_attempts, self.prev_accepted = target, 0, 0
        self.N = self.particles.shape[0]
        self.Lx, self.Ly = np.float64(phys.Lx), np.float64(phys.Ly)
        self.phys, self.beta, self.max_disp = phys, beta, max_disp
        self.rng = np.random.default_rng(seed)
        self.E, self.W = total_energy_pairloop(self.particles, phys)
        self.attempts = self.accepted = 0
        rc = phys.r_cut
        self._e_cut = 4.0 * ((1.0 / rc) ** 6 * (1.0 / rc) ** 6 - (1.0 / rc) ** 6)
        self.samples = []

    def _well(self, pos):
        x, y = pos[0], pos[1]
        Lx, Ly = self.Lx, self.Ly
        centres = [[Lx / 4, Ly / 2]] + ([[3 * Lx / 4, Ly / 2]] if self.phys.num_wells == 2 else [])
        V = np.zeros(1, dtype=np.float64)
        for i, c in enumerate(np.array(centres)):
            dx = np.atleast_1d(x - c[0])
            dy = np.atleast_1d(y - c[1])
            dx -= Lx * np.round(dx / Lx)
            dy -= Ly * np.round(dy / Ly)
            r = np.sqrt(dx ** 2 + dy ** 2)
            V += self.phys.V0[i] * (1 - 0.5 * (1 + np.tanh(self.phys.k * (r - self.phys.r0))))
        return V[0]

    def particle_energy(self, positions, p):
        pos = positions[p]
        others = np.delete(positions, p, axis=0)
        r = np.zeros(len(others))
        for j, q in enumerate(others):
            d = pos - q
            d[0] -= self.Lx * np.round(d[0] / self.Lx)
            d[1] -= self.Ly * np.round(d[1] / self.Ly)
            r[j] = np.linalg.norm(d)
        if np.any(r < self.phys.r_core):
            return float("inf"), float("inf")
        e = np.zeros_like(r)
        w = np.zeros_like(r)
        m = r <= self.phys.r_cut
        sr6 = (1.0 / r[m]) ** 6
        sr12 = sr6 * sr6
        e[m] = 4.0 * (sr12 - sr6)
        w[m] = 48.0 * (sr12 - 0.5 * sr6)
        e[m] -= self._e_cut
        E, W = np.sum(e), np.sum(w)
        if self.phys.num_wells > 0:
            E += self._well(pos)
        return E, W

    def _metropolis(self, old, new):
        if new <= old:
            return True
        if np.isinf(new):
            return False
        return self.rng.random() < np.exp(-self.beta * (new - old))

    def adjust_displacement(self):
        """MonteCarlo.adjust_displacement (monte_carlo.py:375-403)."""
        if self.attempts > self.prev_attempts:
            d_att = self.attempts - self.prev_attempts
            frac = (self.accepted - self.prev_accepted) / d_att
            new = self.max_disp * (frac / self.target)
            ratio = new / self.max_disp
            if ratio > 1.5:
                new = self.max_disp * 1.5
            elif ratio < 0.5:
                new = self.max_disp * 0.5
            self.max_disp = new
            self.prev_attempts, self.prev_accepted = self.attempts, self.accepted

    def local_moves(self, n, adjust_every=0, sample_every=0, step0=0):
        """n particle_displacement calls numbered step0 + 1 .. step0 + n, with
        adjust_displacement after every adjust_every-th and sample() after every
        sample_every-th (the drivers' loops, main_algorithm_1.py:384-390).  Returns the
        per-move accept flags."""
        log = np.zeros(n, np.int8)
        for i in range(n):
            step = step0 + i + 1
            self.attempts += 1
            p = self.rng.integers(self.N)
            eno, viro = self.particle_energy(self.particles, p)
            new = self.particles.copy()
            new[p] += (self.rng.random(2) - 0.5) * self.max_disp
            new[p] = np.array([new[p][0] % self.Lx, new[p][1] % self.Ly])
            enn, virn = self.particle_energy(new, p)
            if self._metropolis(eno, enn):
                self.particles = new
                self.accepted += 1
                self.E += enn - eno
                self.W += virn - viro
                log[i] = 1
            if adjust_every and step % adjust_every == 0:
                self.adjust_displacement()
            if sample_every and step % sample_every == 0:
                area = self.Lx * self.Ly
                self.samples.append((step, self.E / self.N, self.N / area,
                                     self.N / area / self.beta + self.W / (2.0 * area), self.Lx, self.Ly,
                                     self.particles.copy()))
        return log

    def big_move(self, cfg, nll_old, nll_new):
        """nf_big_move (monte_carlo.py:235-301) given both NLLs (reference sign)."""
        self.attempts += 1
        cfg = np.asarray(cfg, np.float32)
        En, Wn = total_energy_pairloop(cfg, self.phys)
        ratio = np.exp(-self.beta * (En - self.E) - (nll_new - nll_old))
        acc = bool(ratio >= 1 or self.rng.random() < ratio)
        if acc:
            self.particles = cfg.copy()
            self.accepted += 1
            self.E, self.W = En, Wn
        else:
            self.E, self.W = total_energy_pairloop(self.particles, self.phys)
        return acc


def pcg64_integers(state6, n):
    """Generator.integers(n) (buffered 32-bit Lemire) on a u64[6] state."""
    return int(lib().oracle_pcg64_integers(_ptr(state6), int(n)))


def pcg64_random6(state6):
    """Generator.random() on a u64[6] state."""
    return float(lib().oracle_pcg64_double6(_ptr(state6)))


def pairwise_sum(a):
    a = np.ascontiguousarray(a, np.float64)
    return lib().oracle_pairwise_sum(_ptr(a), a.shape[0])


def fcc_lattice(N, rho=0.03, aspect=1.0):
    """Restatement of initialise_fcc (MCMC/initialise.py:8-116): float64 (N,2)."""
    import math
    area = N / rho
    bx = np.sqrt(area * aspect)
    by = np.sqrt(area / aspect)
    nx = math.ceil(np.sqrt(N / 2 * aspect))
    ny = math.ceil(N / (2 * nx))
    dx = bx / (nx - 0.5)
    dy = by / (ny - 0.5)
    cand = []
    for i in range(nx):
        for j in range(ny):
            a = np.array([i * dx, j * dy])
            cand.append(np.array([a[0] % bx, a[1] % by]))
            b = np.array([(i + 0.5) * dx, (j + 0.5) * dy])
            cand.append(np.array([b[0] % bx, b[1] % by]))
    cand = np.array(cand)
    center = np.array([bx / 2, by / 2])
    d2 = np.sum((cand - center) ** 2, axis=1)
    return cand[np.argsort(d2)[:N]]
