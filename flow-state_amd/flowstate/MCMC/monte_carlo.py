"""Per-chain MonteCarlo view (reference: MCMC/monte_carlo.py:11-444).

Keeps the reference constructor and the attributes/methods the Algorithm-1
driver touches around ``nf_big_move`` (main_algorithm_1.py:168-186, 372-422).
Each instance is a 1-chain ``BatchedMonteCarlo``; ``nf_big_move(config)``
returns a bool exactly like monte_carlo.py:235-303 (reference acceptance sign,
same PCG64 stream as ``np.random.default_rng(seed)``).  Local moves
(``particle_displacement``) are the next row of SURVEY §8(f) and raise here.
"""
import numpy as np
import torch

from .batched import BatchedMonteCarlo, Physics


class _EnergyView:
    """energy_calculator attribute of the reference MonteCarlo."""

    def __init__(self, mc):
        self._mc = mc

    @property
    def total_energy(self):
        return float(self._mc._b.E_old.item())

    @property
    def total_virial(self):
        return float(self._mc._b.W_old.item())


class MonteCarlo:
    def __init__(self, particles, sim_box, temperature, num_particles, num_wells=0, V0_list=(-0.5, -0.5), r0=1.0,
                 k=10, initial_max_displacement=0.5, target_acceptance=0.5, timing=False, checking=False,
                 logger=None, seed=None, device=None):
        self.sim_box = sim_box
        self.half_width = sim_box.box_size_x / 2
        self.beta = 1.0 / temperature
        self.num_particles = num_particles
        self.num_wells, self.V0_list, self.r0, self.k = num_wells, V0_list, r0, k
        self.max_displacement = initial_max_displacement
        self.target_acceptance = target_acceptance
        self.timing, self.checking, self.logger = timing, checking, logger
        if seed is None:
            seed = int(np.random.SeedSequence().generate_state(1, np.uint64)[0])
        self.seed = int(seed)
        self.device = torch.device("cuda") if device is None else torch.device(device)
        self._particles0 = np.asarray(particles)
        self.physics = Physics(sim_box.box_size_x, sim_box.box_size_y, temperature, num_wells, V0_list, r0, k)
        self.nf_model = None
        self._b = None
        self.energy_calculator = _EnergyView(self)
        self.local_samples = []
        self.testing_samples = []

    @property
    def attempts_displacement(self):
        return int(self._b.attempts.item()) if self._b is not None else 0

    @property
    def accepted_displacement(self):
        return int(self._b.accepted.item()) if self._b is not None else 0

    @property
    def particles(self):
        if self._b is None:
            return self._particles0
        s = self._b.state[0].cpu().numpy()
        return s.astype(np.float32) if int(self._b.state_is_f32[0].item()) else s

    def set_nf_model(self, nf_model):
        """monte_carlo.py:229-233; the chain's device state is created here."""
        self.nf_model = nf_model
        self._b = BatchedMonteCarlo(nf_model, self._particles0[None], self.physics, [self.seed], device=self.device,
                                    state_is_f32=self._particles0.dtype == np.float32)

    def nf_big_move(self, config):
        """monte_carlo.py:235-303: returns True if the NF proposal was accepted."""
        if self._b is None:
            raise RuntimeError("set_nf_model() first")
        cfg = np.asarray(config, dtype=np.float32).reshape(1, self.num_particles, 2)
        acc = self._b.nf_big_move(torch.from_numpy(cfg))
        return bool(acc[0].item())

    def sample(self, cycle_number):
        """monte_carlo.py:416-444."""
        e = self.energy_calculator.total_energy
        vol = self.sim_box.box_size_x * self.sim_box.box_size_y
        rho = self.num_particles / vol
        pressure = rho / self.beta + self.energy_calculator.total_virial / (2.0 * vol)
        return (cycle_number, e / self.num_particles, rho, pressure, self.sim_box.box_size_x,
                self.sim_box.box_size_y, self.particles.copy())

    def particle_displacement(self):
        raise NotImplementedError("local moves (monte_carlo.py:146-189) are the next hot-path row (SURVEY §8(f))")

    def adjust_displacement(self):
        raise NotImplementedError("local moves (monte_carlo.py:375-403) are the next hot-path row (SURVEY §8(f))")
