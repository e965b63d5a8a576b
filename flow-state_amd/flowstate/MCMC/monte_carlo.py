"""Per-chain MonteCarlo view (reference: MCMC/monte_carlo.py:11-444).

Keeps the reference constructor and the attributes/methods the Algorithm-1
driver touches around ``nf_big_move`` (main_algorithm_1.py:168-186, 372-422).
Each instance is a 1-chain ``BatchedMonteCarlo`` created with the chain (its
device state exists before set_nf_model, as the reference equilibrates first).
``particle_displacement`` / ``adjust_displacement`` / ``nf_big_move`` /
``judge_normalizing_flow`` / ``bulk_judge_normalizing_flow`` follow
monte_carlo.py:146-223, 375-403, 235-303 and 305-370 on the same numpy PCG64 stream as
``np.random.default_rng(seed)`` — bit-exact trajectories.  One call = one kernel
launch, so drivers with many chains should use ``BatchedMonteCarlo.local_moves``.
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
        self.target_acceptance = target_acceptance
        self.timing, self.checking, self.logger = timing, checking, logger
        if seed is None:
            seed = int(np.random.SeedSequence().generate_state(1, np.uint64)[0])
        self.seed = int(seed)
        self.device = torch.device("cuda") if device is None else torch.device(device)
        self._particles0 = np.asarray(particles)
        self.physics = Physics(sim_box.box_size_x, sim_box.box_size_y, temperature, num_wells, V0_list, r0, k)
        self.nf_model = None
        self._b = BatchedMonteCarlo(None, self._particles0[None], self.physics, [self.seed], device=self.device,
                                    state_is_f32=self._particles0.dtype == np.float32,
                                    initial_max_displacement=initial_max_displacement,
                                    target_acceptance=target_acceptance)
        self.energy_calculator = _EnergyView(self)
        self.local_samples = []
        self.testing_samples = []

    @property
    def attempts_displacement(self):
        return int(self._b.attempts.item())

    @property
    def accepted_displacement(self):
        return int(self._b.accepted.item())

    @property
    def max_displacement(self):
        return float(self._b.max_disp.item())

    @property
    def rng_state(self):
        """numpy bit_generator.state-style dict of the chain's PCG64 stream."""
        s = self._b.pcg[0].cpu().numpy().view(np.uint64)
        b = self._b.pcg_buf[0].cpu().numpy().view(np.uint64)
        return {"bit_generator": "PCG64",
                "state": {"state": (int(s[0]) << 64) | int(s[1]), "inc": (int(s[2]) << 64) | int(s[3])},
                "has_uint32": int(b[0]), "uinteger": int(b[1])}

    @property
    def particles(self):
        s = self._b.state[0].cpu().numpy()
        return s.astype(np.float32) if int(self._b.state_is_f32[0].item()) else s

    def set_nf_model(self, nf_model):
        """monte_carlo.py:229-233; the chain's device state is created here."""
        self.nf_model = nf_model
        self._b.set_model(nf_model)

    def nf_big_move(self, config):
        """monte_carlo.py:235-303: returns True if the NF proposal was accepted."""
        if self.nf_model is None:
            raise RuntimeError("set_nf_model() first")
        cfg = self._as_config(config).reshape(1, self.num_particles, 2)
        acc = self._b.nf_big_move(torch.from_numpy(cfg))  # energy and accepted state in the config's dtype
        ok = bool(acc[0].item())
        self._b.check_errors()
        return ok

    def _log(self, message, level="info"):
        """monte_carlo.py:129-146: the logger's method for `level`, else print."""
        if self.logger:
            getattr(self.logger, level if level in ("debug", "warning", "error") else "info")(message)
        else:
            print(message)

    @staticmethod
    def _as_config(config):
        cfg = np.asarray(config)
        if cfg.dtype not in (np.float32, np.float64):
            cfg = cfg.astype(np.float64)  # numpy promotes ints / Python floats to float64
        return np.ascontiguousarray(cfg)

    def metropolis_acceptance_particle_move(self, old_energy, new_energy):
        """monte_carlo.py:191-223 on the chain's PCG64 stream (a draw only when
        new_energy > old_energy and finite)."""
        acc = self._b.metropolis_judge(torch.tensor([float(old_energy)], dtype=torch.float64),
                                       torch.tensor([[float(new_energy)]], dtype=torch.float64))
        return bool(acc[0, 0].item())

    def judge_normalizing_flow(self, config):
        """monte_carlo.py:305-329: the Metropolis verdict on `config` against the current
        total energy, without accepting it (attempts_displacement += 1)."""
        cfg = self._as_config(config).reshape(1, self.num_particles, 2)
        return bool(self._b.judge_normalizing_flow(torch.from_numpy(cfg))[0].item())

    def bulk_judge_normalizing_flow(self, configs, ref_energy):
        """monte_carlo.py:331-370: (accepted_moves, attempted_moves) of `configs` judged in
        order against ref_energy; the running total energy / virial are left at the last
        configuration's, as the reference's calculator is (BatchedMonteCarlo
        .bulk_judge_normalizing_flow)."""
        cfgs = [self._as_config(c).reshape(self.num_particles, 2) for c in configs]
        M = len(cfgs)
        if M == 0:
            accepted = 0
        else:
            b = self._b
            E = torch.empty((1, M), dtype=torch.float64, device=b.device)
            W = torch.empty_like(E)
            for dt in (np.float32, np.float64):  # each configuration's energy in its own dtype
                idx = [m for m, c in enumerate(cfgs) if c.dtype == dt]
                if idx:
                    e, w = b._proposal_energies(torch.from_numpy(np.stack([cfgs[m] for m in idx])[None]), len(idx))
                    E[:, idx], W[:, idx] = e, w
            acc = b.metropolis_judge(torch.tensor([float(ref_energy)], dtype=torch.float64), E)
            accepted = int(acc.sum().item())
            b.E_old, b.W_old = E[:, -1].contiguous(), W[:, -1].contiguous()
            b._moved = True
        self._log(f"Bulk judge normalizing flow: {accepted} accepted moves out of {M} attempted moves "
                  f"(reference energy: {ref_energy:.3f}).", level="info")
        return accepted, M

    def sample(self, cycle_number):
        """monte_carlo.py:416-444."""
        e = self.energy_calculator.total_energy
        vol = self.sim_box.box_size_x * self.sim_box.box_size_y
        rho = self.num_particles / vol
        pressure = rho / self.beta + self.energy_calculator.total_virial / (2.0 * vol)
        return (cycle_number, e / self.num_particles, rho, pressure, self.sim_box.box_size_x,
                self.sim_box.box_size_y, self.particles.copy())

    def particle_displacement(self):
        """monte_carlo.py:146-189: one local Metropolis move of a random particle."""
        self._b.local_moves(1)

    def adjust_displacement(self):
        """monte_carlo.py:375-403."""
        self._b.adjust_displacement()
