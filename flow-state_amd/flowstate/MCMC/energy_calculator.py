"""Total LJ + double-well energy on the device (reference: MCMC/energy_calculator.py:10-203).

``total_energy`` runs fs_energy_lj_dw for a batch of configurations;
``EnergyCalculator`` keeps the reference class's attributes
(total_energy / total_virial) for one chain.
"""
import numpy as np
import torch

from .. import _lib


def make_phys(box_x, box_y, num_wells=2, V0_list=(-10.0, -10.5), r0=1.2, k=15.0, beta=1.0):
    p = _lib.Phys()
    p.Lx, p.Ly = float(box_x), float(box_y)
    v0 = list(V0_list) + [0.0] * (2 - len(V0_list))
    p.V0[0], p.V0[1] = float(v0[0]), float(v0[1])
    p.r0, p.k = float(r0), float(k)
    p.num_wells = int(num_wells)
    p.r_cut, p.r_core = 2.5, 0.5  # energy_calculator.py:80, :150
    p.beta = float(beta)
    return p


def total_energy(pos, phys, with_neighbours=False):
    """pos: device tensor (C, N, 2) float32/float64 box coordinates.
    Returns E (C,) f64, W (C,) f64, overlap (C,) u8[, nbr (C, N) u64 bitmasks].
    Runs on pos's device."""
    with _lib.on_device(pos):
        return _total_energy_here(pos, phys, with_neighbours)


def _total_energy_here(pos, phys, with_neighbours):
    _lib.require_device(pos)
    if pos.dim() != 3 or pos.shape[2] != 2 or pos.dtype not in (torch.float32, torch.float64):
        raise ValueError("pos must be (C, N, 2) float32/float64")
    pos = pos.contiguous()
    C, N, _ = pos.shape
    E = torch.empty(C, dtype=torch.float64, device=pos.device)
    W = torch.empty_like(E)
    ov = torch.empty(C, dtype=torch.uint8, device=pos.device)
    nbr = torch.empty((C, N), dtype=torch.int64, device=pos.device) if with_neighbours else None
    _lib.check(_lib.load().fs_energy_lj_dw(phys, _lib.ptr(pos), int(pos.dtype == torch.float32), C, N,
                                           _lib.ptr(E), _lib.ptr(W), _lib.ptr(ov), _lib.ptr(nbr),
                                           _lib.stream_ptr()), "fs_energy_lj_dw")
    if with_neighbours:
        return E, W, ov, nbr
    return E, W, ov


class EnergyCalculator:
    """One chain's energy bookkeeping with the reference attribute names."""

    def __init__(self, num_particles, initial_particles, simulation_box, num_wells=0, V0_list=(-4.0, -4.2),
                 r0=1.0, k=10.0, timing=True, checking=False, device="cuda"):
        self.sim_box = simulation_box
        self.num_particles = num_particles
        self.num_wells = num_wells
        self.V0_list = V0_list
        self.r0 = r0
        self.k = k
        self.device = device
        self.phys = make_phys(simulation_box.box_size_x, simulation_box.box_size_y, num_wells, V0_list, r0, k)
        self.total_energy, self.total_virial = self.calculate_total_energy_virial(initial_particles)

    def calculate_total_energy_virial(self, positions):
        """energy_calculator.py:121-203 (sets total_energy / total_virial)."""
        a = np.asarray(positions)
        t = torch.as_tensor(a.astype(a.dtype if a.dtype in (np.float32, np.float64) else np.float64),
                            device=self.device).reshape(1, self.num_particles, 2)
        E, W, _ = total_energy(t, self.phys)
        self.total_energy, self.total_virial = float(E.item()), float(W.item())
        return self.total_energy, self.total_virial

    def calculate_particle_energy_virial(self, positions, particle_index):
        """energy_calculator.py:48-108: (energy, virial) of one particle with the others
        (+inf both on a hard-core overlap); the running totals are not touched."""
        a = np.asarray(positions)
        a = a if a.dtype in (np.float32, np.float64) else a.astype(np.float64)
        t = torch.as_tensor(np.ascontiguousarray(a), device=self.device).reshape(1, self.num_particles, 2)
        part = torch.tensor([int(particle_index)], dtype=torch.int32, device=t.device)
        E = torch.empty(1, dtype=torch.float64, device=t.device)
        W = torch.empty_like(E)
        with _lib.on_device(t):
            _lib.check(_lib.load().fs_particle_energy(self.phys, _lib.ptr(t), int(t.dtype == torch.float32), 1,
                                                      self.num_particles, _lib.ptr(part), _lib.ptr(E), _lib.ptr(W),
                                                      _lib.stream_ptr()), "fs_particle_energy")
        return float(E.item()), float(W.item())

    def update_total_energy_virial(self, energy_dif, virial_dif):
        self.total_energy += energy_dif
        self.total_virial += virial_dif
