"""initialise_fcc (reference: MCMC/initialise.py:8-116) — setup only, host side."""
import math

import numpy as np

from .simulation_box import SimulationBox


def initialise_fcc(num_particles=48, rho=0.5, aspect_ratio=1.5, visualise=False, checking=False):
    """Two-sublattice grid, the num_particles candidates closest to the box centre."""
    area = num_particles / rho
    box_size_x = np.sqrt(area * aspect_ratio)
    box_size_y = np.sqrt(area / aspect_ratio)
    sim_box = SimulationBox(box_size_x, box_size_y)
    nx = math.ceil(np.sqrt(num_particles / 2 * aspect_ratio))
    ny = math.ceil(num_particles / (2 * nx))
    dx = box_size_x / (nx - 0.5)
    dy = box_size_y / (ny - 0.5)
    cand = []
    for i in range(nx):
        for j in range(ny):
            cand.append(sim_box.apply_pbc(np.array([i * dx, j * dy])))
            cand.append(sim_box.apply_pbc(np.array([(i + 0.5) * dx, (j + 0.5) * dy])))
    cand = np.array(cand)
    center = np.array([box_size_x / 2, box_size_y / 2])
    d2 = np.sum((cand - center) ** 2, axis=1)
    return cand[np.argsort(d2)[:num_particles]], sim_box
