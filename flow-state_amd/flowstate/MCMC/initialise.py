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


def _initialise_low(num_particles, rho, aspect_ratio, centre_frac):
    """A grid of 1..12 particles around (centre_frac * Lx, Ly / 2): ceil(sqrt(n)) columns,
    spacing 1.5 or less so that the grid spans at most half the box width and the box
    height, filled row by row and wrapped with apply_pbc (initialise.py:118-210)."""
    if num_particles < 1 or num_particles > 12:
        raise ValueError("Number of particles for low initialization must be between 1 and 12.")
    area = num_particles / rho
    box_size_x = np.sqrt(area * aspect_ratio)
    box_size_y = np.sqrt(area / aspect_ratio)
    sim_box = SimulationBox(box_size_x, box_size_y)
    cx, cy = centre_frac * box_size_x, box_size_y / 2
    if num_particles == 1:
        return np.array([[cx, cy]]), sim_box
    cols = int(np.ceil(np.sqrt(num_particles)))
    rows = int(np.ceil(num_particles / cols))
    sx = box_size_x / (2 * (cols - 1)) if cols > 1 else float("inf")
    sy = box_size_y / (rows - 1) if rows > 1 else float("inf")
    step = min(1.5, sx, sy)
    x0 = cx - (cols - 1) * step / 2
    y0 = cy - (rows - 1) * step / 2
    pts = [sim_box.apply_pbc(np.array([x0 + (k % cols) * step, y0 + (k // cols) * step]))
           for k in range(num_particles)]
    return np.array(pts), sim_box


def initialise_low_left(num_particles=2, rho=0.5, aspect_ratio=1.0, visualise=False, checking=False):
    """Even runs of Algorithm 1 start in the left well (main_algorithm_1.py:150-157)."""
    return _initialise_low(num_particles, rho, aspect_ratio, 0.25)


def initialise_low_right(num_particles=2, rho=0.5, aspect_ratio=1.0, visualise=False, checking=False):
    """Odd runs start in the right well (main_algorithm_1.py:158-165; initialise.py:213-305)."""
    return _initialise_low(num_particles, rho, aspect_ratio, 0.75)
