"""SimulationBox (reference: MCMC/simulation_box.py:3-65).

Holds the box geometry; the per-pair minimum-image arithmetic lives in the
energy kernel (physics_kernels.hip: dist_f32 / dist_f64).  ``apply_pbc`` keeps
the reference's floored modulo for host-side bookkeeping of single positions.
"""
import numpy as np


class SimulationBox:
    def __init__(self, box_size_x, box_size_y=None):
        if box_size_y is None:
            box_size_y = box_size_x
        self.box_size_x = box_size_x
        self.box_size_y = box_size_y
        self.volume = self.box_size_x * self.box_size_y

    def apply_pbc(self, position, checking=False):
        """simulation_box.py:19-29 (Python floored modulo)."""
        return np.array([position[0] % self.box_size_x, position[1] % self.box_size_y])
