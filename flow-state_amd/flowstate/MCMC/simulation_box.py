"""SimulationBox (reference: MCMC/simulation_box.py:3-65).

Holds the box geometry.  The per-pair minimum-image arithmetic lives in the
device kernels (physics_device.h: wrap_min_image / sqdist_*); ``minimum_image``,
``compute_distance`` and ``compute_distances`` run it through ``fs_min_image``
with numpy's promotion (float32 positions stay float32, wrapped against the
np.float64 box lengths initialise_fcc makes) and return numpy values as the
reference does.  ``apply_pbc`` keeps the reference's floored modulo for host-side
bookkeeping of single positions (initialise.py).
"""
import numpy as np
import torch

from .. import _lib


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

    # ---------------------------------------------------------------- device
    def _phys(self):
        from .energy_calculator import make_phys

        return make_phys(float(self.box_size_x), float(self.box_size_y))

    def _min_image(self, p1, p2s, broadcast):
        a, b = np.asarray(p1), np.asarray(p2s)
        f32 = a.dtype == np.float32 and b.dtype == np.float32  # numpy promotion: both float32 or float64
        dt = np.float32 if f32 else np.float64
        a = torch.from_numpy(np.ascontiguousarray(a, dt).reshape(-1, 2)).cuda()
        b = torch.from_numpy(np.ascontiguousarray(b, dt).reshape(-1, 2)).cuda()
        n = b.shape[0]
        delta = torch.empty((n, 2), dtype=torch.float64, device=b.device)
        r = torch.empty(n, dtype=torch.float64, device=b.device)
        with _lib.on_device(b):
            _lib.check(_lib.load().fs_min_image(self._phys(), _lib.ptr(a), 0 if broadcast else 1, _lib.ptr(b),
                                                int(f32), n, _lib.ptr(delta), _lib.ptr(r), _lib.stream_ptr()),
                       "fs_min_image")
        return delta.cpu().numpy().astype(dt), r.cpu().numpy().astype(dt)

    def minimum_image(self, position_1, position_2, checking=False):
        """simulation_box.py:31-46: the minimum-image displacement position_1 - position_2."""
        d, _ = self._min_image(position_1, position_2, False)
        if checking:
            print("wrapped_delta =", d[0])
        return d[0]

    def compute_distance(self, position_1, position_2, checking=False):
        """simulation_box.py:48-56: np.linalg.norm of the minimum image (a numpy scalar)."""
        _, r = self._min_image(position_1, position_2, False)
        if checking:
            print("np.linalg.norm(min_image) =", r[0])
        return r[0]

    def compute_distances(self, position_1, positions_2, checking=False):
        """simulation_box.py:58-65: distances from position_1 to each row (float64 array)."""
        if len(positions_2) == 0:
            return np.zeros(0)
        _, r = self._min_image(position_1, positions_2, True)
        return r.astype(np.float64)
