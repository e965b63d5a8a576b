"""UniformParticle (reference: NF/normflows/Energy/Uniform.py:4-74)."""
import torch
import torch.nn as nn


class UniformParticle(nn.Module):
    """Uniform base density on [-bound, bound]^(n_particles * n_dimension)."""

    def __init__(self, n_particles, n_dimension, bound, device="cpu"):
        super().__init__()
        self.n_particles = n_particles
        self.n_dimension = n_dimension
        self.bound = bound
        self.device = device

    def sample(self, n_sample):
        z = torch.empty((n_sample, self.n_particles, self.n_dimension), dtype=torch.float32,
                        device=self.device).uniform_(-self.bound, self.bound)
        return z.reshape(n_sample, self.n_particles * self.n_dimension)

    def forward(self, n_sample):
        return self.sample(n_sample)

    def log_prob_constant(self):
        """-D * log(2*bound) in float32, as Uniform.py:70 computes it."""
        D = self.n_particles * self.n_dimension
        return float(-D * torch.log(torch.tensor(2 * self.bound)))

    def log_prob(self, z):
        """Uniform.py:50-74 (elementwise; never on the hot path, which fuses it in-kernel)."""
        in_bounds = ((z >= -self.bound) & (z <= self.bound)).all(dim=1)
        out = torch.full((z.size(0),), self.log_prob_constant(), device=z.device, dtype=z.dtype)
        out[~in_bounds] = -float("inf")
        return out


class SimpleLJ(nn.Module):
    """Pairwise LJ energy of flow samples for reverse_kld (reference:
    NF/normflows/Energy/SimpleLJ.py:5-41): minimum image in a box of 2*bound, an
    extra particle at the origin, linear core below r = 0.82, no cutoff.  The
    reference allocates its zero row on 'cuda' unconditionally; here it follows x."""

    def __init__(self, dim, n_particles, temperature, bound):
        super().__init__()
        self._dim = dim
        self._n_particles = n_particles
        self._n_dimensions = dim // n_particles
        self.temperature = temperature
        self.bound = bound

    def _energy(self, x):
        x = x.contiguous()
        xp = x.clone().reshape(-1, self._n_particles, self._n_dimensions)
        d_norm = xp - 2 * self.bound * torch.round(xp / (self.bound * 2))
        zeros = torch.zeros((d_norm.shape[0], 1, d_norm.shape[2]), device=x.device, dtype=d_norm.dtype)
        d_norm = torch.cat((zeros, d_norm), dim=1)
        e = d_norm.unsqueeze(2)
        dist = torch.norm(e - e.transpose(1, 2), dim=-1)
        n = d_norm.size(1)
        iu = torch.triu_indices(n, n, offset=1, device=x.device)
        r = dist[:, iu[0], iu[1]]
        bk = 0.82
        en = torch.where(r <= bk, -80 * (r - bk) + 30, 4 * (pow(1 / r, 12) - pow(1 / r, 6)))
        return en.sum(dim=1) / self.temperature


class _TargetEnergy(torch.autograd.Function):
    """DoubleWellLJ._energy on the device: fs_target_energy (csrc/target_kernels.hip), one
    launch for the energy and, when x needs a gradient, dE/dx (saved for the backward,
    which is one multiply).  Replaces the ~40 torch kernels of the restatement below
    (pairwise distance matrix, triu gather, where, pow, Python-looped wells)."""

    @staticmethod
    def forward(ctx, x, mod):
        from .. import _lib

        x = x.contiguous()
        B, D = x.shape
        N = mod._n_particles
        E = torch.empty(B, dtype=torch.float32, device=x.device)
        g = torch.empty_like(x) if ctx.needs_input_grad[0] else None
        V0 = [float(v) for v in mod.V0_list.tolist()]
        with _lib.on_device(x):
            _lib.require_device(x)
            _lib.check(_lib.load().fs_target_energy(_lib.ptr(x), B, N, float(mod.bound), float(mod.temperature), 2,
                                                   V0[0], V0[1], float(mod.r0), float(mod.k), _lib.ptr(E),
                                                   _lib.ptr(g), _lib.stream_ptr()), "fs_target_energy")
        if g is not None:
            ctx.save_for_backward(g)
        return E

    @staticmethod
    @torch.autograd.function.once_differentiable
    def backward(ctx, gE):
        # dE/dx is a saved constant: a second derivative raises instead of returning zeros
        (g,) = ctx.saved_tensors
        return gE[:, None].to(g.dtype) * g, None


class DoubleWellLJ(SimpleLJ):
    """SimpleLJ + the two-well external potential (reference: Energy/SimpleLJ.py:44-130),
    wells at (-bound/2, 0) and (bound/2, 0) in the centred frame."""

    def __init__(self, dim, n_particles, temperature, bound, V0_list=None, r0=1.0, k=10.0):
        super().__init__(dim, n_particles, temperature, bound)
        if V0_list is None:
            V0_list = [-4.0, -4.0]
        self.V0_list = torch.tensor(V0_list, dtype=torch.float32)
        self.r0 = r0
        self.k = k
        self.centers = torch.tensor([[-bound / 2, 0.0], [bound / 2, 0.0]], dtype=torch.float32)

    def _on(self, device):
        """centers / V0_list on `device`, copied once (no host->device copy per call, so
        the energy can sit inside a captured HIP graph)."""
        cache = self.__dict__.setdefault("_dev_cache", {})
        key = str(device)
        if key not in cache:
            cache[key] = (self.centers.to(device), self.V0_list.to(device))
        return cache[key]

    def double_well_potential(self, positions):
        """Energy/SimpleLJ.py:63-115, vectorised over particles (the reference loops over
        them in Python; the per-particle terms are identical, the particle sum is a
        tensor reduction)."""
        L = 2 * self.bound
        centers, V0 = self._on(positions.device)
        x = positions[:, :, 0]
        y = positions[:, :, 1]
        Vp = torch.zeros_like(x)
        for i in range(centers.shape[0]):
            dx = x - centers[i, 0]
            dy = y - centers[i, 1]
            dx = dx - L * torch.round(dx / L)
            dy = dy - L * torch.round(dy / L)
            r = torch.sqrt(dx ** 2 + dy ** 2)
            transition = 0.5 * (1 + torch.tanh(self.k * (r - self.r0)))
            Vp = Vp + V0[i] * (1 - transition)
        return Vp.sum(dim=1)

    def _energy(self, x):
        """Device float32 samples of the flow's dimension: the HIP kernel (energy and
        gradient); anything else (CPU tensors, other dtypes): the torch restatement."""
        if x.is_cuda and x.dtype == torch.float32 and x.dim() == 2 and x.shape[1] == self._dim \
                and self._dim == 2 * self._n_particles and len(self.V0_list) == 2:
            return _TargetEnergy.apply(x, self)
        return self._energy_torch(x)

    def _energy_torch(self, x):
        lj = super()._energy(x)
        return lj + self.double_well_potential(x.view(x.shape[0], self._n_particles, self._n_dimensions))
