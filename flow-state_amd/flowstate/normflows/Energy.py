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
