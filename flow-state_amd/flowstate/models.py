"""Builders for the flow stacks the reference drivers construct.

A1: main_algorithm_1.py:59-67,276-284 — K=15 layers, H=256, NUM_BINS=32 bins,
    and NUM_BINS passed positionally as num_blocks (32 residual blocks).
A2: main_algorithm_2.py:43-51,287-294 — 23 layers, H=128, 2 blocks, 15 bins.
"""
from .normflows import NormalizingFlow
from .normflows.Energy import UniformParticle
from .normflows.flows import CircularCoupledRationalQuadraticSpline

A1 = dict(L=15, H=256, nb=32, K=32)
A2 = dict(L=23, H=128, nb=2, K=15)


def half_box(N, rho=0.03, dim=2):
    """HALF_BOX (main_algorithm_1.py:50)."""
    return ((N / rho) ** (1 / dim)) / 2


def build_flow(N, L, H, nb, K, bound=None, device="cpu"):
    bound = half_box(N) if bound is None else bound
    base = UniformParticle(N, 2, bound, device=device)
    layers = [CircularCoupledRationalQuadraticSpline(2 * N, nb, H, range(2 * N), num_bins=K, tail_bound=bound)
              for _ in range(L)]
    return NormalizingFlow(base, layers).to(device)


def flow_from_state_dict(sd, N, L, H, nb, K, bound=None, device="cuda"):
    m = build_flow(N, L, H, nb, K, bound=bound, device="cpu")
    m.load_state_dict(sd, strict=True)
    return m.to(device).eval()
