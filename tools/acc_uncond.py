"""Accuracy diagnostic (not a test): one coupling layer, identity half only (the
unconditional spline, coupling.py:91-95), HIP vs the oracle's float32 (= the
reference bit for bit) and float64: bit-equal fraction and error vs float64."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "flow-state_amd")]
from flowstate.models import flow_from_state_dict, half_box  # noqa: E402
from oracle import flow as OF  # noqa: E402

for (N, H, nb, K) in ((64, 256, 2, 32), (16, 64, 1, 8)):
    dims = OF.FlowDims(N=N, L=1, H=H, nb=nb, K=K, B=half_box(N))
    sd = OF.random_state_dict(dims, seed=7)
    sd64 = {k: (v.double() if v.is_floating_point() else v) for k, v in sd.items()}
    m = flow_from_state_dict(sd, N, 1, H, nb, K, bound=dims.B)
    g = torch.Generator().manual_seed(5)
    x = (torch.rand((4096, dims.D), generator=g) * 2 - 1) * dims.B
    lp32, lp64 = OF.layer_params(sd, 0), OF.layer_params(sd64, 0)
    h = dims.D // 2
    unroll = lambda o: torch.cat([o[:, h:], o[:, :h]], dim=1)
    idf = lp32["idf"]
    o64 = unroll(OF.coupling_density(lp64, x.double(), dims)[0])[:, idf]
    o32 = unroll(OF.coupling_density(lp32, x.clone(), dims)[0])[:, idf]
    og = unroll(m.flows[0].inverse(x.cuda())[0].cpu())[:, idf]
    # the unconditional spline alone, through the oracle's rqs on the same inputs
    ident = x[:, idf]
    u32 = OF._uncond_spline(lp32, ident.clone(), dims.B, inverse=False)[0]
    eq = (og == o32).float().mean().item()
    ulp = (og.view(torch.int32).long() - o32.view(torch.int32).long()).abs()
    print(f"N={N} K={K}: bit-equal {eq:.4f}, max ulp {ulp.max().item()}, "
          f"max|d| vs f64 gpu {(og.double() - o64).abs().max():.2e} ref32 {(o32.double() - o64).abs().max():.2e}, "
          f"mean|d| gpu {(og.double() - o64).abs().mean():.2e} ref32 {(o32.double() - o64).abs().mean():.2e}, "
          f"oracle uncond == coupling ident {bool((u32 == o32).all())}")
