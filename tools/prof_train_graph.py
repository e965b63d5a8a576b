"""Replays of the captured A2 training step only (for rocprofv3 --kernel-trace): the
per-step kernel count and time split of GraphedTrainStep (A2 flow, N=64, batch 256)."""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "flow-state_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

from flowstate.MCMC import initialise_fcc  # noqa: E402
from flowstate.models import A2, build_flow, half_box  # noqa: E402
from flowstate.normflows.Energy import DoubleWellLJ  # noqa: E402
from flowstate.normflows.train import GraphedTrainStep  # noqa: E402


def main(replays=10, batch=256, N=64):
    dev = torch.device("cuda")
    torch.manual_seed(0)
    B = half_box(N)
    m = build_flow(N, bound=B, device="cpu", **A2)
    m.p = DoubleWellLJ(2 * N, N, 1.0, B, V0_list=[-10.0, -10.5], r0=1.2, k=15)
    m = m.to(dev)
    base, _ = initialise_fcc(num_particles=N, rho=0.03, aspect_ratio=1.0)
    rng = np.random.default_rng(3)
    data = np.mod(base[None] + rng.normal(0, 0.3, (batch, N, 2)), 2 * B) - B
    x = torch.from_numpy(data.astype(np.float32).reshape(-1, 2 * N)).to(dev)
    g = GraphedTrainStep(m, batch, lr=0.000543510751759681, weight_decay=9.5857178422352e-05, alpha=1.0, example=x)
    g.step(x)
    torch.cuda.synchronize()
    torch.cuda._sleep(1000)  # marker kernel: tools/trace_window.py summarises what follows
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(replays):
        g.step(x)
    torch.cuda.synchronize()
    print(f"graphed step: {(time.perf_counter() - t0) / replays * 1e3:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
