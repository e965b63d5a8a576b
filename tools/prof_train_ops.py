"""aten-level op counts of one eager A2 training step (torch.profiler), to see which
torch ops remain around the HIP kernels (tools/prof_train_graph.py gives the graph's
kernel split)."""
import os
import sys

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


def main(batch=256, N=64):
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
    g._eager_step(x)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        g._eager_step(x)
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="count", row_limit=40, max_name_column_width=60), flush=True)


if __name__ == "__main__":
    main()
