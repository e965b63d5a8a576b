"""Graphed vs eager training epoch drift (tests/test_gpu_algorithm2.py::
test_config5_cycle_at_reference_sizes): the same epoch from the same start,
graphed (Algorithm2 default) and eager (graphed=False); per parameter tensor the distance
between the two results relative to the graphed update's norm.  Run once per switch setting
(FS_FOLD_BN, FS_DEFER_SPLITK, FS_LEAN_GEMM, FS_COUPLING_WAVES, FS_ADAM_EAGER_F32 ...) to see
which path raises the drift; prints one JSON line."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "flow-state_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

from flowstate.MCMC import BatchedMonteCarlo, Physics, initialise_fcc  # noqa: E402
from flowstate.algorithm2 import Algorithm2  # noqa: E402
from flowstate.models import A2, build_flow, half_box  # noqa: E402
from flowstate.normflows.Energy import DoubleWellLJ  # noqa: E402


def main():
    N, runs = 64, 100
    torch.manual_seed(0)
    B = half_box(N)
    m = build_flow(N, bound=B, device="cpu", **A2)
    m.p = DoubleWellLJ(2 * N, N, 1.0, B, V0_list=[-10.0, -10.5], r0=1.2, k=15)
    m = m.cuda()
    m.q0.device = torch.device("cuda", torch.cuda.current_device())
    base, box = initialise_fcc(num_particles=N, rho=0.03, aspect_ratio=1.0)
    bmc = BatchedMonteCarlo(None, np.repeat(base[None], runs, 0), Physics(box.box_size_x, box.box_size_y),
                            [42 + i for i in range(runs)], device="cuda", initial_max_displacement=0.65)
    bmc.local_moves(10 * N, adjust_every=5 * N)
    a = Algorithm2(bmc, m, batch_size=256, alpha=1.0, sampling_frequency=10, update_num_samples=1000)
    a.production()
    twin = build_flow(N, bound=B, device="cpu", **A2)
    twin.p = DoubleWellLJ(2 * N, N, 1.0, B, V0_list=[-10.0, -10.5], r0=1.2, k=15)
    twin = twin.cuda()
    twin.load_state_dict(m.state_dict())
    twin.q0.device = m.q0.device
    before = {k: v.detach().clone() for k, v in m.state_dict().items()}
    torch.manual_seed(5)
    loss = a.train()
    sd = m.state_dict()
    b2 = Algorithm2(type("E", (), {"C": runs})(), twin, batch_size=256, alpha=1.0, graphed=False)
    b2.training_data = a.training_data
    torch.manual_seed(5)
    loss2 = b2.train()
    worst = []
    for k, v in twin.state_dict().items():
        if "running" in k or not v.is_floating_point():
            continue
        step = (sd[k] - before[k]).norm().item()
        worst.append(((v - sd[k]).norm().item() / (step + 1e-12), k))
    worst.sort(reverse=True)
    env = {k: v for k, v in os.environ.items() if k.startswith("FS_")}
    print(json.dumps({"env": env, "loss": loss, "loss_eager": loss2, "max_drift_over_step": worst[0][0],
                      "worst": worst[:5], "median": float(np.median([w for w, _ in worst]))}))


if __name__ == "__main__":
    main()
