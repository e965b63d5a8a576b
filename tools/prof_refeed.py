"""The Algorithm-2 refeed (config 5: 100 runs, A2 flow, N=64) alone, for rocprofv3
--kernel-trace: two warm cycles, then production + training, a marker kernel
(torch.cuda._sleep; tools/trace_window.py summarises what follows) and one refeed, with
the host-side split of the refeed (repack of the trained weights, the fused step)."""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "flow-state_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

from flowstate.algorithm2 import Algorithm2  # noqa: E402
from flowstate.MCMC import BatchedMonteCarlo, Physics, initialise_fcc  # noqa: E402
from flowstate.models import A2, build_flow, half_box  # noqa: E402
from flowstate.normflows.Energy import DoubleWellLJ  # noqa: E402


def main(N=64, runs=100, bs=256):
    dev = torch.device("cuda")
    torch.manual_seed(0)
    B = half_box(N)
    m = build_flow(N, bound=B, device="cpu", **A2)
    m.p = DoubleWellLJ(2 * N, N, 1.0, B, V0_list=[-10.0, -10.5], r0=1.2, k=15)
    m = m.to(dev)
    m.q0.device = dev
    base, box = initialise_fcc(num_particles=N, rho=0.03, aspect_ratio=1.0)
    bmc = BatchedMonteCarlo(None, np.repeat(base[None], runs, 0), Physics(box.box_size_x, box.box_size_y),
                            [42 + i for i in range(runs)], device=dev, initial_max_displacement=0.65)
    bmc.local_moves(10 * N, adjust_every=5 * N)
    algo = Algorithm2(bmc, m, batch_size=bs, alpha=1.0, sampling_frequency=10, update_num_samples=1000)
    for _ in range(2):
        algo.cycle()
    algo.production()
    algo.train()
    torch.cuda.synchronize()
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    m.eval()
    m.packed()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    algo.refeed()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"refeed: repack {1e3 * (t1 - t0):.2f} ms, step + acceptance {1e3 * (t2 - t1):.2f} ms", flush=True)


if __name__ == "__main__":
    main()
