"""Host-side profile (cProfile) of Algorithm-2 cycles at config-5 sizes after warm-up: where
the Python / ctypes time of production, the graphed epoch and the refeed goes.  Prints the
phase times and the top functions by cumulative and own time."""
import cProfile
import io
import os
import pstats
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


def main(N=64, runs=100, bs=256, cycles=6):
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
    torch.cuda.synchronize()
    t = {"production": 0.0, "training": 0.0, "refeed": 0.0}
    pr = cProfile.Profile()
    for _ in range(cycles):
        for name, fn in (("production", algo.production), ("training", algo.train), ("refeed", algo.refeed)):
            t0 = time.perf_counter()
            pr.enable()
            fn()
            pr.disable()
            torch.cuda.synchronize()
            t[name] += time.perf_counter() - t0
    print({k: round(v / cycles * 1e3, 3) for k, v in t.items()}, "ms per cycle", flush=True)
    for key in ("cumulative", "tottime"):
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats(key).print_stats(28)
        print(s.getvalue()[-6000:])


if __name__ == "__main__":
    main()
