"""BASELINE config 2 (A1 flow, N=16, 4096 chains) at one NF-MH step per launch, as bench.py's
config2 leg runs it, for rocprofv3 --kernel-trace --stats (where the step's time goes).
Usage: python tools/config2_onestep.py [steps]"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "flow-state_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import bench  # noqa: E402
from flowstate.MCMC import BatchedMonteCarlo, Physics  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    C, N = 4096, 16
    model = bench.synthetic_model(N, torch.device("cuda"))
    init, L = bench.synthetic_states(N, C, 0)
    phys = Physics(L, L, temperature=1.0, num_wells=2, V0_list=(-10.0, -10.5), r0=1.2, k=15)
    bmc = BatchedMonteCarlo(model, init, phys, np.arange(42, 42 + C, dtype=np.uint64))
    bench.decorrelate(bmc)
    bmc.MAX_STEPS_PER_LAUNCH = 1
    bmc.step(2)
    torch.cuda.synchronize()
    for _ in range(steps):
        bmc.step(1)
    torch.cuda.synchronize()
    print("ok", steps)


if __name__ == "__main__":
    main()
