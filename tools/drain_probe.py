"""Density-pass timing probe: the same kernel on (a) the bench's own proposals and
(b) uniform random inputs, at 1x, 2x and 4x the bench's 65536 chains (one launch each).
Separates data-dependent clock effects from the tail of the last workgroup round."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flow-state_amd"))
sys.path.insert(0, REPO)
from bench import Stepper, synthetic_model, synthetic_states  # noqa: E402
from flowstate.MCMC import BatchedMonteCarlo, Physics  # noqa: E402

N, C = 64, 65536
dev = torch.device("cuda")
model = synthetic_model(N, dev)
init, L = synthetic_states(N, C, 0)
phys = Physics(L, L)
bmc = BatchedMonteCarlo(model, init, phys, np.arange(42, 42 + C, dtype=np.uint64), device=dev)
st = Stepper(bmc)
st.step(timed=False)
torch.cuda.synchronize()
props = st.centered.clone()


def timeit(x, reps=4):
    model.log_prob(x)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        model.log_prob(x)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return ts


out = {"proposals_65536": timeit(props)}
for mult in (1, 2, 4):
    x = props.repeat(mult, 1)
    out[f"proposals_x{mult}_per65536"] = [t / mult for t in timeit(x)]
    u = (torch.rand((C * mult, 2 * N), device=dev) * 2 - 1) * 23.0
    out[f"uniform_x{mult}_per65536"] = [t / mult for t in timeit(u)]
    del x, u
print(json.dumps(out, indent=1))
