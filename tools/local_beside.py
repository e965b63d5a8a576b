"""A local-move launch of the Algorithm-1 regime's engine (N = 3, 10 chains, 1000 moves,
bench.algorithm1_regime's box and starts): its kernel time (HIP events) alone and with a second stream kept busy by (dens) the regime's 10-row density pass of the
A1 flow in a loop, (dens2) two such loops on two streams, (mfma) f32 matrix products on the whole chip, (mem) large device copies.
One JSON line per background."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "flow-state_amd"))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from flowstate.MCMC import BatchedMonteCarlo, Physics, initialise_low_left, initialise_low_right  # noqa: E402

N, C = 3, 10
dev = torch.device("cuda", 0)
hb = bench.half_box(N)  # the regime's engine (bench.algorithm1_regime): box 2 HALF_BOX, low-left / low-right starts
init = np.array([(initialise_low_left if i % 2 == 0 else initialise_low_right)(N, 0.03, 1.0)[0] for i in range(C)])
b = BatchedMonteCarlo(None, init, Physics(2 * hb), [42 + i for i in range(C)], initial_max_displacement=0.65)
b.local_moves(5000, adjust_every=5000, sample_every=150)
model = bench.synthetic_model(N, dev)
log_prob = model.frozen_log_prob()
err = torch.zeros(1, dtype=torch.int32, device=dev)
x10 = (torch.rand((C, 2 * N), device=dev) - 0.5) * hb
A = torch.randn((8192, 8192), device=dev)
Bm = torch.randn((8192, 8192), device=dev)
big = torch.empty(1 << 28, dtype=torch.uint8, device=dev)
big2 = torch.empty_like(big)
side = torch.cuda.Stream(device=dev)
side2 = torch.cuda.Stream(device=dev)
torch.backends.cuda.matmul.allow_tf32 = False


def background(kind, ms, stream=None):
    """Queue about `ms` of work of `kind` on the side stream."""
    if kind == "dens2":  # two density-pass loops on two streams, as the pipeline's
        background("dens", ms, side)
        background("dens", ms, side2)
        return
    with torch.cuda.stream(stream or side):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        unit = {"dens": lambda: log_prob(x10, err), "mfma": lambda: torch.mm(A, Bm),
                "mem": lambda: big2.copy_(big)}[kind]
        unit()
        e1.record()
        e1.synchronize()
        per = max(e0.elapsed_time(e1), 1e-3)
        for _ in range(int(ms / per) + 1):
            unit()


for kind in ("none", "dens", "dens2", "none"):
    ts = []
    for rep in range(6):
        torch.cuda.synchronize()
        if kind != "none":
            background(kind, 40.0)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        b.local_moves(1000, sample_every=150)
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    print(json.dumps({"background": kind, "ms_per_1000_moves": sorted(ts)[len(ts) // 2], "all": [round(t, 3) for t in ts]}),
          flush=True)
