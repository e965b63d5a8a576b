"""Algorithm-2 training throughput (main_algorithm_2.py:314-331):
one optimizer step = reverse_kld(BATCH) + forward_kld(batch) in train mode,
loss = ALPHA*forward + (1-ALPHA)*reverse (ALPHA = 1), backward, Adam; A2 flow
(L=23, H=128, 2 blocks, 15 bins), N=64, batch 256, synthetic training configs
(FCC + jitter, centred).  Also times the eval-mode proposal generation of the
refeeding phase (model.sample through the HIP kernel).  Prints one JSON line."""
import json
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


def main(steps=20, warmup=3, batch=256, N=64):
    dev = torch.device("cuda")
    torch.manual_seed(0)
    B = half_box(N)
    m = build_flow(N, bound=B, device="cpu", **A2)
    m.p = DoubleWellLJ(2 * N, N, 1.0, B, V0_list=[-10.0, -10.5], r0=1.2, k=15)
    m = m.to(dev)
    m.q0.device = dev
    base, box = initialise_fcc(num_particles=N, rho=0.03, aspect_ratio=1.0)
    rng = np.random.default_rng(3)
    data = np.mod(base[None] + rng.normal(0, 0.3, (batch * (steps + warmup), N, 2)), 2 * B) - B
    data = torch.from_numpy(data.astype(np.float32).reshape(-1, 2 * N)).to(dev)
    opt = torch.optim.Adam(m.parameters(), lr=0.000543510751759681, weight_decay=9.5857178422352e-05)
    m.train()

    def step(i):
        opt.zero_grad()
        energy_loss, _ = m.reverse_kld(batch)
        sample_loss = m.forward_kld(data[i * batch:(i + 1) * batch])
        loss = 1.0 * sample_loss + 0.0 * energy_loss
        ok = bool(~(torch.isnan(loss) | torch.isinf(loss)))
        if ok:
            loss.backward()
            opt.step()
        return loss.item(), ok

    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    losses, skipped = [], 0
    for i in range(warmup, warmup + steps):
        l, ok = step(i)
        losses.append(l)
        skipped += not ok
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    # the same loop through the captured HIP graph (flowstate.normflows.train)
    from flowstate.normflows.train import GraphedTrainStep

    # A/B: the two passes in separate launches first (its graph must be done with before the
    # paired step re-homes the BatchNorm buffers), then shared (the default)
    g = GraphedTrainStep(m, batch, lr=0.000543510751759681, weight_decay=9.5857178422352e-05, alpha=1.0,
                         example=data[:batch], paired=False)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    for i in range(warmup, warmup + steps):
        g.step(data[i * batch:(i + 1) * batch])
    torch.cuda.synchronize()
    dt_sep = time.perf_counter() - t2
    del g
    g = GraphedTrainStep(m, batch, lr=0.000543510751759681, weight_decay=9.5857178422352e-05, alpha=1.0,
                         example=data[:batch])
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    for i in range(warmup, warmup + steps):
        gl = g.step(data[i * batch:(i + 1) * batch])
    torch.cuda.synchronize()
    dtg = time.perf_counter() - t2
    # longer runs: 100 checked steps, then 100 back to back as an epoch replays them
    xb = [data[i * batch:(i + 1) * batch] for i in range(warmup, warmup + steps)]
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    for i in range(100):
        g.step(xb[i % steps])
    torch.cuda.synchronize()
    dt100 = time.perf_counter() - t2
    g.reset_nan()
    flags = []
    t2 = time.perf_counter()
    for i in range(100):
        flags.append(g.step(xb[i % steps], check=False)[1])
    torch.cuda.synchronize()
    dte = time.perf_counter() - t2
    assert not bool(torch.stack(flags).any())
    m.eval()
    with torch.no_grad():
        m.sample(8192)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(5):
            m.sample(65536)
        torch.cuda.synchronize()
        ts = (time.perf_counter() - t1) / 5
    print(json.dumps({
        "metric": "Algorithm-2 NF training steps/s (reverse_kld + forward_kld + Adam, A2 flow, N=64, batch 256; HIP-graph step)",
        "value": steps / dtg, "unit": "steps/s", "ms_per_step": dtg / steps * 1e3, "n_gpus": 1,
        "checked_100_steps_per_s": 100 / dt100, "epoch_100_steps_per_s": 100 / dte,
        "eager_steps_per_s": steps / dt, "graphed_separate_passes_steps_per_s": steps / dt_sep,
        "steps": steps, "warmup": warmup, "dtype": "f32", "data": "synthetic (FCC + jitter configs)",
        "skipped_nan_steps": skipped, "last_loss": losses[-1],
        "sampling_65536_ms": ts * 1e3, "samples_per_s": 65536 / ts,
        "config": {"workload": "A2: L=23 H=128 blocks=2 K=15, N=64, batch 256"}}))


if __name__ == "__main__":
    main()
