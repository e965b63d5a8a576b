"""Local-move throughput: MonteCarlo.particle_displacement
batched over chains on one MI355X, the loop Algorithm 1 runs 1000x between big
moves (main_algorithm_1.py:384-390).

One launch = `--moves` local moves of each of `--chains` chains of N particles
(fs_local_moves; no adjust / sampling, as in the testing loop).  Prints one JSON
line: moves/s over the timed launches, the per-launch kernel time from HIP events,
pair evaluations/s (2(N-1) per move) and the oracle's single-core rate on a
bounded sample (the C restatement, kind "port").
"""
import argparse
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

from flowstate.MCMC import BatchedMonteCarlo, Physics, initialise_fcc  # noqa: E402


def cpu_baseline(N, init, seeds, L, budget_s):
    from oracle import physics as OP

    phys = OP.make_phys(N)
    moves, t0, done = 200, time.perf_counter(), 0
    for c in range(len(init)):
        ch = OP.LocalChain(init[c], int(seeds[c]), phys, max_disp=0.65)
        ch.local_moves(moves)
        done += moves
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": done / dt, "unit": "moves/s", "cores": 1, "kind": "port",
            "sample": f"{done // moves} chains x {moves} moves, oracle C restatement, 1 thread"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--particles", type=int, default=64)
    ap.add_argument("--chains", type=int, default=65536)
    ap.add_argument("--moves", type=int, default=1000)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--cpu-budget", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sample-every", type=int, default=0, help="sample() snapshots every k moves")
    ap.add_argument("--f32-chains", type=int, default=0, help="the first k chains hold float32 states")
    args = ap.parse_args()
    N, C = args.particles, args.chains
    base, box = initialise_fcc(num_particles=N, rho=0.03, aspect_ratio=1.0)
    L = float(box.box_size_x)
    rng = np.random.default_rng(7)
    init = np.mod(base[None] + rng.normal(0, 0.05, (C, N, 2)), L)
    seeds = np.arange(42, 42 + C, dtype=np.uint64)
    if args.f32_chains:
        init[:args.f32_chains] = init[:args.f32_chains].astype(np.float32)
    b = BatchedMonteCarlo(None, init, Physics(L, L), seeds, initial_max_displacement=0.65)
    if args.f32_chains:
        b.state_is_f32[:args.f32_chains] = 1
        b.E_old, b.W_old = b._energy_of_state()
    kw = {"sample_every": args.sample_every} if args.sample_every else {}
    for _ in range(args.warmup):
        b.local_moves(args.moves, **kw)
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    a0 = b.accepted.sum().item()
    t0 = time.perf_counter()
    for e0, e1 in evs:
        e0.record()
        b.local_moves(args.moves, **kw)
        e1.record()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    k_ms = sum(e0.elapsed_time(e1) for e0, e1 in evs) / len(evs)
    n_moves = C * args.moves * args.steps
    out = {
        "metric": "local Metropolis moves/s (particle_displacement), N=64 2D LJ + double well",
        "value": n_moves / dt, "unit": "moves/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": dt / args.steps * 1e3, "kernel_ms_per_launch": k_ms, "higher_is_better": True,
        "dtype": "f64", "data": "synthetic (FCC + jitter, float64 states)",
        "config": {"workload": f"{C} chains x {args.moves} local moves per launch, N={N}",
                   "sample_every": args.sample_every, "f32_chains": args.f32_chains},
        "pair_evals_per_s": n_moves * 2 * (N - 1) / dt,
        "acceptance_rate": (b.accepted.sum().item() - a0) / n_moves,
    }
    if not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(N, init[:256], seeds, L, args.cpu_budget)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
