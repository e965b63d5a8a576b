"""Algorithm-1 testing loop end to end (main_algorithm_1.py:381-395) on one MI355X:
per cycle, BIG_MOVE_INTERVAL = 1000 local moves of every chain (fs_local_moves) then one
NF-proposed big move (fs_nf_mh_step with FS_MH_HYBRID: proposal pass, density pass
of the proposal, density pass of the moved state, energies, accept).  65536 chains,
N=64, A1 flow.  Prints one JSON line: big-move attempts/s, local moves/s and the
per-cycle split.  Options: --N, --C, --cycles, --interval; --single runs every big move as
one fused step (no proposal bank: BatchedMonteCarlo.MAX_STEPS_PER_LAUNCH = 1), the
comparison for small batches, where the bank is used from the second cycle on."""
import argparse
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (REPO, os.path.join(REPO, "flow-state_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

from bench import synthetic_model, synthetic_states  # noqa: E402
from flowstate import parallel  # noqa: E402
from flowstate.MCMC import BatchedMonteCarlo, Physics  # noqa: E402


def main(cycles=3, warmup=1, interval=1000, N=64, C=65536, single=False):
    dev = torch.device("cuda")
    model = synthetic_model(N, dev)
    init, L = synthetic_states(N, C, 0)
    _, seeds = parallel.shard(C, 0)
    b = BatchedMonteCarlo(model, init, Physics(L, L), seeds, device=dev, initial_max_displacement=0.65)
    if single:
        b.MAX_STEPS_PER_LAUNCH = 1
    ev = lambda: torch.cuda.Event(enable_timing=True)
    for _ in range(warmup):
        b.local_moves(interval)
        b.step()
    torch.cuda.synchronize()
    t_local = t_big = 0.0
    a0 = b.n_accept.item()
    t0 = time.perf_counter()
    for _ in range(cycles):
        e0, e1, e2 = ev(), ev(), ev()
        e0.record()
        b.local_moves(interval)
        e1.record()
        b.step()
        e2.record()
        torch.cuda.synchronize()
        t_local += e0.elapsed_time(e1)
        t_big += e1.elapsed_time(e2)
    dt = time.perf_counter() - t0
    print(json.dumps({
        "metric": f"Algorithm-1 cycles ({interval} local moves + 1 NF big move per chain), N={N}, {C} chains",
        "value": C * cycles / dt, "unit": "big-move attempts/s", "local_moves_per_s": C * cycles * interval / dt,
        "ms_per_cycle": dt / cycles * 1e3, "local_ms_per_cycle": t_local / cycles,
        "big_move_ms_per_cycle": t_big / cycles, "n_gpus": 1, "steps": cycles, "warmup": warmup,
        "big_move_acceptance": (b.n_accept.item() - a0) / (C * cycles),
        "proposal_bank_steps": 1 if single else b.steps_per_launch(),
        "dtype": "f64 local / f32 flow", "data": "synthetic (FCC + jitter, random-init A1 flow)",
        "config": {"workload": f"{C} chains x ({interval} local moves + 1 hybrid NF-MH step), N={N}, A1 flow"}}))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--N", type=int, default=64)
    ap.add_argument("--C", type=int, default=65536)
    ap.add_argument("--cycles", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--interval", type=int, default=1000)
    ap.add_argument("--single", action="store_true")
    a = ap.parse_args()
    main(a.cycles, a.warmup, a.interval, a.N, a.C, a.single)
