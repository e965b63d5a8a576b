"""Algorithm-2 update-cycle throughput (BASELINE config 5; main_algorithm_2.py:393-570)
through flowstate.algorithm2: production (local moves + sample() every 10 steps) ->
one training epoch (graphed forward_kld + reverse_kld + Adam, batch 256, fresh Adam)
-> refeed (one fused NF-MH step per run), A2 flow (L=23, H=128, 2 blocks, 15 bins),
N=64, the reference's NUM_MC_RUNS = 100 and UPDATE_NUM_SAMPLES = 1000 by default.

Runs shard over ranks (torchrun, one process per GPU, RCCL): each rank owns
runs/world runs; the training set is all-gathered and the replicated model is
broadcast from rank 0 after the epoch.  Prints one JSON line on rank 0 with
cycles/s and the per-phase split (max over ranks)."""
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

from flowstate import parallel  # noqa: E402
from flowstate.algorithm2 import Algorithm2  # noqa: E402
from flowstate.MCMC import BatchedMonteCarlo, Physics, initialise_fcc  # noqa: E402
from flowstate.models import A2, build_flow, half_box  # noqa: E402
from flowstate.normflows.Energy import DoubleWellLJ  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cycles", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--runs", type=int, default=100, help="NUM_MC_RUNS over all ranks")
    ap.add_argument("--update-samples", type=int, default=1000)
    ap.add_argument("--particles", type=int, default=64)
    ap.add_argument("--backend", default="nccl")
    args = ap.parse_args()
    world, rank, local = parallel.env()
    torch.cuda.set_device(local % max(1, torch.cuda.device_count()))
    dev = torch.device("cuda", torch.cuda.current_device())
    if world > 1:
        import torch.distributed as dist

        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)
    if args.runs % world:
        raise ValueError("runs must divide over the ranks")
    N, C = args.particles, args.runs // world
    c0 = rank * C
    torch.manual_seed(0)  # same initial weights on every rank
    B = half_box(N)
    m = build_flow(N, bound=B, device="cpu", **A2)
    m.p = DoubleWellLJ(2 * N, N, 1.0, B, V0_list=[-10.0, -10.5], r0=1.2, k=15)
    m = m.to(dev)
    m.q0.device = dev
    base, box = initialise_fcc(num_particles=N, rho=0.03, aspect_ratio=1.0)
    init = np.repeat(base[None], C, 0)
    phys = Physics(box.box_size_x, box.box_size_y)
    bmc = BatchedMonteCarlo(None, init, phys, [42 + c0 + i for i in range(C)], device=dev, chain_offset=c0,
                            initial_max_displacement=0.65)
    bmc.local_moves(10 * N, adjust_every=5 * N)
    algo = Algorithm2(bmc, m, batch_size=256, alpha=1.0, sampling_frequency=10,
                      update_num_samples=args.update_samples, num_mc_runs=args.runs)
    t = np.zeros(3)

    def cycle(timed):
        ts = [time.perf_counter()]
        algo.production()
        torch.cuda.synchronize()
        ts.append(time.perf_counter())
        algo.train()
        torch.cuda.synchronize()
        ts.append(time.perf_counter())
        algo.refeed()
        torch.cuda.synchronize()
        ts.append(time.perf_counter())
        if timed:
            t[:] += np.diff(ts)

    for _ in range(args.warmup):
        cycle(False)
    if world > 1:
        import torch.distributed as dist

        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.cycles):
        cycle(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    el = torch.tensor([time.perf_counter() - t0] + list(t), dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    el = el.cpu().numpy()
    if rank == 0:
        print(json.dumps({
            "metric": "Algorithm-2 update cycles/s (production + one training epoch + refeed), A2 flow, N=64",
            "value": args.cycles / el[0], "unit": "cycles/s", "n_gpus": world, "cycles": args.cycles,
            "warmup": args.warmup, "ms_per_cycle": el[0] / args.cycles * 1e3,
            "phase_ms": {"production": el[1] / args.cycles * 1e3, "training": el[2] / args.cycles * 1e3,
                         "refeed": el[3] / args.cycles * 1e3},
            "production_steps_per_run": algo.production_runs, "training_set": int(algo.training_data.shape[0]),
            "train_batches": -(-int(algo.training_data.shape[0]) // 256),
            "last_loss": algo.loss_history[-1], "last_p_acc": algo.p_acc_history[-1],
            "dtype": "f32", "data": "synthetic (FCC start, random-init A2 flow)",
            "config": {"workload": f"A2 cycle: {args.runs} runs, UPDATE_NUM_SAMPLES={args.update_samples}, "
                                   f"L=23 H=128 blocks=2 K=15, N={N}", "parallelism": f"runs sharded over {world}"}}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
