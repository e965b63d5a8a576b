"""Multi-GPU sharding of independent chains.

One process per GPU (torchrun), backend "nccl" (= RCCL over xGMI).  Chains
never interact (main_algorithm_1.py:138-186 builds one MonteCarlo per chain),
so rank g owns global chains [g*C, (g+1)*C): its PCG64 seeds are
42 + global index (main_algorithm_1.py:139: seed = i + MASTER_SEED) and its
proposal-stream rows start at g*C (fs_nf_mh_step chain_offset).  A chain's
trajectory is therefore independent of the number of GPUs.  There is no
per-step collective; the only exchange is the final reduction of the density
histogram (utils.py:488-495) and the well-occupancy counters (utils.py:61-101),
which this module all-reduces (a few tens of KB: latency-bound, one call each).
"""
import numpy as np
import torch

MASTER_SEED = 42  # main_algorithm_1.py:34


def env():
    import os

    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def shard(chains_per_rank, rank, master_seed=MASTER_SEED):
    """(chain_offset, seeds) of this rank's chains."""
    c0 = rank * chains_per_rank
    seeds = np.arange(master_seed + c0, master_seed + c0 + chains_per_rank, dtype=np.uint64)
    return c0, seeds


def all_reduce_stats(hist, well_totals, group=None):
    """Sum the per-rank histogram and well counters in place over the group (no-op
    when torch.distributed is not initialised)."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(hist, group=group)
        dist.all_reduce(well_totals, group=group)
    return hist, well_totals


def free_energy(well_totals):
    """ΔF = ln(p_B / p_A) of calculate_well_statistics (utils.py:92-96), 0 if either is empty."""
    a, b, n = (int(v) for v in torch.as_tensor(well_totals).tolist())
    if n == 0 or a == 0 or b == 0:
        return 0.0
    return float(np.log((b / n) / (a / n)))
