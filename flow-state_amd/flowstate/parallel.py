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


def world_size(group=None):
    """Ranks in `group` (1 without an initialised process group)."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return 1
    return dist.get_world_size(group)


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


def final_reduction(bmc, group=None, bins=100):
    """End-of-run reduction of a sharded run: the density histogram of
    the current states (utils.py:488-495) and the well-occupancy totals (utils.py:61-101)
    all-reduced over the group, and the per-chain counters (all-in-A, all-in-B, samples,
    accepted, attempts) all-gathered in rank order.  Returns (hist (bins-1, bins-1),
    wells (3,), table (world*C, 5)), all int64 on the engine's device."""
    hist = bmc.histogram2d(bins)
    per_chain = bmc.well_counts()
    wells = per_chain.sum(dim=0)
    all_reduce_stats(hist, wells, group=group)
    table = gather_chain_counters(torch.cat([per_chain, bmc.accepted[:, None], bmc.attempts[:, None]], 1),
                                  group=group)
    return hist, wells, table


def allreduce_gradients(model, group=None, bucket_bytes=64 << 20):
    """Average the gradients of `model` over the group (Algorithm 2 data-parallel
    training): gradients are flattened into buckets of at most
    bucket_bytes (A2 N=64: 42.9 MB of parameters -> one bucket; xGMI ring
    all-reduce is per-link bound, so fewer, larger calls) and all-reduced over
    RCCL.  No-op without an initialised process group."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    world = dist.get_world_size(group)
    grads = [p.grad for p in model.parameters() if p.grad is not None]
    buckets, cur, size = [], [], 0
    for g in grads:
        nbytes = g.numel() * g.element_size()
        if cur and size + nbytes > bucket_bytes:
            buckets.append(cur)
            cur, size = [], 0
        cur.append(g)
        size += nbytes
    if cur:
        buckets.append(cur)
    for bucket in buckets:
        flat = torch.cat([t.reshape(-1) for t in bucket])
        dist.all_reduce(flat, group=group)
        flat /= world
        off = 0
        for t in bucket:
            t.copy_(flat[off:off + t.numel()].view_as(t))
            off += t.numel()


def broadcast_state(model, src=0, group=None):
    """Rank `src`'s parameters and buffers (BatchNorm running statistics) to every rank."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return
    with torch.no_grad():
        for t in list(model.parameters()) + list(model.buffers()):
            dist.broadcast(t.data, src=src, group=group)


def all_gather_configs(local, group=None):
    """Concatenate every rank's new training configurations (M_r, N, 2) in rank order
    (main_algorithm_2.py:393-420, per-cycle sample collection)."""
    import torch.distributed as dist

    local = torch.as_tensor(local)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return local
    world = dist.get_world_size(group)
    n = torch.tensor([local.shape[0]], dtype=torch.int64, device=local.device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    m = int(max(int(v.item()) for v in ns))
    pad = torch.zeros((m,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[: local.shape[0]] = local
    outs = [torch.zeros_like(pad) for _ in range(world)]
    dist.all_gather(outs, pad, group=group)
    return torch.cat([o[: int(k.item())] for o, k in zip(outs, ns)], 0)


def gather_chain_counters(counters, group=None):
    """All-gather per-chain order-parameter counters (C, k) int64 — count_A, count_B, n,
    accepts, attempts (utils.py:739-747) — in rank order, so every rank
    (the driver reads rank 0) holds the (world*C, k) table."""
    import torch.distributed as dist

    counters = torch.as_tensor(counters)
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return counters
    outs = [torch.empty_like(counters) for _ in range(dist.get_world_size(group))]
    dist.all_gather(outs, counters.contiguous(), group=group)
    return torch.cat(outs, 0)


def free_energy_stats(counters):
    """Per-chain ΔF = ln(p_B / p_A) (0 unless both wells were visited, utils.py:92-96) and
    its mean / standard error / std over chains as plot_avg_free_energy reports them
    (utils.py:738-747: nanmean, nanstd / sqrt(runs))."""
    c = np.asarray(torch.as_tensor(counters).cpu().numpy(), dtype=np.float64)
    a, b, n = c[:, 0], c[:, 1], c[:, 2]
    with np.errstate(divide="ignore", invalid="ignore"):
        pa, pb = a / n, b / n
        dF = np.where((pa > 0) & (pb > 0), np.log(pb / pa), 0.0)
    return float(np.nanmean(dF)), float(np.nanstd(dF) / np.sqrt(len(dF))), float(np.nanstd(dF))


def free_energy(well_totals):
    """ΔF = ln(p_B / p_A) of calculate_well_statistics (utils.py:92-96), 0 if either is empty."""
    a, b, n = (int(v) for v in torch.as_tensor(well_totals).tolist())
    if n == 0 or a == 0 or b == 0:
        return 0.0
    return float(np.log((b / n) / (a / n)))
