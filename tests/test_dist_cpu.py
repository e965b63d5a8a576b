"""world_size-2 gloo test of the multi-GPU contract on CPU: chain sharding
(seeds / proposal-stream offsets) and the end-of-run RCCL reduction of the
density histogram and well counters (flowstate.parallel), against a single
process holding all chains."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from flowstate import parallel
from oracle import analysis as OA


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _states(c0, C, N, L):
    # deterministic per-GLOBAL-chain configurations, as the device chains are
    out = np.empty((C, N, 2))
    for c in range(C):
        g = c0 + c
        rng = np.random.default_rng(1000 + g)
        if g % 3 == 0:    # every particle inside well A (centre (L/4, L/2), radius 1.1 r0)
            out[c] = np.array([L / 4, L / 2]) + rng.uniform(-0.5, 0.5, (N, 2))
        elif g % 3 == 1:  # ... well B
            out[c] = np.array([3 * L / 4, L / 2]) + rng.uniform(-0.5, 0.5, (N, 2))
        else:
            out[c] = rng.random((N, 2)) * L
    return out


def _stats(states, L):
    B = L / 2
    edges = np.linspace(-B, B, 100)
    xy = (states - B).reshape(-1, 2)
    hist, _, _ = np.histogram2d(xy[:, 0], xy[:, 1], bins=[edges, edges])
    # the reference's classify_particles (utils.py:104-141, via the oracle): all-in-A,
    # all-in-B and samples, as BatchedMonteCarlo.well_counts accumulates them per chain
    _, state, _ = OA.classify(states, L / 2, 1.2)
    wells = np.array([np.sum(state == 1), np.sum(state == 2), len(states)])
    return torch.from_numpy(hist.astype(np.int64)), torch.from_numpy(wells.astype(np.int64))


def _worker(rank, world, port, C, N, L, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c0, seeds = parallel.shard(C, rank)
    hist, wells = _stats(_states(c0, C, N, L), L)
    parallel.all_reduce_stats(hist, wells)
    if rank == 0:
        np.savez(out_path, hist=hist.numpy(), wells=wells.numpy())
    gathered = [None] * world
    dist.all_gather_object(gathered, (c0, seeds.tolist()))
    if rank == 0:
        np.save(out_path + ".seeds.npy", np.array([s for _, ss in sorted(gathered) for s in ss], dtype=np.uint64))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_sharded_reduction_matches_single_process(world, tmp_path):
    C, N = 64, 16
    L = float(np.sqrt(N / 0.03))
    out = str(tmp_path / "red.npz")
    mp.spawn(_worker, args=(world, _free_port(), C, N, L, out), nprocs=world, join=True)
    got = np.load(out)
    want_h, want_w = _stats(_states(0, C * world, N, L), L)
    np.testing.assert_array_equal(got["hist"], want_h.numpy())
    np.testing.assert_array_equal(got["wells"], want_w.numpy())
    assert got["wells"][0] > 0 and got["wells"][1] > 0
    seeds = np.load(out + ".seeds.npy")
    np.testing.assert_array_equal(seeds, np.arange(42, 42 + C * world, dtype=np.uint64))


def test_shard_offsets():
    c0, s = parallel.shard(65536, 3)
    assert c0 == 3 * 65536 and s[0] == 42 + 3 * 65536 and len(s) == 65536


def _gather_worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    c = torch.arange(12, dtype=torch.int64).reshape(4, 3) + 100 * rank
    g = parallel.gather_chain_counters(c)
    if rank == 0:
        np.save(out_path, g.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_gather_chain_counters(tmp_path):
    out = str(tmp_path / "g.npy")
    mp.spawn(_gather_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    g = np.load(out)
    want = np.concatenate([np.arange(12).reshape(4, 3) + 100 * r for r in range(2)])
    np.testing.assert_array_equal(g, want)
    m, sem, sd = parallel.free_energy_stats(np.array([[10, 20, 100], [0, 5, 10], [5, 5, 10]]))
    dF = np.array([np.log(2.0), 0.0, 0.0])
    assert m == pytest.approx(dF.mean()) and sd == pytest.approx(dF.std())
    assert sem == pytest.approx(dF.std() / np.sqrt(3))


def test_free_energy():
    assert parallel.free_energy([10, 20, 100]) == pytest.approx(np.log(2.0))
    assert parallel.free_energy([0, 5, 10]) == 0.0


def _train_worker(rank, world, port, out_path):
    """Algorithm-2 data-parallel pieces on gloo: all-gather of per-rank training configs,
    bucketed gradient averaging, state broadcast."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from flowstate.models import build_flow

    torch.manual_seed(100 + rank)  # ranks start from different weights: broadcast must fix that
    m = build_flow(4, L=2, H=32, nb=1, K=5, bound=5.0, device="cpu")
    parallel.broadcast_state(m)
    local = torch.full((3 + rank, 4, 2), float(rank))
    allc = parallel.all_gather_configs(local)
    x = torch.rand((16, 8), generator=torch.Generator().manual_seed(7 + rank)) * 8 - 4
    m.train()
    m.forward_kld(x).backward()
    own = [p.grad.clone() for p in m.parameters() if p.grad is not None]
    parallel.allreduce_gradients(m, bucket_bytes=4096)  # many small buckets
    got = [p.grad.clone() for p in m.parameters() if p.grad is not None]
    gathered = [None] * world
    dist.all_gather_object(gathered, ([g.numpy() for g in own], [g.numpy() for g in got],
                                      [p.detach().numpy() for p in m.parameters()], allc.numpy()))
    if rank == 0:
        np.save(out_path, np.array(gathered, dtype=object), allow_pickle=True)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 8])
def test_training_collectives(world, tmp_path):
    out = str(tmp_path / "train.npy")
    mp.spawn(_train_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    ranks = np.load(out, allow_pickle=True)
    p0, c0 = ranks[0][2], ranks[0][3]
    for _, _, p, c in ranks[1:]:
        for a, b in zip(p0, p):
            np.testing.assert_array_equal(a, b)  # broadcast made the replicas identical
        np.testing.assert_array_equal(c0, c)
    own = [r[0] for r in ranks]
    for i, g0 in enumerate(ranks[0][1]):
        np.testing.assert_allclose(g0, sum(o[i] for o in own) / world, rtol=1e-5, atol=1e-7)
        for r in ranks[1:]:
            np.testing.assert_array_equal(g0, r[1][i])
    sizes = [3 + r for r in range(world)]
    assert c0.shape == (sum(sizes), 4, 2)
    off = 0
    for r, n in enumerate(sizes):
        assert (c0[off:off + n] == r).all()
        off += n
