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


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _states(c0, C, N, L):
    # deterministic per-GLOBAL-chain configurations, as the device chains are
    out = np.empty((C, N, 2))
    for c in range(C):
        out[c] = np.random.default_rng(1000 + c0 + c).random((N, 2)) * L
    return out


def _stats(states, L):
    B = L / 2
    edges = np.linspace(-B, B, 100)
    xy = (states - B).reshape(-1, 2)
    hist, _, _ = np.histogram2d(xy[:, 0], xy[:, 1], bins=[edges, edges])
    wells = np.array([np.sum(states[:, :, 0] < L / 2), np.sum(states[:, :, 0] >= L / 2), len(states)])
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


@pytest.mark.parametrize("world", [2])
def test_sharded_reduction_matches_single_process(world, tmp_path):
    C, N = 64, 16
    L = float(np.sqrt(N / 0.03))
    out = str(tmp_path / "red.npz")
    mp.spawn(_worker, args=(world, _free_port(), C, N, L, out), nprocs=world, join=True)
    got = np.load(out)
    want_h, want_w = _stats(_states(0, C * world, N, L), L)
    np.testing.assert_array_equal(got["hist"], want_h.numpy())
    np.testing.assert_array_equal(got["wells"], want_w.numpy())
    seeds = np.load(out + ".seeds.npy")
    np.testing.assert_array_equal(seeds, np.arange(42, 42 + C * world, dtype=np.uint64))


def test_shard_offsets():
    c0, s = parallel.shard(65536, 3)
    assert c0 == 3 * 65536 and s[0] == 42 + 3 * 65536 and len(s) == 65536


def test_free_energy():
    assert parallel.free_energy([10, 20, 100]) == pytest.approx(np.log(2.0))
    assert parallel.free_energy([0, 5, 10]) == 0.0
