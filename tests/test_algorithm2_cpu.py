"""One Algorithm-2 training epoch (flowstate.algorithm2.Algorithm2.train) against the
reference's own epoch (tests/golden/train_cycle.npz: get_dataloader shuffle order, a
partial last batch, a fresh Adam, ALPHA = 1 and 0.5 with reverse_kld's base draws from
the default generator), on the CPU; and the replicated multi-rank training of the
data-parallel driver (gloo, world size 2): every rank ends with the single-process
weights."""
import os
import types

import numpy as np
import pytest
import torch

from flowstate.algorithm2 import Algorithm2
from flowstate.models import flow_from_state_dict
from flowstate.normflows.Energy import DoubleWellLJ
from oracle import flow as OF

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
DIMS = dict(L=2, H=32, nb=2, K=15)


def _model():
    dims = OF.FlowDims(N=3, B=OF.half_box(3), **DIMS)
    sd = OF.random_state_dict(dims, seed=17, final_std=0.05)
    m = flow_from_state_dict(sd, 3, bound=dims.B, device="cpu", **DIMS)
    m.p = DoubleWellLJ(dims.D, dims.N, 1.0, dims.B, V0_list=[-10.0, -10.5], r0=1.2, k=15)
    return m


def _driver(model, alpha, group=None):
    bmc = types.SimpleNamespace(C=100)  # training only: no device engine needed
    return Algorithm2(bmc, model, batch_size=256, alpha=alpha, graphed=False, group=group)


def _compare(m, f, tag, params_only=False):
    for k, v in m.state_dict().items():
        ref = torch.from_numpy(f[f"{tag}/{k}"])
        if not v.is_floating_point():
            assert torch.equal(v, ref), k
            continue
        if params_only and "running" in k:
            continue
        torch.testing.assert_close(v, ref, rtol=2e-4, atol=2e-6, msg=k)


@pytest.mark.parametrize("alpha", [1.0, 0.5])
def test_training_epoch_matches_reference(alpha):
    f = np.load(os.path.join(G, "train_cycle.npz"))
    tag = f"a{int(alpha * 10)}"
    m = _model()
    a = _driver(m, alpha)
    a.training_data = torch.tensor(f["data"], dtype=torch.float32).reshape(600, -1)
    torch.manual_seed(23)
    avg = a.train()
    np.testing.assert_allclose(avg, float(f[tag + "_avg"]), rtol=1e-5)
    _compare(m, f, tag)


def _rank(rank, world, port, out):
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        f = np.load(os.path.join(G, "train_cycle.npz"))
        m = _model()
        a = _driver(m, 1.0)
        assert a.world == world
        a.training_data = torch.tensor(f["data"], dtype=torch.float32).reshape(600, -1)
        torch.manual_seed(23 + rank)  # ranks disagree on purpose: rank 0's result wins
        if rank == 0:
            torch.manual_seed(23)
        a.train()
        torch.save({k: v.clone() for k, v in m.state_dict().items()}, os.path.join(out, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_replicated_training_two_ranks(tmp_path):
    import socket

    import torch.multiprocessing as mp

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(_rank, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    f = np.load(os.path.join(G, "train_cycle.npz"))
    sd0 = torch.load(tmp_path / "r0.pt", weights_only=True)
    sd1 = torch.load(tmp_path / "r1.pt", weights_only=True)
    for k in sd0:
        assert torch.equal(sd0[k], sd1[k]), k
    m = _model()
    m.load_state_dict(sd0)
    _compare(m, f, "a10")
