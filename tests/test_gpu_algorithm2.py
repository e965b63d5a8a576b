"""Algorithm-2 update cycle on the GPU (flowstate.algorithm2): the graphed training
epoch against the reference's epoch (tests/golden/train_cycle.npz, ALPHA = 1: the
shuffle order and the partial last batch are the reference's; parameters compared as
per-tensor update norms because Adam turns float32 noise on near-zero gradients into
lr-sized steps), and a full production -> training -> refeed cycle whose refeed sees
the trained weights."""
import os

import numpy as np
import pytest
import torch

from flowstate.algorithm2 import Algorithm2
from flowstate.MCMC import BatchedMonteCarlo, Physics, initialise_low_left, initialise_low_right
from flowstate.models import flow_from_state_dict
from flowstate.normflows.Energy import DoubleWellLJ
from oracle import flow as OF
from test_algorithm2_cpu import _model

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


class _NoEngine:
    C = 100


def test_graphed_training_epoch_matches_reference():
    f = np.load(os.path.join(G, "train_cycle.npz"))
    m = _model().cuda()
    p0 = {k: v.detach().clone() for k, v in m.state_dict().items()}
    a = Algorithm2(_NoEngine(), m, batch_size=256, alpha=1.0, graphed=True)
    assert a.graphed
    a.training_data = torch.tensor(f["data"], dtype=torch.float32).reshape(600, -1).cuda()
    torch.manual_seed(23)
    avg = a.train()
    np.testing.assert_allclose(avg, float(f["a10_avg"]), rtol=1e-4)
    for k, v in m.state_dict().items():
        if "running" in k or not v.is_floating_point():
            continue  # reverse_kld's base draws (CUDA generator) only feed the BN statistics at ALPHA = 1
        ref = torch.from_numpy(f["a10/" + k]).cuda()
        moved = (ref - p0[k]).norm().item()
        assert (v - ref).norm().item() <= 3e-2 * moved + 1e-6, k


def _cycle_model():
    dims = OF.FlowDims(N=3, L=2, H=32, nb=2, K=8, B=OF.half_box(3))  # an instantiated (H, K) of the HIP passes
    sd = OF.random_state_dict(dims, seed=29, final_std=0.05)
    m = flow_from_state_dict(sd, 3, L=2, H=32, nb=2, K=8, bound=dims.B)
    m.p = DoubleWellLJ(dims.D, dims.N, 1.0, dims.B, V0_list=[-10.0, -10.5], r0=1.2, k=15)
    return m


def test_update_cycle_refeeds_with_trained_weights():
    N, runs = 3, 100
    m = _cycle_model()
    B = float(m.flows[0].tail_bound)
    init = np.array([(initialise_low_left if i % 2 == 0 else initialise_low_right)(N, 0.03, 1.0)[0]
                     for i in range(runs)])
    phys = Physics(2 * B)
    bmc = BatchedMonteCarlo(None, init, phys, [42 + i for i in range(runs)], device="cuda",
                            initial_max_displacement=0.65)
    bmc.local_moves(500, adjust_every=100)
    a = Algorithm2(bmc, m, batch_size=256, alpha=1.0, sampling_frequency=10, update_num_samples=1000)
    assert a.production_runs == 100
    torch.manual_seed(0)
    for _ in range(2):
        snap, loss, acc, p = a.cycle()
        assert snap.xy.shape == (runs, 10, N, 2)
        assert a.training_data.shape == (1000, 2 * N)
        assert np.isfinite(loss) and 0.0 <= p <= 1.0
    assert a.total_mcmc_steps == 2 * 100 * runs
    assert len(a.loss_history) == 2 and len(a.p_acc_history) == 2
    # the cached old NLL after the refeed is -log q(state) under the TRAINED weights
    fresh = _cycle_model()
    fresh.load_state_dict(m.state_dict())
    fresh.eval()
    x = (bmc.state - phys.half_width).to(torch.float32).reshape(runs, -1)
    torch.testing.assert_close(bmc.nll_old, -fresh.log_prob(x).double(), rtol=0, atol=0)
