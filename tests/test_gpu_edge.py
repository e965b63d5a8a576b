"""Empty and minimal inputs through the drop-in APIs on the device: zero-row batches
(the reference's torch / numpy code returns empty results for them), single chains,
empty proposal lists."""
import numpy as np
import pytest
import torch

from flowstate.MCMC import BatchedMonteCarlo, MonteCarlo, Physics, SimulationBox
from flowstate.MCMC.energy_calculator import make_phys, total_energy
from flowstate.models import flow_from_state_dict
from flowstate import analysis as A
from oracle import flow as OF
from oracle import physics as OP

pytestmark = pytest.mark.gpu


def small_model(N=16):
    dims = OF.FlowDims(N=N, L=2, H=32, nb=1, K=8, B=OF.half_box(N))
    sd = OF.random_state_dict(dims, seed=3)
    return flow_from_state_dict(sd, N, bound=dims.B, L=2, H=32, nb=1, K=8), dims


def test_flow_zero_rows():
    model, dims = small_model()
    x = torch.empty((0, dims.D), device="cuda")
    assert model.log_prob(x).shape == (0,)
    z, ld = model.forward_and_log_det(x)
    assert z.shape == (0, dims.D) and ld.shape == (0,)
    z, ld = model.inverse_and_log_det(x)
    assert z.shape == (0, dims.D) and ld.shape == (0,)
    assert model.sample(0).shape == (0, dims.D)


def test_energy_and_analysis_zero_rows():
    N = 16
    L = float(np.sqrt(N / 0.03))
    E, W, ov = total_energy(torch.empty((0, N, 2), dtype=torch.float32, device="cuda"), make_phys(L, L))
    assert E.shape == W.shape == ov.shape == (0,)
    cls, state, avg = A.classify_wells(np.empty((0, N, 2), np.float32), L / 2, 1.2)
    assert cls.shape == (0, N) and state.shape == (0,)
    counts = A.pair_histograms(np.empty((0, N, 2), np.float32), L / 2, np.linspace(0, L / 2, 11))
    assert counts.shape == (0, 10)


def test_judge_and_box_empty():
    N = 16
    L = float(np.sqrt(N / 0.03))
    init = OP.fcc_lattice(N)
    bmc = BatchedMonteCarlo(None, init[None], Physics(L, L), [42])
    pcg0 = bmc.pcg.clone()
    acc, att = bmc.bulk_judge_normalizing_flow(np.empty((1, 0, N, 2), np.float32), 0.0)
    assert att == 0 and int(acc.sum()) == 0
    assert torch.equal(bmc.pcg, pcg0)
    mc = MonteCarlo(particles=init, sim_box=SimulationBox(L, L), temperature=1.0, num_particles=N, num_wells=2,
                    V0_list=[-10.0, -10.5], r0=1.2, k=15, seed=42)
    assert mc.bulk_judge_normalizing_flow([], 0.0) == (0, 0)
    assert SimulationBox(L, L).compute_distances(init[0], np.empty((0, 2))).shape == (0,)


def test_single_chain_step():
    model, dims = small_model()
    N = dims.N
    L = float(np.sqrt(N / 0.03))
    bmc = BatchedMonteCarlo(model, OP.fcc_lattice(N)[None], Physics(L, L), [42])
    for _ in range(3):
        bmc.step()
    bmc.check_errors()
    assert int(bmc.attempts.item()) == 3
