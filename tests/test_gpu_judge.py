"""GPU parity of the Metropolis judge API (fs_metropolis_judge):
MonteCarlo.judge_normalizing_flow / bulk_judge_normalizing_flow /
metropolis_acceptance_particle_move (MCMC/monte_carlo.py:191-223, 305-370).

1. The reference's own traces (tests/golden/judge_trace.npz) replayed through the
   drop-in per-chain MonteCarlo: identical verdicts, running energies (1e-12),
   attempt counters, final states and PCG64 states — including the nf_big_move
   after a bulk judge, whose ratio uses the stale running energy bulk leaves.
2. The batched judge on many chains against the oracle's restatement
   (oracle_metropolis_judge) with each chain's own PCG64 stream.
"""
import os

import numpy as np
import pytest
import torch

from flowstate.MCMC import BatchedMonteCarlo, MonteCarlo, Physics, SimulationBox
from flowstate.models import flow_from_state_dict
from oracle import flow as OF
from oracle import physics as OP

pytestmark = pytest.mark.gpu
G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _close(a, b):
    return (np.isinf(a) and np.isinf(b)) or abs(a - b) <= 1e-12 * max(1.0, abs(b))


@pytest.mark.parametrize("N", [16, 64])
def test_reference_judge_traces_replay(N):
    f = np.load(os.path.join(G, "judge_trace.npz"))
    dims = OF.FlowDims(N=N, L=2, H=32, nb=1, K=8, B=OF.half_box(N))
    sd = OF.random_state_dict(dims, seed=int(f[f"N{N}_flow_seed"]))
    model = flow_from_state_dict(sd, N, bound=dims.B, L=2, H=32, nb=1, K=8)
    L = 2 * OF.half_box(N)
    for c in range(int(f[f"N{N}_chains"])):
        k = f"N{N}_c{c}"
        mc = MonteCarlo(particles=f[k + "_init"], sim_box=SimulationBox(L, L), temperature=1.0, num_particles=N,
                        num_wells=2, V0_list=[-10.0, -10.5], r0=1.2, k=15, initial_max_displacement=0.65,
                        target_acceptance=0.5, seed=42 + c)
        mc.set_nf_model(model)
        off = 0
        cfgs = f[k + "_cfgs"]
        for i, (kind, is32, M, a, b) in enumerate(f[k + "_ops"]):
            M = int(M)
            xs = cfgs[off:off + M].astype(np.float32 if is32 else np.float64)
            off += M
            if kind == 0:
                r = float(mc.judge_normalizing_flow(xs[0]))
            elif kind == 1:
                r = float(mc.metropolis_acceptance_particle_move(a, b))
            elif kind == 2:
                acc, att = mc.bulk_judge_normalizing_flow(list(xs), a)
                assert att == M
                r = float(acc)
            else:
                r = float(mc.nf_big_move(xs[0]))
            assert r == f[k + "_result"][i], (k, i, kind)
            assert _close(mc.energy_calculator.total_energy, f[k + "_E"][i]), (k, i)
            assert _close(mc.energy_calculator.total_virial, f[k + "_W"][i]), (k, i)
            assert mc.attempts_displacement == f[k + "_attempts"][i]
        st = mc._b.pcg[0].cpu().numpy().view(np.uint64)
        np.testing.assert_array_equal(st, f[k + "_pcg_state"])
        np.testing.assert_array_equal(np.asarray(mc.particles, np.float64), f[k + "_final"])
        assert (np.asarray(mc.particles).dtype == np.float32) == bool(f[k + "_final_f32"])


def test_batched_bulk_judge_matches_oracle():
    N, C, M = 16, 2048, 7
    L = float(np.sqrt(N / 0.03))
    rng = np.random.default_rng(3)
    init = np.mod(OP.fcc_lattice(N)[None] + rng.normal(0, 0.05, (C, N, 2)), L)
    bmc = BatchedMonteCarlo(None, init, Physics(L, L), np.arange(42, 42 + C, dtype=np.uint64))
    props = np.mod(init[:, None] + rng.normal(0, 0.2, (C, M, N, 2)), L).astype(np.float32)
    props[::5, 3, 1] = props[::5, 3, 0]  # overlaps: rejected without a draw
    E0 = bmc.E_old.cpu().numpy().copy()
    ref = E0 - rng.uniform(-0.5, 1.0, C)
    pcg0 = bmc.pcg.cpu().numpy().view(np.uint64).copy()
    acc, att = bmc.bulk_judge_normalizing_flow(torch.from_numpy(props), torch.from_numpy(ref))
    assert att == M
    E_new = OP.total_energy_batch(props.reshape(C * M, N, 2), OP.make_phys(N))[0].reshape(C, M)
    acc_o = OP.metropolis_judge(ref, E_new, pcg0)
    np.testing.assert_array_equal(acc.cpu().numpy(), acc_o.sum(1))
    np.testing.assert_array_equal(bmc.pcg.cpu().numpy().view(np.uint64), pcg0)
    # the running energy is left at each chain's last proposal (energy_calculator.py:121-203)
    np.testing.assert_allclose(bmc.E_old.cpu().numpy(), E_new[:, -1], rtol=1e-12)
    # judge_normalizing_flow: one proposal each against the running energy, nothing kept
    pcg1 = pcg0.copy()
    one = props[:, 0]
    a1 = bmc.judge_normalizing_flow(torch.from_numpy(one)).cpu().numpy()
    np.testing.assert_array_equal(a1, OP.metropolis_judge(E_new[:, -1], E_new[:, :1], pcg1)[:, 0])
    np.testing.assert_array_equal(bmc.pcg.cpu().numpy().view(np.uint64), pcg1)
    np.testing.assert_allclose(bmc.E_old.cpu().numpy(), E_new[:, -1], rtol=1e-12)
    assert (bmc.attempts.cpu().numpy() == 1).all()
    np.testing.assert_array_equal(bmc.state.cpu().numpy(), init)


@pytest.mark.parametrize("tag", ["N16_f32", "N16_f64", "N64_f32", "N64_f64"])
def test_simulation_box_and_particle_energy_match_reference(tag):
    """SimulationBox.minimum_image / compute_distance / compute_distances and
    EnergyCalculator.calculate_particle_energy_virial on the device (fs_min_image,
    fs_particle_energy) against the reference's own outputs (tests/golden/box_trace.npz):
    bit-exact displacements and distances in the reference's dtype, energies within
    1e-12 (+inf on the hard core)."""
    from flowstate.MCMC import EnergyCalculator

    f = np.load(os.path.join(G, "box_trace.npz"))
    x = f[tag + "_x"]
    N = x.shape[0]
    L = float(f[tag + "_L"])
    box = SimulationBox(L, L)
    ij = f[tag + "_ij"]
    for k, (i, j) in enumerate(ij):
        d = box.minimum_image(x[i], x[j])
        assert d.dtype == (np.float32 if f[tag + "_delta_dtype_f32"] else np.float64)
        np.testing.assert_array_equal(d, f[tag + "_delta"][k])
        r = box.compute_distance(x[i], x[j])
        assert r == f[tag + "_dist"][k] and np.asarray(r).dtype == d.dtype
    for i in range(N):
        rows = box.compute_distances(x[i], np.delete(x, i, axis=0))
        assert rows.dtype == np.float64
        np.testing.assert_array_equal(rows, f[tag + "_rows"][i])
    ec = EnergyCalculator(N, x, box, num_wells=2, V0_list=[-10.0, -10.5], r0=1.2, k=15)
    for p in range(N):
        E, W = ec.calculate_particle_energy_virial(x, p)
        Er, Wr = f[tag + "_particle_ew"][p]
        assert _close(E, Er) and _close(W, Wr), (p, E, Er)
